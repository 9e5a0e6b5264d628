#!/bin/bash
# Pre-verification time per rule set, triage pass (product library) against
# the count pass (diagnostic build with YAMD_TRIAGE_MIN above any count).
#   bash tools/triage_ab.sh "rx fuzz0 C"
set -uo pipefail
for r in $1; do
  printf "%-6s triage " "$r"
  timeout -k 10 120 python tools/verify_time.py --rules $r --reps 10 2>/dev/null | tail -1
  rc=${PIPESTATUS[0]}; if [ $rc -ne 0 ]; then exit $rc; fi
  printf "%-6s count  " "$r"
  YARA_AMD_LIB=$PWD/yara_amd/_diag/libyara_amd.so YAMD_TRIAGE_MIN=1000000000000 \
    timeout -k 10 120 python tools/verify_time.py --rules $r --reps 10 2>/dev/null | tail -1
  rc=${PIPESTATUS[0]}; if [ $rc -ne 0 ]; then exit $rc; fi
done
