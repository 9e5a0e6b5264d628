#!/bin/bash
# A/B of the two byte-key scan kernels (kernels.hip kModeByteKeys = ring,
# kModeByteDirect = direct) through the diagnostic build's YAMD_BYTE_DIRECT
# switch: scan kernel time per rule set, 4 GiB, rounds alternating the order.
#   bash tools/bytekey_ab.sh <rounds> "rx short fuzz0"
set -uo pipefail
ROUNDS=$1; SETS=$2
LIB=$PWD/yara_amd/_diag/libyara_amd.so
for r in $(seq 1 $ROUNDS); do
  for rules in $SETS; do
    for d in 0 1; do
      printf "%-6s direct=%s round %s  " "$rules" "$d" "$r"
      YARA_AMD_LIB=$LIB YAMD_BYTE_DIRECT=$d timeout -k 10 150 python tools/ablate.py --modes 0 \
        --rounds 3 --rules $rules 2>/dev/null | python -c "
import json, sys
d = json.load(sys.stdin); m = d['modes']['product']
print('median %.4f ms  min %.4f  candidates %d' % (m['median_ms'], m['min_ms'], m['candidates']))"
      rc=${PIPESTATUS[0]}
      if [ $rc -ne 0 ]; then exit $rc; fi
    done
  done
done
