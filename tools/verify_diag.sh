#!/bin/bash
# Pre-verification time per rule set for the product build and the
# YAMD_VERIFY_DIAG profiling builds (yara_amd/_variants/vd<N>.so, built with
# make -C yara_amd/csrc OUT=../_variants/vdN.so OBJDIR=../_build_vdN EXTRA=-DYAMD_VERIFY_DIAG=N):
#   bash tools/verify_diag.sh "rx fuzz0 C" base vd1 vd2 vd3 vd4
set -uo pipefail
SETS=$1; shift
for r in $SETS; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=$PWD/yara_amd/libyara_amd.so; else lib=$PWD/yara_amd/_variants/$v.so; fi
    printf "%-6s %-5s " "$r" "$v"
    YARA_AMD_LIB=$lib timeout -k 10 120 python tools/verify_time.py --rules $r --reps 10 2>/dev/null | tail -1
  done
done
