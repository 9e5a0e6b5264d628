#!/bin/bash
# Marginal cost of one instruction per tile step of the product scan kernel,
# by issue class (VERDICT r05 item 2's stage-2 cost model): variant builds that
# add N instructions of one class to every tile step (kernels.hip YAMD_PAD_*,
# four independent dummy chains), timed in one process against the product
# (tools/ab_inproc.py, orders alternating every round).
#   build (here):  bash tools/stage2_cost.sh build
#   run (GPU box): bash tools/stage2_cost.sh run <out.json>
set -euo pipefail
cd "$(dirname "$0")/.."
VARS="pad16v2:-DYAMD_PAD_VOP2=16 pad8v3:-DYAMD_PAD_VOP3=8 pad16s:-DYAMD_PAD_SALU=16 pad8nop:-DYAMD_PAD_NOP=8"
if [ "$1" = build ]; then
  for v in $VARS; do
    n=${v%%:*}; f=${v#*:}
    make -s -C yara_amd/csrc OUT=../_variants/$n.so OBJDIR=../_build_v_$n EXTRA="$f" &
  done
  wait
else
  timeout -k 10 300 python tools/ab_inproc.py base,pad16v2,pad8v3,pad16s,pad8nop --rules C --rounds 16 --reps 5 > "$2"
fi
