#!/bin/bash
# End-to-end scan time, stock libyara vs the GPU shim (same libyara, same rules,
# same bytes; match sets compared by e2e_check), with the GPU side's wall time
# split (yr_gpu_scanner_timing): host copy into the pipeline's pinned staging,
# waiting for the GPU (H2D + scan + pre-verification + records D2H), and the
# host replay of the records into yr_scan_verify_match / re.c.
#   bash tools/e2e_rate.sh <out_dir> [sets] [size] [block]
#     sets: golden rule sets (tests/golden/rules/*.yar, B/C/E, fuzzN), default
#           "short fuzz3 fuzz0 lit rx C"; size default 1 GiB of xorshift seed 1;
#           block: 0 = one scan_mem block (the direct path), else the block
#           iterator with blocks of that many bytes (the pipeline)
set -euo pipefail
OUT=${1:-gpurun_out/e2e_rate}
SETS=${2:-"short fuzz3 fuzz0 lit rx C"}
SIZE=${3:-1073741824}
BLOCK=${4:-0}
mkdir -p $OUT
python3 - "$OUT" $SETS <<'PY'
import os, shutil, sys
sys.path.insert(0, "tests/golden")
import fuzz_rules, gen_rules
out = sys.argv[1]
for n in sys.argv[2:]:
    p = os.path.join("tests", "golden", "rules", n + ".yar")
    if os.path.exists(p):
        shutil.copy(p, os.path.join(out, n + ".yar"))
    elif n.startswith("fuzz"):
        open(os.path.join(out, n + ".yar"), "w").write(fuzz_rules.gen(int(n[4:])))
    else:
        open(os.path.join(out, n + ".yar"), "w").write(gen_rules.gen(n))
PY
for r in $SETS; do
  if [ "$BLOCK" = 0 ]; then args=""; else args="$BLOCK 0"; fi
  E2E_REPEAT=2 timeout -k 10 600 integration/_build/e2e_check $OUT/$r.yar xs:1:$SIZE $args \
    > $OUT/${r}_b${BLOCK}.json
  echo "$r block=$BLOCK $(cat $OUT/${r}_b${BLOCK}.json)"
done
