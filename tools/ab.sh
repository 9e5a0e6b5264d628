#!/bin/bash
# A/B of library builds (yara_amd/_variants/<name>.so; "base" = the product
# build): each round times every variant with tools/ablate.py (mode 0, one
# process per variant, 60 clock warm-up scans), rounds alternate the order.
#   bash tools/ab.sh <rounds> <rules> name1 name2 ...
set -euo pipefail
ROUNDS=$1; RULES=$2; shift 2
OUT=gpurun_out/ab; mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=$PWD/yara_amd/libyara_amd.so; else lib=$PWD/yara_amd/_variants/$v.so; fi
    YARA_AMD_LIB=$lib timeout -k 10 150 python tools/ablate.py --modes 0 --rounds 3 --rules $RULES \
      > $OUT/${RULES}_${v}_$r.json 2> $OUT/${RULES}_${v}_$r.err
    python - "$OUT/${RULES}_${v}_$r.json" "$v" "$r" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
m = d["modes"]["product"]
print("%-14s round %s  %s  median %.4f ms  min %.4f  candidates %d" % (sys.argv[2], sys.argv[3], d["rules"], m["median_ms"], m["min_ms"], m["candidates"]))
PY
  done
done
