#!/bin/bash
# Time build variants of the scan kernel (yara_amd/_variants/<name>.so, built by
# make -C yara_amd/csrc OUT=../_variants/<name>.so OBJDIR=../_build_<name> EXTRA=...)
# with tools/ablate.py, one process per variant.
#   bash tools/variants.sh "<modes>" name1 name2 ...     (name "base" = the product build)
set -euo pipefail
MODES=$1; shift
mkdir -p gpurun_out/variants
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/yara_amd/_variants/$v.so; fi
  YARA_AMD_LIB=$lib timeout -k 10 120 python tools/ablate.py --modes $MODES --rounds 3 \
    > gpurun_out/variants/$v.json 2> gpurun_out/variants/$v.err
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open("gpurun_out/variants/%s.json" % v))
print(v, {k: (m["median_ms"], m["candidates"]) for k, m in d["modes"].items()})
PY
done
