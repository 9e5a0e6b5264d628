#!/bin/bash
# Profile the benchmark on the GPU box: kernel trace + stats (rocprofv3), then a
# separate PMC pass for HBM traffic of the scan kernel (FETCH_SIZE; see
# MI355X_MICROARCH.md "HBM": double it for wide coalesced reads on gfx950).
#   bash tools/profile_round.sh <tag>
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --no-cpu --no-other > $OUT/bench_under_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 20 --no-cpu --no-other > $OUT/bench_under_pmc.log 2>&1
find $OUT -name "*.csv" | head -20
