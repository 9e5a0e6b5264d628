#!/bin/bash
# Live-list sort A/B: the verified path's GPU tests, then per-kernel times
# (rocprofv3) and one-process step times (ab_inproc, both orders) of the
# product against a variant.   bash tools/r6_live_ab.sh <tag> <variant> [sets]
set -euo pipefail
TAG=$1; VAR=$2; SETS=${3:-"fuzz0 rx fuzz3 short"}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_preverify.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/$TAG/tests.txt 2>&1
for r in $SETS; do
  bash tools/r6_prof_variants.sh $TAG $r base $VAR
  timeout -k 10 200 python tools/ab_inproc.py base,$VAR --rules $r --verified-only --rounds 10 --reps 3 > gpurun_out/$TAG/vo_$r.json 2>> gpurun_out/$TAG/err
  timeout -k 10 200 python tools/ab_inproc.py $VAR,base --rules $r --verified-only --rounds 10 --reps 3 > gpurun_out/$TAG/vo_${r}_rev.json 2>> gpurun_out/$TAG/err
done
