#!/bin/bash
# Per-kernel times of the verified path of the dense rule sets (rocprofv3
# --kernel-trace --stats over tools/verified_step.py), then the rule-set rates
# (full vs verified-only).  Outputs under gpurun_out/<tag>/.
#   bash tools/r5_prof_verified.sh <tag> [sets]
set -e
TAG=${1:-r5prof}
SETS=${2:-"rx fuzz0 short fuzz3"}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for r in $SETS; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/$r -o run --output-format csv -- python3 tools/verified_step.py $r > gpurun_out/$TAG/$r.txt 2>&1
done
timeout -k 10 400 python -u tools/ruleset_rates.py --sets $(echo $SETS | tr ' ' ','),C --reps 10 > gpurun_out/$TAG/rates.json 2> gpurun_out/$TAG/rates.err
