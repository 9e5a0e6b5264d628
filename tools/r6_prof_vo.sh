#!/bin/bash
# Per-kernel times of the verified-only step of short/fuzz3 for the product
# build and a variant (rocprofv3 --kernel-trace --stats over tools/verified_step.py)
#   bash tools/r6_prof_vo.sh <tag> <variant> [sets]
set -e
TAG=$1; VAR=$2; SETS=${3:-"short fuzz3"}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for r in $SETS; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/base_$r -o run --output-format csv -- python3 tools/verified_step.py $r > gpurun_out/$TAG/base_$r.txt 2>&1
  YARA_AMD_LIB=$PWD/yara_amd/_variants/$VAR.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/${VAR}_$r -o run --output-format csv -- python3 tools/verified_step.py $r > gpurun_out/$TAG/${VAR}_$r.txt 2>&1
done
