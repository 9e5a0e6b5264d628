#!/bin/bash
# Per-kernel times of one rule set's verified-only step under several builds
# (rocprofv3 --kernel-trace --stats over tools/verified_step.py; "base" = the
# product, others yara_amd/_variants/<name>.so)
#   bash tools/r6_prof_variants.sh <tag> <rules> name...
set -e
TAG=$1; R=$2; shift 2
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in "$@"; do
  if [ "$v" = base ]; then lib=$PWD/yara_amd/libyara_amd.so; else lib=$PWD/yara_amd/_variants/$v.so; fi
  YARA_AMD_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/${v}_$R -o run --output-format csv -- python3 tools/verified_step.py $R > gpurun_out/$TAG/${v}_$R.txt 2>&1
done
