#!/bin/bash
# Per-kernel PMC detail of the scan kernel, one rocprofv3 --pmc pass per
# (counter set, kernel mode); no tracing domains.  Summarise with
#   python tools/pmc_modes.py gpurun_out/pmc_<tag>
#   bash tools/pmc_detail.sh <tag> [modes] [rules]   (modes: tools/ablate.py kernel variants, default 0;
#                                                     rules: a tests/golden/tables set, default C)
set -euo pipefail
TAG=${1:-detail}
MODES=${2:-0}
RULES=${3:-C}
OUT=gpurun_out/pmc_${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for m in ${MODES//,/ }; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $set -d $OUT/m${m}_p$i -o run --output-format csv -- \
      python3 tools/ablate.py --rules $RULES --modes $m --rounds 1 --reps 4 > $OUT/m${m}_p$i.log 2>&1
  done
done
find $OUT -name "*counter_collection.csv" | sort
