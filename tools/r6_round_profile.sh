#!/bin/bash
# Round-6 measurement set: the default bench line, the kernel trace + FETCH_SIZE
# pass (tools/profile_round.sh), the SQ/LDS counter mix of the product kernel
# (tools/pmc_detail.sh) and the ablation ladder (tools/ablate.py).
#   bash tools/r6_round_profile.sh <tag>
set -euo pipefail
TAG=$1
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
bash tools/profile_round.sh $TAG
bash tools/pmc_detail.sh $TAG 0 C
python3 tools/pmc_modes.py gpurun_out/pmc_$TAG --out gpurun_out/$TAG/pmc_detail.json
timeout -k 10 300 python3 tools/ablate.py --rules C --modes 0,3,2,7 --rounds 5 --reps 5 > gpurun_out/$TAG/ablation.json 2> gpurun_out/$TAG/ablation.err
