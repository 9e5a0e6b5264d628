set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_preverify.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/r6e/tests.txt 2>&1 || exit 1
for r in short fuzz3 rx fuzz0; do
  timeout -k 10 200 python tools/ab_inproc.py head,base --rules $r --verified-only --rounds 10 --reps 3 > gpurun_out/r6e/vo_$r.json 2>> gpurun_out/r6e/err || exit 2
  timeout -k 10 200 python tools/ab_inproc.py base,head --rules $r --verified-only --rounds 10 --reps 3 > gpurun_out/r6e/vo_${r}_rev.json 2>> gpurun_out/r6e/err || exit 3
done
