set -e
mkdir -p gpurun_out/ab_carry2
bash tools/variants.sh "0" base carry2 base carry2 base carry2 > gpurun_out/ab_carry2/variants.txt 2>&1
for i in 1 2 3; do
  for v in base carry2; do
    if [ $v = base ]; then lib=""; else lib=$PWD/yara_amd/_variants/$v.so; fi
    YARA_AMD_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/ab_carry2/bench_${v}_$i.json 2>/dev/null
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['roofline']['kernel_ms_avg'], d['ms_per_step'], d['verified_step']['ms_per_step'], {k:v['kernel_ms'] for k,v in d['other_rule_sets'].items()})" gpurun_out/ab_carry2/bench_${v}_$i.json $v | tee -a gpurun_out/ab_carry2/bench.txt
  done
done
cat gpurun_out/ab_carry2/variants.txt
