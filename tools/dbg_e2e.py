import sys, subprocess, os
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo/tests/golden')
import numpy as np, oracle, planted, gen_rules
os.makedirs('gpurun_out', exist_ok=True)
open('gpurun_out/B.yar','w').write(gen_rules.gen('B'))
planted.planted_buffer(oracle.xorshift, gen_rules.gen('B'), 16<<20, 3).tofile('gpurun_out/b16.bin')
for i in range(2):
    r = subprocess.run(['integration/_build/e2e_check','gpurun_out/B.yar','gpurun_out/b16.bin'], capture_output=True, text=True)
    print(r.returncode, r.stdout, r.stderr[-2000:])
