import os, sys, time, json, statistics
sys.path.insert(0, os.getcwd())
import torch, yara_amd
n = 4 << 30
buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
yara_amd.fill_xorshift64(buf.data_ptr(), n, 1)
torch.cuda.synchronize()
out = {}
for name in sys.argv[1].split(","):
    t = yara_amd.Tables.from_npz(os.path.join("tests", "golden", "tables", name + ".npz"), device=0)
    sc = yara_amd.Scanner(t)
    ts = []
    for i in range(25):
        t0 = time.perf_counter()
        sc.scan_device(buf.data_ptr(), n)
        _, c, _ = sc.device_result()
        ts.append((time.perf_counter() - t0) * 1e3)
    out[name] = {"first_ms": round(ts[0], 3), "median_ms_scan_plus_result": round(statistics.median(ts[5:]), 4), "candidates": int(c)}
print(json.dumps(out))
