"""Time on-device pre-verification (yr_amd_verify_device) of a device scan.

    python tools/verify_time.py [--rules C] [--gib 4] [--reps 10]

Prints the wall time per call (median) and the record count; with
YARA_AMD_LIB pointing at a diagnostic build, compares variants.
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rules", default="C")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    import yara_amd
    n = int(a.gib * (1 << 30))
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(buf.data_ptr(), n, 1)
    t = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables", a.rules + ".npz"),
                                 strings=True)
    sc = yara_amd.Scanner(t)
    sc.scan_device(buf.data_ptr(), n)
    _, cand, _ = sc.device_result()
    torch.cuda.synchronize()
    sc.verify_device(0)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        _, nrec = sc.verify_device(0)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"rules": a.rules, "bytes": n, "candidates": cand, "records": nrec,
                      "median_ms": round(statistics.median(ts), 4), "min_ms": round(min(ts), 4)}))


if __name__ == "__main__":
    main()
