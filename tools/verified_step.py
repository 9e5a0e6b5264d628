"""The verified path of one rule set, repeated (for rocprofv3 --kernel-trace
--stats: per-kernel times of the scan, the compaction and pre-verification).

    python tools/verified_step.py <rules> [--gib 4] [--reps 20] [--full]

A scan of the canonical input (seed 1) resident in HBM, its result, and
yr_amd_verify_device, --reps times after a clock warm-up; verified-only scans
unless --full.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rules")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--full", action="store_true")
    a = ap.parse_args()
    import torch
    import yara_amd
    n = int(a.gib * (1 << 30))
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(buf.data_ptr(), n, 1)
    t = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables", a.rules + ".npz"),
                                 device=0, strings=True)
    sc = yara_amd.Scanner(t)
    sc.set_verified_only(not a.full)
    for _ in range(60):
        sc.scan_device(buf.data_ptr(), n)
        sc.device_result()
        sc.verify_device(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        sc.scan_device(buf.data_ptr(), n)
        _, cnt, _ = sc.device_result()
        _, nrec = sc.verify_device(0)
    dt = (time.perf_counter() - t0) / a.reps * 1e3
    print("%s %s: %.4f ms per verified step, %d candidates (stream %d), %d records"
          % (a.rules, "full" if a.full else "verified-only", dt, cnt, sc.stream_length(), nrec))


if __name__ == "__main__":
    main()
