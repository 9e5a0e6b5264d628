"""HBM write and copy rates for the record sizes of the verified path (16.8 M
records of 16 B = 269 MB written): what floor the write pass
(verify.hip verify_write_kernel, 110-117 us on short / fuzz3) has.
    python tools/microbench/write_bw.py
"""
import json

import torch


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3   # us


def main():
    n = 16_841_229 * 16
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    src = torch.empty(16_972_791 * 9, dtype=torch.uint8, device="cuda")
    out = {}
    out["fill_269MB_us"] = timed(lambda: dst.fill_(7))
    out["fill_GBps"] = n / out["fill_269MB_us"] / 1e3
    s2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    out["copy_269MB_us"] = timed(lambda: dst.copy_(s2))
    out["copy_GBps_rw"] = 2 * n / out["copy_269MB_us"] / 1e3
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
