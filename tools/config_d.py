"""Config D (32 GiB, 10k atoms, 8 GPUs) rehearsed on one MI355X.

The whole 32 GiB block is resident in one GPU's HBM (288 GB), scanned and
pre-verified in one piece; then each of the 8 ranks' windows (shard + verify
halos, yara_amd/dist.py, exactly what `bench.py --gpus 8` allocates per rank)
is generated, scanned and pre-verified on its own.  The ranks' candidates and
{offset, pool index} records, concatenated in rank order, must equal the whole
block's (what rank 0 gathers over RCCL), and the first 4 GiB's candidates the
golden C_4G stream.  Per-rank kernel and pre-verification times are the
single-GPU part of the 8-GPU step.

    python tools/config_d.py [--gib 32] [--world 8] > config_d.json
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
GiB = 1 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=32)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    import yara_amd
    from yara_amd import dist as ydist
    from yara_amd._hip import d2h_u64, memcpy
    import oracle

    total = a.gib * GiB
    tables = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables", "C.npz"),
                                      device=0, strings=True)

    def records(sc):
        ptr, n = sc.verify_device(0)
        h = torch.empty(max(n, 1) * 16, dtype=torch.uint8, device="cuda")
        memcpy(h.data_ptr(), ptr, n * 16, 3)
        r = np.frombuffer(h[:n * 16].cpu().numpy().tobytes(), dtype=yara_amd._lib.VERIFY_REC_DTYPE)
        return r["offset"].copy(), r["pool_index"].copy()

    def timed(sc, launch, reps):
        sc.set_timing(True)
        ks, vs = [], []
        for _ in range(reps):
            launch()
            sc.device_result()
            ks.append(sc.kernel_ms())
            t0 = time.perf_counter()
            sc.verify_device(0)
            vs.append((time.perf_counter() - t0) * 1e3)
        sc.set_timing(False)
        return statistics.median(ks), statistics.median(vs)

    # the whole block on one GPU
    buf = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(buf.data_ptr(), total, 1)
    torch.cuda.synchronize()
    sc = yara_amd.Scanner(tables)
    for _ in range(10):   # clock ramp
        sc.scan_device(buf.data_ptr(), min(total, 4 * GiB))
        sc.device_result()
    sc.scan_device(buf.data_ptr(), total)
    ptr, cnt, _ = sc.device_result()
    full_pos = d2h_u64(ptr, cnt)
    full_off, full_idx = records(sc)
    k_full, v_full = timed(sc, lambda: sc.scan_device(buf.data_ptr(), total), 3)
    del buf, sc
    torch.cuda.empty_cache()

    golden = json.load(open(os.path.join(REPO, "tests", "golden", "golden.json")))["cases"]["C_4G"]
    head = full_pos[full_pos <= golden["size"]]
    out = {"what": __doc__.strip().splitlines()[0], "block_bytes": total, "world": a.world,
           "whole_block": {"candidates": int(cnt), "records": int(len(full_off)),
                           "kernel_ms": round(k_full, 3), "verify_ms": round(v_full, 3),
                           "first_4GiB_equals_golden_C_4G":
                               bool(len(head) == golden["candidate_count"] and
                                    oracle.positions_sha(head) == golden["candidate_sha"])},
           "ranks": []}

    before, after = ydist.tables_halos(tables)
    pos_parts, off_parts, idx_parts = [], [], []
    for r in range(a.world):
        begin, end = ydist.shard_bounds(total, a.world, r)
        lo, hi = ydist.shard_window(total, begin, end, before, after)
        w = torch.empty(hi - lo + 16, dtype=torch.uint8, device="cuda")
        yara_amd.fill_xorshift64(w.data_ptr(), hi - lo, 1, lo)
        torch.cuda.synchronize()
        s = yara_amd.Scanner(tables)
        launch = lambda: s.scan_window(w.data_ptr(), lo, hi, total, begin, end)   # noqa: E731
        for _ in range(5):
            launch()
            s.device_result()
        launch()
        p, c, _ = s.device_result()
        pos_parts.append(d2h_u64(p, c))
        o, i = records(s)
        off_parts.append(o)
        idx_parts.append(i)
        k, v = timed(s, launch, a.reps)
        out["ranks"].append({"rank": r, "shard": [begin, end], "window": [lo, hi],
                             "window_bytes": hi - lo, "candidates": int(c), "records": int(len(o)),
                             "kernel_ms": round(k, 4), "GB/s": round((end - begin) / (k * 1e-3) / 1e9, 1),
                             "verify_ms": round(v, 4)})
        del w, s
        torch.cuda.empty_cache()
        print("rank %d done" % r, file=sys.stderr, flush=True)

    out["sharded_equals_whole"] = {
        "candidates": bool(np.array_equal(np.concatenate(pos_parts), full_pos)),
        "records": bool(np.array_equal(np.concatenate(off_parts), full_off) and
                        np.array_equal(np.concatenate(idx_parts), full_idx))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
