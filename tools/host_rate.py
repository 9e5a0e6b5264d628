"""End-to-end rate of host-resident blocks (PCIe-inclusive; not the bench
metric, which times HBM-resident data).  Blocks of a host buffer go through
  (a) yr_amd_scan_block_verified, one block at a time, and
  (b) the block pipeline (yr_amd_pipeline_*) at several depths, with the
      host-memcpy submit and with the DMA submit (yr_amd_pipeline_submit_dma),
  (c) with --devices: the pipeline across N logical devices
      (yr_amd_pipeline_create_multi, DMA submit, depth 2; on a one-GPU box the
      N devices share its link) and the single-call multi-device scan of the
      whole buffer (yr_amd_multi_scan_block_verified: staged through pinned
      memory),
and the records are fetched to the host (the replay into yr_scan_verify_match
is the caller's and is not timed here).

    python tools/host_rate.py [--gib 2] [--block-mib 256] [--rules C] [--devices 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--block-mib", type=int, default=256)
    ap.add_argument("--rules", default="C")
    ap.add_argument("--depths", default="1,2,3")
    ap.add_argument("--devices", default="")
    ap.add_argument("--skip-single", action="store_true")
    a = ap.parse_args()
    import numpy as np
    import oracle
    import yara_amd
    from conftest import tables_npz
    n = int(a.gib * (1 << 30))
    data = oracle.xorshift(n, 1)
    bs = a.block_mib << 20
    blocks = [(b, data[b:b + bs]) for b in range(0, n, bs)]
    tab = yara_amd.Tables.from_npz(tables_npz(a.rules), device=0, strings=True)
    sc = yara_amd.Scanner(tab)
    sc.verify_calls(blocks[0][1])
    res = {"bytes": n, "block_bytes": bs, "rules": a.rules}
    dst = np.empty(bs, np.uint8)
    np.copyto(dst, blocks[0][1])
    t0 = time.perf_counter()
    for _ in range(4):
        np.copyto(dst, blocks[1][1])
    res["host_memcpy_GBps"] = round(4 * bs / (time.perf_counter() - t0) / 1e9, 2)
    t0 = time.perf_counter()
    tot = 0
    for b, blk in blocks:
        tot += len(sc.verify_calls(blk, data_base=b))
    res["single_block_GBps"] = round(n / (time.perf_counter() - t0) / 1e9, 2)
    res["records"] = tot
    for dma in (() if a.skip_single else (False, True)):
        for depth in [int(x) for x in a.depths.split(",")]:
            pipe = yara_amd.Pipeline(tab, depth=depth)

            def run():
                inflight, tot2 = 0, 0
                for b, blk in blocks:
                    if inflight == depth:
                        tot2 += len(pipe.next(copy_data=False)[0])
                        inflight -= 1
                    pipe.submit(blk, base=b, dma=dma)
                    inflight += 1
                while inflight:
                    tot2 += len(pipe.next(copy_data=False)[0])
                    inflight -= 1
                return tot2
            run()   # steady state: slot buffers and device workspaces allocated
            t0 = time.perf_counter()
            tot2 = run()
            key = "pipeline%s_depth%d_GBps" % ("_dma" if dma else "", depth)
            res[key] = round(n / (time.perf_counter() - t0) / 1e9, 2)
            assert tot2 == tot
            pipe.close()
    for nd in [int(x) for x in a.devices.split(",") if x]:
        tabs = [tab] + [yara_amd.Tables.from_npz(tables_npz(a.rules), device=0, strings=True)
                        for _ in range(nd - 1)]
        pipe = yara_amd.Pipeline(tabs if nd > 1 else tab, depth=2)

        def run_multi():
            inflight, tot2 = 0, 0
            for b, blk in blocks:
                if inflight == 2:
                    tot2 += len(pipe.next(copy_data=False)[0])
                    inflight -= 1
                pipe.submit(blk, base=b, dma=True)
                inflight += 1
            while inflight:
                tot2 += len(pipe.next(copy_data=False)[0])
                inflight -= 1
            return tot2
        run_multi()
        t0 = time.perf_counter()
        tot2 = run_multi()
        res["multi_pipeline_dma_n%d_GBps" % nd] = round(n / (time.perf_counter() - t0) / 1e9, 2)
        assert tot2 == tot, (tot2, tot)
        pipe.close()
        m = yara_amd.Multi(tabs)
        whole = len(m.verify_calls(data))
        t0 = time.perf_counter()
        whole = len(m.verify_calls(data))
        res["multi_whole_n%d_GBps" % nd] = round(n / (time.perf_counter() - t0) / 1e9, 2)
        res["multi_whole_records"] = whole
        m.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
