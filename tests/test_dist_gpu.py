"""Verification-complete shards on the GPU (SURVEY.md §8e, config D's path).

World-2/3 process groups (gloo) on the one GPU: every rank allocates ONLY its
window of the block -- its shard plus the tables' verify halos
(yr_amd_tables_info) -- runs the HIP scan (yr_amd_scan_window) and the
on-device pre-verification of its own candidates (yr_amd_verify_device), and
the {offset, pool index} records are gathered to rank 0.  Their rank-ordered
concatenation must equal the single-block pre-verification records, which the
other GPU tests pin to the reference's verify-call stream.
"""
import os

import numpy as np
import pytest

from conftest import case_data, golden, tables_npz

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, rules, case, align, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import yara_amd
    from yara_amd import dist as ydist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        data = case_data(golden()["cases"][case])
        n = data.size
        tables = yara_amd.Tables.from_npz(tables_npz(rules), device=0, strings=True)
        before, after = ydist.tables_halos(tables)
        begin, end = ydist.shard_bounds(n, world, rank, align=align)
        lo, hi = ydist.shard_window(n, begin, end, before, after)
        win = torch.empty(max(hi - lo, 16), dtype=torch.uint8, device="cuda")
        win[:hi - lo] = torch.from_numpy(data[lo:hi].copy()).cuda()
        torch.cuda.synchronize()
        sc = yara_amd.Scanner(tables)
        sc.scan_window(win.data_ptr(), lo, hi, n, begin, end)
        sc.device_result()
        ptr, cnt = sc.verify_device(0)
        rows = ydist.records_to_rows(ptr, cnt, "cuda")
        out = ydist.gather_rows(rows)
        if rank == 0:
            full = yara_amd.Scanner(tables).verify_calls(data)
            want = np.stack([full["offset"].astype(np.int64),
                             full["pool_index"].astype(np.int64)], 1)
            got = out.cpu().numpy()
            q.put((bool(got.shape == want.shape and np.array_equal(got, want)), int(len(want)),
                   int(lo), int(hi), int(before), int(after)))
    except Exception as e:   # report instead of hanging the parent
        if rank == 0:
            q.put((False, repr(e), 0, 0, 0, 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("rules,case,world,align", [
    ("lit", "lit_1M", 2, 1 << 16),
    ("hex", "hex_1M", 2, 1 << 16),
    ("rx", "rx_1M", 3, 1 << 16),
    ("C", "C_planted16M", 2, 1 << 20),
    ("E", "E_planted16M", 3, 1 << 20),
])
def test_sharded_preverify_gathers_full_records(rules, case, world, align):
    import torch.multiprocessing as mp
    if case not in golden()["cases"]:
        pytest.skip("no golden case %s" % case)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + world * 7 + sum(map(ord, case)) % 50
    ps = [ctx.Process(target=_worker, args=(r, world, port, rules, case, align, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = q.get(timeout=240)
    for p in ps:
        p.join(timeout=60)
    assert res[0], res
    assert res[1] > 0, res
