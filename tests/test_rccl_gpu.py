"""The RCCL ("nccl" backend) code path of the multi-GPU shard
on the box's one GPU, world size 1.

bench.py at N > 1 initialises torch.distributed with backend "nccl" (= RCCL on
ROCm) and a device id, all-gathers counts as device tensors and gathers device
positions / records to rank 0 (yara_amd/dist.py).  The CPU tests cover the
same functions over gloo at world 2/3; this test makes sure the RCCL calls
themselves run on MI355X: a fresh child process (spawned, so the parent's HIP
state is not inherited) scans config C's planted buffer, gathers its
candidates and its pre-verified records through RCCL, and checks them against
the un-gathered device results (identity at world size 1).
"""
import os

import pytest

from conftest import case_data, golden, tables_npz

pytestmark = pytest.mark.gpu


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import numpy as np
    import torch
    import torch.distributed as dist
    import yara_amd
    from yara_amd import dist as ydist
    from yara_amd._hip import memcpy
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_backend() == "nccl"
        data = case_data(golden()["cases"]["C_planted16M"])
        n = data.size
        tables = yara_amd.Tables.from_npz(tables_npz("C"), device=0, strings=True)
        buf = torch.from_numpy(data.copy()).to(dev)
        torch.cuda.synchronize()
        sc = yara_amd.Scanner(tables)
        sc.scan_window(buf.data_ptr(), 0, n, n, 0, n)
        ptr, cnt, _ = sc.device_result()
        pos = torch.empty(max(cnt, 1), dtype=torch.int64, device=dev)
        memcpy(pos.data_ptr(), ptr, cnt * 8, 3)
        pos = pos[:cnt]
        # the bench's candidate gather: 32-bit offsets over RCCL
        g32 = ydist.gather_positions(pos, begins=[0], end=n)
        g64 = ydist.gather_positions(pos)
        ok_pos = (g32.device.type == "cuda" and torch.equal(g32, pos) and torch.equal(g64, pos))
        # the records path: {offset, pool index} rows
        rptr, nrec = sc.verify_device(0)
        rows = ydist.records_to_rows(rptr, nrec, dev)
        grows = ydist.gather_rows(rows)
        ok_rows = grows.device.type == "cuda" and torch.equal(grows, rows)
        want = sc.verify_calls(data)
        ok_ref = (np.array_equal(rows[:, 0].cpu().numpy(), want["offset"].astype(np.int64))
                  and np.array_equal(rows[:, 1].cpu().numpy(), want["pool_index"].astype(np.int64)))
        # the bench's per-rank attribution and timing reductions
        t = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
        parts = [torch.empty_like(t)]
        dist.all_gather(parts, t)
        m = torch.tensor([3.25], dtype=torch.float64, device=dev)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        ok_coll = torch.equal(parts[0], t) and float(m.item()) == 3.25
        q.put((bool(ok_pos), bool(ok_rows), bool(ok_ref), bool(ok_coll), int(cnt), int(nrec)))
    except Exception as e:   # report instead of hanging the parent
        q.put(("error", repr(e)))
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rccl_world1_gathers_are_identity():
    import torch.multiprocessing as mp
    if "C_planted16M" not in golden()["cases"]:
        pytest.skip("no golden case C_planted16M")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(29671, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] is True and all(res[:4]), res
    assert res[4] > 0 and res[5] > 0, res
    assert p.exitcode == 0, p.exitcode
