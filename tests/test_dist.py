"""Multi-rank sharding + candidate gather on CPU (gloo, world size 2 and 3).

Each rank scans only its shard (plus the warm-up halo) with the CPU oracle
standing in for the per-GPU scan; the gathered, rank-ordered lists must equal
the single-process candidate stream of the whole block -- including atoms that
straddle a shard boundary.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from conftest import ref_tables
from yara_amd import dist as ydist


def _shard_candidates(tab, data, begin, end):
    lo, _ = ydist.shard_window(len(data), begin, end)
    cand = oracle.candidates(tab, data[lo:end]).astype(np.int64) + lo
    return cand[cand > begin] if begin > 0 else cand   # position 0 only on rank 0


def _worker(rank, world, port, n, period, q, no_gather=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if no_gather:                      # the all_gather path of gather_rows
        ydist._gather_backend = lambda group: "all_gather"
    try:
        import planted
        import gen_rules
        tab = ref_tables("C")
        atoms = [b for b, _ in planted.string_instances(gen_rules.gen("C")) if len(b) >= 4][:64]
        data = planted.boundary_buffer(oracle.xorshift, atoms, n, period)
        b, e = ydist.shard_bounds(n, world, rank, align=period)
        local = torch.from_numpy(_shard_candidates(tab, data, b, e))
        out = ydist.gather_positions(local)
        # 32-bit offsets from each rank's shard begin (bench.py's N > 1 gather)
        begins = [ydist.shard_bounds(n, world, r, align=period)[0] for r in range(world)]
        out32 = ydist.gather_positions(local, begins=begins, end=n)
        # two-column rows (the records path: {offset, pool index})
        rows = torch.stack([local, local * 3 + rank], 1)
        out2 = ydist.gather_rows(rows)
        if rank == 0:
            full = oracle.candidates(tab, data).astype(np.int64)
            ok = bool(np.array_equal(out.numpy(), full)) and out.numel() > 0
            ok &= bool(np.array_equal(out32.numpy(), full))
            ok &= tuple(out2.shape) == (full.size, 2)
            ok &= bool(np.array_equal(out2[:, 0].numpy(), full))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,no_gather", [(2, False), (3, False), (2, True)])
def test_sharded_scan_gathers_full_stream(world, no_gather):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29400 + world + (10 if no_gather else 0)
    n, period = (3 << 20) + 77, 1 << 16
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, period, q, no_gather))
          for r in range(world)]
    for p in ps:
        p.start()
    ok = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
    assert ok


def _edge_worker(rank, world, port, q):
    """Synthetic positions at every shard's edges (rank 0: position 0), gathered
    as 32-bit offsets to a dst other than rank 0, and a block whose shards
    exceed 2^32 positions (the int64 fallback) -- ADVICE r04."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = True
        for n in ((3 << 20) + 77, (9 << 30) + 5, (8 << 32) + 3):
            bounds = [ydist.shard_bounds(n, world, r) for r in range(world)]
            begins = [b for b, _ in bounds]
            b, e = bounds[rank]
            lo = 0 if rank == 0 else b + 1
            local = torch.tensor(sorted({lo, lo + 1, (lo + e) // 2, e - 1, e}), dtype=torch.int64)
            for dst in range(world):
                out = ydist.gather_positions(local, dst=dst, begins=begins, end=n)
                if rank == dst:
                    want = []
                    for r, (rb, re_) in enumerate(bounds):
                        rl = 0 if r == 0 else rb + 1
                        want += sorted({rl, rl + 1, (rl + re_) // 2, re_ - 1, re_})
                    ok &= out.tolist() == want
                else:
                    ok &= out is None
        # only the last rank's input is bad: every rank must raise, none may be
        # left waiting in the collective
        n = 1 << 20
        bounds = [ydist.shard_bounds(n, world, r, align=16) for r in range(world)]
        good = 0 if rank == 0 else bounds[rank][0] + 1
        with_bad = torch.tensor([1 << 40 if rank == world - 1 else good], dtype=torch.int64)
        try:
            ydist.gather_positions(with_bad, begins=[b for b, _ in bounds], end=n)
            ok = False
        except ValueError:
            pass
        # and the group is still usable afterwards
        ok &= ydist.gather_positions(torch.tensor([good], dtype=torch.int64),
                                     begins=[b for b, _ in bounds], end=n,
                                     dst=0) is not None or rank != 0
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_positions_edges_and_large_shards(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29440 + world
    ps = [ctx.Process(target=_edge_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(res.values()), res


def test_shard_bounds_cover_block():
    for n in (0, 15, 1 << 20, (8 << 30) + 12345):
        for world in (1, 2, 3, 8):
            prev = 0
            for r in range(world):
                b, e = ydist.shard_bounds(n, world, r, align=16)
                assert b == prev and b % 16 == 0 and e >= b
                prev = e
            assert prev == n


def test_shard_window_halos():
    n = 10 << 20
    # candidates only: 4-byte warm-up, 16-aligned
    assert ydist.shard_window(n, 0, 1 << 20) == (0, 1 << 20)
    assert ydist.shard_window(n, 1 << 20, 2 << 20) == ((1 << 20) - 16, 2 << 20)
    # verification-complete: halos before/after, clipped to the block
    lo, hi = ydist.shard_window(n, 1 << 20, 2 << 20, 4096 + 16, 4096)
    assert lo % 16 == 0 and lo <= (1 << 20) - 4096 - 16 and hi == (2 << 20) + 4096
    assert ydist.shard_window(n, 9 << 20, n, 5000, 5000) == (((9 << 20) - 5000) // 16 * 16, n)
    with pytest.raises(ValueError):
        ydist.shard_window(n, 5, 4)
