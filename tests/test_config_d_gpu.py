"""Config D (the 10k-string rule set over a 32 GiB block,
8 GPUs) at full size on the one GPU of the box.

The whole 32 GiB block is resident in one MI355X's HBM and scanned +
pre-verified in one piece; then each of the 8 ranks' windows -- shard plus
the rule set's verify halos, exactly what `bench.py --gpus 8` allocates per
rank (yara_amd/dist.py) -- is generated, scanned and pre-verified on its own.

  * every rank's candidate stream equals the per-shard golden
    (tests/golden/config_d.json: count and SHA-256 of its positions; shard 0
    is the stock golden C_4G);
  * the ranks' candidates and {offset, pool index} records, concatenated in
    rank order (what rank 0 gathers over RCCL), equal the whole block's.
"""
import json
import os

import numpy as np
import pytest

import oracle
import yara_amd
from conftest import GOLDEN, tables_npz

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

GiB = 1 << 30
WORLD = 8


def _records(sc):
    import torch
    from yara_amd._hip import memcpy
    ptr, n = sc.verify_device(0)
    h = torch.empty(max(n, 1) * 16, dtype=torch.uint8, device="cuda")
    memcpy(h.data_ptr(), ptr, n * 16, 3)
    r = np.frombuffer(h[:n * 16].cpu().numpy().tobytes(), dtype=yara_amd._lib.VERIFY_REC_DTYPE)
    return r["offset"].copy(), r["pool_index"].copy()


def test_config_d_windows_equal_whole_block_and_goldens():
    import torch
    from yara_amd import dist as ydist
    from yara_amd._hip import d2h_u64

    with open(os.path.join(GOLDEN, "config_d.json")) as f:
        gold = json.load(f)
    shard = gold["shard_bytes"]
    total = WORLD * shard
    if torch.cuda.mem_get_info()[0] < total + 12 * GiB:
        pytest.skip("needs ~44 GiB of free HBM")
    tables = yara_amd.Tables.from_npz(tables_npz("C"), device=0, strings=True)

    buf = torch.empty(total + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(buf.data_ptr(), total, gold["seed"])
    torch.cuda.synchronize()
    sc = yara_amd.Scanner(tables)
    sc.scan_device(buf.data_ptr(), total)
    ptr, cnt, _ = sc.device_result()
    full_pos = d2h_u64(ptr, cnt)
    full_off, full_idx = _records(sc)
    del buf, sc
    torch.cuda.empty_cache()
    assert cnt == sum(s["count"] for s in gold["shards"])

    before, after = ydist.tables_halos(tables)
    pos_parts, off_parts, idx_parts = [], [], []
    for r in range(WORLD):
        begin, end = ydist.shard_bounds(total, WORLD, r)
        assert (begin, end) == (r * shard, (r + 1) * shard)
        lo, hi = ydist.shard_window(total, begin, end, before, after)
        w = torch.empty(hi - lo + 16, dtype=torch.uint8, device="cuda")
        yara_amd.fill_xorshift64(w.data_ptr(), hi - lo, gold["seed"], lo)
        torch.cuda.synchronize()
        s = yara_amd.Scanner(tables)
        s.scan_window(w.data_ptr(), lo, hi, total, begin, end)
        p, c, _ = s.device_result()
        pos = d2h_u64(p, c)
        assert c == gold["shards"][r]["count"], r
        assert oracle.positions_sha(pos) == gold["shards"][r]["sha"], r
        pos_parts.append(pos)
        o, i = _records(s)
        off_parts.append(o)
        idx_parts.append(i)
        del w, s
        torch.cuda.empty_cache()

    np.testing.assert_array_equal(np.concatenate(pos_parts), full_pos)
    np.testing.assert_array_equal(np.concatenate(off_parts), full_off)
    np.testing.assert_array_equal(np.concatenate(idx_parts), full_idx)
    assert len(full_off) > 0
