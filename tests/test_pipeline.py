"""Block pipeline (yr_amd_pipeline_*): blocks come back in
submission order with exactly the records of the one-block-at-a-time path
(yr_amd_scan_block_verified), whatever the depth, block sizes and interleaving
of submit / next."""
import numpy as np
import pytest

import oracle
import planted
from conftest import tables_npz

pytestmark = pytest.mark.gpu


def _blocks(data, sizes):
    out, b = [], 0
    for n in sizes:
        out.append((b, data[b:b + n]))
        b += n
    return out


@pytest.mark.parametrize("dma", [False, True], ids=["memcpy", "dma"])
@pytest.mark.parametrize("depth", [1, 2, 4])
def test_pipeline_equals_single_block_path(depth, dma):
    """Either submit form (host memcpy, or H2D from the caller's buffer with
    the host copy made by D2H into pinned memory): the same records and block
    copies; the caller's buffer is overwritten right after each submit (it
    may be reused on return)."""
    import yara_amd
    data = planted.lit_buffer(oracle.xorshift, 3 << 20, 13)
    tab = yara_amd.Tables.from_npz(tables_npz("lit"), device=0, strings=True)
    sc = yara_amd.Scanner(tab)
    rng = np.random.default_rng(depth)
    sizes = [int(x) for x in rng.integers(0, 300_000, 14)] + [0, 1, 17]
    blocks = _blocks(data, sizes)
    want = [sc.verify_calls(blk, data_base=b) for b, blk in blocks]
    pipe = yara_amd.Pipeline(tab, depth=depth)
    got, inflight = [], 0
    scratch = np.empty(max(sizes), np.uint8)
    for b, blk in blocks:
        if inflight == depth:
            got.append(pipe.next())
            inflight -= 1
        scratch[:len(blk)] = blk                    # the caller's reusable buffer
        pipe.submit(scratch[:len(blk)], base=b, dma=dma)
        scratch[:len(blk)] = 0x5A
        inflight += 1
    while inflight:
        got.append(pipe.next())
        inflight -= 1
    assert len(got) == len(blocks)
    for (b, blk), w, (recs, copy, base) in zip(blocks, want, got):
        assert base == b and np.array_equal(copy, blk)
        assert np.array_equal(recs, w)


def test_pipeline_limits_and_drain():
    import yara_amd
    tab = yara_amd.Tables.from_npz(tables_npz("lit"), device=0, strings=True)
    pipe = yara_amd.Pipeline(tab, depth=2)
    with pytest.raises(yara_amd.YaraAmdError):
        pipe.next()                       # nothing in flight
    blk = oracle.xorshift(1 << 16, 3)
    pipe.submit(blk)
    pipe.submit(blk)
    with pytest.raises(yara_amd.YaraAmdError):
        pipe.submit(blk)                  # depth exceeded
    pipe.drain()
    pipe.submit(blk, base=5)
    recs, copy, base = pipe.next()
    assert base == 5 and np.array_equal(copy, blk)
