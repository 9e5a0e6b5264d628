"""Multi-device block scans behind the C ABI (yr_amd_multi_*).

One process, n logical devices -- here all on the one GPU of the box, each
with its own copy of the tables, stream and scanner, as on an 8-GPU node: a
block is split into per-device windows (shard + the rule set's verify halos),
every device scans and pre-verifies only its window, and the records,
concatenated in device order, must equal the single-device records of the
whole block (yr_amd_scan_block_verified), call for call, candidate indices
included.  The single-device records are themselves pinned to the stock
reference's verify-call stream (test_preverify.py, test_gpu_fuzz.py).
"""
import ctypes

import numpy as np
import pytest

import gen_rules
import oracle
import planted
import yara_amd
from conftest import tables_npz
from yara_amd import _lib

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _data(kind, size):
    if kind == "planted_C":
        return planted.planted_buffer(oracle.xorshift, gen_rules.gen("C"), size, 3)
    if kind == "planted_E":
        return planted.planted_buffer(oracle.xorshift, gen_rules.gen("E"), size, 3)
    if kind == "lit":
        return planted.lit_buffer(oracle.xorshift, size, 13)
    if kind == "hex":
        return planted.hex_buffer(oracle.xorshift, size, 17)
    if kind == "rx":
        return planted.rx_buffer(oracle.xorshift, size, 19)
    if kind == "alpha":
        x = oracle.xorshift(size, 5)
        return np.frombuffer(b"abcdxyzHeloC\x00\x01\xff", np.uint8)[x % 15]
    raise ValueError(kind)


_CACHE = {}


def _tables(rules, n):
    key = (rules, n)
    if key not in _CACHE:
        _CACHE[key] = [yara_amd.Tables.from_npz(tables_npz(rules), device=0, strings=True)
                       for _ in range(n)]
    return _CACHE[key]


CASES = [("C", "planted_C", 16 * MiB + 12345), ("E", "planted_E", 16 * MiB),
         ("lit", "lit", 12 * MiB + 7), ("hex", "hex", 9 * MiB + 1), ("rx", "rx", 8 * MiB + 3),
         ("short", "alpha", 10 * MiB), ("root", "alpha", 3 * MiB + 5)]


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("rules,kind,size", CASES)
def test_multi_device_records_equal_single_device(rules, kind, size, n):
    data = _data(kind, size)
    single = yara_amd.Scanner(_tables(rules, 1)[0]).verify_calls(data, data_base=0x1000)
    m = yara_amd.Multi(_tables(rules, n))
    got = m.verify_calls(data, data_base=0x1000)
    assert len(got) == len(single) and len(single) > 0
    for f in ("offset", "pool_index", "candidate"):
        np.testing.assert_array_equal(got[f], single[f], err_msg=f)
    # every device held only its window: the shards tile the block
    bounds = [m.shard(size, k) for k in range(n)]
    assert bounds[0][0] == 0 and bounds[-1][1] == size
    assert all(bounds[k][1] == bounds[k + 1][0] for k in range(n - 1))
    per = (size // n) // MiB * MiB
    assert sum(1 for b in bounds if b[1] > b[0]) == (n if per else 1)
    m.close()


def test_multi_shards_match_dist_py():
    """The C ABI's device windows are dist.py's rank windows."""
    from yara_amd import dist as ydist
    tabs = _tables("C", 8)
    m = yara_amd.Multi(tabs)
    before, after = ydist.tables_halos(tabs[0])
    for size in (0, 100, 8 * MiB - 1, 8 * MiB, (32 << 30) + 77):
        for k in range(8):
            b, e = ydist.shard_bounds(size, 8, k)
            lo, hi = ydist.shard_window(size, b, e, before, after)
            assert m.shard(size, k) == (b, e, lo, hi), (size, k)
    m.close()


def test_multi_small_and_empty_blocks():
    """Blocks smaller than one 1 MiB slice per device: the last device takes
    all of it, the others scan empty ranges; an empty block has no records."""
    single = yara_amd.Scanner(_tables("lit", 1)[0])
    m = yara_amd.Multi(_tables("lit", 3))
    for size in (0, 1, 17, 4096, MiB + 3):
        data = _data("lit", size) if size > 65536 else oracle.xorshift(size, 7)
        a, b = m.verify_calls(data), single.verify_calls(data)
        np.testing.assert_array_equal(a, b)
    m.close()


def test_multi_refuses_streams_beyond_the_candidate_limit():
    """A device range whose candidates could exceed YR_AMD_VERIFY_MAX_CANDIDATES
    (range + 1 > 2^32) is refused before any work (the libyara shim then
    replays the block on one device instead)."""
    buf = np.zeros(64, np.uint8)
    for n, size in ((1, 1 << 32), (2, (1 << 33) + 1)):
        m = yara_amd.Multi(_tables("C", n))
        ptr = ctypes.POINTER(_lib.VerifyRec)()
        cnt = ctypes.c_uint64()
        rc = _lib.lib().yr_amd_multi_scan_block_verified(
            m._h, buf.ctypes.data_as(_lib._u8p), size, 0, ctypes.byref(ptr), ctypes.byref(cnt))
        assert rc == yara_amd.INVALID_ARGUMENT
        m.close()


def test_multi_needs_matching_tables():
    with pytest.raises(yara_amd.YaraAmdError):
        yara_amd.Multi([_tables("C", 1)[0], _tables("lit", 1)[0]])
    with pytest.raises(yara_amd.YaraAmdError):
        yara_amd.Multi([])


# ---- the block pipeline across devices (yr_amd_pipeline_create_multi) ----

def _blocks(data, sizes):
    out, b = [], 0
    for s in sizes:
        out.append((b, data[b:b + s]))
        b += s
    return out


@pytest.mark.parametrize("dma", [True, False])
@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("rules,kind", [("C", "planted_C"), ("rx", "rx"), ("short", "alpha"),
                                        ("root", "alpha"), ("lit", "lit")])
def test_multi_pipeline_records_equal_single_device(rules, kind, n, dma):
    """Blocks through a pipeline over n logical devices -- those of at least
    split_min bytes split into device windows, the smaller ones whole to one
    device (round-robin) -- come back in order with exactly the single-device
    records of each block (candidate indices rebased onto the block)."""
    sizes = [9 * MiB + 5, 3 * MiB, 1, 0, 6 * MiB + 17, 2 * MiB - 3, 12 * MiB]
    if rules == "root":
        sizes = [s // 8 for s in sizes]
    data = _data(kind, sum(sizes))
    single = yara_amd.Scanner(_tables(rules, 1)[0])
    want = [single.verify_calls(blk, data_base=b) for b, blk in _blocks(data, sizes)]
    tabs = _tables(rules, n)
    pipe = yara_amd.Pipeline(tabs if n > 1 else tabs[0], depth=2, split_min=4 * MiB)
    got, inflight = [], 0
    for b, blk in _blocks(data, sizes):
        if inflight == 2:
            got.append(pipe.next())
            inflight -= 1
        pipe.submit(blk, base=b, dma=dma)
        inflight += 1
    while inflight:
        got.append(pipe.next())
        inflight -= 1
    pipe.close()
    assert len(got) == len(want)
    for (b, blk), w, (recs, bytes_back, base) in zip(_blocks(data, sizes), want, got):
        assert base == b
        np.testing.assert_array_equal(bytes_back, blk)
        for f in ("offset", "pool_index", "candidate"):
            np.testing.assert_array_equal(recs[f], w[f], err_msg=f)
    assert sum(len(w) for w in want) > 0


@pytest.mark.parametrize("n", [1, 3])
def test_pipeline_copy_failure_is_could_not_map(n):
    """The caller's copy function fails one chunk (what the libyara shim's
    YR_TRYCATCH copy reports for a truncated mapping): the submission fails
    with YR_AMD_COULD_NOT_MAP_FILE on the parallel path, and the pipeline keeps
    working for the next block."""
    data = _data("lit", 24 * MiB)
    tabs = _tables("lit", n)
    pipe = yara_amd.Pipeline(tabs if n > 1 else tabs[0], depth=2)
    bad = int(data.ctypes.data) + 13 * MiB + 5

    def failing(d, s, k):
        ctypes.memmove(d, s, k)
        return 1 if s <= bad < s + k else 0
    pipe.set_copy(failing)
    with pytest.raises(yara_amd.YaraAmdError) as e:
        pipe.submit(data, base=0, dma=True)
    assert e.value.code == yara_amd.COULD_NOT_MAP_FILE
    pipe.set_copy(lambda d, s, k: (ctypes.memmove(d, s, k), 0)[1])
    pipe.submit(data, base=0, dma=True)
    recs = pipe.next()[0]
    single = yara_amd.Scanner(_tables("lit", 1)[0]).verify_calls(data)
    np.testing.assert_array_equal(recs, single)
    pipe.close()


def test_multi_copy_failure_is_could_not_map():
    data = _data("lit", 40 * MiB)
    m = yara_amd.Multi(_tables("lit", 3))
    bad = int(data.ctypes.data) + 33 * MiB

    def failing(d, s, k):
        ctypes.memmove(d, s, k)
        return 1 if s <= bad < s + k else 0
    m.set_copy(failing)
    with pytest.raises(yara_amd.YaraAmdError) as e:
        m.verify_calls(data)
    assert e.value.code == yara_amd.COULD_NOT_MAP_FILE
    m.set_copy(None)
    np.testing.assert_array_equal(m.verify_calls(data),
                                  yara_amd.Scanner(_tables("lit", 1)[0]).verify_calls(data))
    m.close()
