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
