"""GPU parity: the HIP path (libyara_amd.so through its C ABI) against the
pinned oracle and the reference's golden streams.

Bar: bit-exact.  The candidate stream (ascending positions with
ac_match_table[state] != 0) must equal the oracle's, and the verify-call
stream produced by GPU candidates + host replay must equal the stream the
stock libyara hot loop produced (golden SHA-256 / full arrays).
"""
import numpy as np
import pytest

import oracle
import yara_amd
from conftest import case_arrays, case_data, golden, ref_tables, tables_npz

pytestmark = pytest.mark.gpu

CASES = golden()["cases"]
_TABLES = {}


def dev_tables(name):
    if name not in _TABLES:
        _TABLES[name] = yara_amd.Tables.from_npz(tables_npz(name), device=0)
    return _TABLES[name]


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


def blocks(size, bsize, overlap):
    if size == 0:
        return [(0, 0)]
    out, base = [], 0
    while base < size:
        n = min(bsize, size - base)
        out.append((base, n))
        base = size if base + n >= size else base + n - overlap
    return out


SINGLE = [k for k, v in CASES.items() if v["size"] <= (64 << 20) and not v["block"]]
MULTI = [k for k, v in CASES.items() if v["block"]]


@pytest.mark.parametrize("case", SINGLE)
def test_candidates_and_verify_stream(case):
    rec = CASES[case]
    data = case_data(rec)
    sc = yara_amd.Scanner(dev_tables(rec["rules"]))
    pos, allp = sc.candidates(data)
    if allp:
        assert rec["rules"] == "root"
    else:
        assert len(pos) == rec["candidate_count"]
        assert oracle.positions_sha(pos) == rec["candidate_sha"]
    P, K = sc.verify_stream(data)
    assert len(P) == rec["verify_count"]
    assert oracle.verify_stream_sha(P, K) == rec["verify_sha"]
    full = case_arrays(case)
    if full is not None:
        np.testing.assert_array_equal(P, full["verify_pos"])
        np.testing.assert_array_equal(K, full["verify_idx"])


@pytest.mark.parametrize("case", MULTI)
def test_multi_block_iterator(case):
    """State resets per YR_MEMORY_BLOCK (scanner.c:69); offsets per block base."""
    rec = CASES[case]
    data = case_data(rec)
    sc = yara_amd.Scanner(dev_tables(rec["rules"]))
    P, K, B = [], [], []
    for base, n in blocks(data.size, rec["block"], rec["overlap"]):
        p, k = sc.verify_stream(data[base:base + n])
        P.append(p); K.append(k); B.append(np.full(p.size, base, np.uint64))
    P, K, B = np.concatenate(P), np.concatenate(K), np.concatenate(B)
    assert len(P) == rec["verify_count"]
    assert oracle.verify_stream_sha(P, K, base=B) == rec["verify_sha"]


@pytest.mark.parametrize("rules", ["B", "C", "E", "short"])
@pytest.mark.parametrize("size", [0, 1, 2, 3, 4, 5, 15, 16, 17, 100, 1023, 1024, 1025,
                                  2047, 2048, 2049, 3071, 3072, 3073,
                                  4095, 4097, 5121, 65535, 65536, 65537, 262144 + 7, 3_000_001])
def test_ragged_sizes_vs_oracle(rules, size):
    """Empty and ragged blocks, tile/segment edges, tails not multiple of 16
    (2047 .. 3073: segments of 1, 2 and 3 full tiles with and without a tail --
    the tile loop's peeled last one or two tiles)."""
    if rules == "short":
        x = oracle.xorshift(size, 17)
        data = np.frombuffer(b"abcdxyzHeloC\x00\x01\xff", np.uint8)[x % 15]
    else:
        data = oracle.xorshift(size, 23)
    tab = ref_tables(rules)
    sc = yara_amd.Scanner(dev_tables(rules))
    pos, allp = sc.candidates(data)
    assert not allp
    np.testing.assert_array_equal(pos, oracle.candidates(tab, data))


@pytest.mark.parametrize("rules", ["B", "C", "E", "rx", "short"])
def test_segment_tile_counts(rules):
    """Segments of 4 to 13 full tiles, with and without a ragged tail: every
    entry and exit of the tile loop (kernels.hip scan_segment: the rounds of
    kPf + 1 steps with kPf tiles in flight, the remaining tiles one ahead,
    the one-ahead loop of segments too short for a round).  A block of
    waves x T KiB makes segments of T tiles (scanner.cpp choose_seg_bytes)."""
    torch = _torch()
    waves = torch.cuda.get_device_properties(0).multi_processor_count * 16
    tab = ref_tables(rules)
    sc = yara_amd.Scanner(dev_tables(rules))
    for t in range(4, 13):
        for extra in (0, 777):
            n = waves * t * 1024 + extra
            data = oracle.xorshift(n, 100 + t)
            if rules == "short":
                data = np.frombuffer(b"abcdxyzHeloC\x00\x01\xff", np.uint8)[data % 15]
            pos, allp = sc.candidates(data)
            assert not allp
            np.testing.assert_array_equal(pos, oracle.candidates(tab, data), err_msg=str((t, extra)))


@pytest.mark.parametrize("hot_mib", [1, 3])
def test_skewed_candidate_density(hot_mib):
    """One dense region (every byte a candidate of a 1-byte key) inside random
    data: a few segments overflow their capacity by orders of magnitude; the
    exact-offset rerun must still give the oracle's stream, and the scanner
    must stay usable for a normal block afterwards."""
    size = 64 << 20
    data = oracle.xorshift(size, 31).copy()
    lo = 20 << 20
    data[lo:lo + (hot_mib << 20)] = ord("a")
    tab = ref_tables("short")
    sc = yara_amd.Scanner(dev_tables("short"))
    pos, allp = sc.candidates(data)
    assert not allp
    ref = oracle.candidates(tab, data)
    assert len(pos) > (hot_mib << 20)
    np.testing.assert_array_equal(pos, ref)
    small = oracle.xorshift(1 << 20, 32)
    np.testing.assert_array_equal(sc.candidates(small)[0], oracle.candidates(tab, small))


@pytest.mark.parametrize("period", [16, 1024, 4096, 65536])
def test_atoms_ending_on_slice_boundaries(period):
    """Adversarial: atoms end exactly at lane/tile/segment edges (+-1 byte)."""
    import planted
    import gen_rules
    tab = ref_tables("C")
    inst = planted.string_instances(gen_rules.gen("C"))
    atoms = [b for b, _ in inst if len(b) >= 4][:500]
    data = planted.boundary_buffer(oracle.xorshift, atoms, 4 << 20, period)
    sc = yara_amd.Scanner(dev_tables("C"))
    pos, _ = sc.candidates(data)
    ref = oracle.candidates(tab, data)
    assert len(ref) > (4 << 20) // period // 2
    np.testing.assert_array_equal(pos, ref)


@pytest.mark.parametrize("stride", [3, 4, 5, 8, 12, 16, 24, 40])
def test_dense_hits_per_lane(stride):
    """4-byte atoms of config C planted every `stride` bytes (period 16 = the
    lane width): lanes with 1, 2 and >2 hits exercise the kernel's deferred
    first-level path (<= 2 hits per lane, incl. more than a wave's worth of
    survivors in one drain) and its synchronous fallback (> 2 hits in a lane).
    Bursts alternate with random stretches so both regimes meet in one drain."""
    import planted
    import gen_rules
    tab = ref_tables("C")
    atoms = [b[:4] for b, _ in planted.string_instances(gen_rules.gen("C")) if len(b) >= 4][:997]
    size = 4 << 20
    data = oracle.xorshift(size, 41).copy()
    k = 0
    for burst in range(0, size, 96 << 10):          # 64 KiB dense, 32 KiB random
        for off in range(burst, min(burst + (64 << 10), size) - 4, stride):
            data[off:off + 4] = np.frombuffer(atoms[k % len(atoms)], np.uint8)
            k += 1
    sc = yara_amd.Scanner(dev_tables("C"))
    pos, _ = sc.candidates(data)
    ref = oracle.candidates(tab, data)
    if stride >= 4:                                 # (stride 3: atoms overwrite each other)
        assert len(ref) > k // 4                    # (not every string's first 4 bytes are a key)
    np.testing.assert_array_equal(pos, ref)


def test_periodic_data_deep_chains():
    """'aaaa...' keeps the automaton in depth-3/4 states (failure chains)."""
    tab = ref_tables("short")
    sc = yara_amd.Scanner(dev_tables("short"))
    for pat in (b"a", b"ab", b"abc", b"abcd", b"aab", b"\x00\x01", b"\xff"):
        data = np.frombuffer(pat * (300_000 // len(pat)), np.uint8)
        pos, _ = sc.candidates(data)
        np.testing.assert_array_equal(pos, oracle.candidates(tab, data))


def test_device_generator_matches_canonical():
    torch = _torch()
    for n in (1, 15, 16, 1000, 65536, 65536 * 3 + 5, 1 << 22):
        d = torch.empty(max(n, 16), dtype=torch.uint8, device="cuda")
        yara_amd.fill_xorshift64(d.data_ptr(), n, 1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(d[:n].cpu().numpy(), oracle.xorshift(n, 1))


def test_device_shards_concatenate_to_full_stream():
    """Shards [a, b) with a 4-byte warm-up read concatenate exactly (multi-GPU basis)."""
    torch = _torch()
    n = (16 << 20) + 12345
    d = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(d.data_ptr(), n, 9)
    torch.cuda.synchronize()
    sc = yara_amd.Scanner(dev_tables("C"))
    sc.scan_device(d.data_ptr(), n)
    full = _d2h(torch, *sc.device_result()[:2])
    rng = np.random.default_rng(5)
    cuts = sorted(set([0, n] + [int(c) // 16 * 16 for c in rng.integers(0, n, 9)]))
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        sc.scan_device(d.data_ptr(), n, a, b)
        parts.append(_d2h(torch, *sc.device_result()[:2]))
    np.testing.assert_array_equal(np.concatenate(parts), full)
    np.testing.assert_array_equal(full, oracle.candidates(ref_tables("C"), d[:n].cpu().numpy()))


def _d2h(torch, ptr, count):
    from yara_amd._hip import d2h_u64
    return d2h_u64(ptr, count)


@pytest.mark.slow
@pytest.mark.parametrize("case", ["C_4G", "E_1G"])
def test_full_size_against_reference(case):
    """BASELINE sizes (4 GiB / 1 GiB): GPU candidates from device-resident data
    equal the oracle's count/SHA recorded at golden time, and GPU candidates +
    replay reproduce the stock libyara verify stream."""
    torch = _torch()
    rec = CASES[case]
    n = rec["size"]
    d = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(d.data_ptr(), n, rec["data"][1])
    torch.cuda.synchronize()
    sc = yara_amd.Scanner(dev_tables(rec["rules"]))
    sc.scan_device(d.data_ptr(), n)
    ptr, cnt, allp = sc.device_result()
    pos = _d2h(torch, ptr, cnt)
    assert cnt == rec["candidate_count"]
    assert oracle.positions_sha(pos) == rec["candidate_sha"]
    assert np.all(np.diff(pos.astype(np.int64)) > 0)
    host = d[:n].cpu().numpy()
    del d
    P, K = [], []
    bt = dev_tables(rec["rules"])._bt

    def verify(k, off):
        K.append(k)
        P.append(off + int(bt[k]))
        return 0
    assert yara_amd.replay(dev_tables(rec["rules"]), host, pos, allp, verify) == 0
    assert len(P) == rec["verify_count"]
    assert oracle.verify_stream_sha(np.array(P, np.uint64), np.array(K, np.uint32)) == rec["verify_sha"]


def test_scan_window_holds_only_the_window():
    """yr_amd_scan_window: the device holds just [lo, hi) of the block (a
    shard + halo, the multi-GPU layout); candidates equal the whole block's in
    (begin, end], and pre-verification records equal the whole block's for the
    same candidates when the window includes the tables' verify halos."""
    torch = _torch()
    from yara_amd import dist as ydist
    rec = CASES["lit_1M"]
    data = case_data(rec)
    n = data.size
    t = yara_amd.Tables.from_npz(tables_npz("lit"), device=0, strings=True)
    full = yara_amd.Scanner(t).verify_calls(data)
    full_pos, _ = yara_amd.Scanner(t).candidates(data)
    before, after = ydist.tables_halos(t)
    assert before >= 4096 and after >= 4096
    sc = yara_amd.Scanner(t)
    for begin, end in [(0, 300000), (300000, 700000), (700000, n), (123456 // 16 * 16, 123456 // 16 * 16)]:
        for halo in ((4, 0), (before, after)):
            lo, hi = ydist.shard_window(n, begin, end, *halo)
            win = torch.empty(max(hi - lo, 16), dtype=torch.uint8, device="cuda")
            win[:hi - lo] = torch.from_numpy(data[lo:hi].copy()).cuda()
            torch.cuda.synchronize()
            sc.scan_window(win.data_ptr(), lo, hi, n, begin, end)
            ptr, cnt, _ = sc.device_result()
            pos = _d2h(torch, ptr, cnt)
            sel = (full_pos > begin) & (full_pos <= end) if begin else (full_pos <= end)
            np.testing.assert_array_equal(pos, full_pos[sel])
            if halo[0] == before:
                p, c = sc.verify_device(0)
                got = np.zeros(c, dtype=yara_amd._lib.VERIFY_REC_DTYPE)
                if c:
                    from yara_amd._hip import memcpy
                    memcpy(got.ctypes.data, p, c * 16, 2)
                i = full["offset"] + t._bt[full["pool_index"]]
                fsel = (i > begin) & (i <= end) if begin else (i <= end)
                np.testing.assert_array_equal(got["offset"], full["offset"][fsel])
                np.testing.assert_array_equal(got["pool_index"], full["pool_index"][fsel])


def test_scan_window_rejects_bad_windows():
    torch = _torch()
    t = dev_tables("C")
    sc = yara_amd.Scanner(t)
    d = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    bad = [(16, 1 << 16, 1 << 20, 16, 1024),      # warm-up before byte 16 not held
           (0, 1 << 16, 1 << 20, 0, (1 << 16) + 16),  # scan past the window
           (8, 1 << 16, 1 << 20, 32, 64),          # window_begin not 16-aligned
           (0, 1 << 21, 1 << 20, 0, 64)]           # window past the block
    for args in bad:
        with pytest.raises(yara_amd.YaraAmdError) as e:
            sc.scan_window(d.data_ptr(), *args)
        assert e.value.code == yara_amd.INVALID_ARGUMENT


@pytest.mark.parametrize("env", [{"YAMD_SEG_KIB": "4"},
                                 {"YAMD_SEG_KIB": "4", "YAMD_SEG_DYNAMIC": "1"},
                                 {"YAMD_SEG_KIB": "8", "YAMD_SEG_DYNAMIC": "1"}])
def test_segment_schedules(env):
    """The profiling switches of the segment schedule (several segments per
    wave, round-robin or claimed from a counter; read once per process by the
    diagnostic build, hence a child process) give the same candidate stream.  48 MiB with 4-8 KiB
    segments: several segments per wave of the full-chip grid."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import sys; sys.path[:0] = [%r, %r, %r]\n"
        "import numpy as np, torch, yara_amd, oracle\n"
        "from conftest import ref_tables, tables_npz\n"
        "n = (48 << 20) + 777\n"
        "d = torch.empty(n + 16, dtype=torch.uint8, device='cuda')\n"
        "yara_amd.fill_xorshift64(d.data_ptr(), n, 3); torch.cuda.synchronize()\n"
        "sc = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz('C'), device=0))\n"
        "from yara_amd._hip import d2h_u64\n"
        "sc.scan_device(d.data_ptr(), n); p, c = sc.device_result()[:2]\n"
        "got = d2h_u64(p, c)\n"
        "ref = oracle.candidates(ref_tables('C'), d[:n].cpu().numpy())\n"
        "assert np.array_equal(got, ref), (len(got), len(ref))\n"
        "print('ok', len(got))\n" % (repo, os.path.join(repo, "tests"),
                                     os.path.join(repo, "tests", "golden")))
    from conftest import DIAG_LIB   # the switches exist in the diagnostic build only
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, YARA_AMD_LIB=DIAG_LIB, **env))
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


def test_byte_keys_stage1_path():
    """1-byte keys (incl. 0x00 and 0xFF) tested byte by byte in stage 1
    (kernels.hip kModeByteKeys) instead of the window filter: candidate streams
    equal the oracle's on ragged sizes, all-zero blocks, and blocks whose last
    bytes are zeros (the ragged tail tile is zero-filled past the block end,
    which must not turn into candidates).  Tables: tests/golden/rules/
    bytekeys.yar compiled by the stock libyara (make_golden.py)."""
    tab = ref_tables("bytekeys")
    sc = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz("bytekeys"), device=0))
    rng = np.random.default_rng(17)
    alpha = np.frombuffer(b"\x00\x41\x51\xffabcwxyzrstQ", np.uint8)
    sizes = [1, 2, 3, 15, 16, 17, 1023, 1024, 1025, 4095, 65537, (1 << 20) + 13, 3 << 20]
    for n in sizes:
        data = alpha[rng.integers(0, len(alpha), n)]
        for variant in (data, np.zeros(n, np.uint8), np.concatenate(
                [data[: n // 2], np.zeros(n - n // 2, np.uint8)])):
            variant = np.ascontiguousarray(variant)
            pos, allp = sc.candidates(variant)
            assert not allp
            np.testing.assert_array_equal(pos, oracle.candidates(tab, variant), err_msg=str(n))
    # random bytes: 1/256 of positions per byte key
    data = oracle.xorshift(8 << 20, 5)
    pos, _ = sc.candidates(data)
    ref = oracle.candidates(tab, data)
    assert len(ref) > 3 * (8 << 20) // 256 * 0.9
    np.testing.assert_array_equal(pos, ref)


def test_byte_key_sets_dense_and_mixed():
    """Rule sets with 1-byte keys (kernels.hip kModeByteKeys) on random blocks,
    blocks drawn from the key bytes (several keys per lane, other filter
    passes next to key bytes, drains yielding more than a wave of hits) and
    blocks with 1 % key bytes, at ragged sizes: candidates equal the oracle's.
    (A direct-output form of this kernel was measured slower and dropped,
    profiles/r03_bytekey_direct_ab.json.)"""
    alpha = np.frombuffer(b"[]ab_d>1xyz\x00\xffA.", np.uint8)
    for rules in ("bytekeys", "rx", "short", "fuzz0", "fuzz3"):
        ref_t = ref_tables(rules)
        sc = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz(rules), device=0))
        for i, n in enumerate(((3 << 20) + 13, 1 << 20, 4095, 17)):
            x = oracle.xorshift(n, 40 + i)
            mixed = x.copy()
            pick = (x % 100) < 1
            mixed[pick] = alpha[(x[pick] >> 3) % len(alpha)]
            for d in (x, np.ascontiguousarray(alpha[x % len(alpha)]), mixed):
                got, allp = sc.candidates(d)
                assert not allp
                np.testing.assert_array_equal(got, oracle.candidates(ref_t, d), err_msg=(rules, n))


@pytest.mark.slow
def test_verify_refuses_more_than_2_32_candidates():
    """yr_amd_verify_device refuses a candidate stream longer than
    YR_AMD_VERIFY_MAX_CANDIDATES (2^32: records carry 32-bit candidate indices)
    before allocating anything, and the libyara shim replays such blocks on the
    host instead (integration/yr_gpu_scanner.c, the same limit).  A zero-filled
    block of 2^32 + 16 bytes under a rule set with the 1-byte key 00 makes
    every position a candidate: the scan gives all 2^32 + 16 of them, the
    pre-verification returns INVALID_ARGUMENT, and the scanner stays usable."""
    torch = _torch()
    n = (1 << 32) + 16
    if torch.cuda.mem_get_info()[0] < 80 << 30:
        pytest.skip("needs ~80 GiB of free HBM (positions of 2^32 candidates)")
    d = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    sc = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz("bytekeys"), device=0, strings=True))
    sc.scan_device(d.data_ptr(), n)
    ptr, cnt, allp = sc.device_result()
    assert not allp and cnt == n
    with pytest.raises(yara_amd.YaraAmdError) as e:
        sc.verify_device(0)
    assert e.value.code == yara_amd.INVALID_ARGUMENT
    del d
    torch.cuda.empty_cache()
    small = oracle.xorshift(1 << 20, 3)
    assert len(sc.verify_calls(small)) > 0


@pytest.mark.slow
def test_verify_exactly_2_32_candidates_with_key_classes():
    """The largest stream yr_amd_verify_device accepts: exactly 2^32 candidates
    (a zero-filled 4 GiB block, 1-byte key 00) under a rule set whose 1-byte
    keys have candidate classes.  The compaction's live-list counter is 32-bit,
    so the scanner decides no classes for a stream past 0xFFFFFFFF candidates
    (scanner.cpp) -- a wrapped counter would have dropped every candidate.  On
    zero bytes the record count is affine in the block size past the first few
    bytes (edge effects at both ends are fixed), so two small blocks predict
    the 4 GiB one exactly."""
    torch = _torch()
    n = 1 << 32
    if torch.cuda.mem_get_info()[0] < 170 << 30:
        pytest.skip("needs ~170 GiB of free HBM (positions, classes and records of 2^32 candidates)")
    sc = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz("bytekeys"), device=0, strings=True))
    counts = {}
    for m in (1 << 20, 1 << 21):
        z = torch.zeros(m + 16, dtype=torch.uint8, device="cuda")
        sc.scan_device(z.data_ptr(), m)
        _, cnt, allp = sc.device_result()
        assert cnt == m
        counts[m] = sc.verify_device(0)[1]
        del z
    slope = (counts[1 << 21] - counts[1 << 20]) // (1 << 20)
    assert slope * (1 << 20) == counts[1 << 21] - counts[1 << 20] and slope > 0
    expect = counts[1 << 20] + slope * (n - (1 << 20))
    d = torch.zeros(n + 16, dtype=torch.uint8, device="cuda")
    sc.scan_device(d.data_ptr(), n)
    _, cnt, allp = sc.device_result()
    assert not allp and cnt == n
    assert sc.verify_device(0)[1] == expect
    del d
    torch.cuda.empty_cache()


def test_block_larger_than_4gib():
    """A single 8 GiB block (past 32-bit byte offsets: 8,192 segments, positions
    above 2^32): its candidates up to 4 GiB equal the golden C_4G stream (the
    input is the same xorshift64 prefix), and the block's stream equals the
    concatenation of three device shards scanned separately."""
    torch = _torch()
    rec = CASES["C_4G"]
    n = (8 << 30) + 4096 + 7
    d = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(d.data_ptr(), n, rec["data"][1])
    torch.cuda.synchronize()
    sc = yara_amd.Scanner(dev_tables("C"))
    sc.scan_device(d.data_ptr(), n)
    full = _d2h(torch, *sc.device_result()[:2])
    assert np.all(np.diff(full.astype(np.int64)) > 0) and int(full[-1]) > (1 << 32)
    head = full[full <= rec["size"]]
    assert len(head) == rec["candidate_count"]
    assert oracle.positions_sha(head) == rec["candidate_sha"]
    cuts = [0, (3 << 30) + 16, (6 << 30) + 4096, n]
    parts = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        sc.scan_device(d.data_ptr(), n, a, b)
        parts.append(_d2h(torch, *sc.device_result()[:2]))
    np.testing.assert_array_equal(np.concatenate(parts), full)
    # on-device pre-verification of the 8 GiB block: its records up to 4 GiB
    # equal those of the 4 GiB block (offsets past 2^32 in the records)
    from yara_amd._hip import memcpy

    def records(scanner, size):
        scanner.scan_device(d.data_ptr(), size)
        scanner.device_result()
        ptr, cnt = scanner.verify_device(0)
        h = torch.empty(max(cnt, 1) * 16, dtype=torch.uint8, device="cuda")
        memcpy(h.data_ptr(), ptr, cnt * 16, 3)
        return np.frombuffer(h[:cnt * 16].cpu().numpy().tobytes(),
                             dtype=yara_amd._lib.VERIFY_REC_DTYPE)
    sv = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz("C"), device=0, strings=True))
    r8 = records(sv, n)
    r4 = records(sv, rec["size"])
    assert len(r4) > 0 and len(r8) > len(r4) and int(r8["offset"].max()) > (1 << 32)
    head8 = r8[r8["offset"] < rec["size"] - 64]
    head4 = r4[r4["offset"] < rec["size"] - 64]
    np.testing.assert_array_equal(head8["offset"], head4["offset"])
    np.testing.assert_array_equal(head8["pool_index"], head4["pool_index"])


def even_planted(rules, stride):
    """Strings of rule set `rules` planted every `stride` bytes (drifting through
    every residue mod 16) into 2 MiB + 12345 random bytes."""
    import planted
    import gen_rules
    inst = [b for b, _ in planted.string_instances(gen_rules.gen(rules))]
    size = (2 << 20) + 12345
    data = oracle.xorshift(size, 43).copy()
    k, off = 0, 3
    while off + 40 < size:
        s = inst[k % len(inst)][: max(4, stride - 1)]
        data[off:off + len(s)] = np.frombuffer(s, np.uint8)
        k += 1
        off += stride + (k % 3 == 0)
    return data


EVEN_STRIDES = [5, 7, 16, 33, 1021]


@pytest.mark.parametrize("rules", ["B", "E"])
@pytest.mark.parametrize("stride", EVEN_STRIDES)
def test_even_filter_planted_keys(rules, stride):
    """Rule sets whose keys are all 4 bytes scan with the even-position filter
    (internal.h kFilterEven: only the windows ending at even positions are
    tested, each key inserted as its 3-byte prefix and suffix).  Strings planted
    every `stride` bytes end at both parities and at every lane byte (lane,
    tile and segment edges included; strides 5 and 7 put several hits in one
    lane, the drains' synchronous path): candidates equal the oracle's."""
    data = even_planted(rules, stride)
    even = dev_tables(rules)
    assert even.info()["filter_mode"] in (1, 2)
    pos, allp = yara_amd.Scanner(even).candidates(data)
    ref = oracle.candidates(ref_tables(rules), data)
    assert not allp and len(ref) > data.size // stride // 8
    np.testing.assert_array_equal(pos, ref)


def test_every_filter_form_on_planted_keys():
    """Every filter form the host can pick -- the plain and the hashed even
    filter and the pair filter -- forced in turn through the diagnostic build's
    switches (one child process): candidates equal the oracle's on the planted
    B and E buffers of every stride."""
    from conftest import run_diag_child
    code = (
        "import os, numpy as np, torch, yara_amd, oracle\n"
        "from conftest import ref_tables, tables_npz\n"
        "from test_gpu_parity import even_planted, EVEN_STRIDES\n"
        "n = 0\n"
        "for rules in ('B', 'E'):\n"
        "  for stride in EVEN_STRIDES:\n"
        "    data = even_planted(rules, stride)\n"
        "    ref = oracle.candidates(ref_tables(rules), data)\n"
        "    for env, val, mode in (('YAMD_EVEN_FILTER', 'plain', 1),\n"
        "                           ('YAMD_EVEN_FILTER', 'hash', 2), ('YAMD_PAIR_FILTER', '1', 0)):\n"
        "      os.environ[env] = val\n"
        "      t = yara_amd.Tables.from_npz(tables_npz(rules), device=0)\n"
        "      del os.environ[env]\n"
        "      assert t.info()['filter_mode'] == mode\n"
        "      got = yara_amd.Scanner(t).candidates(data)[0]\n"
        "      assert np.array_equal(got, ref), (rules, stride, mode)\n"
        "      n += 1\n"
        "print('forms ok', n)\n")
    assert "forms ok 30" in run_diag_child(code, timeout=600)


def test_dense_rescans_after_capacity_learning():
    """A scanner whose scan overflowed the default segment output (1 candidate
    per 256 bytes) sizes the following scans' outputs from it (scanner.cpp
    dense_per_kib): a 64 MiB block with ~1 candidate per 100 bytes overflows
    once, then fits; every scan, and a sparse block after them, gives the
    oracle's candidates."""
    tab = ref_tables("short")
    sc = yara_amd.Scanner(dev_tables("short"))
    n = 64 << 20
    x = oracle.xorshift(n, 19)
    data = x.copy()
    pick = (x % 100) < 1                           # 1 % of the bytes from the key alphabet
    data[pick] = np.frombuffer(b"abcdxyzHeloC\x00\x01\xff", np.uint8)[(x[pick] >> 3) % 15]
    ref = oracle.candidates(tab, data)
    assert n // 256 < len(ref) < n // 80
    for _ in range(3):
        np.testing.assert_array_equal(sc.candidates(data)[0], ref)
    sparse = oracle.xorshift(3 << 20, 20)
    np.testing.assert_array_equal(sc.candidates(sparse)[0], oracle.candidates(tab, sparse))
