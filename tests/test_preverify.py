"""On-device literal pre-verification.

The GPU emits, in the reference's call order, only the yr_scan_verify_match
calls that can have an effect (scan.c:887-990, :1013, :1023).  Parity:
  * CPU: the oracle's keep-mask (oracle_literal_effect, a restatement of the
    scan.c comparisons) never drops a call that produced one of the matches the
    stock libyara reported (golden match sets) -- it is pinned to the reference
    through its final output;
  * GPU: the device records equal the golden verify-call stream filtered by the
    oracle's mask, bit-exact (offset, pool index), for every golden case,
    single- and multi-block (fixed-offset strings see the block base);
  * the end-to-end match sets through the libyara shim with pre-verification
    on are identical to stock libyara (tests/test_e2e_libyara.py).
"""
import numpy as np
import pytest

import oracle
from conftest import case_arrays, case_data, golden, tables_npz

CASES = golden()["cases"]
FULL = [k for k in CASES if case_arrays(k) is not None]
SF_LITERAL = 0x400


def _expected(rec, arr, data):
    """Golden verify stream -> (keep mask, offsets, pool idx, bases)."""
    z = np.load(tables_npz(rec["rules"]))
    pos, idx = arr["verify_pos"], arr["verify_idx"]
    base = arr["verify_base"]
    bt = z["pool_backtrack"]
    keep = np.zeros(len(pos), bool)
    if rec["block"]:
        for b in np.unique(base):
            sel = base == b
            blk = data[int(b):int(b) + rec["block"]]
            keep[sel] = oracle.literal_effect(z, pos[sel], idx[sel], blk, base=int(b))
    else:
        keep = oracle.literal_effect(z, pos, idx, data)
    off = pos.astype(np.uint64) - bt[idx].astype(np.uint64)
    return z, keep, off, idx, base


@pytest.mark.parametrize("case", FULL)
def test_oracle_keeps_every_reported_match(case):
    rec = CASES[case]
    arr = case_arrays(case)
    data = case_data(rec)
    z, keep, off, idx, base = _expected(rec, arr, data)
    ps = z["pool_string"]
    kept = set(zip((base[keep] + off[keep]).tolist(), ps[idx[keep]].tolist()))
    flags = z["str_flags"]
    by_string = {}
    for o_, s_ in kept:
        by_string.setdefault(s_, []).append(o_)
    by_string = {k: np.sort(np.array(v, np.int64)) for k, v in by_string.items()}
    for s, o, n in zip(arr["match_string"].tolist(), arr["match_offset"].tolist(),
                       arr["match_len"].tolist()):
        if flags[s] & SF_LITERAL:
            assert (o, s) in kept, (case, s, o)
        else:
            # regexp / hex: the atom lies inside the reported match, so some
            # kept call of that string has its atom offset in [o, o + len]
            v = by_string.get(s)
            assert v is not None, (case, s, o)
            j = np.searchsorted(v, o)
            assert j < len(v) and v[j] <= o + n, (case, s, o, n)
    # the filter is not a no-op where near misses exist
    if case.startswith(("lit", "hex", "rx")):
        assert keep.sum() < len(keep)


@pytest.mark.gpu
@pytest.mark.parametrize("case", FULL)
def test_device_records_equal_oracle_filtered_reference_stream(case):
    import yara_amd
    rec = CASES[case]
    arr = case_arrays(case)
    data = case_data(rec)
    z, keep, off, idx, base = _expected(rec, arr, data)
    tab = yara_amd.Tables.from_npz(tables_npz(rec["rules"]), device=0, strings=True)
    sc = yara_amd.Scanner(tab)
    if rec["block"]:
        from test_gpu_parity import blocks
        got_off, got_idx, got_base = [], [], []
        for b, n in blocks(rec["size"], rec["block"], rec["overlap"]):
            r = sc.verify_calls(data[b:b + n], data_base=b)
            got_off.append(r["offset"])
            got_idx.append(r["pool_index"])
            got_base.append(np.full(len(r), b, np.uint64))
        g_off, g_idx = np.concatenate(got_off), np.concatenate(got_idx)
        g_base = np.concatenate(got_base)
        assert np.array_equal(g_base, base[keep])
    else:
        r = sc.verify_calls(data)
        g_off, g_idx = r["offset"], r["pool_index"]
    assert len(g_off) == int(keep.sum()), (case, len(g_off), int(keep.sum()))
    assert np.array_equal(g_off, off[keep])
    assert np.array_equal(g_idx, idx[keep])


@pytest.mark.gpu
def test_device_verify_after_sharded_device_scan():
    """yr_amd_verify_device on a device-resident block scanned in two shards
    equals the whole-block host path."""
    import torch
    import yara_amd
    from yara_amd._hip import memcpy
    rec = CASES["lit_1M"]
    data = case_data(rec)
    tab = yara_amd.Tables.from_npz(tables_npz("lit"), device=0, strings=True)
    sc = yara_amd.Scanner(tab)
    want = sc.verify_calls(data)
    d = torch.from_numpy(data.copy()).cuda()
    half = (len(data) // 2) & ~15
    got = []
    for lo, hi in ((0, half), (half, len(data))):
        sc.scan_device(d.data_ptr(), len(data), lo, hi)
        sc.device_result()
        p, n = sc.verify_device(0)
        out = np.zeros(n, dtype=yara_amd._lib.VERIFY_REC_DTYPE)
        if n:
            h = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
            memcpy(h.data_ptr(), p, n * 16, 3)
            out = np.frombuffer(h.cpu().numpy().tobytes(), dtype=yara_amd._lib.VERIFY_REC_DTYPE)
        got.append(out)
    g = np.concatenate(got)
    assert np.array_equal(g["offset"], want["offset"])
    assert np.array_equal(g["pool_index"], want["pool_index"])


@pytest.mark.gpu
@pytest.mark.parametrize("rules,pre,key,after", [
    ("rx", b"\xe8\x11\x22\x33\x44", 0x5B, b"\xc3"),   # { E8 ?? ?? ?? ?? ( 5B | 5D ) C3 }
    ("fuzz0", b"\x64", 0x5F, b"\x00\x3e")])               # { 64 ( .. | 5F | .. ) [0-4] 3E }
@pytest.mark.parametrize("split", [1, 2, 3, 4])
def test_range_scan_keeps_candidates_decided_past_its_end(rules, pre, key, after, split):
    """A byte range scan of a device-resident block reads nothing past the
    range's end (zeros fill its last lane), so a 1-byte key whose guard bytes lie
    beyond it stays undecided (kernels.hip key_class tests the range end, not
    the block's): the range [0, cut) ends 5 bytes into a lane, keys planted
    `split` bytes before the cut with their guard's bytes after it; the range's
    records equal the whole-block host path's up to the cut, planted matches
    included."""
    import torch
    import yara_amd
    from yara_amd._hip import memcpy
    n = (1 << 20) + 77
    data = oracle.xorshift(n, 71).copy()
    cut = ((n // 2) & ~15) + 5
    data[cut - split - len(pre):cut - split] = np.frombuffer(pre, np.uint8)
    data[cut - split] = key
    data[cut - split + 1:cut - split + 1 + len(after)] = np.frombuffer(after, np.uint8)
    tab = yara_amd.Tables.from_npz(tables_npz(rules), device=0, strings=True)
    sc = yara_amd.Scanner(tab)
    want = sc.verify_calls(data)
    want = want[want["offset"] < cut]   # (a record's offset: its key's byte)
    assert np.isin(cut - split, want["offset"])
    d = torch.from_numpy(data.copy()).cuda()
    sc.scan_device(d.data_ptr(), n, 0, cut)
    sc.device_result()
    p, m = sc.verify_device(0)
    got = np.zeros(m, dtype=yara_amd._lib.VERIFY_REC_DTYPE)
    if m:
        h = torch.empty(m * 16, dtype=torch.uint8, device="cuda")
        memcpy(h.data_ptr(), p, m * 16, 3)
        got = np.frombuffer(h.cpu().numpy().tobytes(), dtype=yara_amd._lib.VERIFY_REC_DTYPE)
    assert np.array_equal(got["offset"], want["offset"])
    assert np.array_equal(got["pool_index"], want["pool_index"])


@pytest.mark.gpu
def test_preverify_requires_strings():
    import yara_amd
    tab = yara_amd.Tables.from_npz(tables_npz("lit"), device=0)
    sc = yara_amd.Scanner(tab)
    with pytest.raises(yara_amd.YaraAmdError) as e:
        sc.verify_calls(np.zeros(16, np.uint8))
    assert e.value.code == yara_amd.INVALID_ARGUMENT


def _planted_jumps(seeds=range(7, 15), size=8 << 20):
    """Config C's strings, one instance per string per seed (hex jumps and
    wildcards drawn anew for every seed, so every jump length occurs), planted
    back to back into random bytes."""
    import gen_rules
    import planted
    text = gen_rules.gen("C")
    data = oracle.xorshift(size, 51).copy()
    off = 100
    for seed in seeds:
        for b, _ in planted.string_instances(text, seed=seed):
            if off + len(b) + 64 > size:
                return data
            data[off:off + len(b)] = np.frombuffer(b, np.uint8)
            off += len(b) + 37
    return data


def test_oracle_keeps_planted_hex_matches():
    """The CPU side of the guard test below: the oracle keeps calls of fast-exec
    (hex) strings on the planted instances, i.e. the GPU comparison is not
    vacuous."""
    from conftest import ref_tables
    z = np.load(tables_npz("C"))
    data = _planted_jumps(seeds=range(7, 8), size=1 << 20)
    P, K = oracle.walk_verify(ref_tables("C"), data)
    keep = oracle.literal_effect(z, P, K, data)
    fast = z["re_kind"][K] != 0
    assert (keep & fast).sum() > 1000 and (~keep & fast).sum() > 0


@pytest.mark.gpu
def test_guards_keep_every_planted_match():
    """Fast-exec guards (verify.h DevGuard, checked before any program is
    interpreted) reject only calls whose program cannot match: with config C's
    hex strings planted with every jump length and wildcard byte, the device
    records equal the oracle's kept calls exactly."""
    import yara_amd
    from conftest import ref_tables
    z = np.load(tables_npz("C"))
    data = _planted_jumps()
    P, K = oracle.walk_verify(ref_tables("C"), data)
    keep = oracle.literal_effect(z, P, K, data)
    assert (keep & (z["re_kind"][K] != 0)).sum() > 10000
    r = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz("C"), device=0, strings=True)).verify_calls(data)
    off = P.astype(np.uint64) - z["pool_backtrack"][K].astype(np.uint64)
    np.testing.assert_array_equal(r["offset"], off[keep])
    np.testing.assert_array_equal(r["pool_index"], K[keep])


@pytest.mark.gpu
@pytest.mark.parametrize("case", [k for k in FULL if not CASES[k]["block"]])
def test_profiling_count_only_records(case):
    """yr_amd_tables_set_profiling: besides the kept calls, every dropped call
    that passes yr_scan_verify_match's early returns (offset < size, fixed
    offset, scan.c:1013-1027) -- i.e. every call libyara's profiling counts,
    scan.c:1083 -- comes out as a count-only record, in the reference's call
    order; kept records are unchanged."""
    import yara_amd
    rec = CASES[case]
    arr = case_arrays(case)
    data = case_data(rec)
    z, keep, off, idx, base = _expected(rec, arr, data)
    sf = z["str_flags"][z["pool_string"][idx]]
    fixed = z["str_fixed_offset"][z["pool_string"][idx]]
    counted = (off < len(data)) & (((sf & 0x8000) == 0) | (fixed == off.astype(np.int64)))
    tab = yara_amd.Tables.from_npz(tables_npz(rec["rules"]), device=0, strings=True)
    tab.set_profiling(True)
    r = yara_amd.Scanner(tab).verify_calls(data)
    co = (r["pool_index"] & 0x80000000) != 0
    want = keep | counted
    assert len(r) == int(want.sum()), (case, len(r), int(want.sum()))
    assert np.array_equal(r["offset"], off[want])
    assert np.array_equal(r["pool_index"] & 0x7FFFFFFF, idx[want])
    assert np.array_equal(co, ~keep[want])


@pytest.mark.gpu
@pytest.mark.parametrize("tail", [0, 1, 2, 5, 15, 16, 17, 1000])
def test_scan_side_guard_flags(tail):
    """1-byte keys whose list is one regexp call decided by its forward guard
    (rx's `[` and `]`: the guard tests the key and the next byte, C3) are
    decided from the bytes the scan keeps beside them (kernels.hip key_class,
    in the compaction) and skipped by pre-verification.  Random bytes with `[` / `]` planted at every lane byte, half of
    them followed by C3 (the guard passes, the call is searched), and the block
    cut `tail` bytes after a planted key (regions past the block end are never
    flagged): the device records equal the oracle's kept calls."""
    import yara_amd
    from conftest import ref_tables
    z = np.load(tables_npz("rx"))
    n = (1 << 20) + 77
    data = oracle.xorshift(n, 61).copy()
    k = 0
    for off in range(5, n - 64, 37):
        data[off] = (0x5B, 0x5D)[k & 1]
        if k % 2 == 0:
            data[off + 1] = 0xC3
        k += 1
    cut = (n - 200) + tail
    data[n - 200] = 0x5B
    data = np.ascontiguousarray(data[:cut])
    P, K = oracle.walk_verify(ref_tables("rx"), data)
    keep = oracle.literal_effect(z, P, K, data)
    r = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz("rx"), device=0, strings=True)).verify_calls(data)
    off = P.astype(np.uint64) - z["pool_backtrack"][K].astype(np.uint64)
    np.testing.assert_array_equal(r["offset"], off[keep])
    np.testing.assert_array_equal(r["pool_index"], K[keep])


@pytest.mark.gpu
@pytest.mark.parametrize("tail", [0, 1, 3, 5, 6, 7, 16, 1000])
def test_scan_side_guard_after_key(tail):
    """fuzz0's one 1-byte key (`d`, the hex string { 64 ( .. ) [0-4] 3E }) is
    decided by a guard over the five bytes after it: the scan keeps the bytes
    after the key instead of the one before (scanner.cpp key_classes picks the
    place per table), and near a lane's end or the block's end the candidate
    stays undecided.  `d` planted at every lane byte with `>` 1..7 bytes after
    it (the guard passes for 1..5) and the block cut `tail` bytes after a key:
    the device records equal the oracle's kept calls."""
    import yara_amd
    from conftest import ref_tables
    z = np.load(tables_npz("fuzz0"))
    n = (1 << 20) + 77
    data = oracle.xorshift(n, 67).copy()
    k = 0
    for off in range(5, n - 64, 37):
        data[off] = 0x64
        data[off + 1 + k % 7] = 0x3E
        k += 1
    cut = (n - 200) + tail
    data[n - 200] = 0x64
    data = np.ascontiguousarray(data[:cut])
    P, K = oracle.walk_verify(ref_tables("fuzz0"), data)
    keep = oracle.literal_effect(z, P, K, data)
    r = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz("fuzz0"), device=0, strings=True)).verify_calls(data)
    off = P.astype(np.uint64) - z["pool_backtrack"][K].astype(np.uint64)
    np.testing.assert_array_equal(r["offset"], off[keep])
    np.testing.assert_array_equal(r["pool_index"], K[keep])


def _device_records(sc, d, n, lo=0, hi=None):
    import torch
    import yara_amd
    from yara_amd._hip import memcpy
    sc.scan_device(d.data_ptr(), n, lo, n if hi is None else hi)
    _, cnt, _ = sc.device_result()
    p, m = sc.verify_device(0x2000)
    out = np.zeros(m, dtype=yara_amd._lib.VERIFY_REC_DTYPE)
    if m:
        h = torch.empty(m * 16, dtype=torch.uint8, device="cuda")
        memcpy(h.data_ptr(), p, m * 16, 3)
        out = np.frombuffer(h.cpu().numpy().tobytes(), dtype=yara_amd._lib.VERIFY_REC_DTYPE)
    return out, cnt, sc.stream_length()


def _dense_key_buffer(rules):
    """8 MiB for the drain classes' edge cases (kernels.hip drain_classes): runs
    of the rule set's 1-byte key (a dead candidate at every position, more
    dead per drain than a filter-hit entry's 8-bit count holds), the key
    followed by bytes its guard accepts, zeros, and slices of the rule set's
    planted golden case every 4 KiB (filter hits and live calls inside the
    dense runs)."""
    key = {"rx": 0x5B, "fuzz0": 0x5F, "short": 0x61}[rules]
    planted = case_data(CASES[{"rx": "rx_1M", "fuzz0": "fuzz0_256K", "short": "short_1M"}[rules]])
    d = oracle.xorshift(8 << 20, 7).copy()
    M = 1 << 20
    d[1 * M:3 * M] = key
    alive = {"rx": b"\x5b\xc3", "fuzz0": b"d_>", "short": b"ab"}[rules]
    d[3 * M:4 * M] = np.resize(np.frombuffer(alive, dtype=np.uint8), M)
    d[4 * M:5 * M] = 0
    d[5 * M:6 * M] = np.resize(np.frombuffer(bytes([key]) * 7 + alive, dtype=np.uint8), M)
    for at in range(1 * M, 6 * M, 4096):
        o = (at * 2654435761) % (len(planted) - 256)
        d[at + 1000:at + 1256] = planted[o:o + 256]
    return d


@pytest.mark.gpu
@pytest.mark.parametrize("rules,case", [
    ("rx", "rx_1M"), ("fuzz0", "fuzz0_256K"), ("fuzz3", "fuzz3_256K"), ("short", "short_1M"),
    ("lit", "lit_1M"), ("C", "C_planted16M"),
    ("rx", "xs64M"), ("fuzz0", "xs64M"), ("fuzz3", "xs64M"), ("short", "xs64M"),
    ("rx", "dense"), ("fuzz0", "dense"), ("short", "dense")])
def test_verified_only_scan_keeps_records_and_candidate_indices(rules, case):
    """Verified-only scans (yr_amd_scanner_set_verified_only: the scan kernel
    decides the 1-byte keys' classes from eight bytes around the key and leaves
    the dead candidates out of its result) yield exactly the records of a full
    scan -- the same calls, and candidate fields that still index the full
    candidate stream -- on whole blocks and on byte ranges (the full scan's
    records are pinned to the reference by the tests above)."""
    import torch
    import yara_amd
    if case == "xs64M":
        data = oracle.xorshift(64 << 20, 1)
    elif case == "dense":
        data = _dense_key_buffer(rules)
    else:
        data = case_data(CASES[case])
    n = len(data)
    d = torch.from_numpy(data.copy()).cuda()
    tab = yara_amd.Tables.from_npz(tables_npz(rules), device=0, strings=True)
    sc = yara_amd.Scanner(tab)
    cut = ((n // 3) & ~15)
    for lo, hi in ((0, n), (0, cut + 5), (cut, n)):
        full, cnt_full, len_full = _device_records(sc, d, n, lo, hi)
        sc.set_verified_only(True)
        got, cnt, length = _device_records(sc, d, n, lo, hi)
        sc.set_verified_only(False)
        assert len_full == cnt_full and length == cnt_full, (lo, hi, cnt_full, length)
        assert cnt <= cnt_full
        for f in ("offset", "pool_index", "candidate"):
            np.testing.assert_array_equal(got[f], full[f], err_msg="%s [%d, %d)" % (f, lo, hi))
        if rules in ("rx", "fuzz0") and case == "xs64M":   # dense candidates, most of them dead
            assert cnt < cnt_full // 2, (cnt, cnt_full)


@pytest.mark.gpu
@pytest.mark.parametrize("rules", ["rx", "fuzz0", "short", "fuzz3"])
def test_verified_only_first_scan_of_a_fresh_scanner(rules):
    """A verified-only scan as a FRESH scanner's first scan: its
    segments still have the default capacity, so the dense key runs overflow
    them and the scan is re-run at exact offsets under the verified-only
    instance (the dropped candidates' full-stream counts, the candidate index
    rebuilt; with kept keys, the segment write pass over the re-run's
    layout).  Records and candidate indices equal a separate full-scan
    scanner's."""
    import torch
    import yara_amd
    data = _dense_key_buffer(rules if rules != "fuzz3" else "short")
    n = len(data)
    d = torch.from_numpy(data.copy()).cuda()
    tab = yara_amd.Tables.from_npz(tables_npz(rules), device=0, strings=True)
    vo = yara_amd.Scanner(tab)
    vo.set_verified_only(True)
    got, cnt, length = _device_records(vo, d, n)
    full, cnt_full, len_full = _device_records(yara_amd.Scanner(tab), d, n)
    assert length == cnt_full == len_full and cnt <= cnt_full
    for f in ("offset", "pool_index", "candidate"):
        np.testing.assert_array_equal(got[f], full[f], err_msg=f)
    # and again on the same (now learned-capacity) scanner, over a byte range
    cut = (n // 3) & ~15
    got2, _, _ = _device_records(vo, d, n, cut, n)
    full2, _, _ = _device_records(yara_amd.Scanner(tab), d, n, cut, n)
    for f in ("offset", "pool_index", "candidate"):
        np.testing.assert_array_equal(got2[f], full2[f], err_msg=f)


@pytest.mark.gpu
def test_one_plan_drop_instance_selection():
    """scanner.cpp key_plan: rx's two 1-byte keys ('[' and ']') share one forward
    guard once each key's test of its own byte is left out -- the byte after
    the key is 0xC3 -- so its verified-only scans run the one-plan drop
    instance (kernels.hip kDropPlanModes); fuzz0 (exclusions, a backward guard)
    and the kept-key sets short / fuzz3 keep their own kernels.  (The records
    of every one of these sets are pinned by the verified-only tests above.)
    Read through the diagnostic build's yr_amd__diag_key_classes."""
    from conftest import run_diag_child
    code = (
        "import ctypes, yara_amd\n"
        "from conftest import tables_npz\n"
        "g = yara_amd._lib.lib().yr_amd__diag_key_classes\n"
        "g.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]\n"
        "for name in ('rx', 'fuzz0', 'short', 'fuzz3'):\n"
        "  t = yara_amd.Tables.from_npz(tables_npz(name), device=0, strings=True)\n"
        "  o = (ctypes.c_uint32 * 40)()\n"
        "  assert g(t._h, o) == 0\n"
        "  print('plan', name, o[29], hex(o[30]), hex(o[31]))\n")
    got = {ln.split()[1]: ln.split()[2:] for ln in run_diag_child(code).splitlines()
           if ln.startswith("plan ")}
    assert got["rx"] == ["1", "0xff00", "0xc300"], got
    assert [got[n][0] for n in ("fuzz0", "short", "fuzz3")] == ["0", "0", "0"], got
