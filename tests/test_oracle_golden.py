"""Pin the CPU oracle (oracle/ac_oracle.c) to the reference's own outputs.

Every golden verify-call stream was recorded from the stock libyara build
(hooked calls of _yr_scanner_scan_mem_block -> yr_scan_verify_match,
oracle/refhook.c).  The oracle restatement of scanner.c:45-176 must reproduce
each one exactly -- count, SHA-256 and, where stored, every record.
"""
import numpy as np
import pytest

import oracle
from conftest import case_arrays, case_data, golden, ref_tables

CASES = golden()["cases"]
SMALL = [k for k, v in CASES.items() if v["size"] <= (64 << 20)]


def blocks(size, bsize, overlap):
    """Block layout of the tests/util.c-style overlapping iterator (refdump.c)."""
    if size == 0:
        return [(0, 0)]
    out, base = [], 0
    while base < size:
        n = min(bsize, size - base)
        out.append((base, n))
        base = size if base + n >= size else base + n - overlap
    return out


@pytest.mark.parametrize("case", SMALL)
def test_oracle_matches_reference_verify_stream(case):
    rec = CASES[case]
    tab = ref_tables(rec["rules"])
    data = case_data(rec)
    assert data.size == rec["size"]
    if rec["block"]:
        P, K, B = [], [], []
        for base, n in blocks(data.size, rec["block"], rec["overlap"]):
            p, k = oracle.walk_verify(tab, data[base:base + n])
            P.append(p); K.append(k); B.append(np.full(p.size, base, np.uint64))
        pos, idx, base = np.concatenate(P), np.concatenate(K), np.concatenate(B)
        sha = oracle.verify_stream_sha(pos, idx, base=base)
    else:
        pos, idx = oracle.walk_verify(tab, data)
        base = None
        sha = oracle.verify_stream_sha(pos, idx)
    assert len(pos) == rec["verify_count"]
    assert sha == rec["verify_sha"]
    full = case_arrays(case)
    if full is not None:
        np.testing.assert_array_equal(pos, full["verify_pos"])
        np.testing.assert_array_equal(idx, full["verify_idx"])
        if base is not None:
            np.testing.assert_array_equal(base, full["verify_base"])
    if not rec["block"]:
        cand = oracle.candidates(tab, data)
        assert len(cand) == rec["candidate_count"]
        assert oracle.positions_sha(cand) == rec["candidate_sha"]


def test_oracle_parallel_slices_equal_full_walk():
    """4-byte warm-up slices (the CPU-baseline mode) reproduce the full stream."""
    tab = ref_tables("C")
    data = oracle.xorshift(8 << 20, 1)
    full = oracle.candidates(tab, data)
    for nt in (1, 3, 8):
        assert oracle.count_parallel(tab, data, nt) == len(full)


def test_reference_table_stats_match_survey():
    """Slot/pool counts of the stock compiler."""
    t = golden()["tables"]
    assert (t["B"]["slots"], t["B"]["pool"]) == (6937, 1000)
    assert (t["C"]["slots"], t["C"]["pool"]) == (60136, 11530)
    assert (t["E"]["slots"], t["E"]["pool"]) == (58337, 17000)
    assert t["root"]["root_list"] == 1 and t["C"]["root_list"] == 0


def test_config_d_shards_pinned_to_stock():
    """Config D's per-shard goldens (tests/golden/config_d.json) were computed
    by the stock reference libyara (refdump over each shard's window) and by
    the oracle restatement, asserted equal (make_config_d.py); shard 0 is the
    stock golden C_4G."""
    import json
    import os
    from conftest import GOLDEN
    with open(os.path.join(GOLDEN, "config_d.json")) as f:
        d = json.load(f)
    assert d["provenance"] == "stock" and len(d["shards"]) == 8
    c4 = golden()["cases"]["C_4G"]
    assert (d["shards"][0]["count"], d["shards"][0]["sha"]) == (c4["candidate_count"],
                                                               c4["candidate_sha"])


def test_oracle_equals_stock_deep_in_config_d(tmp_path):
    """A live cross-check where the reference build exists (the build
    container): stock libyara (refdump, "xst:" jump-ahead input) and the oracle
    give the same candidates over 32 MiB starting 28 GiB into config D's
    block (shard 7)."""
    import os
    import subprocess
    import gen_rules
    from conftest import REPO
    refdump = os.path.join(REPO, "oracle", "_ref", "refdump")
    if not os.path.exists(refdump):
        pytest.skip("oracle/_ref/refdump not built (no reference tree)")
    lo, n = (28 << 30) - 64, (32 << 20) + 64
    (tmp_path / "C.yar").write_text(gen_rules.gen("C"))
    subprocess.run([refdump, "scan", str(tmp_path / "C.yar"),
                    "xst:%d:%d" % (oracle.xorshift_state(1, lo), n), str(tmp_path / "s")],
                   check=True, stdout=subprocess.DEVNULL)
    rec = np.fromfile(str(tmp_path / "s.verify"), dtype=[("b", "<u8"), ("p", "<u8"), ("k", "<u4")])
    stock = np.unique(rec["p"])
    stock = stock[stock > 64]
    cand = oracle.candidates(ref_tables("C"), oracle.xorshift_at(n, 1, lo)).astype(np.uint64)
    cand = cand[cand > 64]
    assert stock.size > 1000
    np.testing.assert_array_equal(stock, cand)
