"""Device tables straight from compiled rules files.

Fixtures: tests/golden/yarc/<set>.yarc.gz = stock yarac output for every golden
rule set (tests/golden/make_golden.py).  yr_amd_tables_load_yarc parses the
arena (arena.c:543-625, rules.c:326-370) without libyara; the tables must be
the ones the stock compiler handed YR_RULES (the same flattening statistics, and
a replay of the oracle's candidates through them reproduces the reference's
verify-call stream), and on the GPU the pre-verification records must equal
those of the tables built from the compiler's in-memory arrays.
"""
import gzip
import os

import numpy as np
import pytest

import oracle
import yara_amd
from conftest import GOLDEN, case_arrays, case_data, golden, ref_tables, tables_npz

SETS = ["B", "C", "E", "lit", "hex", "rx", "short", "root", "bytekeys"] + [
    "fuzz%d" % s for s in range(12)]
CASES = golden()["cases"]


def yarc(name):
    with gzip.open(os.path.join(GOLDEN, "yarc", "%s.yarc.gz" % name)) as f:
        return f.read()


@pytest.mark.parametrize("name", SETS)
def test_yarc_tables_equal_compiler_tables(name):
    a = yara_amd.Tables.from_yarc(yarc(name), device=-1).info()
    b = yara_amd.Tables.from_npz(tables_npz(name), device=-1).info()
    assert a == b


@pytest.mark.parametrize("case", [c for c in ("B_64M", "short_1M", "lit_1M", "hex_1M", "rx_1M",
                                               "root_4K", "short_3", "bytekeys_1M")])
def test_yarc_tables_replay_reference_stream(case):
    rec = CASES[case]
    arr = case_arrays(case)
    data = case_data(rec)
    t = yara_amd.Tables.from_yarc(yarc(rec["rules"]), device=-1)
    allp = rec["rules"] == "root"
    cand = None if allp else oracle.candidates(ref_tables(rec["rules"]), data)
    P, K = [], []

    def cb(k, off):
        K.append(k)
        P.append(off)
        return 0
    assert yara_amd.replay(t, data, cand, allp, cb) == 0
    bt = np.load(tables_npz(rec["rules"]))["pool_backtrack"]
    assert np.array_equal(np.array(K, np.uint32), arr["verify_idx"])
    assert np.array_equal(np.array(P, np.uint64) + bt[arr["verify_idx"]], arr["verify_pos"])


def test_yarc_rejects_malformed():
    good = yarc("hex")
    bad = [b"", b"YARA", good[:5], b"XARA" + good[4:], good[:4] + bytes([18]) + good[5:],
           good[:100], good[:-4], good[:-8] + b"\xff\xff\xff\xff\x00\x00\x00\x00"]
    for b in bad:
        with pytest.raises(yara_amd.YaraAmdError) as e:
            yara_amd.Tables.from_yarc(b, device=-1)
        assert e.value.code == yara_amd.INVALID_ARGUMENT


def test_yarc_mutations_never_crash():
    """Random byte flips: either a clean error or valid tables -- never a crash."""
    good = bytearray(yarc("hex"))
    rng = np.random.default_rng(7)
    outcomes = set()
    for _ in range(300):
        b = bytearray(good)
        for p in rng.integers(0, len(b), 3):
            b[int(p)] ^= int(rng.integers(1, 256))
        try:
            yara_amd.Tables.from_yarc(bytes(b), device=-1)
            outcomes.add("ok")
        except yara_amd.YaraAmdError as e:
            outcomes.add(e.code)
    assert outcomes <= {"ok", yara_amd.INVALID_ARGUMENT}


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["lit_1M", "hex_1M", "rx_1M", "C_planted16M", "E_planted16M",
                                  "short_1M", "B_planted4M_blocks"])
def test_yarc_device_tables_preverify_like_compiler_tables(case):
    rec = CASES[case]
    data = case_data(rec)
    a = yara_amd.Scanner(yara_amd.Tables.from_yarc(yarc(rec["rules"]), device=0))
    b = yara_amd.Scanner(yara_amd.Tables.from_npz(tables_npz(rec["rules"]), device=0,
                                                  strings=True))
    ra, rb = a.verify_calls(data), b.verify_calls(data)
    assert len(ra) > 0
    assert np.array_equal(ra, rb)
