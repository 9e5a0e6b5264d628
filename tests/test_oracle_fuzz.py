"""Live randomised check of the oracle against stock libyara (build container only).

For 200 fresh rule sets from tests/golden/fuzz_rules.py (seeds 100..299, beyond
the 12 committed as fixtures) the stock compiler builds the Aho-Corasick tables
(oracle/_ref/refdump tables) and stock yr_rules_scan_mem scans a planted
64 KiB buffer with the verify-call probe (refdump scan, oracle/refhook.c).  The
oracle restatement of scanner.c:45-176 must reproduce every verify call, and
the literal pre-verification restatement (oracle.literal_effect, scan.c) must
keep every match libyara reports for a literal string.

Needs oracle/_ref (built from /root/reference by oracle/ref.mk); skipped where
it is absent, e.g. on the GPU box, which only ever sees the committed fixtures.
"""
import os
import subprocess

import numpy as np
import pytest

import fuzz_rules
import make_golden
import oracle
from conftest import REPO
from oracle.tables import read_tables

REFDUMP = os.path.join(REPO, "oracle", "_ref", "refdump")
SEEDS = range(100, 300)
SIZE = 64 << 10
SF_LITERAL = 0x400   # STRING_FLAGS_LITERAL (types.h)

pytestmark = pytest.mark.skipif(not os.access(REFDUMP, os.X_OK),
                                reason="oracle/_ref/refdump not built (needs /root/reference)")


def _run(tmp, seed):
    rules = os.path.join(tmp, "f.yar")
    with open(rules, "w") as f:
        f.write(fuzz_rules.gen(seed))
    subprocess.run([REFDUMP, "tables", rules, os.path.join(tmp, "t.bin")], check=True,
                   stdout=subprocess.DEVNULL)
    data = fuzz_rules.buffer(oracle.xorshift, seed, SIZE)
    data.tofile(os.path.join(tmp, "d.bin"))
    prefix = os.path.join(tmp, "s")
    res = subprocess.run([REFDUMP, "scan", rules, os.path.join(tmp, "d.bin"), prefix],
                         check=True, capture_output=True, text=True)
    assert "rc=0" in res.stdout, res.stdout
    ver = np.fromfile(prefix + ".verify", dtype=[("b", "<u8"), ("p", "<u8"), ("k", "<u4")])
    mt = np.fromfile(prefix + ".matches",
                     dtype=[("s", "<u4"), ("o", "<u8"), ("l", "<u4"), ("x", "<u4")])
    return read_tables(os.path.join(tmp, "t.bin")), data, ver, mt


@pytest.mark.parametrize("seed", SEEDS)
def test_oracle_verify_stream_equals_stock_libyara(tmp_path, seed):
    t, data, ver, mt = _run(str(tmp_path), seed)
    pos, idx = oracle.walk_verify(t, data)
    assert len(pos) == len(ver)
    np.testing.assert_array_equal(pos, ver["p"])
    np.testing.assert_array_equal(idx, ver["k"])
    # candidates (the device's product) = distinct positions of the stream, plus
    # match-list states near the start whose entries all backtrack past offset 0
    # (scanner.c: verify only when backtrack <= i)
    cand = oracle.candidates(t, data)
    called = np.unique(ver["p"])
    assert np.isin(called, cand).all()
    extra = np.setdiff1d(cand, called)
    assert (extra < int(t.pool_backtrack.max(initial=0))).all(), extra
    # pre-verification (literal compares + fast-exec hex programs) keeps every
    # reported match: literals at their exact offset, hex / regexp strings with
    # an atom offset inside the match
    z = make_golden.tables_dict(t)
    keep = oracle.literal_effect(z, pos, idx, data)
    off = pos.astype(np.int64) - t.pool_backtrack[idx].astype(np.int64)
    kept = set(zip(off[keep].tolist(), t.pool_string[idx[keep]].tolist()))
    by_string = {}
    for o_, s_ in kept:
        by_string.setdefault(s_, []).append(o_)
    by_string = {k: np.sort(np.array(v, np.int64)) for k, v in by_string.items()}
    for s, o, n in zip(mt["s"].tolist(), mt["o"].tolist(), mt["l"].tolist()):
        if z["str_flags"][s] & SF_LITERAL:
            assert (o, s) in kept, (seed, s, o)
        else:
            v = by_string.get(s)
            assert v is not None, (seed, s, o)
            j = np.searchsorted(v, o)
            assert j < len(v) and v[j] <= o + n, (seed, s, o, n)
