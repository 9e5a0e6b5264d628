"""The walk's debug trace (tracing; scanner.c:83-96).

CPU: the oracle's trace restatement (oracle_trace, the sequential walk) is pinned
to the stock golden candidate streams -- its rows with match != 0 are exactly
the positions the stock hot loop dispatched.
GPU: yr_amd_trace_walk (one lane per position, the reference transition rule
over the last <= 4 bytes, trace.hip) equals the oracle's trace row for row, and
its match rows equal the scan kernel's candidate stream.  Bar: bit-exact.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from conftest import REPO, case_data, golden, ref_tables, tables_npz

CASES = golden()["cases"]
SMALL = [k for k, v in CASES.items()
         if v["size"] <= (1 << 20) + 64 and not v["block"] and v["rules"] != "root"]


@pytest.mark.parametrize("case", SMALL)
def test_oracle_trace_matches_golden_candidates(case):
    rec = CASES[case]
    data = case_data(rec)
    pos, st, mt = oracle.trace(ref_tables(rec["rules"]), data)
    assert np.all(st != 0)
    assert np.all(np.diff(pos.astype(np.int64)) > 0)
    cand = pos[mt != 0]
    assert len(cand) == rec["candidate_count"]
    assert oracle.positions_sha(cand) == rec["candidate_sha"]


def test_oracle_trace_root_and_empty():
    tab = ref_tables("C")
    pos, st, mt = oracle.trace(tab, np.zeros(0, np.uint8))
    assert len(pos) == 0
    rec = CASES["root_4K"]
    pos, st, mt = oracle.trace(ref_tables("root"), case_data(rec))
    # a root-accepting rule set: the root itself has a match list, but the
    # trace (like the reference's) lists only the non-root states
    assert np.all(st != 0)


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    return torch


def _device_trace(rules, data, **kw):
    import yara_amd
    torch = _torch()
    tab = yara_amd.Tables.from_npz(tables_npz(rules), device=0)
    sc = yara_amd.Scanner(tab)
    d = torch.from_numpy(data.copy()).to("cuda:0") if data.size else torch.zeros(1, dtype=torch.uint8,
                                                                               device="cuda:0")
    torch.cuda.synchronize()
    rows, total = sc.trace_walk(d.data_ptr(), int(data.size), **kw)
    return sc, d, rows, total


@pytest.mark.gpu
@pytest.mark.parametrize("case", SMALL[:12])
def test_device_trace_equals_oracle(case):
    rec = CASES[case]
    data = case_data(rec)
    sc, d, rows, total = _device_trace(rec["rules"], data)
    pos, st, mt = oracle.trace(ref_tables(rec["rules"]), data)
    assert total == len(pos)
    np.testing.assert_array_equal(rows["position"], pos)
    np.testing.assert_array_equal(rows["state"], st)
    np.testing.assert_array_equal(rows["match"], mt)
    # the trace's match rows are the scan kernel's candidate stream
    sc.scan_device(d.data_ptr(), int(data.size))
    _, cnt, allp = sc.device_result()
    assert not allp and cnt == rec["candidate_count"]
    assert oracle.positions_sha(rows["position"][rows["match"] != 0]) == rec["candidate_sha"]


@pytest.mark.gpu
def test_device_trace_capacity_and_empty():
    rec = CASES["C_planted16M"]
    data = case_data(rec)[: 1 << 20]
    _, _, full, total = _device_trace("C", data)
    assert len(full) == total > 100
    _, _, part, total2 = _device_trace("C", data, cap=100)
    assert total2 == total and len(part) == 100
    np.testing.assert_array_equal(part, full[:100])
    _, _, none, total3 = _device_trace("C", data, cap=0)
    assert total3 == total and len(none) == 0
    _, _, empty, total4 = _device_trace("C", np.zeros(0, np.uint8))
    assert total4 == 0 and len(empty) == 0


@pytest.mark.gpu
def test_device_trace_prints_reference_format():
    """YR_DEBUG_VERBOSITY=2 prints the rows in scanner.c:85-94's format."""
    code = (
        "import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "import numpy as np, torch, yara_amd\n"
        "from conftest import tables_npz\n"
        "t = yara_amd.Tables.from_npz(tables_npz('lit'), device=0)\n"
        "s = yara_amd.Scanner(t)\n"
        "data = np.frombuffer(b'xxhello worldxx' * 4, dtype=np.uint8)\n"
        "d = torch.from_numpy(data.copy()).cuda(); torch.cuda.synchronize()\n"
        "rows, n = s.trace_walk(d.data_ptr(), data.size, data_base=0x1000)\n"
        "print('ROWS', n)\n" % (REPO, os.path.join(REPO, "tests")))
    env = dict(os.environ, YR_DEBUG_VERBOSITY="2")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    n = int(r.stdout.split("ROWS")[1])
    lines = [ln for ln in r.stderr.splitlines() if "// yr_amd_trace_walk()" in ln]
    assert len(lines) == n
    for ln in lines:
        assert ln.startswith("- match_table[state=") and "block->base=0x1000" in ln
