"""C-ABI checks that need no GPU: exports, host-only flattening, replay order,
error behaviour (libyara ERROR_* conventions)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
import yara_amd
from yara_amd import _lib
from conftest import REPO, case_arrays, case_data, golden, ref_tables, run_diag_child, tables_npz

HEADER = os.path.join(REPO, "include", "yara_amd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(yr_amd_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 10
    L = _lib.lib()
    for n in names:
        assert hasattr(L, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (yr_amd_\w+)", out))
    assert set(names) <= exported
    assert set(_lib.PROTOTYPES) == set(names)   # the Python binding covers the ABI exactly


def test_library_is_gfx950_code():
    """The embedded code object targets gfx950 (MI355X) and only gfx950."""
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"gfx90a" not in blob


@pytest.mark.parametrize("name,states,depth,keys", [
    ("B", 3244, [1, 252, 991, 1000, 1000], [0, 0, 0, 0, 1000]),
    ("C", 29923, [1, 256, 9064, 11501, 9101], [0, 0, 0, 2426, 9101]),
    ("E", 28983, [1, 253, 2972, 8757, 17000], [0, 0, 0, 0, 17000]),
])
def test_flattening_stats(name, states, depth, keys):
    t = yara_amd.Tables.from_npz(tables_npz(name), device=-1)
    inf = t.info()
    assert inf["n_states"] == states
    assert inf["states_by_depth"] == depth
    assert inf["keys_by_length"] == keys
    assert inf["max_depth"] == 4 and inf["root_accepting"] == 0
    # filter density bounds the stage-2 rate
    assert inf["filter_set_bits"] / (1 << inf["filter_bits"]) < 0.05
    # 4-byte keys only: the even-position filter (internal.h kFilterEven), its
    # block hashed where that lets fewer random windows pass (config E)
    assert inf["filter_mode"] == {"B": 1, "C": 0, "E": 2}[name]


FORM_CODE = ("import yara_amd\nfrom conftest import tables_npz\n"
             "print('modes', *[yara_amd.Tables.from_npz(tables_npz(n), device=-1).info()"
             "['filter_mode'] for n in ('B', 'E')])\n")


def test_pair_filter_switch():
    """YAMD_PAIR_FILTER (diagnostic build): the pair filter for 4-byte-key sets."""
    assert run_diag_child(FORM_CODE, {"YAMD_PAIR_FILTER": "1"}).split()[-3:] == ["modes", "0", "0"]


@pytest.mark.parametrize("form,mode", [("plain", 1), ("hash", 2)])
def test_even_filter_forms(form, mode):
    """YAMD_EVEN_FILTER (diagnostic build) forces one even-filter block form."""
    out = run_diag_child(FORM_CODE, {"YAMD_EVEN_FILTER": form})
    assert out.split()[-3:] == ["modes", str(mode), str(mode)]


def test_product_library_ignores_ab_switches(monkeypatch):
    """The product library reads none of the A/B switches: with
    them set, B and E still get the host's own filter choice."""
    monkeypatch.setenv("YAMD_PAIR_FILTER", "1")
    monkeypatch.setenv("YAMD_EVEN_FILTER", "plain")
    monkeypatch.setenv("YAMD_NO_GUARDS", "1")
    modes = [yara_amd.Tables.from_npz(tables_npz(n), device=-1).info()["filter_mode"]
             for n in ("B", "E")]
    assert modes == [1, 2]
    assert not hasattr(yara_amd._lib.lib(), "yr_amd__diag_kernel_mode")


def test_short_and_root_tables():
    s = yara_amd.Tables.from_npz(tables_npz("short"), device=-1).info()
    assert s["keys_by_length"][1] >= 1 and s["keys_by_length"][2] >= 1
    r = yara_amd.Tables.from_npz(tables_npz("root"), device=-1).info()
    assert r["root_accepting"] == 1


REPLAY_CASES = ["A_sample", "B_64M", "C_64M", "short_1M", "root_4K", "C_empty", "short_3",
                "C_planted16M"]


@pytest.mark.parametrize("case", REPLAY_CASES)
def test_replay_of_oracle_candidates_reproduces_reference(case):
    """Host replay (product) fed the oracle's candidate stream == reference calls."""
    rec = golden()["cases"][case]
    data = case_data(rec)
    tab = ref_tables(rec["rules"])
    t = yara_amd.Tables.from_npz(tables_npz(rec["rules"]), device=-1)
    allp = bool(t.info()["root_accepting"])
    cand = None if allp else oracle.candidates(tab, data)
    P, K = [], []

    def verify(k, off):
        K.append(k)
        P.append(off + int(tab.pool_backtrack[k]))
        return 0
    assert yara_amd.replay(t, data, cand, allp, verify) == 0
    pos, idx = np.array(P, np.uint64), np.array(K, np.uint32)
    assert len(pos) == rec["verify_count"]
    assert oracle.verify_stream_sha(pos, idx) == rec["verify_sha"]
    full = case_arrays(case)
    np.testing.assert_array_equal(pos, full["verify_pos"])
    np.testing.assert_array_equal(idx, full["verify_idx"])


def test_replay_propagates_verify_error():
    """A failing verify aborts the block (GOTO_EXIT_ON_ERROR, scanner.c:111)."""
    rec = golden()["cases"]["short_1M"]
    data = case_data(rec)
    t = yara_amd.Tables.from_npz(tables_npz("short"), device=-1)
    cand = oracle.candidates(ref_tables("short"), data)
    calls = []

    def verify(k, off):
        calls.append(k)
        return 30 if len(calls) == 5 else 0   # ERROR_TOO_MANY_MATCHES
    assert yara_amd.replay(t, data, cand, False, verify) == 30
    assert len(calls) == 5


def test_replay_rejects_unsorted_and_out_of_range():
    data = case_data(golden()["cases"]["short_1M"])[:4096]
    t = yara_amd.Tables.from_npz(tables_npz("short"), device=-1)
    cand = oracle.candidates(ref_tables("short"), data)
    assert cand.size > 3
    bad = cand.copy()
    bad[[1, 2]] = bad[[2, 1]]
    assert yara_amd.replay(t, data, bad, False, lambda k, o: 0) == _lib.INVALID_ARGUMENT
    assert yara_amd.replay(t, data, np.array([data.size + 1], np.uint64), False,
                           lambda k, o: 0) == _lib.INVALID_ARGUMENT


def test_replay_rejects_non_candidate():
    data = np.zeros(64, np.uint8)   # no atom of `C` is all zeros
    t = yara_amd.Tables.from_npz(tables_npz("C"), device=-1)
    assert yara_amd.replay(t, data, np.array([10], np.uint64), False,
                           lambda k, o: 0) == _lib.INTERNAL_FATAL_ERROR


def _mk(T, M, nx=(), bt=()):
    return yara_amd.Tables(np.array(T, np.uint32), np.array(M, np.uint32),
                           np.array(nx, np.uint32), np.array(bt, np.uint16), device=-1)


def test_rejects_trie_deeper_than_max_atom_length():
    # chain of 5 states each with one child on byte 0x41 ('A'), rows 512 apart
    n = 512 * 7
    T = np.zeros(n, np.uint32)
    M = np.zeros(n, np.uint32)
    rows = [0] + [512 * (k + 1) for k in range(6)]
    for d in range(5):
        s, c = rows[d], rows[d + 1]
        T[s + 0x41 + 1] = (c << 9) | (0x41 + 1)
    M[rows[5]] = 1
    with pytest.raises(yara_amd.YaraAmdError) as e:
        yara_amd.Tables(T, M, np.array([0], np.uint32), np.array([5], np.uint16), device=-1)
    assert e.value.code == _lib.INVALID_ARGUMENT


def test_rejects_cyclic_match_pool():
    T = np.zeros(1024, np.uint32)
    M = np.zeros(1024, np.uint32)
    T[0x41 + 1] = (512 << 9) | (0x41 + 1)   # root --'A'--> state at slot 512
    M[512] = 1
    _mk(T, M, nx=[0, 1], bt=[1, 1])          # well-formed: accepted
    with pytest.raises(yara_amd.YaraAmdError) as e:
        _mk(T, M, nx=[2, 1], bt=[1, 1])      # 1 -> 2 -> 1 ...
    assert e.value.code == _lib.INVALID_ARGUMENT


def test_rejects_failure_links_that_do_not_shorten_and_rows_past_the_table():
    """The walk follows T[state] >> 9 (scanner.c:124-141): a failure link to a
    state that is not shallower could loop forever, a row past the end of T
    would read out of bounds -- both are rejected at creation."""
    T = np.zeros(1024, np.uint32)
    M = np.zeros(1024, np.uint32)
    T[0x41 + 1] = (512 << 9) | (0x41 + 1)   # root --'A'--> slot 512
    M[512] = 1
    _mk(T, M, nx=[0], bt=[1])                # failure of 512 = root: fine
    T2 = T.copy()
    T2[512] = 512 << 9                       # failure link to itself
    with pytest.raises(yara_amd.YaraAmdError) as e:
        _mk(T2, M, nx=[0], bt=[1])
    assert e.value.code == _lib.INVALID_ARGUMENT
    T3 = T.copy()
    T3[512] = 5000 << 9                      # failure link outside T
    with pytest.raises(yara_amd.YaraAmdError) as e:
        _mk(T3, M, nx=[0], bt=[1])
    assert e.value.code == _lib.INVALID_ARGUMENT
    with pytest.raises(yara_amd.YaraAmdError) as e:   # state row 512..768 past n = 700
        _mk(T[:700].copy(), M[:700].copy(), nx=[0], bt=[1])
    assert e.value.code == _lib.INVALID_ARGUMENT


def test_scanner_on_host_only_tables_is_invalid():
    t = yara_amd.Tables.from_npz(tables_npz("B"), device=-1)
    with pytest.raises(yara_amd.YaraAmdError) as e:
        yara_amd.Scanner(t)
    assert e.value.code == _lib.INVALID_ARGUMENT


def test_version():
    assert "gfx950" in yara_amd.version()


def _host_tables(name="lit"):
    return yara_amd.Tables.from_npz(tables_npz(name), device=-1)


def test_set_strings_validates_before_touching_the_device():
    """yr_amd_tables_set_strings: pool/string indexes and byte ranges are checked
    (ERROR_INVALID_ARGUMENT), and host-only tables cannot carry device strings."""
    L = _lib.lib()
    z = np.load(tables_npz("lit"))
    t = _host_tables()
    n_pool, n_str = len(z["pool_string"]), len(z["str_flags"])
    recs = (_lib.String * n_str)()
    blob = np.zeros(64, np.uint8)
    low = np.arange(256, dtype=np.uint8)
    ps = np.ascontiguousarray(z["pool_string"], np.uint32)
    u8 = lambda a: a.ctypes.data_as(_lib._u8p)  # noqa: E731
    u32 = lambda a: a.ctypes.data_as(_lib._u32p)  # noqa: E731
    # wrong pool size
    assert L.yr_amd_tables_set_strings(t.handle, u32(ps), n_pool - 1, recs, n_str, u8(blob), 64,
                                       u8(low)) == yara_amd.INVALID_ARGUMENT
    # string index out of range
    bad = ps.copy()
    bad[0] = n_str
    assert L.yr_amd_tables_set_strings(t.handle, u32(bad), n_pool, recs, n_str, u8(blob), 64,
                                       u8(low)) == yara_amd.INVALID_ARGUMENT
    # bytes out of range
    recs[0].length, recs[0].bytes_offset = 10, 60
    assert L.yr_amd_tables_set_strings(t.handle, u32(ps), n_pool, recs, n_str, u8(blob), 64,
                                       u8(low)) == yara_amd.INVALID_ARGUMENT
    recs[0].length, recs[0].bytes_offset = 0, 0
    # valid, but host-only tables
    assert L.yr_amd_tables_set_strings(t.handle, u32(ps), n_pool, recs, n_str, u8(blob), 64,
                                       u8(low)) == yara_amd.INVALID_ARGUMENT
    # missing lowercase table / null tables
    assert L.yr_amd_tables_set_strings(t.handle, u32(ps), n_pool, recs, n_str, u8(blob), 64,
                                       None) == yara_amd.INVALID_ARGUMENT
    assert L.yr_amd_tables_set_strings(None, u32(ps), n_pool, recs, n_str, u8(blob), 64,
                                       u8(low)) == yara_amd.INVALID_ARGUMENT


def test_set_re_code_requires_strings():
    L = _lib.lib()
    t = _host_tables("hex")
    n = len(np.load(tables_npz("hex"))["pool_next"])
    z = np.zeros(n, np.uint32)
    code = np.array([0xAD], np.uint8)
    assert L.yr_amd_tables_set_re_code(
        t.handle, n, *[z.ctypes.data_as(_lib._u32p)] * 4, code.ctypes.data_as(_lib._u8p),
        1) == yara_amd.INVALID_ARGUMENT


def test_pipeline_and_verify_reject_bad_handles():
    L = _lib.lib()
    p = ctypes.c_void_p()
    assert L.yr_amd_pipeline_create(None, 2, ctypes.byref(p)) == yara_amd.INVALID_ARGUMENT
    t = _host_tables()
    assert L.yr_amd_pipeline_create(t.handle, 0, ctypes.byref(p)) == yara_amd.INVALID_ARGUMENT
    assert L.yr_amd_pipeline_create(t.handle, 9, ctypes.byref(p)) == yara_amd.INVALID_ARGUMENT
    assert L.yr_amd_pipeline_submit(None, None, 0, 0) == yara_amd.INVALID_ARGUMENT
    assert L.yr_amd_pipeline_next(None, None, None, None, None, None) == yara_amd.INVALID_ARGUMENT
    assert L.yr_amd_pipeline_destroy(None) == yara_amd.SUCCESS
    assert L.yr_amd_verify_device(None, 0, None, None) == yara_amd.INVALID_ARGUMENT
    assert L.yr_amd_scan_block_verified(None, None, 0, 0, None, None) == yara_amd.INVALID_ARGUMENT


def test_debug_verbosity_dumps_candidate_states(tmp_path):
    """YR_DEBUG_VERBOSITY=2 (libyara's own switch, globals.h:51-90): the host
    replay prints every candidate's state and match-table entry, the analogue
    of scanner.c:83-96 (CPU: host-only tables, oracle candidates)."""
    import subprocess
    import sys
    code = (
        "import sys, numpy as np; sys.path[:0] = %r\n"
        "import oracle, yara_amd\n"
        "from conftest import ref_tables, tables_npz\n"
        "t = yara_amd.Tables.from_npz(tables_npz('short'), device=-1)\n"
        "d = np.frombuffer(b'xxabcdxxaaaa', np.uint8)\n"
        "c = oracle.candidates(ref_tables('short'), d)\n"
        "yara_amd.replay(t, d, c, False, lambda k, o: 0)\n"
        "print(len(c))\n" % [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")])
    env = dict(os.environ, YR_DEBUG_VERBOSITY="2")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=120)
    assert p.returncode == 0, p.stderr
    n = int(p.stdout.strip().splitlines()[-1])
    lines = [l for l in p.stderr.splitlines() if "match_table[state=" in l]
    assert n > 0 and len(lines) == n, (n, p.stderr[-2000:])
