"""End-to-end match-set parity against the stock reference libyara.

integration/_build/e2e_check compiles the rules with the stock libyara
compiler and scans the same bytes twice: through stock yr_scanner_scan_mem
(scanner.c:633) and through the re-hosted driver of integration/yr_gpu_scanner.c
(GPU candidate stream -> reference-ordered replay -> the unmodified
yr_scan_verify_match / yr_execute_code of that same libyara).  Every match of
every string ({string, base+offset, length, xor key}) and every rule report
must be identical.  The reference build (oracle/_ref) and the shim are built
in the build container and travel to the GPU box as shared objects.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import gen_rules
import oracle
import planted
from conftest import ALPHA, GOLDEN, REPO

pytestmark = pytest.mark.gpu

CHECK = os.path.join(REPO, "integration", "_build", "e2e_check")
# the same checker built against libyara + integration/libyara-block-scanner.patch:
# its GPU side calls libyara's OWN yr_scanner_scan_* with the block scanner attached
CHECK_HOOK = os.path.join(REPO, "integration", "_build", "e2e_check_hook")
needs_check = pytest.mark.skipif(not os.path.exists(CHECK),
                                 reason="integration/_build/e2e_check not built "
                                        "(needs the reference headers at build time)")


def _rules_file(tmp_path, name):
    p = tmp_path / ("%s.yar" % name)
    if name in ("short", "root", "lit", "hex", "rx", "bytekeys"):
        p.write_text(open(os.path.join(GOLDEN, "rules", name + ".yar")).read())
    else:
        p.write_text(gen_rules.gen(name))
    return str(p)


def _run(rules, data_spec, block=0, overlap=0, preverify=True, mode="mem", check=None, **extra):
    cmd = [check or CHECK, rules, data_spec] + ([str(block), str(overlap)] if block else [])
    env = dict(os.environ, E2E_PREVERIFY="1" if preverify else "0", E2E_MODE=mode, **extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.stdout, r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    return r.returncode, res


def _data_file(tmp_path, arr, name):
    p = tmp_path / name
    np.asarray(arr, dtype=np.uint8).tofile(str(p))
    return str(p)


CASES = [
    ("B", "planted", 16 << 20, 0, 0),
    ("C", "planted", 16 << 20, 0, 0),
    ("E", "planted", 16 << 20, 0, 0),
    ("C", "xs", 64 << 20, 0, 0),
    ("B", "planted", 4 << 20, 1024, 256),
    ("C", "planted", 2 << 20, 4096, 512),
    ("short", "alpha", 1 << 20, 0, 0),
    ("short", "alpha", 1 << 20, 1024, 256),
    ("root", "alpha", 4096, 0, 0),
    ("lit", "lit", 1 << 20, 0, 0),
    ("lit", "lit", 1 << 20, 4096, 512),
    ("lit", "lit", 8 << 20, 65536, 100),
    ("hex", "hex", 1 << 20, 0, 0),
    ("hex", "hex", 1 << 20, 8192, 1024),
    ("hex", "hex", 4 << 20, 3000, 64),
    ("rx", "rx", 1 << 20, 0, 0),
    ("rx", "rx", 1 << 20, 8192, 1024),
    ("rx", "rx", 4 << 20, 3000, 64),
    ("bytekeys", "alpha", 2 << 20, 0, 0),          # 1-byte keys in stage 1 (kModeByteKeys)
    ("bytekeys", "alpha", 2 << 20, 4096, 512),
]


@needs_check
@pytest.mark.parametrize("preverify", [True, False], ids=["preverify", "full-replay"])
@pytest.mark.parametrize("rules,kind,size,block,overlap", CASES)
def test_match_set_equals_stock_libyara(tmp_path, rules, kind, size, block, overlap, preverify):
    rf = _rules_file(tmp_path, rules)
    if kind == "xs":
        spec = "xs:1:%d" % size
    elif kind == "lit":
        spec = _data_file(tmp_path, planted.lit_buffer(oracle.xorshift, size, 13), "d.bin")
    elif kind == "hex":
        spec = _data_file(tmp_path, planted.hex_buffer(oracle.xorshift, size, 17), "d.bin")
    elif kind == "rx":
        spec = _data_file(tmp_path, planted.rx_buffer(oracle.xorshift, size, 19), "d.bin")
    elif kind == "planted":
        spec = _data_file(tmp_path, planted.planted_buffer(oracle.xorshift, gen_rules.gen(rules),
                                                           size, 3), "d.bin")
    else:
        x = oracle.xorshift(size, 5)
        spec = _data_file(tmp_path, np.frombuffer(ALPHA, np.uint8)[x % len(ALPHA)], "d.bin")
    rc, res = _run(rf, spec, block, overlap, preverify)
    assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, res
    assert res["same_matches"] and res["same_rule_reports"], res
    assert res["finished"] == [1, 1], res
    if kind in ("planted", "lit", "hex", "rx"):
        assert res["matches_stock"] > 0 and res["rules_matching"] > 0, res
    assert rc == 0


@needs_check
@pytest.mark.parametrize("mode", ["file", "fd", "proc"])
@pytest.mark.parametrize("rules", ["lit", "C"])
def test_file_fd_proc_entry_points_equal_stock(tmp_path, rules, mode):
    """yr_gpu_scanner_scan_file / _fd / _proc vs yr_scanner_scan_file / _fd /
    _proc (scanner.c:674-722): mmap'ed files and a stopped process's memory
    regions (proc/linux.c iterator: many blocks through the pipeline)."""
    rf = _rules_file(tmp_path, rules)
    if rules == "lit":
        buf = planted.lit_buffer(oracle.xorshift, 4 << 20, 13)
    else:
        buf = planted.planted_buffer(oracle.xorshift, gen_rules.gen("C"), 4 << 20, 3)
    spec = _data_file(tmp_path, buf, "d.bin")
    rc, res = _run(rf, spec, mode=mode)
    if mode == "proc" and res["rc_stock"] != 0:
        pytest.skip("process memory not readable here (rc %d)" % res["rc_stock"])
    assert res["mode"] == mode
    assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, res
    assert res["same_matches"] and res["same_rule_reports"], res
    assert res["matches_stock"] > 0, res
    assert rc == 0


@needs_check
@pytest.mark.parametrize("preverify", [True, False], ids=["preverify", "full-replay"])
def test_fast_mode_abort_and_too_many_matches(tmp_path, preverify):
    """Scanner semantics that depend on the order and effect of the verify
    calls: SCAN_FLAGS_FAST_MODE (scan.c:1019-1021), CALLBACK_ABORT from the
    rule-report loop (scanner.c:540-548), and strings disabled after
    YR_MAX_STRING_MATCHES with CALLBACK_MSG_TOO_MANY_MATCHES (scan.c:1055-1076)."""
    lit = _rules_file(tmp_path, "lit")
    spec = _data_file(tmp_path, planted.lit_buffer(oracle.xorshift, 2 << 20, 13), "d.bin")
    for extra in ({"E2E_FAST": "1"}, {"E2E_ABORT": "2"}, {"E2E_FAST": "1", "E2E_ABORT": "3"}):
        rc, res = _run(lit, spec, preverify=preverify, **extra)
        assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, (extra, res)
        assert res["same_matches"] and res["same_rule_reports"], (extra, res)
        want_finished = [0, 0] if "E2E_ABORT" in extra else [1, 1]
        assert res["finished"] == want_finished, (extra, res)
    # > 1,000,000 matches of "a" in 16 MiB of the 15-letter alphabet buffer
    short = _rules_file(tmp_path, "short")
    x = oracle.xorshift(16 << 20, 5)
    spec = _data_file(tmp_path, np.frombuffer(ALPHA, np.uint8)[x % len(ALPHA)], "a.bin")
    rc, res = _run(short, spec, preverify=preverify)
    assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, res
    assert res["too_many"][0] > 0 and res["too_many"] == [res["too_many"][0]] * 2, res
    assert res["same_matches"] and res["same_rule_reports"], res


@needs_check
@pytest.mark.parametrize("preverify", [True, False], ids=["preverify", "full-replay"])
def test_regexp_fiber_limit_error_is_preserved(tmp_path, preverify):
    """A yr_re_exec call that fails with ERROR_TOO_MANY_RE_FIBERS (re.c:1228,
    RE_MAX_FIBERS = 1024) fails the stock scan even though it matches nothing;
    pre-verification must keep that call (its search budget is below the fiber
    limit), so the shim reports the same error."""
    rf = tmp_path / "fib.yar"
    rf.write_text('rule fib { strings: $a = /x(a{1,40}){1,40}b/ condition: $a }\n'
                  'rule other { strings: $b = "needle" condition: $b }\n')
    d = np.zeros(64 << 10, np.uint8)
    d[100:106] = np.frombuffer(b"needle", np.uint8)
    run = b"x" + b"a" * 3000 + b"c"
    d[4096:4096 + len(run)] = np.frombuffer(run, np.uint8)
    rc, res = _run(str(rf), _data_file(tmp_path, d, "d.bin"), preverify=preverify)
    assert res["rc_stock"] == 46 and res["rc_gpu"] == 46, res   # ERROR_TOO_MANY_RE_FIBERS


def _alpha_file(tmp_path, size, name="a.bin"):
    x = oracle.xorshift(size, 5)
    return _data_file(tmp_path, np.frombuffer(ALPHA, np.uint8)[x % len(ALPHA)], name)


@needs_check
@pytest.mark.parametrize("preverify", [True, False], ids=["preverify", "full-replay"])
@pytest.mark.parametrize("block", [0, 1 << 20], ids=["one-block", "pipeline"])
def test_scan_timeout_inside_a_block(tmp_path, preverify, block):
    """ERROR_SCAN_TIMEOUT from the walk's own checks (scanner.c:74-81: every
    4096 positions of a block).  The callback sleeps past the 1 s timeout when
    CALLBACK_MSG_TOO_MANY_MATCHES arrives (inside yr_scan_verify_match, in the
    middle of the 16 MiB buffer); the next check of the reference walk fires,
    and the GPU replay must make that check too (before this round it checked
    only around the GPU pass, so it returned ERROR_SUCCESS)."""
    short = _rules_file(tmp_path, "short")
    spec = _alpha_file(tmp_path, 16 << 20)
    rc, res = _run(short, spec, block, 0 if not block else 64, preverify,
                   E2E_TIMEOUT="1", E2E_SLEEP_TOO_MANY="1200")
    assert res["too_many"][0] >= 1 and res["too_many"][1] >= 1, res
    assert res["rc_stock"] == 26 and res["rc_gpu"] == 26, res   # ERROR_SCAN_TIMEOUT


@needs_check
def test_no_timeout_without_sleep(tmp_path):
    """Same scan, same 1 s timeout, no sleep: both finish (the timeout checks
    themselves change nothing)."""
    short = _rules_file(tmp_path, "short")
    spec = _alpha_file(tmp_path, 16 << 20)
    rc, res = _run(short, spec, E2E_TIMEOUT="5")
    assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, res
    assert res["same_matches"] and res["same_rule_reports"], res


@needs_check
@pytest.mark.parametrize("preverify", [True, False], ids=["preverify", "full-replay"])
def test_scan_mem_of_truncated_mapping(tmp_path, preverify):
    """yr_scanner_scan_mem over an mmap whose file was truncated underneath:
    the stock walk faults inside YR_TRYCATCH -> ERROR_COULD_NOT_MAP_FILE
    (scanner.c:493-496).  The shim's in-place scan_mem touches the caller's
    pages inside the trycatch before its H2D, so it returns the same code
    instead of faulting inside the HIP runtime."""
    lit = _rules_file(tmp_path, "lit")
    spec = _data_file(tmp_path, planted.lit_buffer(oracle.xorshift, 4 << 20, 13), "d.bin")
    rc, res = _run(lit, spec, preverify=preverify, mode="truncmap")
    assert res["rc_stock"] == 4 and res["rc_gpu"] == 4, res   # ERROR_COULD_NOT_MAP_FILE
    assert res["finished"] == [0, 0], res


@needs_check
@pytest.mark.parametrize("block,devices", [(12 << 20, None), (12 << 20, "0,0,0"), (0, "0,0")],
                         ids=["pipeline", "pipeline-3-devices", "scan_mem-2-devices"])
def test_truncated_mapping_through_pinned_staging(tmp_path, block, devices):
    """The same truncated mapping through the paths that copy the block into
    pinned staging with helper threads (yr_amd_pipeline_submit_dma, the
    multi-device pipeline, the staged multi-device scan_mem): every chunk is
    copied by the shim's _guarded_copy inside YR_TRYCATCH, so the pages past
    the truncation fault on a helper thread and the scan returns
    ERROR_COULD_NOT_MAP_FILE like the stock walk -- no SIGBUS, no hang
    (ADVICE r03).  12 MiB blocks: the parallel copy path (>= 8 MiB); the file
    is cut in the middle of the second block."""
    lit = _rules_file(tmp_path, "lit")
    spec = _data_file(tmp_path, planted.lit_buffer(oracle.xorshift, 32 << 20, 13), "d.bin")
    extra = {} if devices is None else {"E2E_DEVICES": devices, "E2E_MULTI_MIN": str(1 << 20)}
    rc, res = _run(lit, spec, block=block, mode="truncmap", **extra)
    assert res["rc_stock"] == 4 and res["rc_gpu"] == 4, res   # ERROR_COULD_NOT_MAP_FILE
    assert res["finished"] == [0, 0], res


@needs_check
@pytest.mark.parametrize("rules,block", [("C", 0), ("lit", 65536)])
def test_threads_share_one_gpu_rules(tmp_path, rules, block):
    """N threads, each with its own YR_SCANNER and YR_GPU_SCANNER, scanning
    concurrently on ONE shared YR_GPU_RULES (as N scanners share one YR_RULES,
    docs/capi.rst:330-347, cli/yara.c:1564-1608): every scan's match set and
    rule reports equal stock."""
    rf = _rules_file(tmp_path, rules)
    if rules == "lit":
        buf = planted.lit_buffer(oracle.xorshift, 4 << 20, 13)
    else:
        buf = planted.planted_buffer(oracle.xorshift, gen_rules.gen("C"), 4 << 20, 3)
    spec = _data_file(tmp_path, buf, "d.bin")
    rc, res = _run(rf, spec, block, 100 if block else 0, E2E_THREADS="6", E2E_THREAD_REPS="3")
    assert res["threads"] == 6 and res["threads_ok"], res
    assert res["same_matches"] and res["matches_stock"] > 0, res
    assert rc == 0


needs_hook = pytest.mark.skipif(not os.path.exists(CHECK_HOOK),
                                reason="integration/_build/e2e_check_hook not built "
                                       "(oracle/refpatch.mk needs the reference tree)")


@needs_hook
@pytest.mark.parametrize("mode,block", [("mem", 0), ("mem", 65536), ("file", 0), ("fd", 0),
                                        ("proc", 0), ("truncmap", 0)])
@pytest.mark.parametrize("rules", ["lit", "rx", "C"])
def test_patched_libyara_block_scanner(tmp_path, rules, mode, block):
    """libyara patched with integration/libyara-block-scanner.patch: the GPU
    scanner attached with yr_gpu_scanner_attach, the scan made through
    libyara's own yr_scanner_scan_mem / _mem_blocks / _file / _fd / _proc.
    Match sets and rule reports equal the same library's CPU walk (no block
    scanner attached = stock behaviour)."""
    rf = _rules_file(tmp_path, rules)
    if rules == "lit":
        buf = planted.lit_buffer(oracle.xorshift, 4 << 20, 13)
    elif rules == "rx":
        buf = planted.rx_buffer(oracle.xorshift, 4 << 20, 19)
    else:
        buf = planted.planted_buffer(oracle.xorshift, gen_rules.gen("C"), 4 << 20, 3)
    spec = _data_file(tmp_path, buf, "d.bin")
    rc, res = _run(rf, spec, block, 100 if block else 0, mode=mode, check=CHECK_HOOK)
    if mode == "proc" and res["rc_stock"] != 0:
        pytest.skip("process memory not readable here (rc %d)" % res["rc_stock"])
    if mode == "truncmap":
        assert res["rc_stock"] == 4 and res["rc_gpu"] == 4, res
        return
    assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, res
    assert res["same_matches"] and res["same_rule_reports"] and res["matches_stock"] > 0, res
    assert rc == 0


@needs_hook
def test_patched_libyara_timeout_and_threads(tmp_path):
    short = _rules_file(tmp_path, "short")
    spec = _alpha_file(tmp_path, 16 << 20)
    rc, res = _run(short, spec, 1 << 20, 64, check=CHECK_HOOK, E2E_TIMEOUT="1",
                   E2E_SLEEP_TOO_MANY="1200")
    assert res["rc_stock"] == 26 and res["rc_gpu"] == 26, res
    rf = _rules_file(tmp_path, "C")
    buf = planted.planted_buffer(oracle.xorshift, gen_rules.gen("C"), 4 << 20, 3)
    rc, res = _run(rf, _data_file(tmp_path, buf, "d.bin"), check=CHECK_HOOK, E2E_THREADS="4",
                   E2E_THREAD_REPS="2")
    assert res["threads_ok"] and res["same_matches"], res


MULTI_CASES = [
    ("C", "planted", 24 << 20, 0, 0, "0,0,0"),
    ("lit", "lit", 16 << 20, 0, 0, "0,0,0,0,0,0,0,0"),
    ("hex", "hex", 8 << 20, 0, 0, "0,0"),
    ("rx", "rx", 12 << 20, 5 << 20, 1024, "0,0,0"),      # blocks of 5 MiB, each split
    ("bytekeys", "alpha", 6 << 20, 0, 0, "0,0,0"),
]


def _spec(tmp_path, rules, kind, size):
    if kind == "lit":
        return _data_file(tmp_path, planted.lit_buffer(oracle.xorshift, size, 13), "d.bin")
    if kind == "hex":
        return _data_file(tmp_path, planted.hex_buffer(oracle.xorshift, size, 17), "d.bin")
    if kind == "rx":
        return _data_file(tmp_path, planted.rx_buffer(oracle.xorshift, size, 19), "d.bin")
    if kind == "planted":
        return _data_file(tmp_path, planted.planted_buffer(oracle.xorshift, gen_rules.gen(rules),
                                                           size, 3), "d.bin")
    x = oracle.xorshift(size, 5)
    return _data_file(tmp_path, np.frombuffer(ALPHA, np.uint8)[x % len(ALPHA)], "d.bin")


@needs_check
@pytest.mark.parametrize("rules,kind,size,block,overlap,devices", MULTI_CASES)
def test_multi_device_match_set_equals_stock(tmp_path, rules, kind, size, block, overlap, devices):
    """Multi-device scans through the shim (yr_gpu_rules_create_multi, N
    logical devices on the box's GPU): every block of >= 1 MiB is split
    across the devices (shard + verify halos each), and the match set and
    rule reports equal stock libyara's."""
    rf = _rules_file(tmp_path, rules)
    spec = _spec(tmp_path, rules, kind, size)
    rc, res = _run(rf, spec, block, overlap, E2E_DEVICES=devices, E2E_MULTI_MIN=str(1 << 20))
    assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, res
    assert res["same_matches"] and res["same_rule_reports"], res
    assert res["devices"] == devices.count(",") + 1 and res["multi_blocks"] > 0, res
    if kind != "alpha":
        assert res["matches_stock"] > 0, res
    assert rc == 0


CHECK_PROF = os.path.join(REPO, "integration", "_build", "e2e_check_prof")
needs_prof = pytest.mark.skipif(not os.path.exists(CHECK_PROF),
                                reason="integration/_build/e2e_check_prof not built "
                                       "(oracle/refprof.mk needs the reference at build time)")


@needs_prof
@pytest.mark.parametrize("rules,kind,size,block,overlap,extra", [
    ("lit", "lit", 1 << 20, 0, 0, {}),
    ("lit", "lit", 1 << 20, 4096, 512, {"E2E_FAST": "1"}),
    ("C", "planted", 4 << 20, 0, 0, {}),
    ("hex", "hex", 1 << 20, 0, 0, {}),
    ("rx", "rx", 1 << 20, 8192, 1024, {}),
    ("short", "alpha", 16 << 20, 0, 0, {}),        # strings disabled after too many matches
    ("C", "planted", 8 << 20, 0, 0, {"E2E_DEVICES": "0,0,0", "E2E_MULTI_MIN": str(1 << 20)}),
])
def test_profiling_counters_equal_stock(tmp_path, rules, kind, size, block, overlap, extra):
    """libyara built with YR_PROFILING_ENABLED (oracle/refprof.mk): the
    per-rule atom_matches counters (scan.c:1077-1083, reported by
    yr_scanner_get_profiling_info, scanner.c:758-829) of the GPU scan equal
    stock's, pre-verification on -- dropped calls come back as count-only
    records counted on the host in the reference's call order."""
    rf = _rules_file(tmp_path, rules)
    spec = _spec(tmp_path, rules, kind, size)
    cmd = [CHECK_PROF, rf, spec] + ([str(block), str(overlap)] if block else [])
    env = dict(os.environ, E2E_PREVERIFY="1", E2E_MODE="mem", **extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    lines = [json.loads(x) for x in r.stdout.strip().splitlines() if x.startswith("{")]
    prof, res = lines[-2], lines[-1]
    assert res["rc_stock"] == 0 and res["rc_gpu"] == 0, res
    assert res["same_matches"] and res["same_rule_reports"], res
    assert prof["atom_matches_equal"], prof
    assert prof["atom_matches_stock"] > 0, prof
