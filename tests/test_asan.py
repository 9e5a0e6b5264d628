"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

yara_amd/csrc/Makefile `asan` builds the library's host side (tables.cpp
flattening, yarc.cpp's arena parser, scanner.cpp's replay and regexp program
validation) with -fsanitize=address,undefined (host only; the gfx950 code
objects are untouched and never run here) and links tests/asan/host_check.
Every run below must exit 0: a sanitizer report aborts the process.
"""
import gzip
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO, case_data, golden, tables_npz

HOST_CHECK = os.path.join(REPO, "tests", "asan", "_build", "host_check")
pytestmark = pytest.mark.skipif(not os.path.exists(HOST_CHECK),
                                reason="tests/asan/_build/host_check not built (make -C yara_amd/csrc asan)")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _run(*args):
    p = subprocess.run([HOST_CHECK] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=600, env=ENV)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    return p.stdout


@pytest.mark.parametrize("case", ["short_1M", "lit_1M", "hex_1M", "rx_1M", "root_4K", "short_3",
                                  "C_empty", "fuzz3_256K", "E_planted16M"])
def test_flatten_and_replay_under_sanitizers(case, tmp_path):
    rec = golden()["cases"][case]
    z = np.load(tables_npz(rec["rules"]))
    z["T"].astype(np.uint32).tofile(str(tmp_path / "T.bin"))
    z["M"].astype(np.uint32).tofile(str(tmp_path / "M.bin"))
    z["pool_next"].astype(np.uint32).tofile(str(tmp_path / "nx.bin"))
    z["pool_backtrack"].astype(np.uint16).tofile(str(tmp_path / "bt.bin"))
    case_data(rec).astype(np.uint8).tofile(str(tmp_path / "data.bin"))
    (tmp_path / "expect.txt").write_text("%d\n" % rec["verify_count"])
    out = _run("tables", tmp_path)
    assert "verify calls" in out


@pytest.mark.parametrize("name", ["B", "C", "E", "lit", "hex", "rx", "short", "root", "fuzz0",
                                  "fuzz5", "fuzz9"])
def test_yarc_mutations_under_sanitizers(name, tmp_path):
    with gzip.open(os.path.join(GOLDEN, "yarc", "%s.yarc.gz" % name)) as f:
        (tmp_path / "r.yarc").write_bytes(f.read())
    out = _run("yarc", tmp_path / "r.yarc", 300, sum(map(ord, name)))
    assert "300 mutations" in out


@pytest.mark.parametrize("name", ["rx", "hex", "fuzz0", "fuzz3"])
def test_regexp_program_validation_under_sanitizers(name, tmp_path):
    z = np.load(tables_npz(name))
    code = z["re_code"].astype(np.uint8)
    if code.size == 0:
        pytest.skip("no programs")
    code.tofile(str(tmp_path / "code.bin"))
    out = _run("re", tmp_path / "code.bin")
    assert "well-formed" in out


def test_copy_pool_under_sanitizers():
    """The parallel host copy (yara_amd/csrc/hostio.h CopyPool) behind
    yr_amd_pipeline_submit_dma and the multi-device staging: back-to-back jobs
    on the multi-threaded path (>= 8 MiB), injected copy failures reported for
    exactly their job, every byte copied (a helper could take a
    chunk of the next job)."""
    out = _run("copypool", 60, 7)
    assert "60 copy jobs" in out


def test_copy_pool_across_the_generation_wrap():
    """The ticket holds 24 bits of the job generation (hostio.h kGenShift = 40):
    jobs started 20 before the wrap point run on through it (a
    full-width generation no longer matched its own ticket from job 2^24 on and
    copy() waited forever)."""
    out = _run("copypool", 40, 11, (1 << 24) - 20)
    assert "40 copy jobs" in out
