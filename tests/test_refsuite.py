"""libyara's own known-answer suites through the GPU scan path.

tests/test-rules.c (every string / hex / xor / wide / base64 / regexp group of
the reference, three iterator passes: default single block, test iterator,
1024-byte blocks with 256-byte overlap -- test-rules.c:3694-3825),
tests/test-async.c (three interleaved scanners with ERROR_BLOCK_NOT_READY
resumption, test-async.c:45-216) and tests/test-api.c (scanner API,
ERROR_TOO_MANY_MATCHES, report flags, scan_file, too-many-matches warnings,
test-api.c:43-996) are compiled in place from the reference by
oracle/refsuite.mk twice:

  <suite>      linked with the stock libyara: must pass (pins the fixtures)
  <suite>-gpu  every scan entry point renamed into integration/refsuite_gpu.c,
               i.e. the GPU candidate stream (+ on-device pre-verification)
               replayed into the unmodified yr_scan_verify_match

The data files the suites read (tests/data/{base64,xor*.out,baz.yar,foo.yar,
include/bar.yar}) are committed fixtures under tests/golden/refdata; x.txt is
1,000,099 bytes of 'X' and is written at run time.
"""
import os
import re
import shutil
import subprocess

import pytest

from conftest import REPO, gpu_available

SUITE = os.path.join(REPO, "oracle", "_ref", "suite")
REFDATA = os.path.join(REPO, "tests", "golden", "refdata")
SUITES = ["test-rules", "test-async", "test-api"]


@pytest.fixture(scope="module")
def topdir(tmp_path_factory):
    d = tmp_path_factory.mktemp("refsuite")
    shutil.copytree(os.path.join(REFDATA, "tests"), str(d / "tests"))
    with open(str(d / "tests" / "data" / "x.txt"), "wb") as f:
        f.write(b"X" * 1000099)
    return str(d)


def _run(binary, topdir, env_extra=None, timeout=600):
    if not os.path.exists(binary):
        pytest.skip("%s not built (oracle/refsuite.mk needs the reference tree)" % binary)
    env = dict(os.environ, TOP_SRCDIR=topdir)
    env.update(env_extra or {})
    p = subprocess.run([binary], cwd=topdir, env=env, capture_output=True, text=True,
                       timeout=timeout)
    return p


@pytest.mark.parametrize("suite", SUITES)
def test_stock_suite_passes(suite, topdir):
    """The upstream suites pass on the stock reference build with the committed
    fixtures (what the GPU runs below are held to)."""
    p = _run(os.path.join(SUITE, suite), topdir)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-2000:])


def test_gpu_suites_are_redirected():
    """The -gpu builds call no stock scan entry point: every scan goes through
    refsuite_gpu.c (nm: the only libyara scan/destroy symbols they import are
    the two destroy calls refsuite_gpu.c itself forwards to)."""
    for s in SUITES:
        b = os.path.join(SUITE, s + "-gpu")
        if not os.path.exists(b):
            pytest.skip("suite not built")
        out = subprocess.run(["nm", "-u", b], capture_output=True, text=True).stdout
        imported = set(re.findall(r"\b(yr_(?:rules|scanner)_(?:scan\w*|destroy))\b", out))
        assert imported <= {"yr_rules_destroy", "yr_scanner_destroy"}, imported
        defined = subprocess.run(["nm", b], capture_output=True, text=True).stdout
        assert "ygt_rules_scan_mem" in defined and "ygt_scanner_scan_mem_blocks" in defined


@pytest.mark.gpu
@pytest.mark.parametrize("preverify", ["1", "0"])
@pytest.mark.parametrize("suite", SUITES)
def test_reference_suite_through_gpu(suite, preverify, topdir):
    assert gpu_available()
    p = _run(os.path.join(SUITE, suite + "-gpu"), topdir, {"YR_GPU_PREVERIFY": preverify})
    tail = (p.stdout[-3000:], p.stderr[-3000:])
    assert p.returncode == 0, tail
    m = re.search(r"refsuite-gpu: (\d+) scans through yr_gpu_scanner, (\d+) GPU rule sets, "
                  r"preverify=(\d)", p.stderr)
    assert m, tail
    assert int(m.group(1)) > 0 and int(m.group(2)) > 0 and m.group(3) == preverify
    if suite == "test-rules":
        assert "--- PASS 3 ---" in p.stdout
        # ~650 assert_*_rule scans per pass, three passes
        assert int(m.group(1)) > 1500, m.group(0)
    print(m.group(0))
