"""Shared fixtures.  CPU tests run everywhere; @pytest.mark.gpu tests need a GPU.

The golden vectors under tests/golden/ were produced by the stock reference
libyara (tests/golden/make_golden.py); the reference itself is never needed
here, so the GPU box runs all of this from the committed fixtures.
"""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libyara_amd.so)")
    config.addinivalue_line("markers", "slow: multi-GiB parity cases")


def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def tables_npz(name):
    return os.path.join(GOLDEN, "tables", "%s.npz" % name)


def ref_tables(name):
    """Reference tables as a plain namespace for the oracle."""
    from oracle.tables import RefTables
    z = np.load(tables_npz(name))
    return RefTables(z["T"], z["M"], z["pool_next"], z["pool_string"], z["pool_backtrack"])


def case_arrays(case):
    p = os.path.join(GOLDEN, "cases", "%s.npz" % case)
    return np.load(p) if os.path.exists(p) else None


ALPHA = b"abcdxyzHeloC\x00\x01\xff"


def case_data(rec):
    """Rebuild the exact input bytes of a golden case (deterministic generators)."""
    import oracle
    import gen_rules
    import planted
    spec = rec["data"]
    kind = spec[0]
    if kind == "xs":
        return oracle.xorshift(spec[2], spec[1])
    if kind == "planted":
        return planted.planted_buffer(oracle.xorshift, gen_rules.gen(spec[1]), spec[3], spec[2])
    if kind == "fuzz":
        import fuzz_rules
        return fuzz_rules.buffer(oracle.xorshift, spec[1], spec[2])
    if kind == "alpha":
        x = oracle.xorshift(spec[2], spec[1])
        return np.frombuffer(ALPHA, dtype=np.uint8)[x % len(ALPHA)]
    if kind == "lit":
        return planted.lit_buffer(oracle.xorshift, spec[2], spec[1])
    if kind == "hex":
        return planted.hex_buffer(oracle.xorshift, spec[2], spec[1])
    if kind == "rx":
        return planted.rx_buffer(oracle.xorshift, spec[2], spec[1])
    if kind == "file":
        return np.frombuffer(bytes.fromhex(rec["data_bytes_hex"]), dtype=np.uint8)
    raise ValueError(kind)


# The diagnostic build of the library (make -C yara_amd/csrc diag): the only
# one that reads the A/B environment switches (internal.h YAMD_DIAG).
DIAG_LIB = os.path.join(REPO, "yara_amd", "_diag", "libyara_amd.so")


def run_diag_child(code, env=None, timeout=240):
    """Run `code` in a child Python with the diagnostic library loaded (the
    switches are read once per process); returns its stdout, asserts exit 0."""
    import subprocess
    prelude = "import sys; sys.path[:0] = [%r, %r, %r]\n" % (
        REPO, os.path.join(REPO, "tests"), GOLDEN)
    r = subprocess.run([sys.executable, "-c", prelude + code], capture_output=True, text=True,
                       timeout=timeout, env=dict(os.environ, YARA_AMD_LIB=DIAG_LIB, **(env or {})))
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gold():
    return golden()
