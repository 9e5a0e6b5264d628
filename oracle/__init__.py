"""CPU parity oracle for the yara_amd hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker.  The product
(``yara_amd`` / ``libyara_amd.so``) never imports, links or calls it.

* ``ac_oracle.c`` restates the reference hot loop (libyara/scanner.c:45-176).
* ``tables.py`` reads table dumps produced by the stock libyara compiler.
* ``ref.mk`` / ``refdump.c`` / ``refhook.c`` build and drive the reference itself
  (only in the build container, where /root/reference exists) to produce the
  committed golden vectors under ``tests/golden/``.
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    """Compile oracle/_build/liboracle.so with gcc (cheap; also done on the GPU box)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(_HERE, "ac_oracle.c")
        if (not os.path.exists(_LIB_PATH)
                or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_walk_verify.restype = ctypes.c_int64
        L.oracle_walk_verify.argtypes = [_u32p, _u32p, _u32p, _u16p, _u8p, ctypes.c_uint64,
                                         _u64p, _u32p, ctypes.c_int64]
        L.oracle_candidates.restype = ctypes.c_int64
        L.oracle_candidates.argtypes = [_u32p, _u32p, _u8p, ctypes.c_uint64, _u64p, ctypes.c_int64]
        L.oracle_count_slice.restype = ctypes.c_int64
        L.oracle_count_slice.argtypes = [_u32p, _u32p, _u8p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint32]
        L.oracle_count_parallel.restype = ctypes.c_int64
        L.oracle_count_parallel.argtypes = [_u32p, _u32p, _u8p, ctypes.c_uint64, ctypes.c_int]
        L.oracle_xorshift_fill.restype = None
        L.oracle_xorshift_fill.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_step.restype = ctypes.c_uint32
        L.oracle_step.argtypes = [_u32p, ctypes.c_uint32, ctypes.c_uint8]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def xorshift(n: int, seed: int) -> np.ndarray:
    """SURVEY.md Appendix A buffer generator (bit-exact with refdump's)."""
    buf = np.empty(max(n, 1), dtype=np.uint8)
    lib().oracle_xorshift_fill(_p(buf, _u8p), n, seed)
    return buf[:n]


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def walk_verify(tab, data: np.ndarray):
    """Reference verify-call stream (position i, pool index) for one block."""
    T, M = _c(tab.T, np.uint32), _c(tab.M, np.uint32)
    nx, bt = _c(tab.pool_next, np.uint32), _c(tab.pool_backtrack, np.uint16)
    d = _c(data, np.uint8)
    if d.size == 0:
        d = np.zeros(1, np.uint8)
    n = data.size
    L = lib()
    cap = 1 << 16
    while True:
        pos = np.empty(cap, np.uint64)
        idx = np.empty(cap, np.uint32)
        cnt = L.oracle_walk_verify(_p(T, _u32p), _p(M, _u32p), _p(nx, _u32p), _p(bt, _u16p),
                                   _p(d, _u8p), n, _p(pos, _u64p), _p(idx, _u32p), cap)
        if cnt <= cap:
            return pos[:cnt], idx[:cnt]
        cap = int(cnt)


def candidates(tab, data: np.ndarray) -> np.ndarray:
    """Positions i in [0, len(data)] where ac_match_table[state_i] != 0."""
    T, M = _c(tab.T, np.uint32), _c(tab.M, np.uint32)
    d = _c(data, np.uint8)
    if d.size == 0:
        d = np.zeros(1, np.uint8)
    L = lib()
    cap = 1 << 16
    while True:
        out = np.empty(cap, np.uint64)
        cnt = L.oracle_candidates(_p(T, _u32p), _p(M, _u32p), _p(d, _u8p), data.size,
                                  _p(out, _u64p), cap)
        if cnt <= cap:
            return out[:cnt]
        cap = int(cnt)


def count_parallel(tab, data: np.ndarray, nthreads: int) -> int:
    T, M = _c(tab.T, np.uint32), _c(tab.M, np.uint32)
    return int(lib().oracle_count_parallel(_p(T, _u32p), _p(M, _u32p), _p(data, _u8p),
                                           data.size, nthreads))


def verify_stream_sha(pos, idx, base=None) -> str:
    """Canonical digest of a verify-call stream.

    Records are little-endian packed {u64 position, u32 pool index}
    (or {u64 block base, u64 position, u32 pool index} for multi-block scans).
    """
    n = len(pos)
    if base is None:
        rec = np.zeros(n, dtype=[("p", "<u8"), ("k", "<u4")])
    else:
        rec = np.zeros(n, dtype=[("b", "<u8"), ("p", "<u8"), ("k", "<u4")])
        rec["b"] = base
    rec["p"] = pos
    rec["k"] = idx
    return hashlib.sha256(rec.tobytes()).hexdigest()


def positions_sha(pos) -> str:
    return hashlib.sha256(np.asarray(pos, dtype="<u8").tobytes()).hexdigest()
