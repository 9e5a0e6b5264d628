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
        L.oracle_trace.restype = ctypes.c_int64
        L.oracle_trace.argtypes = [_u32p, _u32p, _u8p, ctypes.c_uint64, _u64p, _u32p, _u32p,
                                   ctypes.c_int64]
        L.oracle_count_slice.restype = ctypes.c_int64
        L.oracle_count_slice.argtypes = [_u32p, _u32p, _u8p, ctypes.c_uint64, ctypes.c_uint64,
                                         ctypes.c_uint32]
        L.oracle_count_parallel.restype = ctypes.c_int64
        L.oracle_count_parallel.argtypes = [_u32p, _u32p, _u8p, ctypes.c_uint64, ctypes.c_int]
        L.oracle_xorshift_fill.restype = None
        L.oracle_xorshift_fill.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_xorshift_continue.restype = None
        L.oracle_xorshift_continue.argtypes = [_u8p, ctypes.c_uint64,
                                               ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_literal_effect.restype = ctypes.c_int64
        L.oracle_literal_effect.argtypes = [_u64p, _u32p, ctypes.c_uint64, _u16p, _u32p, _u32p,
                                            _u32p, ctypes.POINTER(ctypes.c_int64), _u64p, _u8p,
                                            _u8p, _u8p, ctypes.c_uint64, ctypes.c_uint64, _u8p,
                                            _u8p, _u32p, _u32p, _u32p, _u32p, _u8p]
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


def xorshift_state(seed: int, offset: int) -> int:
    """Generator state after `offset` bytes (GF(2) jump-ahead: xorshift64 is
    linear over GF(2)^64, so the state after m steps is A^m x0)."""
    def step(x):
        x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
        x ^= x >> 7
        x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
        return x

    def apply(cols, v):
        r = 0
        j = 0
        while v:
            if v & 1:
                r ^= cols[j]
            v >>= 1
            j += 1
        return r

    def compose(a, b):   # a(b(.))
        return [apply(a, c) for c in b]

    base = [step(1 << j) for j in range(64)]
    acc = [1 << j for j in range(64)]
    m = offset
    while m:
        if m & 1:
            acc = compose(base, acc)
        base = compose(base, base)
        m >>= 1
    return apply(acc, (0x9E3779B97F4A7C15 * seed) & 0xFFFFFFFFFFFFFFFF)


def xorshift_at(n: int, seed: int, offset: int) -> np.ndarray:
    """Bytes [offset, offset + n) of the canonical input of `seed`."""
    buf = np.empty(max(n, 1), dtype=np.uint8)
    st = ctypes.c_uint64(xorshift_state(seed, offset))
    lib().oracle_xorshift_continue(_p(buf, _u8p), n, ctypes.byref(st))
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


def trace(tab, data: np.ndarray):
    """The walk's debug trace (scanner.c:83-96): (positions, states, matches) of
    every position i in [0, len(data)] whose state is not the root."""
    T, M = _c(tab.T, np.uint32), _c(tab.M, np.uint32)
    d = _c(data, np.uint8)
    if d.size == 0:
        d = np.zeros(1, np.uint8)
    L = lib()
    cap = 1 << 16
    while True:
        pos = np.empty(cap, np.uint64)
        st = np.empty(cap, np.uint32)
        mt = np.empty(cap, np.uint32)
        cnt = L.oracle_trace(_p(T, _u32p), _p(M, _u32p), _p(d, _u8p), data.size, _p(pos, _u64p),
                             _p(st, _u32p), _p(mt, _u32p), cap)
        if cnt <= cap:
            return pos[:cnt], st[:cnt], mt[:cnt]
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


def ascii_lowercase() -> np.ndarray:
    """libyara's yr_lowercase under the C locale (libyara.c:258, tolower)."""
    low = np.arange(256, dtype=np.uint8)
    low[ord("A"):ord("Z") + 1] += 32
    return low


def literal_effect(npz, pos, idx, data: np.ndarray, base: int = 0, lowercase=None,
                   regex: bool = True) -> np.ndarray:
    """Keep-mask of a verify-call stream (positions, pool indexes): True where
    yr_scan_verify_match can have an effect (ac_oracle.c oracle_literal_effect:
    literal comparisons, and with ``regex`` the fast-exec hex programs).
    ``npz`` = a tests/golden/tables/*.npz mapping (pool + YR_STRING records +
    RE programs)."""
    pos = _c(pos, np.uint64)
    idx = _c(idx, np.uint32)
    n = pos.size
    out = np.zeros(max(n, 1), np.uint8)
    offs = _c(npz["str_offsets"], np.int64)
    str_off = _c(offs[:-1], np.uint64) if offs.size > 1 else np.zeros(1, np.uint64)
    str_len = _c(np.diff(offs), np.uint32) if offs.size > 1 else np.zeros(1, np.uint32)
    flags = _c(npz["str_flags"], np.uint32) if len(npz["str_flags"]) else np.zeros(1, np.uint32)
    fixed = _c(npz["str_fixed_offset"], np.int64) if len(npz["str_fixed_offset"]) else np.zeros(1, np.int64)
    blob = _c(npz["str_bytes"], np.uint8) if len(npz["str_bytes"]) else np.zeros(1, np.uint8)
    bt = _c(npz["pool_backtrack"], np.uint16)
    ps = _c(npz["pool_string"], np.uint32)
    low = _c(ascii_lowercase() if lowercase is None else lowercase, np.uint8)
    d = _c(data, np.uint8) if data.size else np.zeros(1, np.uint8)
    re = [None] * 6
    if regex and "re_kind" in npz:
        re = [_c(npz["re_kind"], np.uint8), _c(npz["re_fwd_off"], np.uint32),
              _c(npz["re_fwd_len"], np.uint32), _c(npz["re_bwd_off"], np.uint32),
              _c(npz["re_bwd_len"], np.uint32), _c(npz["re_code"], np.uint8)]
    re_p = [None if a is None else _p(a, t) for a, t in
            zip(re, [_u8p, _u32p, _u32p, _u32p, _u32p, _u8p])]
    lib().oracle_literal_effect(
        _p(pos, _u64p) if n else None, _p(idx, _u32p) if n else None, n, _p(bt, _u16p),
        _p(ps, _u32p), _p(flags, _u32p), _p(str_len, _u32p),
        fixed.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), _p(str_off, _u64p),
        _p(blob, _u8p), _p(low, _u8p), _p(d, _u8p), int(data.size), base, _p(out, _u8p), *re_p)
    return out[:n].astype(bool)
