"""yara_amd -- MI355X-native Aho-Corasick atom scanner for libyara.

Python mirror of the hot-path interface (the C ABI in include/yara_amd.h is
the product boundary; this module is a thin ctypes host layer over it, used by
the tests, the benchmark and smoke()).

Reference interface mirrored (HoundThe/yara, libyara 4.2.1):
  * ``Tables``      <- the AC tables of a compiled YR_RULES
                       (rules->ac_transition_table / ac_match_table /
                       ac_match_pool, rules.c:356-363)
  * ``Scanner.scan_mem_block(data, verify)`` <- ``_yr_scanner_scan_mem_block``
                       (scanner.c:45-176): same dispatch order, same verify
                       arguments (pool index, offset) as its calls to
                       ``yr_scan_verify_match`` (scan.c:992), same int error
                       convention (ERROR_* values of error.h).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import (CALLBACK_ERROR, COULD_NOT_MAP_FILE, INSUFFICIENT_MEMORY,  # noqa: F401
                   INTERNAL_FATAL_ERROR, INVALID_ARGUMENT, MAX_ATOM_LENGTH, SCAN_TIMEOUT, SUCCESS,
                   YaraAmdError)

__all__ = ["Tables", "Scanner", "Pipeline", "replay", "fill_xorshift64", "version",
           "YaraAmdError"]


def _arr(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


def version() -> str:
    return _lib.lib().yr_amd_version().decode()


class Tables:
    """Flattened, device-resident scan tables (one per compiled rule set).

    ``device=-1`` builds host-only tables: flattening + replay, no scanner.
    """

    def __init__(self, T=None, M=None, pool_next=None, pool_backtrack=None, device: int = 0,
                 _handle=None):
        if _handle is not None:          # from_yarc
            self._h = _handle
            self.device = device
            return
        L = _lib.lib()
        self._T = _arr(T, np.uint32)
        self._M = _arr(M, np.uint32)
        self._nx = _arr(pool_next, np.uint32)
        self._bt = _arr(pool_backtrack, np.uint16)
        if self._T.size != self._M.size:
            raise ValueError("transition and match tables differ in length")
        if self._nx.size != self._bt.size:
            raise ValueError("pool arrays differ in length")
        nx = self._nx if self._nx.size else np.zeros(1, np.uint32)
        bt = self._bt if self._bt.size else np.zeros(1, np.uint16)
        h = ctypes.c_void_p()
        rc = L.yr_amd_tables_create(
            self._T.ctypes.data_as(_lib._u32p), self._M.ctypes.data_as(_lib._u32p), self._T.size,
            nx.ctypes.data_as(_lib._u32p), bt.ctypes.data_as(_lib._u16p), self._nx.size, device,
            ctypes.byref(h))
        _lib.check("yr_amd_tables_create", rc)
        self._h = h
        self.device = device

    @classmethod
    def from_yarc(cls, data, device: int = 0):
        """Tables from the bytes (or path) of a compiled rules file (yarac
        output; yr_amd_tables_load_yarc) -- no libyara involved."""
        if isinstance(data, (str, bytes)) and not isinstance(data, bytes):
            with open(data, "rb") as f:
                data = f.read()
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        h = ctypes.c_void_p()
        _lib.check("yr_amd_tables_load_yarc", _lib.lib().yr_amd_tables_load_yarc(
            buf.ctypes.data_as(_lib._u8p), len(data), device, ctypes.byref(h)))
        return cls(device=device, _handle=h)

    @classmethod
    def from_npz(cls, path, device: int = 0, strings: bool = False, regex: bool = True):
        """Tables from a tests/golden/tables/*.npz dump; ``strings=True`` also
        attaches the YR_STRING records (needed by Scanner.verify_calls) and,
        with ``regex``, the fast-exec programs of the hex strings."""
        z = np.load(path)
        t = cls(z["T"], z["M"], z["pool_next"], z["pool_backtrack"], device=device)
        t.pool_string = z["pool_string"] if "pool_string" in z else None
        if strings:
            offs = z["str_offsets"]
            t.set_strings(z["pool_string"], z["str_flags"], np.diff(offs), z["str_fixed_offset"],
                          z["str_bytes"], offs[:-1])
            if regex and "re_kind" in z:
                fl = np.where(z["re_kind"] != 0, z["re_fwd_len"], 0)
                t.set_re_code(z["re_fwd_off"], fl, z["re_bwd_off"], z["re_bwd_len"], z["re_code"])
        return t

    def set_re_code(self, fwd_off, fwd_len, bwd_off, bwd_len, code):
        """Attach fast-exec RE programs (yr_amd_tables_set_re_code)."""
        arrs = [_arr(a, np.uint32) for a in (fwd_off, fwd_len, bwd_off, bwd_len)]
        arrs = [a if a.size else np.zeros(1, np.uint32) for a in arrs]
        self._re = arrs + [_arr(code, np.uint8) if len(code) else np.zeros(1, np.uint8)]
        _lib.check("yr_amd_tables_set_re_code", _lib.lib().yr_amd_tables_set_re_code(
            self._h, len(fwd_off), *[a.ctypes.data_as(_lib._u32p) for a in arrs],
            self._re[4].ctypes.data_as(_lib._u8p), len(code)))

    def set_strings(self, pool_string, flags, lengths, fixed_offsets, blob, bytes_offsets,
                    lowercase=None):
        """Attach YR_STRING records (yr_amd_tables_set_strings).  ``lowercase``
        defaults to C-locale tolower, i.e. libyara's yr_lowercase (libyara.c:258)."""
        n = len(flags)
        recs = (_lib.String * max(n, 1))()
        for k in range(n):
            recs[k].flags = int(flags[k])
            recs[k].length = int(lengths[k])
            recs[k].fixed_offset = int(fixed_offsets[k])
            recs[k].bytes_offset = int(bytes_offsets[k])
        if lowercase is None:
            lowercase = np.arange(256, dtype=np.uint8)
            lowercase[ord("A"):ord("Z") + 1] += 32
        self._ps = _arr(pool_string, np.uint32)
        self._blob = _arr(blob, np.uint8) if len(blob) else np.zeros(1, np.uint8)
        self._lower = _arr(lowercase, np.uint8)
        ps = self._ps if self._ps.size else np.zeros(1, np.uint32)
        _lib.check("yr_amd_tables_set_strings", _lib.lib().yr_amd_tables_set_strings(
            self._h, ps.ctypes.data_as(_lib._u32p), self._ps.size, recs, n,
            self._blob.ctypes.data_as(_lib._u8p), len(blob), self._lower.ctypes.data_as(_lib._u8p)))

    def set_profiling(self, enable: bool = True):
        """Count-only records for libyara's profiling counters
        (yr_amd_tables_set_profiling)."""
        _lib.check("yr_amd_tables_set_profiling",
                   _lib.lib().yr_amd_tables_set_profiling(self._h, int(enable)))

    @property
    def handle(self):
        return self._h

    def info(self) -> dict:
        inf = _lib.TablesInfo()
        _lib.check("yr_amd_tables_get_info", _lib.lib().yr_amd_tables_get_info(self._h, ctypes.byref(inf)))
        d = {}
        for name, _ in inf._fields_:
            v = getattr(inf, name)
            d[name] = list(v) if not isinstance(v, int) else v
        return d

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().yr_amd_tables_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def replay(tables: Tables, data: np.ndarray, positions, all_positions: bool, verify) -> int:
    """Replay a candidate stream into ``verify(pool_index, offset) -> int``.

    Returns the first non-zero verify result, or 0.  Order and arguments are
    those of the reference's calls to yr_scan_verify_match (scanner.c:105-121).
    """
    d = _arr(data, np.uint8)
    if d.size == 0:
        d = np.zeros(1, np.uint8)
    pos = _arr(positions if positions is not None else [], np.uint64)
    pos_p = pos.ctypes.data_as(_lib._u64p) if pos.size else None
    err = []

    def _cb(_user, k, off):
        try:
            return int(verify(int(k), int(off)))
        except Exception as e:  # never unwind through C
            err.append(e)
            return CALLBACK_ERROR

    cb = _lib.VERIFY_FN(_cb)
    rc = _lib.lib().yr_amd_replay(tables.handle, d.ctypes.data_as(_lib._u8p), int(data.size), pos_p,
                                  int(pos.size), 1 if all_positions else 0, cb, None)
    if err:
        raise err[0]
    return rc


class Scanner:
    """One scan at a time on its own HIP stream (or on ``stream``)."""

    def __init__(self, tables: Tables, stream: int = 0):
        h = ctypes.c_void_p()
        _lib.check("yr_amd_scanner_create",
                   _lib.lib().yr_amd_scanner_create(tables.handle, ctypes.c_void_p(stream or None),
                                                    ctypes.byref(h)))
        self._h = h
        self.tables = tables

    # -- host block: the _yr_scanner_scan_mem_block replacement ---------------
    def candidates(self, data: np.ndarray):
        """(positions uint64[], all_positions) for a block in host memory."""
        d = _arr(data, np.uint8)
        ptr = ctypes.POINTER(ctypes.c_uint64)()
        cnt = ctypes.c_uint64()
        allp = ctypes.c_int()
        dp = d.ctypes.data_as(_lib._u8p) if d.size else None
        _lib.check("yr_amd_scan_block",
                   _lib.lib().yr_amd_scan_block(self._h, dp, d.size, ctypes.byref(ptr),
                                                ctypes.byref(cnt), ctypes.byref(allp)))
        n = cnt.value
        pos = np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
        return pos, bool(allp.value)

    def scan_mem_block(self, data: np.ndarray, verify) -> int:
        """Mirror of _yr_scanner_scan_mem_block (scanner.c:45-176): GPU candidate
        detection, then the reference-ordered verify calls.  Returns an ERROR_* code."""
        try:
            pos, allp = self.candidates(data)
        except YaraAmdError as e:
            return e.code
        return replay(self.tables, data, pos, allp, verify)

    def verify_stream(self, data: np.ndarray):
        """(positions, pool indexes) of every verify call the block would make."""
        P, K = [], []

        def cb(k, off):
            K.append(k)
            P.append(off + int(self.tables._bt[k]))
            return 0
        rc = self.scan_mem_block(data, cb)
        _lib.check("scan_mem_block", rc)
        return np.array(P, dtype=np.uint64), np.array(K, dtype=np.uint32)

    def verify_calls(self, data: np.ndarray, data_base: int = 0):
        """On-device pre-verification (yr_amd_scan_block_verified): the verify
        calls of the block that can have an effect, in the reference's order,
        as a structured array {offset, pool_index, candidate}."""
        d = _arr(data, np.uint8)
        ptr = ctypes.POINTER(_lib.VerifyRec)()
        cnt = ctypes.c_uint64()
        dp = d.ctypes.data_as(_lib._u8p) if d.size else None
        _lib.check("yr_amd_scan_block_verified",
                   _lib.lib().yr_amd_scan_block_verified(self._h, dp, d.size, data_base,
                                                         ctypes.byref(ptr), ctypes.byref(cnt)))
        n = cnt.value
        out = np.zeros(n, dtype=_lib.VERIFY_REC_DTYPE)
        if n:
            ctypes.memmove(out.ctypes.data, ptr, n * 16)
        return out

    def verify_device(self, data_base: int = 0):
        """(device pointer to yr_amd_verify_rec[], count) for the last
        completed device scan (yr_amd_verify_device)."""
        p = ctypes.c_void_p()
        cnt = ctypes.c_uint64()
        _lib.check("yr_amd_verify_device",
                   _lib.lib().yr_amd_verify_device(self._h, data_base, ctypes.byref(p),
                                                   ctypes.byref(cnt)))
        return p.value or 0, cnt.value

    # -- device-resident block (benchmark path) -------------------------------
    def scan_device(self, d_ptr: int, block_size: int, byte_begin: int = 0, byte_end=None):
        if byte_end is None:
            byte_end = block_size
        _lib.check("yr_amd_scan_device",
                   _lib.lib().yr_amd_scan_device(self._h, ctypes.c_void_p(d_ptr), block_size,
                                                 byte_begin, byte_end))

    def scan_window(self, d_ptr: int, window_begin: int, window_end: int, block_size: int,
                    byte_begin: int, byte_end: int):
        """Scan [byte_begin, byte_end) of a block of which the device holds only
        bytes [window_begin, window_end) at d_ptr (yr_amd_scan_window: shards)."""
        _lib.check("yr_amd_scan_window",
                   _lib.lib().yr_amd_scan_window(self._h, ctypes.c_void_p(d_ptr), window_begin,
                                                 window_end, block_size, byte_begin, byte_end))

    def device_result(self):
        """(device pointer to uint64 positions, count, all_positions) --
        yr_amd_scan_device_result.  The positions are complete in the
        scanner's stream order: a reader on another stream (or the host) must
        synchronise that stream first.  On a verified-only scanner
        (set_verified_only) the call returns before the compaction has written
        them: such a scan serves verify_device, which queues behind them."""
        p = ctypes.c_void_p()
        cnt = ctypes.c_uint64()
        allp = ctypes.c_int()
        _lib.check("yr_amd_scan_device_result",
                   _lib.lib().yr_amd_scan_device_result(self._h, ctypes.byref(p), ctypes.byref(cnt),
                                                        ctypes.byref(allp)))
        return p.value or 0, cnt.value, bool(allp.value)

    def trace_walk(self, d_ptr: int, size: int, data_base: int = 0, cap=None):
        """Device trace of the walk over a device-resident block (yr_amd_trace_walk,
        the analogue of scanner.c:83-96): structured array of (position, state,
        match) for every position in [0, size] whose state is not the root."""
        cnt = ctypes.c_uint64()
        if cap is None:
            _lib.check("yr_amd_trace_walk",
                       _lib.lib().yr_amd_trace_walk(self._h, ctypes.c_void_p(d_ptr), size, data_base,
                                                    None, 0, ctypes.byref(cnt)))
            cap = cnt.value
        out = np.zeros(cap, dtype=_lib.TRACE_REC_DTYPE)
        _lib.check("yr_amd_trace_walk",
                   _lib.lib().yr_amd_trace_walk(self._h, ctypes.c_void_p(d_ptr), size, data_base,
                                                ctypes.c_void_p(out.ctypes.data if cap else 0), cap,
                                                ctypes.byref(cnt)))
        return out[:min(cap, cnt.value)], cnt.value

    def set_verified_only(self, enable: bool = True):
        """Scans serve verify_device only (yr_amd_scanner_set_verified_only):
        the result may leave out candidates whose calls the scan proves dead."""
        _lib.check("yr_amd_scanner_set_verified_only",
                   _lib.lib().yr_amd_scanner_set_verified_only(self._h, int(enable)))

    def stream_length(self) -> int:
        """Length of the last scan's full candidate stream."""
        n = ctypes.c_uint64()
        _lib.check("yr_amd_scan_device_stream_length",
                   _lib.lib().yr_amd_scan_device_stream_length(self._h, ctypes.byref(n)))
        return n.value

    def set_timing(self, enable: bool = True):
        _lib.check("yr_amd_scanner_set_timing", _lib.lib().yr_amd_scanner_set_timing(self._h, int(enable)))

    def kernel_ms(self) -> float:
        """Duration of the last scan kernel launch (HIP events on the scan stream)."""
        ms = ctypes.c_float()
        _lib.check("yr_amd_scanner_kernel_ms", _lib.lib().yr_amd_scanner_kernel_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def scan_ms(self) -> float:
        """Duration of the last scan and its compaction (HIP events on the scan stream)."""
        ms = ctypes.c_float()
        _lib.check("yr_amd_scanner_scan_ms", _lib.lib().yr_amd_scanner_scan_ms(self._h, ctypes.byref(ms)))
        return ms.value

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().yr_amd_scanner_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fill_xorshift64(d_ptr: int, n: int, seed: int, offset: int = 0, stream: int = 0):
    """Fill device memory with bytes [offset, offset+n) of the SURVEY.md App. A
    synthetic buffer (bench/test utility)."""
    _lib.check("yr_amd_fill_xorshift64",
               _lib.lib().yr_amd_fill_xorshift64(ctypes.c_void_p(d_ptr), n, seed, offset,
                                                 ctypes.c_void_p(stream or None)))


class Pipeline:
    """Block pipeline (yr_amd_pipeline_*): up to ``depth`` blocks copied,
    scanned and pre-verified on the GPU while the caller consumes the oldest.
    Mirrors the block loop of yr_scanner_scan_mem_blocks (scanner.c:417-583)."""

    def __init__(self, tables, depth: int = 2, split_min: int = 0):
        """``tables``: one Tables, or a list of them (one per logical device:
        yr_amd_pipeline_create_multi -- each block split across the devices,
        blocks below ``split_min`` bytes whole to one device)."""
        h = ctypes.c_void_p()
        if isinstance(tables, (list, tuple)):
            self.tables = list(tables)
            arr = (ctypes.c_void_p * len(self.tables))(*[t.handle.value for t in self.tables])
            _lib.check("yr_amd_pipeline_create_multi",
                       _lib.lib().yr_amd_pipeline_create_multi(arr, len(self.tables), depth,
                                                               ctypes.byref(h)))
        else:
            self.tables = tables
            _lib.check("yr_amd_pipeline_create",
                       _lib.lib().yr_amd_pipeline_create(tables.handle, depth, ctypes.byref(h)))
        self._h = h
        self.depth = depth
        self._copy_fn = None
        if split_min:
            _lib.check("yr_amd_pipeline_set_split_min",
                       _lib.lib().yr_amd_pipeline_set_split_min(self._h, split_min))

    def set_copy(self, fn):
        """fn(dst_ptr, src_ptr, n) -> 0 / nonzero: the copy into the pinned
        staging (yr_amd_pipeline_set_copy; None: memcpy).  Test hook for the
        fault path: a nonzero return fails the submission."""
        if fn is None:
            self._copy_fn = None
            _lib.check("yr_amd_pipeline_set_copy",
                       _lib.lib().yr_amd_pipeline_set_copy(self._h, _lib.COPY_FN(), None))
            return
        self._copy_fn = _lib.COPY_FN(lambda _u, d, s, n: fn(d, s, n))
        _lib.check("yr_amd_pipeline_set_copy",
                   _lib.lib().yr_amd_pipeline_set_copy(self._h, self._copy_fn, None))

    def submit(self, data: np.ndarray, base: int = 0, dma: bool = False):
        """Submit a block: host memcpy in this thread (yr_amd_pipeline_submit),
        or with ``dma`` straight to the device (yr_amd_pipeline_submit_dma)."""
        d = _arr(data, np.uint8)
        dp = d.ctypes.data_as(_lib._u8p) if d.size else None
        fn = "yr_amd_pipeline_submit_dma" if dma else "yr_amd_pipeline_submit"
        _lib.check(fn, getattr(_lib.lib(), fn)(self._h, dp, d.size, base))

    def next(self, copy_data: bool = True):
        """(records {offset, pool_index, candidate}, block bytes copy or None,
        base) of the oldest submitted block."""
        recs = ctypes.POINTER(_lib.VerifyRec)()
        cnt = ctypes.c_uint64()
        data = ctypes.POINTER(ctypes.c_uint8)()
        size = ctypes.c_size_t()
        base = ctypes.c_uint64()
        _lib.check("yr_amd_pipeline_next",
                   _lib.lib().yr_amd_pipeline_next(self._h, ctypes.byref(recs), ctypes.byref(cnt),
                                                   ctypes.byref(data), ctypes.byref(size),
                                                   ctypes.byref(base)))
        n = cnt.value
        out = np.zeros(n, dtype=_lib.VERIFY_REC_DTYPE)
        if n:
            ctypes.memmove(out.ctypes.data, recs, n * 16)
        b = None
        if copy_data:
            b = np.empty(size.value, np.uint8)
            if size.value:
                ctypes.memmove(b.ctypes.data, data, size.value)
        return out, b, base.value

    def drain(self):
        _lib.check("yr_amd_pipeline_drain", _lib.lib().yr_amd_pipeline_drain(self._h))

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().yr_amd_pipeline_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """Multi-device block scans in one process (yr_amd_multi_*): the block is
    split into per-device windows (shard + verify halos), each scanned and
    pre-verified on its device; records concatenated in device order."""

    def __init__(self, tables_list):
        self.tables = list(tables_list)
        arr = (ctypes.c_void_p * len(self.tables))(*[t.handle.value for t in self.tables])
        h = ctypes.c_void_p()
        _lib.check("yr_amd_multi_create",
                   _lib.lib().yr_amd_multi_create(arr, len(self.tables), ctypes.byref(h)))
        self._h = h

    def set_copy(self, fn):
        """As Pipeline.set_copy, for the staging of yr_amd_multi_scan_block_verified."""
        self._copy_fn = None if fn is None else _lib.COPY_FN(lambda _u, d, s, n: fn(d, s, n))
        _lib.check("yr_amd_multi_set_copy",
                   _lib.lib().yr_amd_multi_set_copy(self._h, self._copy_fn or _lib.COPY_FN(), None))

    def shard(self, size: int, k: int):
        """(begin, end, window_begin, window_end) of device k."""
        v = [ctypes.c_uint64() for _ in range(4)]
        _lib.check("yr_amd_multi_shard",
                   _lib.lib().yr_amd_multi_shard(self._h, size, k, *[ctypes.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def verify_calls(self, data: np.ndarray, data_base: int = 0):
        """yr_amd_multi_scan_block_verified: the block's effective verify calls
        as a structured array {offset, pool_index, candidate}."""
        d = _arr(data, np.uint8)
        ptr = ctypes.POINTER(_lib.VerifyRec)()
        cnt = ctypes.c_uint64()
        dp = d.ctypes.data_as(_lib._u8p) if d.size else None
        _lib.check("yr_amd_multi_scan_block_verified",
                   _lib.lib().yr_amd_multi_scan_block_verified(self._h, dp, d.size, data_base,
                                                               ctypes.byref(ptr), ctypes.byref(cnt)))
        n = cnt.value
        out = np.zeros(n, dtype=_lib.VERIFY_REC_DTYPE)
        if n:
            ctypes.memmove(out.ctypes.data, ptr, n * 16)
        return out

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().yr_amd_multi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
