"""ctypes binding of libyara_amd.so (the C ABI declared in include/yara_amd.h).

The HIP library is the product; this module only loads it.  There is no
fallback: if the shared object is missing or fails to load, importing raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# YARA_AMD_LIB: another build of the same library (tools/ablate.py variants)
LIB_PATH = os.environ.get("YARA_AMD_LIB") or os.path.join(_HERE, "libyara_amd.so")

# error codes (libyara/include/yara/error.h values)
SUCCESS = 0
INSUFFICIENT_MEMORY = 1
COULD_NOT_MAP_FILE = 4
SCAN_TIMEOUT = 26
CALLBACK_ERROR = 28
INVALID_ARGUMENT = 29
INTERNAL_FATAL_ERROR = 31
MAX_ATOM_LENGTH = 4

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_int = ctypes.c_int

VERIFY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64)
# yr_amd_copy_fn: (user, dst, src, n) -> 0 / nonzero (source unreadable)
COPY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_size_t)


class TablesInfo(ctypes.Structure):
    _fields_ = [
        ("n_slots", ctypes.c_uint32),
        ("n_states", ctypes.c_uint32),
        ("max_depth", ctypes.c_uint32),
        ("states_by_depth", ctypes.c_uint32 * (MAX_ATOM_LENGTH + 1)),
        ("accepting_states", ctypes.c_uint32),
        ("keys_by_length", ctypes.c_uint32 * (MAX_ATOM_LENGTH + 1)),
        ("root_accepting", ctypes.c_uint32),
        ("filter_bits", ctypes.c_uint32),
        ("filter_set_bits", ctypes.c_uint32),
        ("exact_slots", ctypes.c_uint32),
        ("max_backtrack", ctypes.c_uint32),
        ("verify_halo_before", ctypes.c_uint64),
        ("verify_halo_after", ctypes.c_uint64),
        ("filter_mode", ctypes.c_uint32),
    ]


class String(ctypes.Structure):
    """yr_amd_string (include/yara_amd.h)."""
    _fields_ = [("flags", ctypes.c_uint32), ("length", ctypes.c_uint32),
                ("fixed_offset", ctypes.c_int64), ("bytes_offset", ctypes.c_uint64)]


class VerifyRec(ctypes.Structure):
    """yr_amd_verify_rec (include/yara_amd.h)."""
    _fields_ = [("offset", ctypes.c_uint64), ("pool_index", ctypes.c_uint32),
                ("candidate", ctypes.c_uint32)]


VERIFY_REC_DTYPE = [("offset", "<u8"), ("pool_index", "<u4"), ("candidate", "<u4")]
TRACE_REC_DTYPE = [("position", "<u8"), ("state", "<u4"), ("match", "<u4")]   # yr_amd_trace_rec

# name -> (restype, argtypes); every function include/yara_amd.h declares
PROTOTYPES = {
    "yr_amd_tables_create": (_int, [_u32p, _u32p, ctypes.c_uint32, _u32p, _u16p, ctypes.c_uint32,
                                    _int, ctypes.POINTER(_vp)]),
    "yr_amd_tables_destroy": (_int, [_vp]),
    "yr_amd_tables_load_yarc": (_int, [_u8p, ctypes.c_size_t, _int, ctypes.POINTER(_vp)]),
    "yr_amd_tables_get_info": (_int, [_vp, ctypes.POINTER(TablesInfo)]),
    "yr_amd_scanner_create": (_int, [_vp, _vp, ctypes.POINTER(_vp)]),
    "yr_amd_scanner_destroy": (_int, [_vp]),
    "yr_amd_scan_block": (_int, [_vp, _u8p, ctypes.c_size_t, ctypes.POINTER(_u64p),
                                 ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_int)]),
    "yr_amd_scan_device": (_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
    "yr_amd_scan_window": (_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                  ctypes.c_uint64, ctypes.c_uint64]),
    "yr_amd_scan_device_result": (_int, [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_uint64),
                                         ctypes.POINTER(_int)]),
    "yr_amd_replay": (_int, [_vp, _u8p, ctypes.c_size_t, _u64p, ctypes.c_uint64, _int, VERIFY_FN,
                             _vp]),
    "yr_amd_trace_walk": (_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                 ctypes.POINTER(ctypes.c_uint64)]),
    "yr_amd_fill_xorshift64": (_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp]),
    "yr_amd_scanner_set_timing": (_int, [_vp, _int]),
    "yr_amd_scanner_set_verified_only": (_int, [_vp, _int]),
    "yr_amd_scan_device_stream_length": (_int, [_vp, _u64p]),
    "yr_amd_scanner_kernel_ms": (_int, [_vp, ctypes.POINTER(ctypes.c_float)]),
    "yr_amd_scanner_scan_ms": (_int, [_vp, ctypes.POINTER(ctypes.c_float)]),
    "yr_amd_version": (ctypes.c_char_p, []),
    "yr_amd_tables_set_strings": (_int, [_vp, _u32p, ctypes.c_uint32, ctypes.POINTER(String),
                                         ctypes.c_uint32, _u8p, ctypes.c_uint64, _u8p]),
    "yr_amd_tables_set_re_code": (_int, [_vp, ctypes.c_uint32, _u32p, _u32p, _u32p, _u32p, _u8p,
                                         ctypes.c_uint64]),
    "yr_amd_re_code_extent": (_int, [_u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]),
    "yr_amd_verify_device": (_int, [_vp, ctypes.c_uint64, ctypes.POINTER(_vp),
                                    ctypes.POINTER(ctypes.c_uint64)]),
    "yr_amd_pipeline_create": (_int, [_vp, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "yr_amd_pipeline_destroy": (_int, [_vp]),
    "yr_amd_pipeline_submit": (_int, [_vp, _u8p, ctypes.c_size_t, ctypes.c_uint64]),
    "yr_amd_pipeline_submit_dma": (_int, [_vp, _u8p, ctypes.c_size_t, ctypes.c_uint64]),
    "yr_amd_pipeline_next": (_int, [_vp, ctypes.POINTER(ctypes.POINTER(VerifyRec)),
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(_u8p),
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_uint64)]),
    "yr_amd_pipeline_drain": (_int, [_vp]),
    "yr_amd_pipeline_create_multi": (_int, [ctypes.POINTER(_vp), ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.POINTER(_vp)]),
    "yr_amd_pipeline_set_copy": (_int, [_vp, COPY_FN, _vp]),
    "yr_amd_pipeline_set_split_min": (_int, [_vp, ctypes.c_uint64]),
    "yr_amd_multi_set_copy": (_int, [_vp, COPY_FN, _vp]),
    "yr_amd_scan_block_verified": (_int, [_vp, _u8p, ctypes.c_size_t, ctypes.c_uint64,
                                          ctypes.POINTER(ctypes.POINTER(VerifyRec)),
                                          ctypes.POINTER(ctypes.c_uint64)]),
    "yr_amd_multi_create": (_int, [ctypes.POINTER(_vp), ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "yr_amd_multi_destroy": (_int, [_vp]),
    "yr_amd_multi_shard": (_int, [_vp, ctypes.c_uint64, ctypes.c_uint32] +
                           [ctypes.POINTER(ctypes.c_uint64)] * 4),
    "yr_amd_multi_scan_block_verified": (_int, [_vp, _u8p, ctypes.c_size_t, ctypes.c_uint64,
                                                ctypes.POINTER(ctypes.POINTER(VerifyRec)),
                                                ctypes.POINTER(ctypes.c_uint64)]),
    "yr_amd_tables_device": (_int, [_vp]),
    "yr_amd_tables_set_profiling": (_int, [_vp, _int]),
}

_lib = None


class YaraAmdError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__("%s failed with error %d" % (fn, code))
        self.code = code


def lib():
    """Load libyara_amd.so (raises if it is missing: no CPU fallback exists)."""
    global _lib
    if _lib is None:
        # Share ONE HIP runtime with PyTorch: torch ships its own libamdhip64.so.7;
        # loading it first makes the dynamic linker bind libyara_amd.so's
        # DT_NEEDED libamdhip64.so.7 to that same instance, so torch tensors,
        # streams and RCCL and our kernels live in one HIP/HSA runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError("libyara_amd.so not built (%s); run __graft_entry__.build() or "
                              "make -C yara_amd/csrc" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(fn, code):
    if code != SUCCESS:
        raise YaraAmdError(fn, code)
