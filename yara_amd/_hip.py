"""Minimal HIP runtime access (device<->host copies) for the Python host layer."""
import ctypes
import os

import numpy as np

_hip = None


def hip():
    global _hip
    if _hip is None:
        try:
            import torch  # noqa: F401  (share torch's HIP runtime, see _lib.py)
        except ImportError:
            pass
        for cand in ("libamdhip64.so.7", "libamdhip64.so", os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"),
                                                     "lib", "libamdhip64.so")):
            try:
                _hip = ctypes.CDLL(cand)
                break
            except OSError:
                continue
        if _hip is None:
            raise ImportError("libamdhip64.so not found")
        _hip.hipMemcpy.restype = ctypes.c_int
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipDeviceSynchronize.restype = ctypes.c_int
    return _hip


def memcpy(dst: int, src: int, nbytes: int, kind: int):
    """hipMemcpy; kind 1 = H2D, 2 = D2H, 3 = D2D."""
    if nbytes:
        rc = hip().hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, kind)
        if rc != 0:
            raise RuntimeError("hipMemcpy failed: %d" % rc)


def d2h_u64(ptr: int, count: int) -> np.ndarray:
    out = np.empty(count, np.uint64)
    if count:
        rc = hip().hipMemcpy(out.ctypes.data, ctypes.c_void_p(ptr), count * 8, 2)  # D2H
        if rc != 0:
            raise RuntimeError("hipMemcpy D2H failed: %d" % rc)
    return out
