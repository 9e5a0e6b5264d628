"""A/B of scan-kernel builds INSIDE ONE PROCESS (measurement tool).

Every variant library (yara_amd/_variants/<name>.so; "base" = the product
build yara_amd/libyara_amd.so) is loaded side by side with its own ctypes
handle, tables and scanner on the same device-resident input; the variants
then take turns, `--reps` timed scans each per round, in an order that
alternates every round, for `--rounds` rounds.  Same process, same clock
state, interleaved at sub-second granularity: the box-to-box and
process-to-process drift of separate runs (2-4 %) cancels, so 1 % effects
resolve.  Reports per variant the median / min kernel time (HIP events around
the scan kernel) and the median per-round ratio to the first variant.

    python tools/ab_inproc.py --rules C base,r3 [--rounds 20] [--reps 5] [--strings] [--verify]

--strings attaches the rule set's string records and regexp programs (as
tools/ruleset_rates.py does), so the compaction also decides the 1-byte-key
candidates' classes and builds the live list; --verify (implies --strings)
also times the on-device pre-verification after each scan (wall clock);
--verified-only (implies --verify) runs the scanners in verified-only mode
(yr_amd_scanner_set_verified_only) and reports the whole step's wall time.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_vp = ctypes.c_void_p


def load(name):
    name = name.split(":")[0]   # (a ":vo" suffix: that variant's scanner in verified-only mode)
    path = (os.path.join(REPO, "yara_amd", "libyara_amd.so") if name == "base"
            else os.path.join(REPO, "yara_amd", "_variants", name + ".so"))
    L = ctypes.CDLL(path, mode=getattr(os, "RTLD_LOCAL", 0) | os.RTLD_NOW)
    for fn, args in (("yr_amd_tables_create", [_vp, _vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint32,
                                                ctypes.c_int, ctypes.POINTER(_vp)]),
                     ("yr_amd_scanner_create", [_vp, _vp, ctypes.POINTER(_vp)]),
                     ("yr_amd_scan_device", [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]),
                     ("yr_amd_scan_device_result", [_vp, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_uint64),
                                                    ctypes.POINTER(ctypes.c_int)]),
                     ("yr_amd_scanner_set_timing", [_vp, ctypes.c_int]),
                     ("yr_amd_scanner_kernel_ms", [_vp, ctypes.POINTER(ctypes.c_float)]),
                     ("yr_amd_scanner_scan_ms", [_vp, ctypes.POINTER(ctypes.c_float)]),
                     ("yr_amd_fill_xorshift64", [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _vp]),
                     ("yr_amd_tables_set_strings", [_vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp,
                                                    ctypes.c_uint64, _vp]),
                     ("yr_amd_tables_set_re_code", [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64]),
                     ("yr_amd_verify_device", [_vp, ctypes.c_uint64, ctypes.POINTER(_vp),
                                               ctypes.POINTER(ctypes.c_uint64)])):
        getattr(L, fn).argtypes = args
        getattr(L, fn).restype = ctypes.c_int
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants")
    ap.add_argument("--rules", default="C")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warm-s", type=float, default=1.0)
    ap.add_argument("--strings", action="store_true")
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--verified-only", action="store_true")
    a = ap.parse_args()
    a.verify = a.verify or a.verified_only
    a.strings = a.strings or a.verify
    import torch
    names = a.variants.split(",")
    n = int(a.gib * (1 << 30))
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    libs = [load(v) for v in names]
    assert libs[0].yr_amd_fill_xorshift64(_vp(buf.data_ptr()), n, 1, 0, None) == 0
    torch.cuda.synchronize()
    z = np.load(os.path.join(REPO, "tests", "golden", "tables", a.rules + ".npz"))
    T = np.ascontiguousarray(z["T"], np.uint32)
    M = np.ascontiguousarray(z["M"], np.uint32)
    nx = np.ascontiguousarray(z["pool_next"], np.uint32)
    bt = np.ascontiguousarray(z["pool_backtrack"], np.uint16)
    keep = []
    if a.strings:
        # the same records as yara_amd.Tables.from_npz(strings=True)
        class String(ctypes.Structure):   # yr_amd_string (include/yara_amd.h)
            _fields_ = [("flags", ctypes.c_uint32), ("length", ctypes.c_uint32),
                        ("fixed_offset", ctypes.c_int64), ("bytes_offset", ctypes.c_uint64)]
        offs = z["str_offsets"]
        n_str = len(z["str_flags"])
        recs = (String * max(n_str, 1))()
        for k in range(n_str):
            recs[k].flags = int(z["str_flags"][k])
            recs[k].length = int(offs[k + 1] - offs[k])
            recs[k].fixed_offset = int(z["str_fixed_offset"][k])
            recs[k].bytes_offset = int(offs[k])
        ps = np.ascontiguousarray(z["pool_string"], np.uint32)
        ps = ps if ps.size else np.zeros(1, np.uint32)
        blob = np.ascontiguousarray(z["str_bytes"], np.uint8)
        blob_n = blob.size
        blob = blob if blob.size else np.zeros(1, np.uint8)
        lower = np.arange(256, dtype=np.uint8)
        lower[ord("A"):ord("Z") + 1] += 32
        re_arrs = None
        if "re_kind" in z:
            fl = np.where(z["re_kind"] != 0, z["re_fwd_len"], 0)
            re_arrs = [np.ascontiguousarray(x, np.uint32) for x in (z["re_fwd_off"], fl, z["re_bwd_off"], z["re_bwd_len"])]
            re_arrs = [x if x.size else np.zeros(1, np.uint32) for x in re_arrs]
            code = np.ascontiguousarray(z["re_code"], np.uint8)
            re_n = code.size
            code = code if code.size else np.zeros(1, np.uint8)
        keep += [recs, ps, blob, lower, re_arrs]
    scanners = []
    for L in libs:
        t, s = _vp(), _vp()
        assert L.yr_amd_tables_create(T.ctypes.data, M.ctypes.data, T.size, nx.ctypes.data,
                                      bt.ctypes.data, nx.size, 0, ctypes.byref(t)) == 0
        if a.strings:
            assert L.yr_amd_tables_set_strings(t, ps.ctypes.data, int(z["pool_string"].size), ctypes.addressof(recs),
                                               n_str, blob.ctypes.data, blob_n, lower.ctypes.data) == 0
            if re_arrs is not None:
                assert L.yr_amd_tables_set_re_code(t, len(z["re_fwd_off"]), *[x.ctypes.data for x in re_arrs],
                                                   code.ctypes.data, re_n) == 0
        assert L.yr_amd_scanner_create(t, None, ctypes.byref(s)) == 0
        L.yr_amd_scanner_set_timing(s, 1)
        if a.verified_only or names[len(scanners)].endswith(":vo"):
            L.yr_amd_scanner_set_verified_only.argtypes = [_vp, ctypes.c_int]
            assert L.yr_amd_scanner_set_verified_only(s, 1) == 0
        scanners.append((L, t, s))

    import time
    wall = {v: [] for v in names}

    def scan(i):
        L, _, s = scanners[i]
        cnt = ctypes.c_uint64()
        w0 = time.perf_counter()
        assert L.yr_amd_scan_device(s, _vp(buf.data_ptr()), n, 0, n) == 0
        assert L.yr_amd_scan_device_result(s, None, ctypes.byref(cnt), None) == 0
        km, sm = ctypes.c_float(), ctypes.c_float()
        L.yr_amd_scanner_kernel_ms(s, ctypes.byref(km))
        L.yr_amd_scanner_scan_ms(s, ctypes.byref(sm))
        vms = 0.0
        if a.verify:
            nrec = ctypes.c_uint64()
            t0 = time.perf_counter()
            assert L.yr_amd_verify_device(s, 0, None, ctypes.byref(nrec)) == 0
            vms = (time.perf_counter() - t0) * 1e3
        wall[names[i]].append((time.perf_counter() - w0) * 1e3)
        return km.value, sm.value, cnt.value, vms

    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < a.warm_s:   # clock ramp (bench.py)
        scan(k % len(names))
        k += 1
    kern = {v: [] for v in names}
    wall.update({v: [] for v in names})
    scanms = {v: [] for v in names}
    verms = {v: [] for v in names}
    counts = {}
    ratios = {v: [] for v in names}
    for r in range(a.rounds):
        order = list(range(len(names))) if r % 2 == 0 else list(reversed(range(len(names))))
        med = {}
        for i in order:
            ks = []
            for _ in range(a.reps):
                km, sm, c, vm = scan(i)
                ks.append(km)
                scanms[names[i]].append(sm)
                verms[names[i]].append(vm)
                counts[names[i]] = c
            kern[names[i]] += ks
            med[names[i]] = statistics.median(ks)
        for v in names:
            ratios[v].append(med[v] / med[names[0]])
    out = {"rules": a.rules, "bytes": n, "rounds": a.rounds, "reps": a.reps, "strings": a.strings,
           "variants": {}}
    for v in names:
        out["variants"][v] = {"kernel_median_ms": round(statistics.median(kern[v]), 4),
                              "kernel_min_ms": round(min(kern[v]), 4),
                              "scan_median_ms": round(statistics.median(scanms[v]), 4),
                              "ratio_to_first_median": round(statistics.median(ratios[v]), 4),
                              **({"verify_median_ms": round(statistics.median(verms[v]), 4),
                                  "step_wall_median_ms": round(statistics.median(wall[v]), 4)} if a.verify else {}),
                              "candidates": counts[v]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
