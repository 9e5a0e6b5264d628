"""Where the host replay of dense-match rule sets spends its time (VERDICT r04
"next round" item 6), on the CPU alone: the records a block's pre-verification
hands the host are replayed into libyara three ways on the same scanner state
(integration/yr_gpu_scanner.c yr_gpu_replay_profile):

  shim      the shim's replay (_replay_records: the walk's timeout checks,
            scanner.c:74-81, then yr_scan_verify_match per record)
  shim_only the shim's per-record work without the libyara call
  libyara   yr_scan_verify_match alone, one call per record (scan.c:992-1089,
            _yr_scan_match_callback scan.c:634-765 inside it)

Records: the stock hooked scan of the block (oracle/_ref/refdump: every call
the reference loop makes, scanner.c:105-121) filtered by the oracle's
restatement of the device's decisions (oracle.literal_effect: the records
yr_amd_verify_device returns, pinned by tests/test_preverify.py).  The stock
yr_rules_scan_mem of the same block is timed beside it.

    python tools/replay_profile.py [--sets short,fuzz3] [--mib 1024] [--reps 7] > profiles/r06_replay_profile.json

Each mode runs once per repetition, the modes interleaved in a rotating order;
the tool reports medians with their spread and exits non-zero if a part (the
libyara calls alone, the shim's own work alone) measures longer than the whole.
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]


class Rec(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("pool_index", ctypes.c_uint32), ("candidate", ctypes.c_uint32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", default="short,fuzz3")
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import gen_rules
    import oracle
    from conftest import tables_npz
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libyara_ref.so"), mode=ctypes.RTLD_GLOBAL)
    shim = ctypes.CDLL(os.path.join(REPO, "integration", "_build", "libyara_gpu_shim.so"))
    ref.yr_initialize()
    n = a.mib << 20
    data = oracle.xorshift(n, 1)
    out = {"what": __doc__.split("\n\n")[0], "block_mib": a.mib, "cpu": open("/proc/cpuinfo").read()
           .split("model name")[1].split("\n")[0].strip(": "), "sets": {}}
    def text(name):
        if name.startswith("fuzz"):
            import fuzz_rules
            return fuzz_rules.gen(int(name[4:]))
        p = os.path.join(REPO, "tests", "golden", "rules", name + ".yar")
        return open(p).read() if os.path.exists(p) else gen_rules.gen(name)
    bad = []
    for name in a.sets.split(","):
        src = text(name)
        with tempfile.TemporaryDirectory() as td:
            rp = os.path.join(td, "r.yar")
            open(rp, "w").write(src)
            subprocess.run([os.path.join(REPO, "oracle", "_ref", "refdump"), "scan", rp,
                            "xs:1:%d" % n, os.path.join(td, "s")], check=True, stdout=subprocess.DEVNULL)
            v = np.fromfile(os.path.join(td, "s.verify"), dtype=[("b", "<u8"), ("p", "<u8"), ("k", "<u4")])
        z = np.load(tables_npz(name))
        P, K = v["p"], v["k"]
        keep = oracle.literal_effect(z, P, K, data)
        off = (P - z["pool_backtrack"][K].astype(np.uint64))[keep]
        recs = np.zeros(int(keep.sum()), dtype=[("offset", "<u8"), ("pool_index", "<u4"), ("candidate", "<u4")])
        recs["offset"] = off
        recs["pool_index"] = K[keep]
        # rules + scanner from the stock library (the shim links the same one)
        comp = ctypes.c_void_p()
        assert ref.yr_compiler_create(ctypes.byref(comp)) == 0
        ref.yr_compiler_add_string.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
        assert ref.yr_compiler_add_string(comp, src.encode(), None) == 0
        rules = ctypes.c_void_p()
        assert ref.yr_compiler_get_rules(comp, ctypes.byref(rules)) == 0
        scanner = ctypes.c_void_p()
        assert ref.yr_scanner_create(rules, ctypes.byref(scanner)) == 0
        CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
        cb = CB(lambda c, m, d, u: 0)
        ref.yr_scanner_set_callback.argtypes = [ctypes.c_void_p, CB, ctypes.c_void_p]
        ref.yr_scanner_set_callback(scanner, cb, None)
        shim.yr_gpu_replay_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                               ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64,
                                               ctypes.POINTER(ctypes.c_double)]
        res = {"records": int(len(recs)), "stock_verify_calls": int(len(v))}
        modes = (("shim", 0, 0), ("shim_timeout", 0, 10 ** 15), ("shim_only", 1, 0),
                 ("shim_only_timeout", 1, 10 ** 15), ("libyara", 2, 0))
        times = {label: [] for label, _, _ in modes}
        # the modes interleaved, the order rotated every repetition (one pass
        # of each per repetition), so that a slow stretch of a shared host or a
        # cache warmed by the previous mode lands on every mode alike
        for r in range(a.reps):
            for q in range(len(modes)):
                label, mode, tmo = modes[(q + r) % len(modes)]
                sec = ctypes.c_double()
                rc = shim.yr_gpu_replay_profile(scanner, recs.ctypes.data, len(recs), data.ctypes.data, n,
                                                mode, tmo, ctypes.byref(sec))
                assert rc == 0, (label, rc)
                times[label].append(sec.value)
        for label, _, _ in modes:
            t = sorted(times[label])
            med = statistics.median(t)
            res[label + "_s"] = {"median": round(med, 4), "min": round(t[0], 4), "max": round(t[-1], 4),
                                 "spread": round((t[-1] - t[0]) / med, 3)}
            res[label + "_ns_per_record"] = round(med / max(len(recs), 1) * 1e9, 1)
        # shares: medians of the per-repetition ratios (each repetition's parts
        # against the same repetition's whole) and their range
        for part, whole in (("libyara", "shim"), ("shim_only", "shim")):
            q = sorted(x / y for x, y in zip(times[part], times[whole]))
            res["share_%s_of_%s" % (part, whole)] = {"median": round(statistics.median(q), 4),
                                                    "min": round(q[0], 4), "max": round(q[-1], 4)}
        ref.yr_rules_scan_mem.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, CB,
                                          ctypes.c_void_p, ctypes.c_int]
        t0 = time.perf_counter()
        assert ref.yr_rules_scan_mem(rules, data.ctypes.data, n, 0, cb, None, 0) == 0
        res["stock_scan_s"] = round(time.perf_counter() - t0, 3)
        res["share_inside_libyara"] = res["share_libyara_of_shim"]["median"]
        # a part cannot take longer than the whole it is part of: a median share
        # above 1 means the measurement is noise, not a profile
        if res["share_inside_libyara"] > 1.0 or res["share_shim_only_of_shim"]["median"] > 1.0:
            bad.append(name)
        out["sets"][name] = res
        print(name, res, file=sys.stderr, flush=True)
        ref.yr_scanner_destroy(scanner)
        ref.yr_rules_destroy(rules)
    out["reps"] = a.reps
    out["method"] = ("each mode once per repetition, interleaved, order rotated per repetition; "
                     "medians, min/max and spread = (max - min) / median over the repetitions; "
                     "shares = medians of per-repetition ratios")
    print(json.dumps(out, indent=1))
    if bad:
        sys.exit("replay_profile: a part measured longer than the whole for %s" % ",".join(bad))


if __name__ == "__main__":
    main()
