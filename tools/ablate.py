"""Profiling ablations of the scan kernel (diagnostic only; modes != 0 are wrong
by construction).  Interleaved rounds in one process (guide §5.4 rule 24).

    python tools/ablate.py [--gib 4] [--rules C] [--rounds 5] [--modes 0,1,2,3]

Modes other than 0 exist only in the diagnostic build (make -C yara_amd/csrc
diag -> yara_amd/_diag/libyara_amd.so), which is loaded unless YARA_AMD_LIB
names another build; with --modes 0 any build (e.g. a variant) is timed.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

NAMES = {0: "product", 1: "no-exact-check", 2: "stage1-only", 3: "stream-only",
         4: "stage1-conflict-free-lds", 5: "stage1-valu-no-lds",
         6: "stage1-lds-no-test", 7: "stage1+appends-no-drain", 8: "stage1+append-arith-no-lds-writes",
         9: "drain-one-l2-load", 10: "drain-exact-valu-no-loads", 11: "product-reads-first",
         12: "first-level-only", 13: "stage1+appends-index-dword-only", 24: "bytekeys-detected-not-appended", 25: "bytekeys-not-detected",
         # ablations of the byte-key variant the product runs for the rule set (its filter)
         101: "bk-stage1-only", 102: "bk-appends-drains-drop", 103: "bk-keys-detected-not-appended",
         104: "bk-keys-not-detected"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--rules", default="C")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="0,1,2,3,4,5,6")
    a = ap.parse_args()
    modes = [int(m) for m in a.modes.split(",")]
    if any(modes) and not os.environ.get("YARA_AMD_LIB"):
        os.environ["YARA_AMD_LIB"] = os.path.join(REPO, "yara_amd", "_diag", "libyara_amd.so")
    import torch
    import yara_amd
    from yara_amd import _lib
    L = _lib.lib()
    set_mode = getattr(L, "yr_amd__diag_kernel_mode", None)
    if set_mode is not None:
        set_mode.argtypes = [ctypes.c_void_p, ctypes.c_int]
    elif any(modes):
        raise SystemExit("modes != 0 need the diagnostic build (make -C yara_amd/csrc diag)")
    n = int(a.gib * (1 << 30))
    buf = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(buf.data_ptr(), n, 1)
    t = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables", a.rules + ".npz"))
    sc = yara_amd.Scanner(t)
    sc.set_timing(True)
    res = {m: [] for m in modes}
    counts = {}
    for _ in range(60):                 # clock ramp (see bench.py)
        sc.scan_device(buf.data_ptr(), n)
        sc.device_result()
    for _ in range(a.rounds):
        for m in modes:
            if set_mode is not None:
                assert set_mode(sc._h, m) == 0
            for _ in range(a.reps):
                sc.scan_device(buf.data_ptr(), n)
                counts[m] = sc.device_result()[1]
                res[m].append(sc.kernel_ms())
    if set_mode is not None:
        set_mode(sc._h, 0)
    out = {}
    for m in modes:
        med = statistics.median(res[m])
        out[NAMES.get(m, "mode%d" % m)] = {"median_ms": round(med, 4), "min_ms": round(min(res[m]), 4),
                         "GB/s": round(n / (med * 1e-3) / 1e9, 1), "candidates": counts[m]}
    print(json.dumps({"rules": a.rules, "bytes": n, "modes": out}, indent=1))


if __name__ == "__main__":
    main()
