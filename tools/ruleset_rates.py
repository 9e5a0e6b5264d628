"""Scan-kernel and pre-verification times of many rule-set shapes on the same
device-resident input (SURVEY.md §8d data generator, seed 1).

For each rule set: the scan kernel's HIP-event time (median of --reps after a
warm-up), the candidate count, the filter's pass rate, and the on-device
pre-verification time and record count.  Root-accepting sets make every
position a candidate; their verify pass is limited to blocks below 2^32
candidates, so they run on --root-gib.

    python tools/ruleset_rates.py [--gib 4] [--sets short,rx,...] > rates.json
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--root-gib", type=float, default=1.0)
    ap.add_argument("--sets", default="C,B,E,lit,hex,rx,short,fuzz0,fuzz3,fuzz7,root")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--warm-s", type=float, default=1.0)
    ap.add_argument("--step-reps", type=int, default=30)
    a = ap.parse_args()
    import torch
    import yara_amd
    n_max = int(a.gib * (1 << 30))
    buf = torch.empty(n_max + 16, dtype=torch.uint8, device="cuda")
    yara_amd.fill_xorshift64(buf.data_ptr(), n_max, 1)
    torch.cuda.synchronize()
    # clock ramp (bench.py): ~25 ms of scan work before anything is timed
    warm = yara_amd.Scanner(yara_amd.Tables.from_npz(
        os.path.join(REPO, "tests", "golden", "tables", "C.npz"), device=0))
    for _ in range(60):
        warm.scan_device(buf.data_ptr(), n_max)
        warm.device_result()
    del warm
    out = {}
    for name in a.sets.split(","):
        t = yara_amd.Tables.from_npz(os.path.join(REPO, "tests", "golden", "tables", name + ".npz"),
                                     device=0, strings=True)
        info = t.info()
        n = int(a.root_gib * (1 << 30)) if info["root_accepting"] else n_max
        sc = yara_amd.Scanner(t)
        for _ in range(40):   # the tables' host build idled the GPU: ramp the clocks again
            sc.scan_device(buf.data_ptr(), n)
            sc.device_result()
        rec = {"bytes": n}
        if info["root_accepting"]:
            # every position is a candidate: no scan kernel runs at all
            rec.update({"kernel_ms": 0.0, "candidates": n + 1})
        else:
            sc.set_timing(True)
            ks, ss, cnt = [], [], 0
            for _ in range(a.reps):
                sc.scan_device(buf.data_ptr(), n)
                cnt = sc.device_result()[1]
                ks.append(sc.kernel_ms())
                ss.append(sc.scan_ms())
            sc.set_timing(False)
            k = statistics.median(ks)
            # scan_ms: the scan kernel and its compaction (the position list and
            # the candidate classes)
            rec.update({"kernel_ms": round(k, 4), "scan_ms": round(statistics.median(ss), 4),
                        "GB/s": round(n / (k * 1e-3) / 1e9, 1),
                        "frac": round(n / (k * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "candidates": int(cnt)})
        rec.update({"root_accepting": bool(info["root_accepting"]),
               "keys_by_length": info["keys_by_length"],
               "filter_fill": round(info["filter_set_bits"] / float(1 << info["filter_bits"]), 4)})
        if not a.no_verify:
            sc.scan_device(buf.data_ptr(), n)
            sc.device_result()
            sc.verify_device(0)
            vs = []
            for _ in range(3):
                sc.scan_device(buf.data_ptr(), n)
                sc.device_result()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                _, nrec = sc.verify_device(0)
                vs.append((time.perf_counter() - t0) * 1e3)
            rec["verify_ms"] = round(statistics.median(vs), 3)
            rec["records"] = int(nrec)
            # the verified path as the libyara side runs it (verified-only scans,
            # yr_amd_scanner_set_verified_only): scan kernel and compaction (HIP
            # events), then pre-verification; and the whole step's wall time
            # (scan + result + verify, host waits included)
            if not info["root_accepting"]:
                for mode in ("full", "verified_only"):
                    # (a scanner per mode: each learns its own output capacity)
                    sc = yara_amd.Scanner(t)
                    sc.set_verified_only(mode == "verified_only")
                    # whole steps for --warm-s first: a step idles the GPU while
                    # the host waits, and five of them left the clocks below
                    # their steady state (rx's verified-only kernel 1.02 ms here
                    # against 0.94 in tools/ab_inproc.py, gpurun r5h53)
                    t0 = time.perf_counter()
                    while time.perf_counter() - t0 < a.warm_s:
                        sc.scan_device(buf.data_ptr(), n)
                        sc.device_result()
                        sc.verify_device(0)
                    sc.set_timing(True)
                    ks, ss, ws, vv = [], [], [], []
                    for _ in range(a.step_reps):
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        sc.scan_device(buf.data_ptr(), n)
                        cnt = sc.device_result()[1]
                        t1 = time.perf_counter()
                        _, nrec = sc.verify_device(0)
                        t2 = time.perf_counter()
                        ks.append(sc.kernel_ms())
                        ss.append(sc.scan_ms())
                        vv.append((t2 - t1) * 1e3)
                        ws.append((t2 - t0) * 1e3)
                    sc.set_timing(False)
                    km, sm, vm = statistics.median(ks), statistics.median(ss), statistics.median(vv)
                    # (a verified-only scan's pre-verification is queued while its
                    # compaction still runs, so scan_ms + verify_ms counts that
                    # overlap twice: step_wall_ms, the whole step on the host's
                    # clock, is the measure of the verified path)
                    wm = statistics.median(ws)
                    rec[mode] = {"kernel_ms": round(km, 4), "scan_ms": round(sm, 4),
                                 "verify_ms": round(vm, 4), "scan_plus_verify_ms": round(sm + vm, 4),
                                 "frac_scan_plus_verify": round(n / ((sm + vm) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "step_wall_ms": round(wm, 4),
                                 "frac_step_wall": round(n / (wm * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "candidates": int(cnt), "stream_length": int(sc.stream_length()),
                                 "records": int(nrec)}
                sc.set_verified_only(False)
        out[name] = rec
        print(name, rec, file=sys.stderr, flush=True)
        del sc, t
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
