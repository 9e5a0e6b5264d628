"""Summarise rocprofv3 kernel stats of tools/r5_prof_verified.sh runs:
    python tools/prof_summary.py gpurun_out/<tag> [sets]"""
import csv
import json
import os
import sys

d = sys.argv[1]
sets = sys.argv[2:] or ["rx", "fuzz0", "short", "fuzz3"]
for r in sets:
    p = os.path.join(d, r, "run_kernel_stats.csv")
    if not os.path.exists(p):
        continue
    line = [l for l in open(os.path.join(d, r + ".txt")) if "verified step" in l]
    print(line[0].strip() if line else r)
    for x in csv.DictReader(open(p)):
        if "xorshift" in x["Name"]:
            continue
        print("   %-50s calls %5s avg %9.1f us" % (x["Name"][:50], x["Calls"], float(x["AverageNs"]) / 1000))
rp = os.path.join(d, "rates.json")
if os.path.exists(rp):
    for k, v in json.load(open(rp)).items():
        for m in ("full", "verified_only"):
            if m in v:
                x = v[m]
                print("%-6s %-14s kernel %.4f scan %.4f verify %.4f sum %.4f (frac %.3f) wall %.4f cands %d records %d"
                      % (k, m, x["kernel_ms"], x["scan_ms"], x["verify_ms"], x["scan_plus_verify_ms"],
                         x["frac_scan_plus_verify"], x["step_wall_ms"], x["candidates"], x["records"]))
