"""Summarise a rocprofv3 PMC pass (FETCH_SIZE) of the scan kernel into
profiles/pmc_traffic.json, applying the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) counts half the bytes of a wide
coalesced streaming read -> hbm_bytes = 2 * FETCH_SIZE * 1024.

    python tools/pmc_summary.py <run_counter_collection.csv> <input_bytes> [out.json] [label]

label (e.g. "round r02, commit abc1234") is stored as "measured": bench.py
prints it with roofline.traffic so a stale profile is visible as such.
"""
import csv
import json
import sys

KERNEL = "scan_segments_kernel<0>"


def main():
    path, nbytes = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    label = sys.argv[4] if len(sys.argv) > 4 else "unlabelled"
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    if not vals:
        raise SystemExit("no FETCH_SIZE rows for %s" % KERNEL)
    fetch_kb = sum(vals) / len(vals)
    hbm = int(2 * fetch_kb * 1024)
    rec = {"kernel": KERNEL, "counter": "FETCH_SIZE", "launches": len(vals),
           "fetch_size_kb_per_launch": fetch_kb,
           "correction": "x2 (gfx950 FETCH_SIZE reads half of 16-B/lane streaming bytes)",
           "hbm_bytes_per_launch": hbm, "input_bytes": nbytes,
           "traffic_over_algorithmic": round(hbm / nbytes, 4), "measured": label}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
