"""Summarise tools/pmc_detail.sh output: per kernel mode, the chip-wide counters
of the scan kernel averaged over the last `reps` launches of each pass (the
earlier launches are tools/ablate.py's mode-0 clock warm-up).

    python tools/pmc_modes.py gpurun_out/pmc_<tag> [--reps 4] [--out file.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--out")
    a = ap.parse_args()
    res = collections.defaultdict(dict)
    for path in sorted(glob.glob(os.path.join(a.dir, "m*_p*", "**", "*counter_collection.csv"),
                                 recursive=True)):
        mode = int(re.search(r"/m(\d+)_p\d+", path).group(1))
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            if "scan_segments_kernel" not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        for name, d in per.items():
            last = [d[k] for k in sorted(d)][-a.reps:]
            res[mode][name] = sum(last) / len(last)
    out = {}
    for mode, c in sorted(res.items()):
        g = c.get("GRBM_GUI_ACTIVE", 0)
        der = {}
        if g:
            cus = 256
            der["kernel_us_at_clock"] = None
            der["valu_busy_frac"] = c.get("SQ_ACTIVE_INST_VALU", 0) / (g * cus * 4)
            der["lds_idx_active_frac"] = c.get("SQ_LDS_IDX_ACTIVE", 0) / (g * cus)
            der["lds_conflict_frac_of_active"] = (c.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                  max(1.0, c.get("SQ_LDS_IDX_ACTIVE", 0)))
            der["wait_any_per_wave_cycle"] = c.get("SQ_WAIT_ANY", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 0))
            der["valu_insts_per_wave_tile"] = c.get("SQ_INSTS_VALU", 0) / (4 << 20)
            der["lds_insts_per_wave_tile"] = c.get("SQ_INSTS_LDS", 0) / (4 << 20)
            der["salu_insts_per_wave_tile"] = c.get("SQ_INSTS_SALU", 0) / (4 << 20)
        out[mode] = {"counters": c, "derived": der}
    txt = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
