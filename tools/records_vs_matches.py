"""Pre-verification effect per golden case: the stock libyara verify calls of
the case (golden verify_count), the records the device keeps
(yr_amd_verify_device), and the matches stock libyara reports (golden
match_count).  A record can produce zero or several matches; records ==
matches means no call without an effect survives.

    python tools/records_vs_matches.py [--max-mib 64] > records.json
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=64)
    a = ap.parse_args()
    import yara_amd
    from conftest import case_data, golden, tables_npz
    out = {}
    for name, rec in sorted(golden()["cases"].items()):
        if rec["block"] or rec["size"] > (a.max_mib << 20):
            continue
        tab = yara_amd.Tables.from_npz(tables_npz(rec["rules"]), device=0, strings=True)
        r = yara_amd.Scanner(tab).verify_calls(case_data(rec))
        out[name] = {"rules": rec["rules"], "bytes": rec["size"],
                     "verify_calls": rec["verify_count"], "records": int(len(r)),
                     "matches": rec["match_count"]}
        print(name, out[name], file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
