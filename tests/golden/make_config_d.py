"""Per-shard goldens of config D: the config C rule set over one
32 GiB block of the canonical input (xorshift64 seed 1), sharded as
bench.py / yara_amd.dist do with 4 GiB per GPU: shard r owns candidate
positions (4r GiB, 4(r+1) GiB] (shard 0 also position 0).  The shard bounds
do not depend on the number of ranks (total = 4 GiB x ranks), so the same
eight records check N = 1, 2, 4 and 8.

Test infrastructure: computed with the oracle's restatement of scanner.c:45-176
(oracle/ac_oracle.c, pinned to the stock reference build by
test_oracle_golden.py / test_oracle_fuzz.py); shard 0 must equal the stock
golden C_4G (count and SHA-256), which this script asserts.  Each shard is
generated in 1 GiB chunks, each with its 4-byte warm-up (libyara's trie is at
most 4 deep, limits.h:68).

    python tests/golden/make_config_d.py [--jobs 4]   ->  tests/golden/config_d.json
"""
import argparse
import hashlib
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), HERE]

GiB = 1 << 30
SHARD = 4 * GiB
N_SHARDS = 8
CHUNK = GiB
SEED = 1


def shard_positions_digest(r):
    import oracle
    from conftest import ref_tables
    tab = ref_tables("C")
    b, e = r * SHARD, (r + 1) * SHARD
    h = hashlib.sha256()
    count = 0
    for c0 in range(b, e, CHUNK):
        c1 = min(e, c0 + CHUNK)
        lo = max(0, c0 - 4)
        data = oracle.xorshift_at(c1 - lo, SEED, lo)
        pos = oracle.candidates(tab, data).astype(np.uint64) + np.uint64(lo)
        keep = pos > c0 if c0 > 0 else pos >= 0
        pos = pos[keep & (pos <= c1)]
        h.update(np.asarray(pos, dtype="<u8").tobytes())
        count += int(pos.size)
    return r, count, h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=4)
    a = ap.parse_args()
    t0 = time.time()
    with Pool(a.jobs) as pool:
        res = sorted(pool.map(shard_positions_digest, range(N_SHARDS)))
    with open(os.path.join(HERE, "golden.json")) as f:
        c4 = json.load(f)["cases"]["C_4G"]
    assert res[0][1] == c4["candidate_count"] and res[0][2] == c4["candidate_sha"], \
        "shard 0 differs from the stock golden C_4G"
    out = {"rules": "C", "seed": SEED, "shard_bytes": SHARD,
           "what": "candidate positions (4r GiB, 4(r+1) GiB] of the 32 GiB config-D block "
                   "(shard 0 also position 0): count and SHA-256 of the little-endian u64 "
                   "positions; oracle restatement, shard 0 == stock golden C_4G",
           "shards": [{"count": c, "sha": s} for _, c, s in res]}
    with open(os.path.join(HERE, "config_d.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("config_d.json: %s (%.0f s)" % ([c for _, c, _ in res], time.time() - t0))


if __name__ == "__main__":
    main()
