"""Per-shard goldens of config D: the config C rule set over one
32 GiB block of the canonical input (xorshift64 seed 1), sharded as
bench.py / yara_amd.dist do with 4 GiB per GPU: shard r owns candidate
positions (4r GiB, 4(r+1) GiB] (shard 0 also position 0).  The shard bounds
do not depend on the number of ranks (total = 4 GiB x ranks), so the same
eight records check N = 1, 2, 4 and 8.

Test infrastructure, computed twice and asserted equal:
  * stock: the reference libyara itself (oracle/_ref/refdump, the hooked stock
    scanner.c) scans each shard's window [4r GiB - 64, 4(r+1) GiB) of the
    canonical stream (generated from the jump-ahead state, refdump's "xst:"
    spec); the candidates are the distinct positions of its verify calls
    past the window's first 64 bytes (every candidate there makes calls: the
    largest backtrack is 16, and the walk restarts exactly after 4 bytes,
    limits.h:68);
  * port: the oracle's restatement of scanner.c:45-176 (oracle/ac_oracle.c) in
    1 GiB chunks, each with its 4-byte warm-up.
Shard 0 must also equal the stock golden C_4G (count and SHA-256).

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


def shard_stock_digest(r):
    """The same shard from the stock reference build (build container only)."""
    import subprocess
    import tempfile
    import oracle
    refdump = os.path.join(REPO, "oracle", "_ref", "refdump")
    b, e = r * SHARD, (r + 1) * SHARD
    lo = max(0, b - 64)
    with tempfile.TemporaryDirectory() as td:
        rules = os.path.join(td, "C.yar")
        import gen_rules
        with open(rules, "w") as f:
            f.write(gen_rules.gen("C"))
        spec = "xst:%d:%d" % (oracle.xorshift_state(SEED, lo), e - lo)
        subprocess.run([refdump, "scan", rules, spec, os.path.join(td, "s")], check=True,
                       stdout=subprocess.DEVNULL)
        rec = np.fromfile(os.path.join(td, "s.verify"),
                          dtype=[("b", "<u8"), ("p", "<u8"), ("k", "<u4")])
    pos = np.unique(rec["p"]).astype(np.uint64) + np.uint64(lo)
    pos = pos[(pos > b) if b > 0 else (pos >= 0)]
    pos = pos[pos <= e]
    return r, int(pos.size), hashlib.sha256(np.asarray(pos, dtype="<u8").tobytes()).hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=4)
    a = ap.parse_args()
    t0 = time.time()
    with Pool(a.jobs) as pool:
        res = sorted(pool.map(shard_positions_digest, range(N_SHARDS)))
        stock = sorted(pool.map(shard_stock_digest, range(N_SHARDS)))
    assert stock == res, "stock shards differ from the restatement: %s vs %s" % (stock, res)
    with open(os.path.join(HERE, "golden.json")) as f:
        c4 = json.load(f)["cases"]["C_4G"]
    assert res[0][1] == c4["candidate_count"] and res[0][2] == c4["candidate_sha"], \
        "shard 0 differs from the stock golden C_4G"
    out = {"rules": "C", "seed": SEED, "shard_bytes": SHARD,
           "what": "candidate positions (4r GiB, 4(r+1) GiB] of the 32 GiB config-D block "
                   "(shard 0 also position 0): count and SHA-256 of the little-endian u64 "
                   "positions; every shard computed by the stock reference libyara (refdump, "
                   "hooked scanner.c) and by the oracle restatement, asserted equal; shard 0 == "
                   "stock golden C_4G",
           "provenance": "stock",
           "shards": [{"count": c, "sha": s} for _, c, s in res]}
    with open(os.path.join(HERE, "config_d.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("config_d.json: %s (%.0f s)" % ([c for _, c, _ in res], time.time() - t0))


if __name__ == "__main__":
    main()
