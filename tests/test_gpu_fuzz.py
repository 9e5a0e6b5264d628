"""Randomised GPU parity on fresh rule sets (beyond the committed fixtures).

For 48 rule sets from tests/golden/fuzz_rules.py (seeds 300..347, disjoint from
the 12 fixtures and the 200 CPU fuzz seeds) the stock compiler builds the
Aho-Corasick tables and string records (oracle/_ref/refdump, compiled in the
build container; it reads only the generated rules file) and the HIP path
scans a planted 1 MiB buffer:

  * the candidate stream equals the oracle's restatement of scanner.c:45-176
    (oracle.candidates, itself pinned to stock libyara by test_oracle_fuzz.py);
  * the on-device pre-verification records equal the oracle's verify-call
    stream (oracle.walk_verify) filtered by the oracle's restatement of the
    scan.c / re.c decisions (oracle.literal_effect), call for call;
  * three shards of the block, each scanned from a device window holding only
    the shard plus the rule set's verify halos (yr_amd_scan_window, the
    multi-GPU path), give the same records concatenated.

The sets mix 1- to 4-byte atoms (incl. the stage-1 byte-key kernel variant),
literal flags and hex / regexp strings.  Skipped where refdump is absent.
"""
import os
import subprocess

import numpy as np
import pytest

import fuzz_rules
import make_golden
import oracle
import yara_amd
from conftest import REPO
from oracle.tables import read_tables

REFDUMP = os.path.join(REPO, "oracle", "_ref", "refdump")
# (YAMD_FUZZ_SEEDS="a-b": another range, for an extended one-off run)
_seeds = os.environ.get("YAMD_FUZZ_SEEDS", "300-347").split("-")
SEEDS = range(int(_seeds[0]), int(_seeds[1]) + 1)
SIZE = 1 << 20

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.access(REFDUMP, os.X_OK),
                                 reason="oracle/_ref/refdump not built (needs /root/reference)")]


@pytest.mark.parametrize("seed", SEEDS)
def test_fresh_rule_set_on_gpu(tmp_path, seed):
    rules = str(tmp_path / "f.yar")
    with open(rules, "w") as f:
        f.write(fuzz_rules.gen(seed))
    subprocess.run([REFDUMP, "tables", rules, str(tmp_path / "t.bin")], check=True,
                   stdout=subprocess.DEVNULL)
    t = read_tables(str(tmp_path / "t.bin"))
    z = make_golden.tables_dict(t)
    npz = str(tmp_path / "t.npz")
    np.savez(npz, **z)
    data = fuzz_rules.buffer(oracle.xorshift, seed, SIZE)

    sc = yara_amd.Scanner(yara_amd.Tables.from_npz(npz, device=0, strings=True))
    pos, allp = sc.candidates(data)
    if t.M[0] != 0:
        assert allp
    else:
        assert not allp
        np.testing.assert_array_equal(pos, oracle.candidates(t, data))

    vpos, vidx = oracle.walk_verify(t, data)
    keep = oracle.literal_effect(np.load(npz), vpos, vidx, data)
    want_off = (vpos.astype(np.int64) - t.pool_backtrack[vidx].astype(np.int64))[keep]
    recs = sc.verify_calls(data)
    np.testing.assert_array_equal(recs["offset"].astype(np.int64), want_off)
    np.testing.assert_array_equal(recs["pool_index"], vidx[keep])

    # (verify_calls runs yr_amd_scan_block_verified: a verified-only scan, the
    # libyara path's mode, whose byte-key kernels decide classes and drop dead
    # candidates.)  The same records from a full device scan, candidate
    # indices included: the verified-only records index the full stream.
    import torch
    from yara_amd._hip import memcpy
    d = torch.from_numpy(np.ascontiguousarray(data)).cuda()
    sv = yara_amd.Scanner(sc.tables)
    sv.scan_device(d.data_ptr(), SIZE)
    sv.device_result()
    ptr, cnt = sv.verify_device(0)
    h = torch.empty(max(cnt, 1) * 16, dtype=torch.uint8, device="cuda")
    memcpy(h.data_ptr(), ptr, cnt * 16, 3)
    vo = np.frombuffer(h[:cnt * 16].cpu().numpy().tobytes(), dtype=yara_amd._lib.VERIFY_REC_DTYPE)
    np.testing.assert_array_equal(vo["offset"].astype(np.int64), want_off)
    np.testing.assert_array_equal(vo["pool_index"], vidx[keep])
    np.testing.assert_array_equal(vo["candidate"], recs["candidate"])

    if t.M[0] != 0:
        return
    from yara_amd import dist as ydist
    before, after = ydist.tables_halos(sc.tables)
    got = []
    for r in range(3):
        b, e = ydist.shard_bounds(SIZE, 3, r, align=1 << 12)
        lo, hi = ydist.shard_window(SIZE, b, e, before, after)
        win = torch.from_numpy(np.ascontiguousarray(data[lo:hi])).cuda()
        sc.scan_window(win.data_ptr(), lo, hi, SIZE, b, e)
        sc.device_result()
        ptr, cnt = sc.verify_device(0)
        h = torch.empty(max(cnt, 1) * 16, dtype=torch.uint8, device="cuda")
        memcpy(h.data_ptr(), ptr, cnt * 16, 3)
        got.append(np.frombuffer(h[:cnt * 16].cpu().numpy().tobytes(),
                                 dtype=yara_amd._lib.VERIFY_REC_DTYPE))
    got = np.concatenate(got)
    np.testing.assert_array_equal(got["offset"].astype(np.int64), want_off)
    np.testing.assert_array_equal(got["pool_index"], vidx[keep])
