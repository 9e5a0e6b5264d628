"""CPU model of the scan kernel's stage-1 filter designs on config C (VERDICT r04
"next round" item 2): for each design, the filter's pass rate on random input,
what it implies for the per-tile work (lanes passing, tiles that append, ring
entries per tile), the stage-1 issue slots read from the design's instruction
list, and a predicted kernel time from a model fitted to measured ablations.

Keys: the minimal accepting trie strings of config C's
stock tables (tests/golden/tables/C.npz), from a walk of the transition table
T (ahocorasick.h:37-50 encoding) -- the same set tables.cpp extracts.

Designs (filter bits as tables.cpp builds them, tested as kernels.hip does):
  pair       the product: 2^14 blocks of 64 bits, one ds_read_b64 per two
             positions, each key window in both roles (internal.h filter_probe_*)
  pair_xor   the same with b[0..1] XOR-folded into the block index (two
             instructions more per pair; both windows of a pair still share it)
  single     one block per position, the left role only (16 reads per tile)
  pair_k3    the pair filter with a third bit per window from a second dword pair
             (one more ds_read_b64 and shifts per pair)
  pair_1bit  one bit per window, 64-bit index (a v_lshrrev_b64 per window)
  pair_1w    one bit per window in a 32-bit word: the left role in the block's
             low word (a[0..4]), the right role in its high word (d[0..4])
  pair_mask  the product's filter, stage 1 keeping the per-position mask in the
             ring entry (SDWA form, as the drain's re-test) so that drains do not
             re-test
Model (ms, config C, 4 GiB; calibrated on profiles/r04_ablation.json h37:
stream 0.637, stage 1 0.666, + appends 0.771, product 0.839):
  t = 0.839 + a * (stage-1 slots - 120) + b * (tiles appending - 0.98)
            + c * (entries per tile - 3.90) * drain_share
  a = 7 us per VOP2-equivalent slot per tile (issue-bound product, DESIGN.md
  section 5), b = 0.105 / 0.98 ms, c = 0.068 / 3.90 ms (drains per entry per
  tile; drain_share = the part of a drain that remains for the design).
  issue_model: tables.cpp's filter-choice model (round 3, fitted to seven rule
  sets' kernels): VALU per tile = stage-1 VALU + 12 x tiles appending + 5 x
  filter-pass entries, 7 us each, relative to the product's 122.5.

    python tools/filter_model.py [--mib 64] > profiles/r05_filter_model.json
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]


def keys_of(T, M):
    """Minimal accepting strings of length 1..4 as {length: set(int little endian)}."""
    states = {0: b""}
    frontier = [0]
    acc = {}
    for depth in range(1, 5):
        nxt = []
        for s in frontier:
            base = states[s]
            for b in range(256):
                slot = s + b + 1
                if slot >= len(T):
                    continue
                t = int(T[slot])
                if (t & 0x1FF) != b + 1:
                    continue
                c = t >> 9
                states[c] = base + bytes([b])
                nxt.append(c)
                if M[c] != 0:
                    acc[states[c]] = True
        frontier = nxt
    keys = {1: set(), 2: set(), 3: set(), 4: set()}
    for s in acc:
        if any(s[i:] in acc for i in range(1, len(s))):
            continue   # has an accepting proper suffix: not minimal
        keys[len(s)].add(int.from_bytes(s, "little"))
    return keys


def windows3(keys):
    """The 3-byte windows the filter holds (tables.cpp: a 4-byte key's last 3
    bytes, a 3-byte key itself; no 1-/2-byte keys in config C)."""
    assert not keys[1] and not keys[2]
    return sorted({k >> 8 for k in keys[4]} | set(keys[3]))


class Filter:
    def __init__(self, blocks_log2=14):
        self.lo = np.zeros(1 << blocks_log2, np.uint32)
        self.hi = np.zeros(1 << blocks_log2, np.uint32)
        self.third = np.zeros(1 << blocks_log2, np.uint32)


def left(w):   # filter_probe_left: block x[10..23], bits x[0..4], x[5..9]
    return (w >> 10) & 0x3FFF, w & 31, (w >> 5) & 31


def right(w):  # filter_probe_right
    return (w >> 2) & 0x3FFF, (w >> 16) & 31, ((w >> 21) & 7) | ((w & 3) << 3)


def fold(blk, w, role):
    """pair_xor: b[0..1] (the two bits of b the block index leaves out; both
    windows of a pair share b, so they still read one block) XOR-ed into the
    block index's top bits."""
    b = (w >> 8) & 0xFF if role is left else w & 0xFF
    return blk ^ ((b & 3) << 12)


def build(design, W):
    f = Filter()
    W = np.array(W, dtype=np.int64)
    roles = [left] if design == "single" else [left, right]
    for role in roles:
        blk, bl, bh = role(W)
        if design == "pair_xor":
            blk = fold(blk, W, role)
        if design == "pair_1w":   # one bit per window: lo word (left role) / hi word (right role)
            if role is left:
                np.bitwise_or.at(f.lo, blk, (np.uint32(1) << bl.astype(np.uint32)).astype(np.uint32))
            else:
                np.bitwise_or.at(f.hi, blk, (np.uint32(1) << bl.astype(np.uint32)).astype(np.uint32))
            continue
        if design == "pair_1bit":
            idx = (bl | (bh << 5)) & 63
            np.bitwise_or.at(f.lo, blk, np.where(idx < 32, np.uint32(1) << (idx & 31), 0).astype(np.uint32))
            np.bitwise_or.at(f.hi, blk, np.where(idx >= 32, np.uint32(1) << (idx & 31), 0).astype(np.uint32))
            continue
        np.bitwise_or.at(f.lo, blk, (np.uint32(1) << bl.astype(np.uint32)).astype(np.uint32))
        np.bitwise_or.at(f.hi, blk, (np.uint32(1) << bh.astype(np.uint32)).astype(np.uint32))
        if design == "pair_k3":
            b3 = ((W * 0x9E3779) >> 11) & 31
            np.bitwise_or.at(f.third, blk, (np.uint32(1) << b3.astype(np.uint32)).astype(np.uint32))
    return f


def test(design, f, w, pos_parity):
    """Pass bit of the window w (3 bytes) at positions of the given parity
    (pair designs: even positions are the left role of their pair)."""
    role = left if (design == "single" or pos_parity == 0) else right
    blk, bl, bh = role(w)
    if design == "pair_xor":
        blk = fold(blk, w, role)
    if design == "pair_1w":
        return ((f.lo[blk] if role is left else f.hi[blk]) >> bl) & 1
    if design == "pair_1bit":
        idx = (bl | (bh << 5)) & 63
        word = np.where(idx < 32, f.lo[blk], f.hi[blk])
        return (word >> (idx & 31)) & 1
    p = ((f.lo[blk] >> bl) & (f.hi[blk] >> bh)) & 1
    if design == "pair_k3":
        b3 = ((w * 0x9E3779) >> 11) & 31
        p &= (f.third[blk] >> b3) & 1
    return p


# stage-1 VOP2-equivalent issue slots per 1 KiB wave-tile (product: 120 read
# from the ISA, profiles/r04_isa_budget.json) and LDS reads per tile; the
# differences are the design's extra / fewer instructions
STAGE1 = {
    "pair": (120, 8),
    "pair_xor": (120 + 8 * 2, 8),                  # + a v_and and a v_xor (the fold) per pair
    "single": (8.5 * 16, 16),                      # per position: addr 2, window 1.5, lo 1, hi 2, acc 2
    "pair_k3": (120 + 8 * 2 * 3, 16),              # + hash (2 VOP3 = 3 eq) per window, + a read per pair
    "pair_1bit": (120 - 8 * 2 * 2 + 8 * 2 * 1, 8),  # 64-bit shift (2 eq) instead of field + 2 shifts + and
    "pair_mask": (120 + 10, 8),                    # SDWA accumulation + the 16-bit mask combine
    "pair_1w": (120 - 8 * 6, 8),                   # per pair: no hi fields (2 x (shift + shift)), one OR3
}
DRAIN_SHARE = {"pair_mask": 100.0 / 233.0}         # the re-test (133 of ~233 slots per drain) skipped


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    a = ap.parse_args()
    import oracle
    z = np.load(os.path.join(REPO, "tests", "golden", "tables", "C.npz"))
    keys = keys_of(z["T"], z["M"])
    W = windows3(keys)
    data = oracle.xorshift(a.mib << 20, 1).astype(np.int64)
    n = data.size
    # the 3-byte window ending at every position (bytes i-3, i-2, i-1 for position i)
    w = data[:-2] | (data[1:-1] << 8) | (data[2:] << 16)
    par = np.arange(2, n) & 1              # parity of the window's last byte
    key3 = np.isin(w, np.array(W))         # inherent: the window is a key window
    out = {"what": __doc__.split("\n\n")[0], "keys_by_length": {k: len(v) for k, v in keys.items()},
           "key_windows": len(W), "sample_mib": a.mib, "inherent_window_rate": float(key3.mean()),
           "designs": {}}
    base = None
    for d in ("pair", "pair_xor", "single", "pair_k3", "pair_1bit", "pair_mask", "pair_1w"):
        f = build("pair" if d == "pair_mask" else d, W)
        p = np.zeros(w.size, np.int64)
        for parity in (0, 1):
            m = par == parity
            p[m] = test("pair" if d == "pair_mask" else d, f, w[m], parity)
        rate = float(p.mean())
        assert (p[key3] == 1).all(), d     # never a false negative
        lane = 1 - (1 - rate) ** 16
        tile = 1 - (1 - lane) ** 64
        entries = 64 * lane
        slots, lds = STAGE1[d]
        rec = {"pass_rate": round(rate, 5), "false_pass_rate": round(rate - float(key3.mean()), 5),
               "lane_pass": round(lane, 4), "tiles_appending": round(tile, 4),
               "entries_per_tile": round(entries, 3), "stage1_slots": slots, "stage1_lds_reads": lds}
        if d == "pair":
            base = rec
        t = 0.839 + 0.007 * (slots - 120) + (0.105 / 0.98) * (tile - base["tiles_appending"]) + \
            (0.068 / base["entries_per_tile"]) * (entries * DRAIN_SHARE.get(d, 1.0) - base["entries_per_tile"])
        rec["predicted_ms"] = round(t, 4)
        # the issue model tables.cpp picks filters with (fitted in round 3 to the
        # measured kernels of seven rule sets, profiles/r03_even_shapes_ab.json):
        # VALU-equivalents per tile = stage-1 VALU + 12 per appending tile + 5
        # per filter-pass entry (first level), ~7 us of a 4 GiB scan each
        valu = {"pair": 91, "pair_xor": 107, "single": 112, "pair_k3": 139, "pair_1bit": 83,
                "pair_mask": 101, "pair_1w": 55}[d]
        rec["issue_model_valu_per_tile"] = round(valu + 12 * tile + 5 * entries * DRAIN_SHARE.get(d, 1.0), 1)
        rec["issue_model_ms"] = round(0.839 + 0.007 * (rec["issue_model_valu_per_tile"] - 122.5), 4)
        out["designs"][d] = rec
        print(d, rec, file=sys.stderr)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
