// gfx950 kernels of the Aho-Corasick atom scanner.
//
// What is computed (reference semantics, libyara/scanner.c:45-176): the
// positions i in (byte_begin, byte_end] of a block at which the AC walk's state
// has a non-empty match list (ac_match_table[state] != 0, scanner.c:98/:144).
//
// How: libyara's trie is at most 4 deep (YR_MAX_ATOM_LENGTH, limits.h:68) and
// its match lists are closed under failure links (ahocorasick.c:254-300), so
// ac_match_table[state_i] != 0 iff some "key" -- a minimal accepting trie
// string, 1..4 bytes -- ends at position i (host flattening: tables.cpp).
// That makes every position independent of every other: no sequential state
// chain, just a window test.
//
//   stage 1 (every byte, LDS):  a pair filter (2^20 bits) over the 3-byte
//             window ending at each byte (internal.h filter_probe_left/right).
//             128 KiB, staged once per workgroup; one ds_read_b64 per two
//             input bytes.  Superset of the keys (config C: 0.39% pass).
//             The main loop only asks "does some position of the lane pass".
//   stage 2 (filter hits):  lanes that pass append their 20 bytes of window
//             context, in position order, to a per-wave LDS ring; a drain
//             (one entry per lane) re-tests the 16 positions, sends each hit
//             through a first-level word filter (L2) and the survivors
//             through bucketed two-choice tables (L2); exact hits are
//             compacted in order (ballot + mbcnt / DPP prefix sums) into the
//             segment's output.
//
// Memory: the input is streamed once, 16 B per lane (1 KiB per wave per step,
// buffer loads), tiles t+1 and t+2 in flight while tile t is filtered
// (t+3 too in the 1-byte-key kernels, one ahead in the plain even-filter
// kernel).  Roofline: HBM
// read bandwidth (1 algorithmic byte per input byte); in practice the kernel
// is VALU-issue bound.
#include <hip/hip_ext.h>

#include "internal.h"

namespace yamd {

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// LDS accesses by 32-bit byte address (the ring, pending list and filter are
// at fixed offsets of the dynamic LDS block, which starts at address 0):
// keeps the address arithmetic in 32-bit VALU ops.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <typename T>
__device__ __forceinline__ T lds_load(uint32_t addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) T*>((uintptr_t)addr);
}
__device__ __forceinline__ void lds_store2(uint32_t addr, uint32_t x, uint32_t y) {
  u32x2 v;
  v.x = x;
  v.y = y;
  *reinterpret_cast<__attribute__((address_space(3))) u32x2*>((uintptr_t)addr) = v;
}

// Inclusive prefix sum over the 64 lanes with DPP (no LDS traffic):
// Hillis-Steele inside each 16-lane row, then row_bcast:15 / row_bcast:31.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return v;
}

// Does some of the 8 bucket slots hold `k`?  (min over slot ^ k == 0: two
// v_min3 and one v_min instead of a compare/select chain.)
__device__ __forceinline__ bool bucket_pair_has(const uint4& a, const uint4& b, uint32_t k) {
  const uint32_t x = min(min(a.x ^ k, a.y ^ k), a.z ^ k);
  const uint32_t y = min(min(a.w ^ k, b.x ^ k), b.y ^ k);
  const uint32_t z = min(min(b.z ^ k, b.w ^ k), min(x, y));
  return z == 0u;
}

// Exact test of one position `pos` of the block: does a key of length
// L <= min(4, pos) equal the last L bytes before it?  w4 = those 4 bytes,
// little endian (oldest lowest; zeros before the block start).  Every load
// (bitmap words, both candidate buckets of each table) is issued before any
// result is used -- one round trip -- and the branches are wave-uniform (the
// key-length set `len_mask`); tables that are not in use are never read.
template <bool kLoads = true>
__device__ __forceinline__ bool exact_check(uint32_t w4, uint64_t pos, const ScanParams& p) {
  const uint32_t* __restrict__ ex = p.exact;
  const uint32_t lm = p.len_mask;
  const uint32_t k1 = w4 >> 24, k2 = w4 >> 16, k3 = (w4 >> 8) | (1u << 24), k4 = w4;
  uint32_t v1 = 0, v2 = 0;
  uint4 a3 = make_uint4(0, 0, 0, 0), b3 = a3, a4 = a3, b4 = a3;
  if (lm & 2u) v1 = ex[kExactBm1 + (k1 >> 5)];
  if (lm & 4u) v2 = ex[kExactBm2 + (k2 >> 5)];
  if constexpr (!kLoads) {   // ablation: the same VALU, no memory round trip
    const uint32_t h3 = bucket_hash1(k3) & p.t3_mask, g3 = bucket_hash2(k3) & p.t3_mask;
    const uint32_t h4 = bucket_hash1(k4) & p.t4_mask, g4 = bucket_hash2(k4) & p.t4_mask;
    a3 = make_uint4(h3, h3 + 1, h3 + 2, h3 + 3);
    b3 = make_uint4(g3, g3 + 1, g3 + 2, g3 + 3);
    a4 = make_uint4(h4, h4 + 1, h4 + 2, h4 + 3);
    b4 = make_uint4(g4, g4 + 1, g4 + 2, g4 + 3);
  } else {
    if (lm & 8u) {
      a3 = *reinterpret_cast<const uint4*>(ex + p.t3_off + (bucket_hash1(k3) & p.t3_mask) * 4);
      b3 = *reinterpret_cast<const uint4*>(ex + p.t3_off + (bucket_hash2(k3) & p.t3_mask) * 4);
    }
    if (lm & 16u) {
      a4 = *reinterpret_cast<const uint4*>(ex + p.t4_off + (bucket_hash1(k4) & p.t4_mask) * 4);
      b4 = *reinterpret_cast<const uint4*>(ex + p.t4_off + (bucket_hash2(k4) & p.t4_mask) * 4);
    }
  }
  bool hit = false;
  if (lm & 2u) hit |= pos >= 1 && ((v1 >> (k1 & 31)) & 1u);
  if (lm & 4u) hit |= pos >= 2 && ((v2 >> (k2 & 31)) & 1u);
  if (lm & 8u) hit |= pos >= 3 && bucket_pair_has(a3, b3, k3);   // k3 != 0: empty slots never match
  if (lm & 16u)
    hit |= pos >= 4 && (k4 == 0 ? (p.exact_flags & kExactZero4) != 0 : bucket_pair_has(a4, b4, k4));
  return hit;
}

// First level (internal.h fl_word): false proves that no key ends at the
// position; true sends it to exact_check.  Rule sets with 1- or 2-byte keys
// skip this level (every hit goes to exact_check).
__device__ __forceinline__ bool first_level_test(uint32_t d, uint32_t w4) {
  return ((d >> fl_bit3(w4)) | (d >> fl_bit4(w4))) & 1u;   // (the masks fold into the shifts)
}
__device__ __forceinline__ bool first_level(uint32_t w4, const ScanParams& p) {
  if (p.len_mask & 6u) return true;
  return first_level_test(p.exact[kExactFl + fl_word(w4)], w4);
}

// Ring entry layout (24 bytes, WaveQueue): the 4 bytes before the lane at
// kEntCtx, the lane's 16 bytes at kEntData, the lane index word at kEntIdx.
// Context first: the 20 bytes are in stream order, so the 4 bytes ending at
// any lane byte are one unaligned LDS dword (gfx950 runs LDS in unaligned
// mode; the compiler emits one ds_read_b32).
constexpr uint32_t kEntCtx = 0u;
constexpr uint32_t kEntData = 4u;
constexpr uint32_t kEntIdx = 20u;
typedef uint32_t u32_una __attribute__((aligned(1)));

// Lane byte j of a ring entry (j = -4 .. -1: the context bytes).
__device__ __forceinline__ uint32_t entry_byte_addr(uint32_t ent, int32_t j) {
  return ent + kEntData + (uint32_t)j;
}

// The 4 bytes ending at lane byte j (0..15) of a ring entry: lane bytes
// j-3 .. j (the context bytes for j < 3).
__device__ __forceinline__ uint32_t window4(uint32_t ent, uint32_t j) {
  return *reinterpret_cast<const __attribute__((address_space(3))) u32_una*>((uintptr_t)(ent + kEntData + j - 3));
}

// Lane byte (0..15) of bit b of a tile hit mask: bit 8n + r <=> byte 4n + r.
__device__ __forceinline__ uint32_t mask_position(uint32_t b) { return ((b >> 3) << 2) | (b & 3u); }

// The 4 bytes around pair j (lane bytes 2j, 2j+1) of a window context S
// (S[0] = the 4 bytes before the lane, S[1..4] its 16 bytes): lane bytes
// 2j-2 .. 2j+1 = context bytes 2j+2 .. 2j+5 (an aligned dword or one alignbyte).
__device__ __forceinline__ uint32_t pair_window(const uint32_t (&S)[6], uint32_t j) {
  const uint32_t o = 2 * j + 2;
  return (o & 3) == 0 ? S[o >> 2] : __builtin_amdgcn_alignbyte(S[(o >> 2) + 1], S[o >> 2], 2);
}

// Per-wave LDS ring of filter hits awaiting the exact check.  One entry (24
// bytes) per (tile, lane) with at least one hit: the lane's 16 bytes, the 4
// bytes before them, and the lane byte offset in the segment / 16.
// Entries are appended in lane order, so ring order is ascending position
// order.  A drain takes the whole ring (one entry per lane), recomputes the
// filter per position from the context, and needs no global load of the
// input, only table probes.
//
// Drains run the first level of the exact check (internal.h fl_word: one
// dword per hit) over 64 entries; the few hits that pass it go, in order, to
// a per-wave pending list of (window, offset) pairs, and the bucket probes
// run once that list holds a wave's worth -- one lane per hit, one round
// trip per 64 hits instead of one per drain.  (Rounds 1-5 deferred the
// first-level loads to the next tile step; with more than one tile in flight
// that costs more than it hides -- DESIGN.md section 5.2.)
struct WaveQueue {
  uint32_t ring;    // LDS address: kQueueCap entries of kQueueEntryWords dwords
  uint32_t count;   // wave-uniform: entries in the ring (a drain takes all of them)
  uint32_t pend;    // LDS address: kWave pairs {w4, segment offset}
  uint32_t pend_n;  // wave-uniform
  uint32_t full;    // wave-uniform (byte-key kernels): candidates of the segment's full
                    // stream flushed so far (verified-only scans leave the dead out)
  uint32_t dacc;    // wave-uniform (kDrainClass): the drains' dead not yet in `full`
  uint32_t kcv;     // per lane (byte-key kernels): the key class records (scan_key_rec)
  uint32_t facc;    // per lane (byte-key kernels, kBkSkipF): OR of the stage-1 filter
                    // and 2-byte-key tests of the tiles queued since the last drain
};

// A key count read where it is tested: an opaque copy, so the compiler does not
// hoist the loop-exit tests out of the tile loop as lane masks (it spilled
// them to VGPR lanes: two v_readlane per key and tile)
__device__ __forceinline__ uint32_t uniform_count(uint32_t n) {
  asm volatile("" : "+s"(n));
  return n;
}

// Kernel variant: the product kernel for rule sets whose 1-byte keys are tested
// byte by byte in stage 1 (byte_keys_any below) instead of in the filter.
constexpr int kModeByteKeys = 20;
// ... and the same with the next lane's first two bytes in each ring entry, for
// the five bytes kept beside certain candidates near a lane's end (tables with
// guard-decided 1-byte keys: ScanParams::kx_next)
constexpr int kModeByteKeysNext = 23;
// Kernel variant: the product kernel for the even-position filter
// (internal.h kFilterEven: tables.cpp picks it for sets of 4-byte keys, and
// for other shapes when its issue model says so).
constexpr int kModeEven = 21;
// ... with the hashed block index (internal.h kFilterEvenHash).
constexpr int kModeEvenHash = 22;
// The byte-key kernels (20, 23) with the even-position filter, plain / hashed.
constexpr int kModeByteKeysEven = 26;
constexpr int kModeByteKeysEvenHash = 27;
constexpr int kModeByteKeysNextEven = 28;
constexpr int kModeByteKeysNextEvenHash = 29;
// Profiling ablations of a product variant V (diagnostic builds): MODE =
// 100 * A + V, A = 1 stage 1 only (the filter and the byte/pair key tests, no
// ring), 2 ring appends whose drains drop the entries, 3 the 1-byte keys
// detected but not appended (the ring holds the filter hits only), 4 the
// 1-byte keys not detected.  Output wrong by construction.
// MODE + kDropModes: the same kernel for verified-only scans (ScanParams::
// drop_dead; byte-key variants only): a separate instance, so that the class
// decisions add nothing to the others.
constexpr int kDropModes = 1000;
template <int MODE>
constexpr bool kDrop = MODE >= kDropModes;
// MODE + kDropBgModes: the drop instance for tables whose key classes include
// backward guards (ScanParams::kd_bguard) -- kept apart because the extra test,
// inlined at every drain site, costs the other tables' drop kernels ~4 %
constexpr int kDropBgModes = 2000;
template <int MODE>
constexpr bool kDropBg = MODE >= kDropBgModes && MODE < 3000;
// MODE + kDropPlanModes: the drop instance for tables whose keys all share one
// forward guard (ScanParams::kp_on, scanner.cpp key_plan): the drain's classes
// in straight-line code (rx's drop kernel 0.94 -> 0.825 ms, gpurun r06v2; with
// the plan's parameters as compile-time constants 0.81, r06x)
constexpr int kDropPlanModes = 3000;
template <int MODE>
constexpr bool kDropPlan = MODE >= kDropPlanModes;
template <int MODE>
constexpr int kBase = MODE % kDropModes >= 100 ? MODE % 100 : MODE % kDropModes;
template <int MODE>
constexpr int kAbl = MODE % kDropModes >= 100 ? (MODE % kDropModes) / 100 : 0;
template <int MODE>
constexpr bool kByteKeys = kBase<MODE> == kModeByteKeys || kBase<MODE> == kModeByteKeysNext ||
                           (kBase<MODE> >= kModeByteKeysEven && kBase<MODE> <= kModeByteKeysNextEvenHash);
// ring entries carry the next lane's first two bytes (ScanParams::kx_next)
template <int MODE>
constexpr bool kNextBytes = kBase<MODE> == kModeByteKeysNext || kBase<MODE> == kModeByteKeysNextEven ||
                            kBase<MODE> == kModeByteKeysNextEvenHash;
template <int MODE>
constexpr bool kEven = kBase<MODE> == kModeEven || kBase<MODE> == kModeEvenHash ||
                       (kBase<MODE> >= kModeByteKeysEven && kBase<MODE> <= kModeByteKeysNextEvenHash);
template <int MODE>
constexpr bool kEvenHash = kBase<MODE> == kModeEvenHash || kBase<MODE> == kModeByteKeysEvenHash ||
                           kBase<MODE> == kModeByteKeysNextEvenHash;
// the stage-1 filter test a kernel variant runs (stage1's MODE argument)
template <int MODE>
constexpr int kStage1Mode = !(kByteKeys<MODE> || MODE == 24 || MODE == 25) ? kBase<MODE>
                            : kEvenHash<MODE>                              ? kModeEvenHash
                            : kEven<MODE>                                  ? kModeEven
                                                                           : 0;
// Profiling ablations of the byte-key kernel (diagnostic builds): 24 = the 1-byte
// keys detected but not appended (the ring holds the filter hits only), 25 =
// not even detected.  Both on a 1-byte-key rule set; output wrong by construction.
template <int MODE>
constexpr bool kByteKeyAblation = MODE == 24 || MODE == 25;
// The ring entry's index word holds the lane's byte offset in the segment
// (else its 16-byte unit index, with the next lane's first two bytes on top)
template <int MODE>
constexpr bool kIdxBytes = !kNextBytes<MODE>;
// A pending entry's offset with this bit set is a certain candidate (its last
// byte is a 1-byte key): no bucket probe.  (Segment offsets are < 2^20.)
// a pending entry becomes the output entry: certain iff its key place is set
constexpr uint32_t kCertainMask = 7u << kOutKeyShift;
static_assert(kSegment <= kOutOffsetMask + 1u, "segment offsets must leave the top bits free");

// b one of the (up to 8, repeated to fill) bytes of x0, x1: zero-byte test
__device__ __forceinline__ bool excluded(uint32_t b, uint32_t x0, uint32_t x1) {
  const uint32_t pv = b * 0x01010101u, a = pv ^ x0, c = pv ^ x1;
  return ((((a - 0x01010101u) & ~a) | ((c - 0x01010101u) & ~c)) & 0x80808080u) != 0u;
}
static_assert(kQueueCap == kWave, "a drain takes the whole ring, one entry per lane");

// The class of a certain candidate (internal.h kClass*), one lane per output
// entry in the compaction.  For a 1-byte key whose state is its own node
// (ScanParams::kd_*, scanner.cpp key_classes) either every call of the list is
// kept whatever the bytes ("kept" keys: plain literals that fit in the atom),
// or the list is one call decided by a guard on the bytes next to the key.  w
// = the five bytes the scan kept for the candidate, the key at byte kp of them
// (-1: just before them; then the table has one 1-byte key): the byte before
// the key (or the scan's test of it, deep) and the guard are decided only if
// every byte they test lies in w and the scanned range.  Pre-verification then never
// reads the input for the candidate.
// A 1-byte key's class parameters (ScanParams::kd_*), one 32-byte record per
// key in LDS: the compaction finds a candidate's key by a zero-byte test on
// the packed key bytes and reads its record (two ds_read_b128) instead of
// selecting every field over the keys.
struct KeyClassRec {
  uint32_t info, m, v, x0, x1, min_pos, bm, bv;
};
// last = the last valid byte of w (4: the five kept bytes; 7: eight bytes the
// compaction read from the input, the key at byte 2).  *more (if given) is
// set when the class is undecided only because a byte it needs lies outside
// w, and eight bytes with the key at byte 2 would hold them.
// rec(k): key k's KeyClassRec (the compaction: an LDS table; the scan kernel:
// selects over its arguments, scan_key_rec).
template <bool kBg = true, typename Rec>
__device__ __forceinline__ uint32_t key_class(const ScanParams& p, Rec rec, uint64_t w,
                                              int32_t kp, bool deep, uint64_t pos, int32_t last = 4,
                                              bool* more = nullptr) {
  if (kp < 0 && p.n_byte_keys != 1) {
    if (more) *more = true;
    return 0;
  }
  const uint32_t key = kp < 0 ? (p.byte_keys & 0xFFu) : (uint32_t)(w >> (8 * kp)) & 0xFFu;
  // the key's index: the lowest zero byte of byte_keys ^ key x 4 among the
  // first n_byte_keys bytes (the lowest flag of the zero-byte test is exact)
  const uint32_t t = p.byte_keys ^ (key * 0x01010101u);
  const uint32_t nmask = p.n_byte_keys >= 4 ? 0x80808080u : 0x80808080u & ((1u << (8 * p.n_byte_keys)) - 1u);
  const uint32_t z = (t - 0x01010101u) & ~t & nmask;
  if (z == 0) return 0;
  const uint32_t kidx = (uint32_t)__builtin_ctz(z) >> 3;
  const KeyClassRec r = rec(kidx);
  const uint32_t info = r.info, m = r.m, v = r.v, x0 = r.x0, x1 = r.x1, min_pos = r.min_pos;
  if (!(info & 1u)) return 0;
  if (info & 2u) {   // the byte before the key among the exclusions: a deeper state
    if (kp >= 1) {
      if (excluded((uint32_t)(w >> (8 * kp - 8)) & 0xFFu, x0, x1)) return 0;
    } else if (!p.kx_deep || deep) {
      if (more && !p.kx_deep) *more = true;   // (the byte before the key is not in w)
      return 0;
    }
  }
  if (info & 4u) return pos >= min_pos ? (kClassKept | kidx << 2) : 0u;
  // Each guard: shift jj tests w bytes s0 + jj + t for the t <= tmax with mask
  // byte t set; a guard that fails proves the call dead, one whose bytes are
  // not all in w (or in the scanned range) decides nothing.
  // The backward guard (info bit 3; min_pos: its first tested byte relative
  // to the key byte (int8) | last tested byte << 12; one position,
  // scanner.cpp key_classes): bytes before the key, all at or after
  // byte_begin.  Computed without branches (the scan kernel inlines this at
  // every drain site, where new exec masks spill its SGPRs) and folded into
  // the forward guard's result at the end.
  bool bdead = false, bmore = false;
  if constexpr (kBg) {
    const bool on = p.kd_bguard != 0u && (info & 8u) != 0u;
    const int32_t g = (int32_t)(int8_t)min_pos, s0 = kp + g;
    const int32_t tmax = (int32_t)((min_pos >> 12) & 3u);
    const bool inrange = (int64_t)pos - 1 + g >= (int64_t)p.byte_begin;
    const bool inw = s0 >= 0 && s0 + tmax <= last;
    const uint32_t x = (uint32_t)(w >> (8 * (uint32_t)(inw ? s0 : 0)));
    bdead = on && inrange && inw && (x & r.bm) != r.bv;
    bmore = on && inrange && !inw && 2 + g >= 0 && 2 + g + tmax <= 7;
  }
  // the forward guard
  const int32_t g = (int32_t)(int8_t)(info >> 8), s0 = kp + g;
  const uint32_t span = (info >> 16) & 15u, tmax = (info >> 20) & 3u;
  // (the scan read nothing past byte_end: a range of a larger block has zeros there)
  const int64_t end = (int64_t)pos + (int8_t)(info >> 24);
  uint32_t res = 0u;
  if (end > (int64_t)p.byte_end) {
    // undecided
  } else if (s0 < 0 || s0 + (int32_t)(span + tmax) > last) {
    if (more && 2 + g >= 0 && 2 + g + (int32_t)(span + tmax) <= 7) *more = true;
  } else {
    bool hit = false;
    // (not vectorized: the vectorizer's masked form of this short loop cost the
    // compaction ~30 spilled SGPRs)
#pragma clang loop vectorize(disable) interleave(disable)
    for (uint32_t jj = 0; jj <= span; ++jj) hit |= ((uint32_t)(w >> (8 * ((uint32_t)s0 + jj))) & m) == v;
    res = hit ? 0u : kClassDead;
  }
  if (more && bmore) *more = true;
  return bdead ? kClassDead : res;
}

// Key k's class record in the scan kernel (k lane-varying): lane 8k + f of
// kcv holds field f of key k (ScanParams::kc, loaded once per kernel), fetched
// by lane permutes -- no memory access, and no SGPRs held for 24 arguments.
// (bg: the table has backward guards -- wave-uniform, so the two permutes for
// them run with every lane active or not at all)
__device__ __forceinline__ KeyClassRec scan_key_rec(uint32_t kcv, uint32_t k, bool bg) {
  const int b = (int)(k * 32u);   // ds_bpermute byte address of lane 8k
  auto f = [&](int i) { return (uint32_t)__builtin_amdgcn_ds_bpermute(b + 4 * i, (int)kcv); };
  KeyClassRec r{f(0), f(1), f(2), f(3), f(4), f(5), 0u, 0u};
  if (bg) {
    r.bm = f(6);
    r.bv = f(7);
  }
  return r;
}

// Bucket-probe every pending hit (one lane each) and append the survivors,
// in order, to the segment's output.  Verified-only scans (p.drop_dead):
// certain candidates of class dead are left out but still counted in the
// segment's full stream (q.full), and seg_x gets each output candidate's
// index in that stream.
template <int MODE>
__device__ __forceinline__ void flush_pending(const ScanParams& p, WaveQueue& q, uint32_t lane,
                                              uint64_t seg_start, uint32_t* out, uint32_t& found) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  bool keep = false, dead = false;
  uint32_t off = 0, xv = 0, dx = 0;
  if constexpr (kByteKeys<MODE>) {
    // confirmed entries need no probe; a flush of nothing else makes no
    // memory round trip at all
    u32x2 e = {0u, 0u};
    if (lane < q.pend_n) e = lds_load<u32x2>(q.pend + 8 * lane);
    const bool conf = (e.y & kCertainMask) != 0u;
    // (a certain entry's bits for key_class with it; a non-certain one's dead
    // count, kDrainClass, in the class byte's place)
    off = conf ? e.y : e.y & kOutOffsetMask;
    const bool probe = lane < q.pend_n && !conf;
    dead = kDrop<MODE> && lane < q.pend_n && conf &&
           ((e.y >> kOutByteShift) & 0xFFu) == kClassDead;
    keep = lane < q.pend_n && conf && !dead;
    if (__ballot(probe) != 0 && probe) keep = exact_check(e.x, seg_start + off + 1, p);
    xv = e.x;
    dx = conf ? e.x : (e.y >> kOutByteShift) & 0xFFu;   // (kDrop: the dead its drain dropped before it)
  } else if (lane < q.pend_n) {
    const u32x2 e = lds_load<u32x2>(q.pend + 8 * lane);
    off = e.y;
    keep = MODE == 12 ? true : exact_check(e.x, seg_start + off + 1, p);   // 12: ablation
  }
  const uint64_t b = __ballot(keep);
  uint64_t bf = b;   // the segment's full stream: kept and dead candidates
  if constexpr (kByteKeys<MODE>) {
    if constexpr (kDrop<MODE>) {
      bf = __ballot(keep || dead);
      xv = q.full + dx +
           __builtin_amdgcn_mbcnt_hi((uint32_t)(bf >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bf, 0u));
    }
  }
  if (keep) {
    const uint32_t idx = found + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    if (idx < p.seg_cap) {
      // (plain stores: non-temporal ones cost the dense sets' kernels 2-4 %, r5h25)
      out[idx] = off;
      if (kByteKeys<MODE> && p.seg_x != nullptr) p.seg_x[(out - p.seg_out) + idx] = xv;
    }
  }
  found += (uint32_t)__popcll(b);
  if constexpr (kByteKeys<MODE>) q.full += (uint32_t)__popcll(bf);
  q.pend_n = 0;
}

// Append hits (bit j of `keep` = lane byte j at segment offset off0 + j) to
// the segment's output in order.  incl = inclusive scan of popcount(keep).
__device__ __forceinline__ void append_hits(const ScanParams& p, uint32_t keep, uint32_t c,
                                            uint32_t incl, uint32_t off0, uint32_t* out,
                                            uint32_t& found) {
  uint32_t idx = found + incl - c;
  while (keep) {
    const uint32_t j = (uint32_t)__builtin_ctz(keep);
    keep &= keep - 1;
    if (idx < p.seg_cap) out[idx] = off0 + j;
    ++idx;
  }
  found += __builtin_amdgcn_readlane(incl, kWave - 1);
}

template <int MODE, bool kAny>
__device__ __forceinline__ uint32_t stage1(const uint32_t (&S)[6], uint32_t lane);

// stage1's per-position mask (bit 8n + r <=> lane byte 4n + r) -> bit j <=> byte j.
__device__ __forceinline__ uint32_t dense_mask(uint32_t h) {
  h &= 0x0F0F0F0Fu;
  h = (h | (h >> 4)) & 0x00FF00FFu;
  return (h | (h >> 8)) & 0xFFFFu;
}

// LDS byte address of the even-position filter block of window x[0..23]
// (internal.h filter_block_even: one v_mul_u32_u24, a shift and a mask).
template <bool kHash>
__device__ __forceinline__ uint32_t even_addr(uint32_t x) {
  if constexpr (kHash) return (__umul24(x, kEvenHashK) >> 15) & (kFilterBytes - 8);
  return (x >> 7) & (kFilterBytes - 8);
}

// Per-position filter hits of a lane under the even-position filter (drains):
// a pass of the window ending at even lane byte 2j makes bytes 2j and 2j + 1
// hits (bit j <=> lane byte j).
template <bool kHash>
__device__ __forceinline__ uint32_t even_mask(const uint32_t (&S)[6]) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < kBytesPerLane / 2; ++j) {
    const uint32_t x = pair_window(S, (uint32_t)j);
    const u32x2 w = lds_load<u32x2>(even_addr<kHash>(x));
    m |= ((w.x >> (x & 31u)) & (w.y >> ((x >> 5) & 31u)) & 1u) << (2 * j);
  }
  return m | (m << 1);
}

// The product kernel for rule sets with up to kMaxByteKeys 1-byte keys: those
// keys are not in the window filter (each would set 65,536 windows of it) but
// tested here, on every byte of the lane, with the zero-byte test of
// x ^ key * 0x01010101 -- one v_xor, one v_add and one v_bitop3 per dword and
// key.  Positions whose last byte is such a key are 1/256 of random input per
// key: they are candidates in their own right, not filter noise.
// Does some byte of the lane's 16 equal a 1-byte key?  (nonzero = yes)
__device__ __forceinline__ uint32_t byte_keys_any(const uint32_t (&S)[6], const ScanParams& p) {
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t k = 0; k < kMaxByteKeys; ++k) {   // 1..kMaxByteKeys keys (wave-uniform)
    if (k != 0 && k >= uniform_count(p.n_byte_keys)) break;
    const uint32_t v = ((p.byte_keys >> (8 * k)) & 0xFFu) * 0x01010101u;   // (k: a constant)
#pragma unroll
    for (int d = 1; d <= 4; ++d) {
      const uint32_t t = S[d] ^ v;
      // acc |= (t - 0x01010101) & ~t: nonzero in bit 7 of some byte iff a byte of t is 0
      asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xba" : "+v"(acc) : "v"(t - 0x01010101u), "v"(t));
    }
  }
  return acc & 0x80808080u;
}

// Even-position filters: the 2-byte keys (p, q) ending at an odd position k + 1
// are the aligned half-words p | q << 8 of the lane (tables.cpp pair_test;
// their (*, *, p) windows would make every byte p a filter pass).  Same
// zero test as byte_keys_any, per 16-bit half: nonzero iff some half matches.
__device__ __forceinline__ uint32_t pair_keys_any(const uint32_t (&S)[6], const ScanParams& p) {
  uint32_t acc = 0;
#pragma unroll
  for (uint32_t k = 0; k < kMaxPairKeys; ++k) {   // 1..kMaxPairKeys keys (wave-uniform)
    if (k != 0 && k >= uniform_count(p.n_pair_keys)) break;
    const uint32_t v = ((p.pair_keys[k >> 1] >> (16 * (k & 1u))) & 0xFFFFu) * 0x00010001u;
#pragma unroll
    for (int d = 1; d <= 4; ++d) {
      const uint32_t t = S[d] ^ v;
      asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xba" : "+v"(acc) : "v"(t - 0x00010001u), "v"(t));
    }
  }
  return acc & 0x80008000u;
}

// Per-position form (drains): bit j (odd) <=> lane bytes j - 1, j are a 2-byte key.
__device__ __forceinline__ uint32_t pair_keys_mask(const uint32_t (&S)[6], const ScanParams& p) {
  uint32_t z[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t k = 0; k < kMaxPairKeys; ++k) {
    if (k != 0 && k >= uniform_count(p.n_pair_keys)) break;
    const uint32_t v = ((p.pair_keys[k >> 1] >> (16 * (k & 1u))) & 0xFFFFu) * 0x00010001u;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t t = S[1 + d] ^ v;
      // bit 15 / 31 set iff that half is 0 (exact: no carry between the halves)
      asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xab"
          : "+v"(z[d]) : "v"((t & 0x7FFF7FFFu) + 0x7FFF7FFFu), "v"(t));
    }
  }
  // flags in bytes 1 and 3 of each dword: the byte-key gather puts them at bits
  // 4d + 1 and 4d + 3
  const uint32_t lo = __builtin_amdgcn_udot4(z[1] & 0x80008000u, 0x80402010u,
                                             __builtin_amdgcn_udot4(z[0] & 0x80008000u, 0x08040201u, 0u, false),
                                             false);
  const uint32_t hi = __builtin_amdgcn_udot4(z[3] & 0x80008000u, 0x80402010u,
                                             __builtin_amdgcn_udot4(z[2] & 0x80008000u, 0x08040201u, 0u, false),
                                             false);
  return (lo >> 7) | (hi << 1);
}

// Per-position form (drains): bit j <=> lane byte j equals a 1-byte key.
// Exact zero-byte flags (bit 7 of each byte of z_d) OR-ed over the keys, then
// each dword's four flags gathered by one v_dot4_u32_u8 against the place
// values 2^r (two dwords per chain: bytes of 0x80 times 1..128 stay below 2^16).
// (first: if given and the table has more than one key, the first key's own
// mask -- the drain classes' per-key split)
__device__ __forceinline__ uint32_t byte_keys_mask(const uint32_t (&S)[6], const ScanParams& p,
                                                   uint32_t* first = nullptr) {
  uint32_t z[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (uint32_t k = 0; k < kMaxByteKeys; ++k) {
    if (k != 0 && k >= uniform_count(p.n_byte_keys)) break;
    if (k == 1 && first != nullptr) {
      const uint32_t lo = __builtin_amdgcn_udot4(z[1] & 0x80808080u, 0x80402010u,
                                                 __builtin_amdgcn_udot4(z[0] & 0x80808080u, 0x08040201u, 0u, false),
                                                 false);
      const uint32_t hi = __builtin_amdgcn_udot4(z[3] & 0x80808080u, 0x80402010u,
                                                 __builtin_amdgcn_udot4(z[2] & 0x80808080u, 0x08040201u, 0u, false),
                                                 false);
      *first = (lo >> 7) | (hi << 1);
    }
    const uint32_t v = ((p.byte_keys >> (8 * k)) & 0xFFu) * 0x01010101u;   // (k: a constant)
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t t = S[1 + d] ^ v;
      // z |= ~(((t & 0x7F7F7F7F) + 0x7F7F7F7F) | t): bit 7 of a byte set iff it is 0
      asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xab"
          : "+v"(z[d]) : "v"((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu), "v"(t));
    }
  }
  const uint32_t lo = __builtin_amdgcn_udot4(z[1] & 0x80808080u, 0x80402010u,
                                             __builtin_amdgcn_udot4(z[0] & 0x80808080u, 0x08040201u, 0u, false),
                                             false);
  const uint32_t hi = __builtin_amdgcn_udot4(z[3] & 0x80808080u, 0x80402010u,
                                             __builtin_amdgcn_udot4(z[2] & 0x80808080u, 0x08040201u, 0u, false),
                                             false);
  return (lo >> 7) | (hi << 1);   // (x 128: bytes 0..7 in bits 7..14, 8..15 in 15..22)
}


// Wave priorities: the streaming waves (stage 1, the appends) run at
// s_setprio 1, a wave inside a drain at 0,
// so the arbiter issues the waves that keep the input stream going first while
// a drain's long VALU burst fills the gaps (C -1.3 to -2.5 %, rx -2 %, B/E
// within noise: profiles/r03_copy_prio_ab.json, r03_prio_ab.json,
// r03_prio3_ab.json).
//
// Branch-weight hints on the tile step's rare path (an append that fills the
// ring): the common
// path falls through with no taken branch (C -1.2 %).
#define YAMD_EXPECT(c, v) __builtin_expect((c), (v))
// Tiles in flight ahead of the one in the tile step (scan_segment).  Two
// instead of one: C -4 %, rx -8 %, E -2 % (profiles/r06_prefetch_ab/) --
// once the drains check the first level themselves instead of deferring its
// loads to the next tile step (rounds 1-5): vmcnt retires in issue order, so a
// step that consumed the words loaded at the end of the previous one also
// waited for the tile issued after them, and two tiles in flight measured no
// faster with the deferral (round 2; r07c).  The deferral itself was worth
// nothing by then (C equal without it, r07c) and is gone; the plain
// even-position filter kernel without 1-byte keys (B) stays at one tile ahead
// (two: +2 %).  (YAMD_PF / YAMD_PF_EVEN / YAMD_PF_BK / YAMD_NO_PRIO:
// variant builds; without the wave priorities C is 2-4 %
// slower, rx and fuzz3 2-3 %, r07k.)
#ifndef YAMD_PF
#define YAMD_PF 2
#endif
#ifndef YAMD_PF_EVEN
#define YAMD_PF_EVEN 1
#endif
#ifndef YAMD_PF_BK
#define YAMD_PF_BK 3   // (the 1-byte-key kernels: three ahead, rx -1.5-2 %, fuzz3 -1.3 % against two, r07k)
#endif
#ifndef YAMD_NO_PRIO
#define YAMD_NO_PRIO 0
#endif
template <int MODE>
constexpr uint32_t kPf = kBase<MODE> == kModeEven ? YAMD_PF_EVEN : kByteKeys<MODE> ? YAMD_PF_BK : YAMD_PF;
// Byte-key drains re-test the filter and the 2-byte keys only when some tile
// queued since the last drain passed them in stage 1 (a per-lane OR, one
// v_or per tile, balloted once per drain): rx's drains skip ~90 of their ~140
// VALU nearly always (its ring holds 1-byte-key hits).
template <int MODE>
constexpr bool kBkSkipF = kByteKeys<MODE> && kAbl<MODE> == 0;

// The output entry of a certain candidate (its last byte a 1-byte key) at lane
// byte j of ring entry ent: it needs no window for the exact check, so the scan
// keeps five bytes next to it for key_class instead, lane bytes e - 3 .. e + 1,
// the key at place j + 3 - e of them: e = min(j + kx_end, 16), where bytes 16
// and 17 are the next lane's first two (ring entry bytes 22, 23; not in the
// entry of a tile's last lane: e <= 14 there).  y: in, the segment offset;
// out, with the key place, the fifth byte and the deep flag.
template <int MODE>
__device__ __forceinline__ void certain_entry(const ScanParams& p, uint32_t ent, uint32_t j,
                                              uint32_t& x, uint32_t& y) {
  const uint32_t li = lds_load<uint32_t>(ent + kEntIdx);
  const uint32_t e =
      min(j + p.kx_end, kNextBytes<MODE> && (li & (kWave - 1)) != kWave - 1 ? 16u : 14u);
  uint32_t b5;
  if (e <= 14u) {
    x = window4(ent, e);
    b5 = lds_load<uint8_t>(entry_byte_addr(ent, (int32_t)e + 1));
  } else {   // lane bytes 12..17
    const uint64_t w6 = lds_load<uint32_t>(ent + kEntData + 12) | (uint64_t)(li >> 16) << 32;
    x = (uint32_t)(w6 >> (8 * (e - 15u)));
    b5 = (uint32_t)(w6 >> (8 * (e - 11u))) & 0xFFu;
  }
  y |= b5 << kOutByteShift | (j + 5 - e) << kOutKeyShift;
  if (p.kx_deep != 0u) {   // (the byte before the key; j = 0: the last context byte)
    const uint32_t b = lds_load<uint8_t>(entry_byte_addr(ent, (int32_t)j - 1));
    if (excluded(b, p.kd_x0[0], p.kd_x1[0])) y |= kOutDeep;
  }
}

// Byte-key kernels: a drain's hits go to the pending list
// RAW (the ring entry, the lane byte, a certain flag: one LDS store per hit in
// the per-lane loop, whose trip count is the wave's largest per-lane hit
// count), and the window / certain-candidate bytes are then computed for the
// entries [from, pend_n) one lane each, while the ring entries are still
// valid.  One-process A/B in both variant orders (profiles/r04_ab_inproc.json,
// gpurun h7, h8): rx -1.5 %, short -2.5 to -3.3 %, fuzz0 / fuzz3 within 1 %.
// (A first single-order call had it 5 % slower: a per-process placement
// offset, DESIGN.md section 5 "Measurement method".)
template <int MODE>
constexpr bool kBkResolve = kByteKeys<MODE>;

// A raw pending entry's first word: the ring entry's LDS address (< 2^18), the
// lane byte j, and -- drain classes, below -- how many candidates of the same
// drain before it were dropped as dead (< 1024: 64 entries of 16 bytes).
static_assert(kFilterBytes + kQueueBytes + kWavesPerWG * kWave * 8 <= (1u << 18),
              "raw pending entries hold LDS addresses in 18 bits");
__device__ __forceinline__ uint32_t raw_x(uint32_t ent, uint32_t j, uint32_t d) {
  return ent | j << 18 | d << 22;
}
__device__ __forceinline__ uint32_t raw_ent(uint32_t x) { return x & 0x3FFFFu; }
__device__ __forceinline__ uint32_t raw_j(uint32_t x) { return (x >> 18) & 15u; }
__device__ __forceinline__ uint32_t raw_dead(uint32_t x) { return x >> 22; }

// Drain classes (verified-only scans, the drop instances): the drain decides
// the classes of its entries' certain candidates itself, sixteen positions at
// a time, from the bytes the entry holds -- key_class's decision in byte-wise
// SWAR form.  Dead candidates never reach the pending list (only counted, for
// the full stream's indices); kept / undecided ones whose bytes all lie in the
// entry go there resolved, so the drain needs no resolve_pending for them.  The
// rest (a guard's bytes past the entry, a block edge) stay raw for
// scan_class_entry.  (The upper bound, every certain candidate dropped in the
// drain: rx's kernel 1.028 -> 0.769 ms, fuzz0's 1.043 -> 0.844, gpurun r5h41.)
#ifndef YAMD_DRAIN_CLASS
#define YAMD_DRAIN_CLASS 1
#endif
template <int MODE>
constexpr bool kDrainClass = kDrop<MODE> && YAMD_DRAIN_CLASS;

// bit 7 of each byte set iff that byte of t is 0 (exact for every byte)
__device__ __forceinline__ uint32_t zero_flags(uint32_t t) {
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
// Bit-7 flags of lane bytes 4d .. 4d + 3 in z[d] -> bit j <=> lane byte j
// (byte_keys_mask's v_dot4 gather).
__device__ __forceinline__ uint32_t gather16(const uint32_t (&z)[4]) {
  const uint32_t lo = __builtin_amdgcn_udot4(z[1], 0x80402010u, __builtin_amdgcn_udot4(z[0], 0x08040201u, 0u, false),
                                             false);
  const uint32_t hi = __builtin_amdgcn_udot4(z[3], 0x80402010u, __builtin_amdgcn_udot4(z[2], 0x08040201u, 0u, false),
                                             false);
  return (lo >> 7) | (hi << 1);
}
// Byte tests over a drain entry's 24 bytes, lane bytes -4 .. 19 (the context
// dword, the lane's sixteen, the next lane's dword -- its first two bytes, or
// zeros): bit b + 4 of the result <=> (byte b & mt) == vt, for one mask / value
// byte pair and all 24 bytes at once (six zero-byte tests and a v_dot4
// gather).  A test at offset o from each of the sixteen positions is then a
// shift: bit j of (T >> (o + 4)).  (Shifting bytes instead -- a select of
// dwords per offset and v_alignbyte -- cost as much as the drain saved.)
__device__ __forceinline__ uint32_t byte_test24(const uint32_t (&E)[6], uint32_t mt, uint32_t vt) {
  const uint32_t M = mt * 0x01010101u, V = vt * 0x01010101u;
  uint32_t z0, z1, z2, z3, z4, z5;
  if (mt == 0xFFu) {   // (wave-uniform: no mask, one instruction less per dword)
    z0 = zero_flags(E[0] ^ V), z1 = zero_flags(E[1] ^ V), z2 = zero_flags(E[2] ^ V);
    z3 = zero_flags(E[3] ^ V), z4 = zero_flags(E[4] ^ V), z5 = zero_flags(E[5] ^ V);
  } else {
    z0 = zero_flags((E[0] & M) ^ V), z1 = zero_flags((E[1] & M) ^ V), z2 = zero_flags((E[2] & M) ^ V);
    z3 = zero_flags((E[3] & M) ^ V), z4 = zero_flags((E[4] & M) ^ V), z5 = zero_flags((E[5] & M) ^ V);
  }
  const uint32_t lo = __builtin_amdgcn_udot4(z1, 0x80402010u, __builtin_amdgcn_udot4(z0, 0x08040201u, 0u, false),
                                             false);
  const uint32_t mid = __builtin_amdgcn_udot4(z3, 0x80402010u, __builtin_amdgcn_udot4(z2, 0x08040201u, 0u, false),
                                              false);
  const uint32_t hi = __builtin_amdgcn_udot4(z5, 0x80402010u, __builtin_amdgcn_udot4(z4, 0x08040201u, 0u, false),
                                             false);
  return (lo >> 7) | (mid << 1) | (hi << 9);
}

// bit b + 4 <=> lane byte b (-4 .. 15) is one of the bytes of x0, x1 (the
// exclusions: the first one repeated to fill), OR-ed before one gather
__device__ __forceinline__ uint32_t byte_set_test20(const uint32_t (&E)[6], uint32_t x0, uint32_t x1) {
  uint32_t z0 = 0u, z1 = 0u, z2 = 0u, z3 = 0u, z4 = 0u;
  auto acc = [](uint32_t& z, uint32_t t) { z |= ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t); };
#pragma unroll 1
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t b = ((i < 4 ? x0 : x1) >> (8 * (i & 3u))) & 0xFFu;
    if (i != 0 && b == (x0 & 0xFFu)) break;
    const uint32_t V = b * 0x01010101u;
    acc(z0, E[0] ^ V);
    acc(z1, E[1] ^ V);
    acc(z2, E[2] ^ V);
    acc(z3, E[3] ^ V);
    acc(z4, E[4] ^ V);
  }
  const uint32_t k = 0x80808080u;
  const uint32_t lo = __builtin_amdgcn_udot4(z1 & k, 0x80402010u, __builtin_amdgcn_udot4(z0 & k, 0x08040201u, 0u, false),
                                             false);
  const uint32_t mid = __builtin_amdgcn_udot4(z3 & k, 0x80402010u,
                                              __builtin_amdgcn_udot4(z2 & k, 0x08040201u, 0u, false), false);
  const uint32_t hi = __builtin_amdgcn_udot4(z4 & k, 0x08040201u, 0u, false);
  return (lo >> 7) | (mid << 1) | (hi << 9);
}

// One drain entry's certain candidates (m: its 1-byte-key hits, tail-masked;
// first: those of the first key, with two or more keys; pos0: the block
// position of lane byte 0): dead = decided dead;
// res = decided and kept (class kept if in `kept`, the key index's bits in kid
// -- bit j: bit 0, bit 16 + j: bit 1 --, kClassFetch if in `fetch`, else class
// 0).  key_class (kp = 2) for
// sixteen positions at a time, on the same records (kcv, read by v_readlane:
// the key loop is wave-uniform); what it cannot decide is in neither mask.
struct DrainClasses {
  uint32_t dead, res, kept, kid, fetch;
};
template <int MODE>
__device__ __forceinline__ DrainClasses drain_classes(const ScanParams& p, uint32_t kcv, const uint32_t (&S)[6],
                                                      uint32_t eidx, uint32_t m, uint32_t first, uint64_t pos0) {
  DrainClasses c{0u, 0u, 0u, 0u, 0u};
  // the next lane's first two bytes: kept by the kernels with kNextBytes,
  // except in a tile's last lane
  const bool nx = kNextBytes<MODE> && (eidx & (kWave - 1)) != kWave - 1;
  const uint32_t E[6] = {S[0], S[1], S[2], S[3], S[4], nx ? eidx >> 16 : 0u};
  const int32_t last = nx ? 17 : 15;   // last lane byte held
  if constexpr (kDropPlan<MODE>) {
    // one forward guard -- one full-byte compare -- for every key (scanner.cpp
    // key_plan): the per-key loop below in one pass over all of m, its three
    // parameters read from the records' VGPR (kc[kKcPlan..] sit in lanes 32..34
    // of kcv: no memory access in the drain, no SGPRs held across the tile
    // loop), no per-key split of m, no loop over tested bytes, no test-reuse branch
    (void)first;
    const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)kcv, (int)kKcPlan);
    const uint32_t V = (uint32_t)__builtin_amdgcn_readlane((int)kcv, (int)kKcPlan + 1);
    const uint32_t sh = (uint32_t)__builtin_amdgcn_readlane((int)kcv, (int)kKcPlan + 2);
    const int32_t rs = (int32_t)(int8_t)(info >> 8);
    const uint32_t span = (info >> 16) & 15u, tmax = (info >> 20) & 3u;
    const int64_t endo = (int8_t)(info >> 24);
    // the one full-byte compare, on all 24 bytes (byte_test24's unmasked form)
    const uint32_t z0 = zero_flags(E[0] ^ V), z1 = zero_flags(E[1] ^ V), z2 = zero_flags(E[2] ^ V);
    const uint32_t z3 = zero_flags(E[3] ^ V), z4 = zero_flags(E[4] ^ V), z5 = zero_flags(E[5] ^ V);
    const uint32_t lo = __builtin_amdgcn_udot4(z1, 0x80402010u, __builtin_amdgcn_udot4(z0, 0x08040201u, 0u, false),
                                               false);
    const uint32_t mid = __builtin_amdgcn_udot4(z3, 0x80402010u, __builtin_amdgcn_udot4(z2, 0x08040201u, 0u, false),
                                                false);
    const uint32_t hi = __builtin_amdgcn_udot4(z5, 0x80402010u, __builtin_amdgcn_udot4(z4, 0x08040201u, 0u, false),
                                               false);
    const uint32_t A = ((lo >> 7) | (mid << 1) | (hi << 9)) >> sh;
    uint32_t fp = A;
#pragma unroll 1
    for (uint32_t jj = 1; jj <= span; ++jj) fp |= A >> jj;
    const int32_t lim = last - (rs + (int32_t)(span + tmax));
    const uint32_t avail = lim < 0 ? 0u : lim >= 15 ? 0xFFFFu : (2u << lim) - 1u;
    const uint32_t rng = (int64_t)pos0 + 16 + endo > (int64_t)p.byte_end ? 0u : 0xFFFFu;
    c.dead = m & ~fp & avail & rng;
    c.res = m & rng & ~c.dead;
    c.fetch = m & rng & ~avail & ~c.dead;
    return c;
  }
  uint32_t seen = 0u;                  // the keys' candidates so far
  // one test remembered across keys and guards (rx: both keys test the byte
  // after them against 0xC3)
  uint32_t cm = 0u, cv = 0u, ct = 0u;
  auto test = [&](uint32_t mt, uint32_t vt) {
    // (readfirstlane: provably uniform, so the reuse test is a scalar branch)
    mt = __builtin_amdgcn_readfirstlane(mt);
    vt = __builtin_amdgcn_readfirstlane(vt);
    if (mt != __builtin_amdgcn_readfirstlane(cm) || vt != __builtin_amdgcn_readfirstlane(cv)) {
      cm = mt;
      cv = vt;
      ct = byte_test24(E, mt, vt);
    }
    return ct;
  };
  // (rolled loops, over the keys and the tested bytes: unrolled, with the
  // test's reuse branch, the drop kernels' code grew four-fold)
  const uint32_t nk = uniform_count(p.n_byte_keys);
#pragma unroll 1
  for (uint32_t k = 0; k < nk; ++k) {
    auto f = [&](uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)kcv, (int)(8 * k + i)); };
    const uint32_t key = (p.byte_keys >> (8 * k)) & 0xFFu;
    uint32_t K;   // this key's candidates (the first: byte_keys_mask's; the last: the rest of m)
    if (k + 1 == nk) {
      K = m & ~seen;
    } else if (k == 0) {
      K = first;
      seen = K;
    } else {
      uint32_t z[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) z[d] = zero_flags(S[1 + d] ^ key * 0x01010101u);
      K = gather16(z) & m;
      seen |= K;
    }
    const uint32_t info = f(0);
    if (!(info & 1u)) {   // no class: 0
      c.res |= K;
      continue;
    }
    uint32_t Kn = K;
    if (info & 2u) {   // the byte before the key among the exclusions (a deeper trie state): class 0
      const uint32_t X = byte_set_test20(E, f(3), f(4)) >> 3 & K;
      c.res |= X;
      Kn = K & ~X;
    }
    if (info & 4u) {   // kept, from min_pos on (pos >= min_pos for every j of the entry)
      if (pos0 + 1 >= (uint64_t)f(5)) {
        c.res |= Kn;
        c.kept |= Kn;
        c.kid |= ((k & 1u) ? Kn : 0u) | ((k & 2u) ? Kn << 16 : 0u);
      }
      continue;
    }
    // the forward guard: dead iff no shift jj <= span passes; decided where its
    // bytes lie in the entry (avail) and end <= byte_end for every j of the
    // entry (rng)
    const uint32_t gm = f(1), gv = f(2);
    const int32_t rs = (int32_t)(int8_t)(info >> 8);
    const uint32_t span = (info >> 16) & 15u, tmax = (info >> 20) & 3u;
    const int64_t endo = (int8_t)(info >> 24);
    // A: bit j <=> position j passes every tested byte at shift 0 (rs + t + 4
    // >= 0: rs >= -1, fits() in scanner.cpp); shift jj is A >> jj
    uint32_t A = ~0u;
#pragma unroll 1
    for (uint32_t t = 0; t <= tmax; ++t) {
      const uint32_t mt = (gm >> (8 * t)) & 0xFFu, vt = (gv >> (8 * t)) & 0xFFu;
      // (a test of the key byte itself holds at every candidate)
      if (mt == 0u || (rs + (int32_t)t == 0 && mt == 0xFFu && vt == key)) continue;
      A &= test(mt, vt) >> (uint32_t)(rs + (int32_t)t + 4);
    }
    uint32_t fp = 0u;
#pragma unroll 1
    for (uint32_t jj = 0; jj <= span; ++jj) fp |= A >> jj;
    const int32_t lim = last - (rs + (int32_t)(span + tmax));   // held: j <= lim
    const uint32_t avail = lim < 0 ? 0u : lim >= 15 ? 0xFFFFu : (2u << lim) - 1u;
    const uint32_t rng = (int64_t)pos0 + 16 + endo > (int64_t)p.byte_end ? 0u : 0xFFFFu;
    uint32_t dead = Kn & ~fp & avail & rng;
    // the backward guard (one position, its bytes before the key: always held)
    if (p.kd_bguard != 0u && (info & 8u)) {
      const uint32_t mp = f(5), bm = f(6), bv = f(7);
      const int32_t g = (int32_t)(int8_t)mp;
      const uint32_t btmax = (mp >> 12) & 3u;
      if ((int64_t)pos0 + g >= (int64_t)p.byte_begin) {
        uint32_t a = ~0u;
#pragma unroll 1
        for (uint32_t t = 0; t <= btmax; ++t) {
          const uint32_t mt = (bm >> (8 * t)) & 0xFFu, vt = (bv >> (8 * t)) & 0xFFu;
          if (mt == 0u) continue;
          a &= test(mt, vt) >> (uint32_t)(g + (int32_t)t + 4);
        }
        dead |= Kn & ~a;
      }
    }
    c.dead |= dead;
    // alive: class 0 where the guard's bytes were held, else (within byte_end)
    // kClassFetch -- key_class's "more": the compaction's eight bytes around
    // the key hold them (fits(): rs >= -1, rs + span + tmax <= 5)
    c.res |= Kn & rng & ~dead;
    c.fetch |= Kn & rng & ~avail & ~dead;
  }
  return c;
}

// Verified-only scans: the class of the certain candidate at lane byte j of
// ring entry ent (key_class over the eight lane bytes j - 2 .. j + 5, the key at
// byte 2 -- lane bytes 16, 17 are the next lane's first two, kept in the
// index word's top half by the kernels with kNextBytes), as an output entry:
// the segment offset, the class code (kClassFetch: undecided only because
// some byte lies past what the entry holds) and key place 7.
template <int MODE>
__device__ __forceinline__ uint32_t scan_class_entry(const ScanParams& p, uint32_t kcv_, uint32_t ent,
                                                     uint32_t j, uint32_t off, uint64_t seg_start) {
  const uint32_t li = lds_load<uint32_t>(ent + kEntIdx);
  // lane bytes j - 2 .. j + 5 = entry bytes j + 2 .. j + 9 (past lane byte 15:
  // the index word, replaced below)
  const auto una = [](uint32_t a) {
    return *reinterpret_cast<const __attribute__((address_space(3))) u32_una*>((uintptr_t)a);
  };
  uint64_t w = una(ent + kEntData + j - 2) | (uint64_t)una(ent + kEntData + j + 2) << 32;
  int32_t have = 18 - (int32_t)j;   // lane bytes j - 2 .. 15
  if (have < 8) {
    w &= (1ull << (8 * have)) - 1ull;
    if (kNextBytes<MODE> && (li & (kWave - 1)) != kWave - 1) {
      w |= (uint64_t)(li >> 16) << (8 * have);
      have += 2;
    }
  }
  // the key's record, fetched by lane permutes before any divergent branch (a
  // permute reading a lane outside EXEC would not see its record): key_class's
  // own index computation, branch-free
  const uint32_t key = (uint32_t)(w >> 16) & 0xFFu;
  const uint32_t t = p.byte_keys ^ (key * 0x01010101u);
  const uint32_t z = (t - 0x01010101u) & ~t & 0x80808080u;
  constexpr bool kBg = kDropBg<MODE>;
  const KeyClassRec r = scan_key_rec(kcv_, (uint32_t)__builtin_ctz(z | 0x80000000u) >> 3, kBg);
  bool more = false;
  const uint32_t cls = key_class<kBg>(p, [r](uint32_t) { return r; }, w, 2, false, seg_start + off + 1,
                                 min(have, 8) - 1, &more);
  return off | (cls == 0u && more ? kClassFetch : cls) << kOutByteShift |
         kOutPlaceScanClass << kOutKeyShift;
}

template <int MODE>
__device__ __forceinline__ void resolve_pending(const ScanParams& p, WaveQueue& q, uint32_t lane,
                                                uint32_t from, uint64_t seg_start) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const bool act = lane >= from && lane < q.pend_n;
  if constexpr (kDrop<MODE>) {
    // every lane (EXEC is full here: the drains run on wave-uniform paths) --
    // scan_class_entry's permutes need their source lanes active; an idle
    // lane computes on pending entry `from`'s (raw) entry and stores nothing
    const u32x2 e = lds_load<u32x2>(q.pend + 8 * (act ? lane : from));
    const uint32_t ent = raw_ent(e.x), j = raw_j(e.x);
    const uint32_t yc = scan_class_entry<MODE>(p, q.kcv, ent, j, e.y & 0x7FFFFFFFu, seg_start);
    // (entries the drain resolved itself, kDrainClass, stay as they are; an
    // idle lane's entry may be one of them: its reads stay inside the LDS)
    if (act && (e.y & kCertainMask) == 0u) {
      uint32_t x = raw_dead(e.x), y = yc;
      if (!(e.y >> 31)) {   // non-certain: the dead count (< 256) in the class byte's place
        x = window4(ent, j);
        y = e.y | raw_dead(e.x) << kOutByteShift;
      }
      lds_store2(q.pend + 8 * lane, x, y);
    }
    return;
  }
  if (act) {
    const u32x2 e = lds_load<u32x2>(q.pend + 8 * lane);
    const uint32_t ent = raw_ent(e.x), j = raw_j(e.x);
    uint32_t x = 0u, y = e.y & 0x7FFFFFFFu;
    if (e.y >> 31) certain_entry<MODE>(p, ent, j, x, y);
    else x = window4(ent, j);
    lds_store2(q.pend + 8 * lane, x, y);
  }
}

// First-level check of the hits of up to 64 ring entries; survivors go to
// the pending list.  kInLoop: a drain inside the tile loop (a full ring),
// whose entries all lie in full tiles.
template <int MODE, bool kInLoop = false>
__device__ __forceinline__ void drain(const ScanParams& p, WaveQueue& q, uint32_t lane,
                                      uint64_t seg_start, uint32_t seg_len, uint32_t* out,
                                      uint32_t& found) {
  const uint32_t n = q.count;   // <= kQueueCap = kWave
  q.count = 0;
  bool need_f = true;   // (kBkSkipF: some queued tile passed the filter / a 2-byte key)
  if constexpr (kBkSkipF<MODE>) {
    need_f = __ballot(q.facc != 0u) != 0;
    q.facc = 0u;
  }
  if constexpr (MODE == 7 || MODE == 8 || MODE == 13 || kAbl<MODE> == 2) return;   // ablations: entries dropped
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t maybe = 0, off0 = 0, m = 0;   // m: bit j = lane byte j passes the filter
  uint32_t kmask = 0;                    // bit j = lane byte j is a 1-byte key (certain)
  DrainClasses dc{0u, 0u, 0u, 0u, 0u};   // (kDrainClass)
  uint32_t kfirst = 0u;                  // (kDrainClass, tables with 2+ keys: bits of the first one)
  const uint32_t ent = q.ring + lane * (kQueueEntryWords * 4);
  uint32_t S[6] = {0u, 0u, 0u, 0u, 0u, 0u}, eidx = 0u;
  if (lane < n) {
    // the entry's 16 positions again, now with a per-position result: the
    // same pair tests as stage 1 over the entry's window context
    const u32x2 e01 = lds_load<u32x2>(ent);
    const u32x2 e23 = lds_load<u32x2>(ent + 8);
    const u32x2 e45 = lds_load<u32x2>(ent + 16);
    S[0] = e01.x;
    S[1] = e01.y;
    S[2] = e23.x;
    S[3] = e23.y;
    S[4] = e45.x;
    eidx = e45.y;
    off0 = kIdxBytes<MODE> ? eidx : (eidx & 0xFFFFu) * kBytesPerLane;
    if (need_f) {
      if constexpr (kEven<MODE>) {
        m = even_mask<kEvenHash<MODE>>(S);
        if (p.n_pair_keys != 0) m |= pair_keys_mask(S, p);
      } else {
        m = dense_mask(stage1<0, false>(S, lane));
      }
    }
    if constexpr (kByteKeys<MODE>) {
      kmask = byte_keys_mask(S, p, kDrainClass<MODE> ? &kfirst : nullptr);
      m |= kmask;
    }
    // the segment's partial last tile (its entries are appended after the main
    // loop's last drain, so only the final drain can hold them)
    if (!kInLoop && off0 + kBytesPerLane > seg_len) {
      const uint32_t lim = off0 >= seg_len ? 0u : seg_len - off0;
      m &= lim >= 16u ? 0xFFFFu : (1u << lim) - 1u;
    }
  }
  // (kDrainClass: nc = some lane holds a filter hit, a non-certain entry)
  const bool nc = kDrainClass<MODE> && __ballot((m & ~kmask) != 0u) != 0;
  // (every lane, in uniform control flow -- lanes without an entry have no
  // hits: the class code's wave-uniform values stay in SGPRs)
  if constexpr (kDrainClass<MODE>)
    dc = drain_classes<MODE>(p, q.kcv, S, eidx, m & kmask, kfirst & m, seg_start + off0);
  if ((MODE == 0 || kByteKeys<MODE> || kByteKeyAblation<MODE>) && (p.len_mask & 6u) != 0u) {
    maybe = m;   // 1-/2-byte keys: no first level, every hit goes to the buckets
  } else {
    while (m) {
      const uint32_t j = (uint32_t)__builtin_ctz(m);
      m &= m - 1;
      bool hit;
      if constexpr (MODE == 1) {
        hit = ((off0 + j) & 1023u) == 7u;
      } else if constexpr (MODE == 9) {   // one L2 dword per hit, minimal VALU
        hit = (p.exact[kExactBm2 + (window4(ent, j) & 2047u)] >> 31) != 0u;
      } else if constexpr (MODE == 10) {
        hit = exact_check<false>(window4(ent, j), seg_start + off0 + j + 1, p);
      } else {
        hit = first_level(window4(ent, j), p);
      }
      maybe |= (uint32_t)hit << j;
    }
  }
  // (kDrainClass: the dead are counted, per lane dd = how many, dbase = how
  // many in the lanes below, dtotal = in the drain -- one scan for both sums)
  uint32_t dd = 0u, dbase = 0u, dtotal = 0u;
  const uint32_t maybe0 = maybe;
  if constexpr (kDrainClass<MODE>) {
    maybe &= ~dc.dead;
    dd = __popc(dc.dead);
  }
  uint32_t c = __popc(maybe);
  uint32_t incl;
  if constexpr (kDrainClass<MODE>) {
    const uint32_t both = wave_inclusive_scan(c | dd << 16);   // (sums <= 1024)
    incl = both & 0xFFFFu;
    dbase = (both >> 16) - dd;
    dtotal = __builtin_amdgcn_readlane(both, kWave - 1) >> 16;
    if (nc && dtotal >= 256u) {
      // a non-certain entry carries its dead count in 8 bits: a drain with
      // more dead than that and a filter hit keeps all of its entries (rare:
      // 16 dead per lane of a dense 1-byte key)
      dc = DrainClasses{0u, 0u, 0u, 0u, 0u};
      maybe = maybe0;
      c = __popc(maybe);
      incl = wave_inclusive_scan(c);
      dd = dbase = dtotal = 0u;
    }
  } else {
    incl = wave_inclusive_scan(c);
  }
  if constexpr (MODE == 1 || MODE == 9 || MODE == 10) {   // ablations: output as is
    append_hits(p, maybe, c, incl, off0, out, found);
    return;
  }
  const uint32_t total = __builtin_amdgcn_readlane(incl, kWave - 1);
  if (total != 0) {
    // any entry left raw (kDrainClass: a drain that resolved all of its own
    // entries skips resolve_pending)
    const bool raw = !kDrainClass<MODE> || __ballot((maybe & ~dc.res) != 0u) != 0;
    if constexpr (kDrainClass<MODE>) {
      // the dead not yet counted (q.dacc) join the full stream before any
      // entry that cannot carry their number -- a non-certain one past 8 bits
      // of it, a raw one past 10 -- after the pending entries before them
      if (q.dacc != 0u && ((nc && q.dacc + dtotal >= 256u) || (raw && q.dacc + dtotal >= 1024u))) {
        if (q.pend_n != 0u) flush_pending<MODE>(p, q, lane, seg_start, out, found);
        q.full += q.dacc;
        q.dacc = 0u;
      }
    }
    // in order to the pending list, bucket-probed (one round trip for 64 hits)
    // each time it fills up -- dense true hits (1-byte keys) can yield up to 16
    // per lane; probing them in place would cost one round trip per hit
    const uint32_t end = q.pend_n + total;
    uint32_t idx = q.pend_n + incl - c;
    uint32_t from = q.pend_n;   // (kBkResolve: the first pending entry still raw)
    for (uint32_t base = 0;; base += kWave) {
      while (maybe != 0u && idx < base + kWave) {
        const uint32_t j = (uint32_t)__builtin_ctz(maybe);
        maybe &= maybe - 1;
        uint32_t y = off0 + j, x;
        if constexpr (kBkResolve<MODE>) {
          // the dead of this drain before the candidate
          const uint32_t dj = kDrainClass<MODE> ? q.dacc + dbase + __popc(dc.dead & ((1u << j) - 1u)) : 0u;
          if (kDrainClass<MODE> && ((dc.res >> j) & 1u)) {
            // resolved here: scan_class_entry's output entry, the dead count in x
            const uint32_t kidx = ((dc.kid >> j) & 1u) | ((dc.kid >> (15 + j)) & 2u);
            const uint32_t cls = ((dc.kept >> j) & 1u)    ? (kClassKept | kidx << 2)
                                 : ((dc.fetch >> j) & 1u) ? kClassFetch
                                                          : 0u;
            x = dj;
            y |= cls << kOutByteShift | kOutPlaceScanClass << kOutKeyShift;
          } else {
            // raw: the ring entry, the lane byte and "certain"; resolved below
            x = raw_x(ent, j, dj);
            y |= ((kmask >> j) & 1u) << 31;
          }
        } else if (kByteKeys<MODE> && ((kmask >> j) & 1u)) {
          certain_entry<MODE>(p, ent, j, x, y);
        } else {
          x = window4(ent, j);
        }
        lds_store2(q.pend + 8 * (idx - base), x, y);
        ++idx;
      }
      if (end <= base + kWave) {
        q.pend_n = end - base;
        if constexpr (kBkResolve<MODE>)
          if (raw) resolve_pending<MODE>(p, q, lane, from, seg_start);
        break;
      }
      q.pend_n = kWave;
      if constexpr (kBkResolve<MODE>)
        if (raw) resolve_pending<MODE>(p, q, lane, from, seg_start);
      from = 0;
      flush_pending<MODE>(p, q, lane, seg_start, out, found);
    }
  }
  if constexpr (kDrainClass<MODE>) {
    // the drain's dead, counted into the full stream once no pending entry
    // precedes them (each pending entry carries the number before it)
    q.dacc += dtotal;
    if (q.pend_n == 0u) {
      q.full += q.dacc;
      q.dacc = 0u;
    }
  }
}

// A tile entirely inside the block: one 16-byte non-temporal load per lane
// (read-once stream; keeps the exact tables' L2 lines).
// Buffer load: the resource (segment base) and the tile offset live in SGPRs,
// the lane's 16-byte offset is a loop-invariant VGPR -- no per-tile address
// VALU.  aux 2 = nt (gfx950 cache policy).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t segment_rsrc(const uint8_t* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, 0x7FFFFFFF,
                                           0x00020000);
}
__device__ __forceinline__ uint4 load_tile_full(__amdgpu_buffer_rsrc_t rsrc, uint32_t tile_off,
                                                uint32_t lane16) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane16, tile_off, 2);
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint4 load_tile(const uint8_t* base, uint32_t tile_off, uint32_t lane,
                                           uint64_t avail) {
  const uint32_t off = tile_off + lane * kBytesPerLane;
  if (tile_off + (uint64_t)kTile <= avail) {
    // read-once stream: non-temporal, so the filter staging and the exact
    // tables keep their L2 lines
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + off));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  // ragged block tail (at most one tile per launch)
  uint4 v = make_uint4(0, 0, 0, 0);
  if (off + (uint64_t)kBytesPerLane <= avail) {
    v = *reinterpret_cast<const uint4*>(base + off);
  } else if (off < avail) {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < kBytesPerLane; ++i) {
      const uint32_t b = off + i < avail ? (uint32_t)base[off + i] : 0u;
      w[i >> 2] |= b << (8 * (i & 3));
    }
    v = make_uint4(w[0], w[1], w[2], w[3]);
  }
  return v;
}

struct SegState {
  uint64_t seg_start;
  uint32_t seg_len;
  uint32_t* out;
  uint32_t found;
  uint32_t carry;   // lane 0: the 4 bytes before the current tile (its window head)
};

// Stage 1 of one 1 KiB tile: the filter over its 1024 byte positions.  Returns
// the lane's hit mask (bit 8n + r <=> lane byte 4n + r), or with kAny only
// whether some position of the lane passes (bit 0).
template <int MODE, bool kAny>
__device__ __forceinline__ uint32_t stage1(const uint32_t (&S)[6], uint32_t lane) {
  // Phase A: the lane's 8 position pairs and their 8 filter-block reads.
  // Pair j covers lane bytes k = 2j and k + 1; xs[j] = bytes k-2 .. k+1
  // (stream offset k + 2: even, so an aligned dword or one alignbyte).
  constexpr int kPairs = kBytesPerLane / 2;
  uint32_t xs[kPairs];
  uint2 ws[kPairs];
#pragma unroll
  for (int j = 0; j < kPairs; ++j) {
    xs[j] = pair_window(S, j);
    if constexpr (MODE != 3) {
      const uint32_t x = xs[j];
      uint32_t addr = MODE == kModeEvenHash ? even_addr<true>(x)      // hashed block
                                            : (x >> 7) & (kFilterBytes - 8);   // block x[10..23], 8 B each
      if constexpr (MODE == 4) addr = ((lane & 31u) * 8u + (uint32_t)j * 256u) & (kFilterBytes - 8);
      if constexpr (MODE == 5) {
        ws[j] = make_uint2(addr ^ x, addr + x);
      } else {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x2*>(
            (uintptr_t)addr);   // filter sits at LDS offset 0: no base add
        ws[j] = make_uint2(v.x, v.y);
      }
    }
  }
  if constexpr (MODE == 11) __builtin_amdgcn_sched_barrier(0);   // ablation: all 8 reads first
  // Phase B: the two windows of each pair against their block (internal.h
  // filter_probe_left / _right): left (position k) bit x[0..4] of the lo word
  // and x[5..9] of the hi word; right (position k + 1) the same fields of
  // y = d | b << 8 (one v_perm).  The shifter reads only the low 5 bits of the
  // amount.  The AND of the two shifted words is written by one SDWA v_and
  // straight into byte n of accumulator r (position 4n + r), so bit 0 of that
  // byte is the position's result and no separate accumulate instruction is
  // needed; bits 1..7 of each byte are don't-care and masked off below.
  if constexpr (kAny && kEven<MODE>) {
    // the even-position filter: the left windows only (pairs 0-3, 4-7 into
    // two accumulators), any pass of the lane in bit 0
    uint32_t a[2];
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      const uint32_t x = xs[j];
      const uint32_t ul = ws[j].x >> (x & 31u), vl = ws[j].y >> ((x >> 5) & 31u);
      uint32_t& aq = a[j >> 2];
      if ((j & 3) == 0) aq = ul & vl;
      else asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xea" : "+v"(aq) : "v"(ul), "v"(vl));
    }
    uint32_t t;
    asm("v_bitop3_b32 %0, %1, %2, 1 bitop3:0xa8" : "=v"(t) : "v"(a[0]), "v"(a[1]));
    return t;
  } else if constexpr (kAny && MODE != 3 && MODE != 6) {
    // the main loop only needs "does any position of this lane pass?": OR the
    // shifted-word ANDs together (v_bitop3: full rate, unlike SDWA) and keep
    // bit 0; the drain recomputes the per-position results of the few lanes
    // that do.  Two accumulators (pairs 0-3, 4-7) for some ILP.
    uint32_t a[2];
    // the right windows of pairs 2m and 2m+1 from ONE v_perm of the context
    // dwords S[m], S[m+1]: y2 = d(2m) | b(2m) << 8 | d(2m+1) << 16 | b(2m+1) << 24
    // (0.9 % faster than one v_perm per pair, profiles/r02_pair_perm_ab.json)
    uint32_t y2[kPairs / 2];
#pragma unroll
    for (int m = 0; m < kPairs / 2; ++m) y2[m] = __builtin_amdgcn_perm(S[m + 1], S[m], 0x05070305u);
#pragma unroll
    for (int j = 0; j < kPairs; ++j) {
      const uint32_t x = xs[j];
      const uint32_t ul = ws[j].x >> (x & 31u), vl = ws[j].y >> ((x >> 5) & 31u);
      const uint32_t y = (j & 1) ? y2[j >> 1] >> 16 : y2[j >> 1];   // d | b << 8 (low 10 bits)
      const uint32_t ur = ws[j].x >> (y & 31u), vr = ws[j].y >> ((y >> 5) & 31u);
      uint32_t& aq = a[j >> 2];
      if ((j & 3) == 0) aq = ul & vl;
      // acc |= u & v in one v_bitop3 (S0 = u, S1 = v, S2 = acc: 0xF0 & 0xCC | 0xAA)
      else asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xea" : "+v"(aq) : "v"(ul), "v"(vl));
      asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xea" : "+v"(aq) : "v"(ur), "v"(vr));
    }
    if constexpr (MODE == 2 || MODE == 4 || MODE == 5) {   // ablations: no ring
      asm volatile("" ::"v"(a[0] | a[1]));
      return 0u;
    }
    // (a0 | a1) & 1 in one v_bitop3 (S0 = a0, S1 = a1, S2 = 1: (0xF0 | 0xCC) & 0xAA)
    uint32_t t;
    asm("v_bitop3_b32 %0, %1, %2, 1 bitop3:0xa8" : "=v"(t) : "v"(a[0]), "v"(a[1]));
    return t;
  }
  uint32_t acc[4];   // byte 0 written first (zero-padding the rest), then bytes 1..3
  if constexpr (MODE == 3 || MODE == 6) acc[0] = acc[1] = acc[2] = acc[3] = 0u;
#define YAMD_SDWA_AND(K, U, V)                                                                   \
  switch ((K) >> 2) {                                                                            \
    case 0: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD" \
                : "=v"(acc[(K) & 3]) : "v"(U), "v"(V)); break;                                   \
    case 1: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" \
                : "+v"(acc[(K) & 3]) : "v"(U), "v"(V)); break;                                   \
    case 2: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" \
                : "+v"(acc[(K) & 3]) : "v"(U), "v"(V)); break;                                   \
    default: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD" \
                 : "+v"(acc[(K) & 3]) : "v"(U), "v"(V)); break;                                  \
  }
  // (the right windows' d | b << 8 of two pairs from one v_perm, as in the
  // kAny form above)
  uint32_t y2[kPairs / 2];
#pragma unroll
  for (int m = 0; m < kPairs / 2; ++m) y2[m] = __builtin_amdgcn_perm(S[m + 1], S[m], 0x05070305u);
#pragma unroll
  for (int j = 0; j < kPairs; ++j) {
    const int k = 2 * j;
    (void)y2;
    if constexpr (MODE == 3) {
      acc[k & 3] ^= xs[j];
    } else if constexpr (MODE == 6) {
      acc[k & 3] ^= ws[j].x ^ ws[j].y;
    } else {
      const uint32_t x = xs[j];
      const uint32_t ul = ws[j].x >> (x & 31u), vl = ws[j].y >> ((x >> 5) & 31u);
      YAMD_SDWA_AND(k, ul, vl);
      const uint32_t y = (j & 1) ? y2[j >> 1] >> 16 : y2[j >> 1];   // d | b << 8 (low 10 bits)
      const uint32_t ur = ws[j].x >> (y & 31u), vr = ws[j].y >> ((y >> 5) & 31u);
      YAMD_SDWA_AND(k + 1, ur, vr);
    }
  }
#undef YAMD_SDWA_AND
  if constexpr (MODE >= 2 && MODE <= 6) {
    asm volatile("" ::"v"(acc[0] ^ acc[1] ^ acc[2] ^ acc[3]));
    return 0u;
  }
  // hit mask: bit 8n + r <=> position 4n + r of the lane (mask_position())
  return (acc[0] & 0x01010101u) | ((acc[1] & 0x01010101u) << 1) |
         ((acc[2] & 0x01010101u) << 2) | ((acc[3] & 0x01010101u) << 3);
}

// One ring entry: the 16-byte unit's bytes S[1..4] (as loaded: no register
// moves), the 4 bytes before them S[0], and the unit's place in the segment:
// its byte offset (kIdxBytes: one VOP2 from the tile offset in an SGPR and the
// lane's loop-invariant offset), or, for the kernels that keep the next lane's
// first two bytes in the top half (kNextBytes), its index (offset / 16).
template <int MODE>
__device__ __forceinline__ void write_entry(uint32_t ent, const uint32_t (&S)[6], uint32_t unit) {
  const uint32_t idx = unit | (kNextBytes<MODE> ? S[5] << 16 : 0u);
  // three ds_write2_b32: context, the 16 bytes as loaded, index
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
  u32x4 d;
  d.x = S[1];
  d.y = S[2];
  d.z = S[3];
  d.w = S[4];
  *reinterpret_cast<__attribute__((address_space(3))) u32x4_a4*>((uintptr_t)(ent + kEntData)) = d;
  *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>((uintptr_t)(ent + kEntCtx)) = S[0];
  *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>((uintptr_t)(ent + kEntIdx)) = idx;
}

// The ordered append of a tile's hits to the wave ring.  TAIL: the segment's
// last, partial tile (positions past seg_len are masked off).
// The common path (~98 % of config C's tiles: some lane passes, the ring has
// room) is straight-line scalar code: one compare for the rare path, and a
// tile without a passing lane takes the common path too -- its masked-off
// writes cost less than a branch around them
// (tools/stage2_cost.sh: a SALU or branch instruction per tile costs config C
// 2.5 us per 4 GiB, a VOP2 4.5 us).
template <int MODE, bool TAIL>
__device__ __forceinline__ void ring_append(const ScanParams& p, WaveQueue& q, SegState& st,
                                            const uint32_t (&S)[6], uint32_t any,
                                            uint32_t tile_off, uint32_t lane) {
  if constexpr (MODE >= 2 && MODE <= 6) return;
  const uint32_t lane_off = tile_off + lane * kBytesPerLane;
  if constexpr (TAIL) {
    if (lane_off >= st.seg_len) any = 0u;   // lanes wholly past the segment end
  }
  const uint64_t lanes = __ballot(any != 0);
  const uint32_t n = (uint32_t)__popcll(lanes);
  if (YAMD_EXPECT(q.count + n > kQueueCap, 0)) {
    if (!YAMD_NO_PRIO) __builtin_amdgcn_s_setprio(0);   // (streaming waves first)
    drain<MODE, true>(p, q, lane, st.seg_start, st.seg_len, st.out, st.found);
    if (!YAMD_NO_PRIO) __builtin_amdgcn_s_setprio(1);
  }
  if (any != 0) {
    // slot = count (scalar, folded into the base) + the appending lanes below
    // (gfx950's VOP3 reads one SGPR: count as the mbcnt's addend would cost a
    // v_mov instead of the two SALU of the base)
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(
        (uint32_t)(lanes >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lanes, 0u));
    static_assert(kQueueEntryWords * 4 == 24, "entry size is the asm's inline constant");
    const uint32_t base = q.ring + q.count * (kQueueEntryWords * 4);   // scalar
    uint32_t ent;   // (asm: the compiler would re-associate into a 64-bit mad)
    asm("v_mad_u32_u24 %0, %1, 24, %2" : "=v"(ent) : "v"(below), "s"(base));
    // 24-byte entry: the lane's 16 bytes (as loaded: no register moves),
    // the 4 bytes before them, the lane's place in the segment
    if constexpr (MODE == 8) {   // ablation: the append's slot arithmetic, no LDS writes
      asm volatile("" ::"v"(ent), "v"(lane_off));
    } else if constexpr (MODE == 13) {   // ablation: an entry of the index dword only
      *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>((uintptr_t)(ent + kEntIdx)) = lane_off;
    } else {
      write_entry<MODE>(ent, S, kIdxBytes<MODE> ? lane_off : (tile_off >> 4) + lane);
    }
  }
  q.count += n;
}

// The lane's window context: the previous lane's last dword (lane 0: the
// previous tile's, or the halo), then its own 16 bytes.
__device__ __forceinline__ void tile_context(SegState& st, const uint4& cur, uint32_t (&S)[6]) {
  // wave_ror:1 gives lanes 1..63 the previous lane's last dword and lane 0
  // this tile's lane 63 -- the next tile's lane-0 context; lane 0 takes the
  // one kept from the previous tile (st.carry, meaningful in lane 0 only).
  // (One DPP move and one select: 1 % faster than a wave_shr:1 into the
  // carry plus a v_readlane of the next one, profiles/r02_carry_ror_ab.json.)
  const uint32_t rot = __builtin_amdgcn_mov_dpp(cur.w, 0x13C, 0xF, 0xF, true);
  // wave_shr:1 without bound_ctrl leaves lane 0 its old value (the carry):
  // a second DPP move instead of a select on a lane-0 SGPR mask
  // (profiles/r02_carry_dpp2_ab.json)
  S[0] = __builtin_amdgcn_update_dpp(st.carry, cur.w, 0x138, 0xF, 0xF, false);
  st.carry = rot;
  S[1] = cur.x;
  S[2] = cur.y;
  S[3] = cur.z;
  S[4] = cur.w;
  S[5] = 0u;
}

// One 1 KiB tile: stage-1 filter over its 1024 byte positions, then the ordered
// append of the hits to the wave ring.
template <int MODE, bool TAIL>
__device__ __forceinline__ void tile_step(const ScanParams& p, WaveQueue& q, SegState& st,
                                          uint4 cur, uint32_t tile_off, uint32_t lane) {
  uint32_t S[6];
  tile_context(st, cur, S);
  // the next lane's first dword (wave_shl:1; lane 63: 0), for the five bytes
  // kept beside a certain candidate near the lane's end (drain)
  if constexpr (kNextBytes<MODE>) S[5] = __builtin_amdgcn_mov_dpp(cur.x, 0x130, 0xF, 0xF, true);
  uint32_t any = stage1<kStage1Mode<MODE>, true>(S, lane);
  if constexpr (kEven<MODE>)
    if (p.n_pair_keys != 0) any |= pair_keys_any(S, p);
  const uint32_t any_f = any;   // (the filter and 2-byte-key part: kBkSkipF)
  if constexpr (kByteKeys<MODE>) {
    if constexpr (kAbl<MODE> == 3) asm volatile("" ::"v"(byte_keys_any(S, p)));   // ablation
    else if constexpr (kAbl<MODE> != 4) any |= byte_keys_any(S, p);
  }
  if constexpr (MODE == 24) asm volatile("" ::"v"(byte_keys_any(S, p)));
#if defined(YAMD_PAD_VOP2) || defined(YAMD_PAD_VOP3) || defined(YAMD_PAD_SALU) || defined(YAMD_PAD_NOP)
  // cost model (tools/stage2_cost.sh, variant builds only): N extra instructions
  // of one issue class per tile step of the product kernel, on four independent
  // dummy chains -- the marginal cost of one instruction of that class per tile
  if constexpr (MODE == 0) {
    uint32_t t0 = S[1], t1 = S[2], t2 = S[3], t3 = S[4];
#ifdef YAMD_PAD_VOP2
#pragma unroll
    for (int i = 0; i < YAMD_PAD_VOP2; i += 4)
      asm volatile("v_add_u32_e32 %0, 1, %0\n v_add_u32_e32 %1, 1, %1\n v_add_u32_e32 %2, 1, %2\n v_add_u32_e32 %3, 1, %3"
                   : "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3));
#endif
#ifdef YAMD_PAD_VOP3
#pragma unroll
    for (int i = 0; i < YAMD_PAD_VOP3; i += 4)
      asm volatile("v_add3_u32 %0, %0, 1, 2\n v_add3_u32 %1, %1, 1, 2\n v_add3_u32 %2, %2, 1, 2\n v_add3_u32 %3, %3, 1, 2"
                   : "+v"(t0), "+v"(t1), "+v"(t2), "+v"(t3));
#endif
#ifdef YAMD_PAD_NOP
#pragma unroll
    for (int i = 0; i < YAMD_PAD_NOP; ++i) asm volatile("s_nop 0");
#endif
    asm volatile("" ::"v"(t0 ^ t1 ^ t2 ^ t3));
#ifdef YAMD_PAD_SALU
    uint32_t u0 = tile_off, u1 = tile_off + 1, u2 = tile_off + 2, u3 = tile_off + 3;
#pragma unroll
    for (int i = 0; i < YAMD_PAD_SALU; i += 4)
      asm volatile("s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n s_add_u32 %3, %3, 1"
                   : "+s"(u0), "+s"(u1), "+s"(u2), "+s"(u3) : : "scc");
    asm volatile("" ::"s"(u0 ^ u1 ^ u2 ^ u3));
#endif
  }
#endif
  if constexpr (kAbl<MODE> == 1) {   // ablation: stage 1 only
    asm volatile("" ::"v"(any));
  } else {
    ring_append<MODE, TAIL>(p, q, st, S, any, tile_off, lane);
  }
  // (after the append: a drain inside it takes only the earlier tiles' entries)
  if constexpr (kBkSkipF<MODE>) q.facc |= any_f;
}

// Stream one segment [seg_start, seg_start + seg_len) of the block: full tiles
// in the main loop (unmasked; the next tile's loads in flight, two tile
// registers used alternately so no copy waits for a load), then the partial
// tail tile if any.
// MODE: 0 = the product kernel.  Others are profiling ablations only (their
// output is wrong by construction): 1 = no exact check, 2 = stage 1 only
// (no queue), 3 = input streaming only (no filter), 4 = stage 1 with
// bank-conflict-free LDS addresses, 5 = stage 1 VALU without the LDS reads,
// 6 = stage 1 addresses + LDS reads without the bit tests, 7 = stage 1 +
// ring appends, drains drop the entries, 8 = 7 without the ring's LDS writes, 9 = exact check replaced by one L2 dword
// load per hit, 10 = exact-check VALU with the bucket loads replaced by values,
// 11 = product with all 8 filter reads of a tile issued before any test,
// 12 = product without the bucket probes (first level only), 13 = 7 with
// ring entries of the index dword only (what an offset-only entry would cost).
//
// (An earlier version rotated each segment's tile order so that the waves of
// the chip would not read the same offsets of their equal segments at the
// same time; it helped the filter alone but made the product kernel 2-4 %
// slower -- the waves' drains de-synchronise them anyway.)
template <int MODE>
__device__ __forceinline__ void scan_segment(const ScanParams& p, WaveQueue& q, uint32_t seg, uint32_t lane) {
  SegState st;
  st.seg_start = p.byte_begin + (uint64_t)seg * p.seg_bytes;
  const uint64_t seg_end = min(st.seg_start + p.seg_bytes, p.byte_end);
  st.seg_len = (uint32_t)(seg_end - st.seg_start);
  st.out = p.seg_out + (p.seg_base ? p.seg_base[seg] : (size_t)seg * p.seg_cap);
  st.found = 0;
  // bytes read: [seg_start - 4, seg_end) only -- never past byte_end, so a
  // shard that holds just its window of the block is never read beyond it
  const uint64_t avail = p.byte_end - st.seg_start;
  const uint8_t* base = p.data + st.seg_start;

  // 4 bytes before the segment (warm-up halo); zeros before the block start.
  // (readfirstlane: waited for here, so no load is pending on the carry's
  // register when the tile loop starts)
  st.carry = __builtin_amdgcn_readfirstlane(
      st.seg_start >= 4 ? *reinterpret_cast<const uint32_t*>(base - 4) : 0u);
  q.count = 0;
  q.pend_n = 0;
  q.full = 0;
  q.dacc = 0;
  q.facc = 0u;

  const uint32_t n_full = st.seg_len / kTile;            // tiles needing no mask / bounds
  if (n_full > 0) {
    const uint32_t full_end = n_full * kTile;
    const __amdgpu_buffer_rsrc_t rsrc = segment_rsrc(base);
    const uint32_t lane16 = lane * kBytesPerLane;
    // kPf tiles in flight ahead of the one in the step: kPf + 1 tile registers
    // in rotation, the main loop unrolled over them (no copies, so no wait is
    // attached to a copy); the loop runs on the tile's byte offset (the loads'
    // SGPR offset; the tile's place in the round folds into the instruction's
    // offset field), only while a round's loads stay inside the full tiles
    constexpr uint32_t kP = kPf<MODE>, kR = kP + 1;
    uint4 t[kR];
#pragma unroll
    for (uint32_t i = 0; i < kP; ++i)
      if (i * kTile < full_end) t[i] = load_tile_full(rsrc, i * kTile, lane16);
    // the first tile waited for before the loop: no path into the loop
    // arrives with a load pending on t[0] (without the wait: equal,
    // profiles/r06_prefetch_ab/r07m_*)
    asm volatile("" : "+v"(t[0].x), "+v"(t[0].y), "+v"(t[0].z), "+v"(t[0].w));
    uint32_t off = 0;
    if (full_end >= (2 * kR - 1) * kTile) {
      const uint32_t lim = full_end - (2 * kR - 1) * kTile;   // (every load of a round inside)
      do {
#pragma unroll
        for (uint32_t i = 0; i < kR; ++i) {
          t[(i + kP) % kR] = load_tile_full(rsrc, off + (i + kP) * kTile, lane16);
          tile_step<MODE, false>(p, q, st, t[i], off + i * kTile, lane);
        }
        off += kR * kTile;
      } while (off <= lim);
    }
    // the rest (fewer than 2 kR tiles; short segments all of theirs): the
    // same rotation with every load and step guarded (scalar tests)
    while (off < full_end) {
#pragma unroll
      for (uint32_t i = 0; i < kR; ++i) {
        if (off + i * kTile < full_end) {
          if (off + (i + kP) * kTile < full_end)
            t[(i + kP) % kR] = load_tile_full(rsrc, off + (i + kP) * kTile, lane16);
          tile_step<MODE, false>(p, q, st, t[i], off + i * kTile, lane);
        }
      }
      off += kR * kTile;
    }
  }
  if (st.seg_len % kTile != 0)   // the ragged tail tile
    tile_step<MODE, true>(p, q, st, load_tile(base, n_full * kTile, lane, avail), n_full * kTile,
                          lane);
  // everything queued to the segment's output, in order
  if (q.count != 0) drain<MODE>(p, q, lane, st.seg_start, st.seg_len, st.out, st.found);
  if (q.pend_n != 0) flush_pending<MODE>(p, q, lane, st.seg_start, st.out, st.found);
  if (lane == 0) {
    p.seg_count[seg] = st.found;
    if (kDrop<MODE>) p.seg_full[seg] = q.full + q.dacc;
  }
}

template <int MODE>
__global__ __launch_bounds__(kWGThreads, 1) void scan_segments_kernel(ScanParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* filt = lds;
  {
    // 128 KiB: 8 x 16 B per thread, all 8 loads in flight before the stores
    // (a loop over blockDim.x waited for each load in turn: 8 L2 round trips
    // before the first tile)
    const uint4* src = reinterpret_cast<const uint4*>(p.filter);
    uint4* dst = reinterpret_cast<uint4*>(filt);
    constexpr uint32_t kPer = kFilterWords / 4 / kWGThreads;
    static_assert(kPer * kWGThreads * 4 == kFilterWords, "filter copy: whole uint4s per thread");
    uint4 v[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) v[k] = src[threadIdx.x + k * kWGThreads];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) dst[threadIdx.x + k * kWGThreads] = v[k];
  }
  __syncthreads();
  const uint32_t lane = lane_id();
  // wave index, provably wave-uniform: everything derived from it (segment
  // bounds, loop counts, ring base) stays in SGPRs with scalar branches
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t total_waves = gridDim.x * kWavesPerWG;
  uint32_t seg = blockIdx.x * kWavesPerWG + wid;
  uint32_t kcv = 0u;
  if constexpr (kDrop<MODE>)
    if (lane < kKcWords) kcv = p.kc[lane];   // (the records, and the plan in lanes 32..)
  while (seg < p.n_segments) {
    WaveQueue q;   // (per segment: its per-lane state then stays in registers)
    q.kcv = kcv;
    q.ring = kFilterBytes + wid * (kQueueCap * kQueueEntryWords * 4);
    q.pend = kFilterBytes + kQueueBytes + wid * (kWave * 8);
    __builtin_amdgcn_s_setprio(1);
    scan_segment<MODE>(p, q, seg, lane);
    if (p.seg_next == nullptr) {
      seg += total_waves;
    } else {
      // dynamic: the next unclaimed segment (one vector atomic per wave)
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(p.seg_next, 1u);
      seg = __builtin_amdgcn_readfirstlane(t);
    }
  }
}

// ---------------------------------------------------------------------------
// Candidate compaction: per-segment counts -> offsets (one workgroup), then a
// scatter of every segment's ascending entries into one ascending uint64 array.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void seg_offsets_kernel(const uint32_t* seg_count, uint32_t n,
                                                           uint32_t cap, uint64_t* seg_offset,
                                                           uint64_t* summary) {
  // each thread a contiguous run of segments; wave scans by shuffles, then
  // one wave scans the 16 wave totals (two barriers in all)
  __shared__ uint64_t wsum[kWGThreads / kWave];
  __shared__ uint32_t wmax[kWGThreads / kWave];
  const uint32_t t = threadIdx.x, lane = t % kWave, w = t / kWave;
  const uint32_t per = (n + kWGThreads - 1) / kWGThreads;
  const uint32_t lo = min(t * per, n), hi = min(lo + per, n);
  uint64_t s = 0;
  uint32_t mx = 0;
  // the run's first kKeep counts stay in registers for the offsets below (one
  // global round trip fewer; runs are 4 segments per thread at 4 GiB)
  constexpr uint32_t kKeep = 8;
  uint32_t keep[kKeep];
#pragma unroll
  for (uint32_t k = 0; k < kKeep; ++k) {
    keep[k] = lo + k < hi ? seg_count[lo + k] : 0u;
    s += min(keep[k], cap);
    mx = max(mx, keep[k]);
  }
  // (unrolled: the loads of a run are independent and go out together -- one
  // round trip per 16 segments instead of one per segment)
#pragma unroll 16
  for (uint32_t i = lo + kKeep; i < hi; ++i) {
    const uint32_t c = seg_count[i];
    s += min(c, cap);
    mx = max(mx, c);
  }
  uint64_t incl = s;
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t v = __shfl_up(incl, d, kWave);
    if (lane >= (uint32_t)d) incl += v;
  }
  for (int d = kWave / 2; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, d, kWave));
  if (lane == kWave - 1) wsum[w] = incl;
  if (lane == 0) wmax[w] = mx;
  __syncthreads();
  if (w == 0) {
    constexpr uint32_t kWaves = kWGThreads / kWave;
    const uint64_t v = lane < kWaves ? wsum[lane] : 0;
    uint32_t m = lane < kWaves ? wmax[lane] : 0;
    uint64_t inc = v;
    for (int d = 1; d < kWave; d <<= 1) {
      const uint64_t u = __shfl_up(inc, d, kWave);
      if (lane >= (uint32_t)d) inc += u;
    }
    for (int d = kWave / 2; d >= 1; d >>= 1) m = max(m, (uint32_t)__shfl_xor(m, d, kWave));
    if (lane < kWaves) wsum[lane] = inc - v;   // exclusive
    if (lane == kWaves - 1) {
      // (host-mapped coherent memory: system-scope stores)
      __hip_atomic_store(&summary[0], inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&summary[1], (uint64_t)m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      seg_offset[n] = inc;   // (the total for device-side readers)
    }
  }
  __syncthreads();
  uint64_t run = wsum[w] + incl - s;
#pragma unroll
  for (uint32_t k = 0; k < kKeep; ++k) {
    if (lo + k < hi) seg_offset[lo + k] = run;
    run += min(keep[k], cap);
  }
#pragma unroll 16
  for (uint32_t i = lo + kKeep; i < hi; ++i) {
    seg_offset[i] = run;
    run += min(seg_count[i], cap);
  }
}

constexpr uint32_t kScatterWaves = 8;   // waves per segment in the scatter (dense segments; 4, 16: no better, r5h24)

// The compaction reads the input bytes a certain candidate's class needs when
// the scan's five kept bytes do not hold them (key_class's `more`):
// fuzz0's pre-verification 0.63 -> 0.32 ms for 0.08 ms more compaction, rx
// +0.02 ms, short / fuzz3 unchanged (profiles/r04_ab_inproc.json, gpurun h8).

template <uint32_t W>
__global__ __launch_bounds__(W * kWave) void seg_scatter_kernel(
    ScanParams p, const uint64_t* seg_offset, uint64_t* positions) {
  // one block of W waves per segment (segments hold up to ~10^4 candidates),
  // its waves interleaved 64 candidates apart
  __shared__ KeyClassRec kc[kMaxByteKeys];
  __shared__ uint32_t lcount;
  // the classes of a chunk of kChunk candidates, staged here and written out as
  // aligned dwords (one byte store per candidate ran at ~1.4 TB/s:
  // profiles/r04_ab_inproc.json h31); +4: the chunk's start is placed at its
  // absolute index mod 4
  constexpr uint32_t kChunk = W * kWave * (W == 2 ? 16u : 8u);
  __shared__ __attribute__((aligned(4))) uint8_t cbuf[kChunk + 4];
  const bool classes = p.dead != nullptr;   // (uniform)
  if (threadIdx.x < kMaxByteKeys) {
    const uint32_t k = threadIdx.x;
    // (the backward guards from the scan kernel's record table, kc fields 6, 7)
    kc[k] = KeyClassRec{p.kd_info[k], p.kd_m[k], p.kd_v[k], p.kd_x0[k], p.kd_x1[k], p.kd_min_pos[k],
                        p.kc != nullptr ? p.kc[8 * k + 6] : 0u, p.kc != nullptr ? p.kc[8 * k + 7] : 0u};
  }
  if (threadIdx.x == 0) lcount = 0;
  __syncthreads();
  const uint32_t seg = blockIdx.x;
  const uint32_t c = min(p.seg_count[seg], p.seg_cap);
  const uint64_t base = p.byte_begin + (uint64_t)seg * p.seg_bytes + 1;  // position = byte + 1
  const size_t at0 = p.seg_base ? p.seg_base[seg] : (size_t)seg * p.seg_cap;
  const uint32_t* src = p.seg_out + at0;
  const uint32_t* sx = classes ? p.seg_x + at0 : nullptr;
  const uint64_t first = seg_offset[seg];
  uint64_t* dst = positions + first;
  // verified-only scans: the full stream's index of every output candidate,
  // when some candidate was left out (otherwise it is the output index)
  uint32_t* cidx = nullptr;
  uint32_t full0 = 0;
  if (p.drop_dead != 0u && p.seg_full_offset[p.n_segments] != seg_offset[p.n_segments]) {
    cidx = p.cand_index + first;
    full0 = (uint32_t)p.seg_full_offset[seg];
  }
  // (w through readfirstlane: the compiler then knows the loop's trips are
  // wave-uniform -- otherwise it runs the loop under an exec mask and carries
  // every wave-uniform value of it as a lane mask)
  const uint32_t lane = threadIdx.x % kWave, w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  constexpr uint32_t kStride = W * kWave;
  // Latency-bound (a few hundred candidates per wave): every iteration's
  // entry and kept bytes are loaded one iteration ahead.
  uint32_t e = 0, x = 0;
  {
    const uint32_t i = w * kWave + lane;
    if (i < c) {
      e = src[i];
      if (classes) x = sx[i];
    }
  }
  for (uint32_t chunk = 0; chunk < c; chunk += kChunk) {   // (block-uniform: the barriers)
    const uint32_t cend = c - chunk > kChunk ? chunk + kChunk : c;
    const uint32_t sh0 = (uint32_t)(first + chunk) & 3u;   // cbuf[sh0 + k] = class of chunk + k
    for (uint32_t i0 = chunk + w * kWave; i0 < cend; i0 += kStride) {   // (wave-uniform trips: the ballots)
      const uint32_t i = i0 + lane;
      const bool valid = i < c;
      const uint32_t ec = e, xc = x;
      e = x = 0u;
      if (i + kStride < c) {
        e = src[i + kStride];
        if (classes) x = sx[i + kStride];
      }
      const uint64_t pos = base + (ec & kOutOffsetMask);
      // (non-temporal: short's verified step -2 %, fuzz3's -1 %, the
      // pre-verification that reads them back included, gpurun r5h24)
      if (valid) __builtin_nontemporal_store(pos, dst + i);
      if (valid && cidx != nullptr) cidx[i] = full0 + xc;   // (mod 2^32, as the records')
      if (!classes) continue;
      // the certain candidates' classes from the bytes the scan kept beside them
      // (verified-only scans: decided by the scan, kernels.hip scan_class_entry)
      uint32_t cls = 0u;
      if (valid && (ec & kCertainMask) != 0u) {
        bool more = false;
        if ((ec >> kOutKeyShift & 7u) == kOutPlaceScanClass) {
          cls = ec >> kOutByteShift & 0xFFu;
          more = cls == kClassFetch;
          if (more) cls = 0u;
        } else {
          cls = key_class(p, [](uint32_t k) { return kc[k]; },
                          xc | (uint64_t)(ec >> kOutByteShift & 0xFFu) << 32,
                          (int32_t)(ec >> kOutKeyShift & 7u) - 2, (ec & kOutDeep) != 0u, pos, 4, &more);
        }
        // Undecided only because the guard's bytes (or the byte before the key)
        // lie outside the five the scan kept -- the key near its lane's end:
        // read eight bytes around the key from the input (three aligned dwords
        // inside [byte_begin - 4, byte_end), the bytes the scan itself may read)
        // and decide again, rather than leave the candidate to the live list.
        if (more) {
          const uint64_t kb = pos - 1;   // the key's byte
          const uint64_t a4 = (kb - 2) & ~3ull;
          if (kb >= 2 && a4 + 4 >= p.byte_begin && a4 + 12 <= p.byte_end) {
            const uint32_t* d = reinterpret_cast<const uint32_t*>(p.data + a4);
            const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
            const uint32_t sh = (uint32_t)(kb - 2 - a4);
            const uint64_t w8 = __builtin_amdgcn_alignbyte(d1, d0, sh) |
                                (uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32;
            cls = key_class(p, [](uint32_t k) { return kc[k]; }, w8, 2, false, pos, 7);
          }
        }
      }
      if (valid) {
        cbuf[sh0 + (i - chunk)] = (uint8_t)cls;
      }
      // the undecided ones onto the segment's live list (any order), in the
      // segment's own range of p.live -- an LDS counter, no global atomic (one
      // per segment on one global counter serialised ~4,096 of them: rx's
      // compaction 51 us for 230 k candidates, gpurun r5h4)
      const bool live = valid && cls == 0u;
      const uint64_t lm = __ballot(live);
      if (lm != 0) {
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(&lcount, (uint32_t)__popcll(lm));
        b = __builtin_amdgcn_readfirstlane(b);
        const uint32_t slot =
            b + __builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
        if (live) p.live[first + slot] = (uint32_t)(first + i);
      }
    }
    {
      if (classes) {
        // the chunk's classes: absolute bytes [a, a + m) of p.dead -- head and
        // tail bytes (shared with the neighbouring segments' blocks) byte by
        // byte, the aligned dwords between them whole
        __syncthreads();
        const uint64_t a = first + chunk;
        const uint32_t m = cend - chunk;
        const uint32_t head = min((4u - sh0) & 3u, m);
        const uint32_t nd = (m - head) / 4u, tail = m - head - 4u * nd;
        uint8_t* out = p.dead + a;
        for (uint32_t t = threadIdx.x; t < nd; t += kStride)
          *reinterpret_cast<uint32_t*>(out + head + 4u * t) =
              *reinterpret_cast<const uint32_t*>(cbuf + sh0 + head + 4u * t);
        if (threadIdx.x < head) out[threadIdx.x] = cbuf[sh0 + threadIdx.x];
        if (threadIdx.x < tail) out[head + 4u * nd + threadIdx.x] = cbuf[sh0 + head + 4u * nd + threadIdx.x];
        __syncthreads();
      }
    }
  }
  if (!classes) return;
  __syncthreads();
  if (threadIdx.x == 0) p.live_count[seg] = lcount;
}

// ---------------------------------------------------------------------------
// Synthetic input (SURVEY.md App. A xorshift64), one chunk per thread, each
// chunk's start state precomputed on the host by GF(2) jump-ahead.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void xorshift_fill_kernel(uint8_t* buf, uint64_t n,
                                                            const uint64_t* states,
                                                            uint32_t n_chunks, uint32_t chunk) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_chunks) return;
  uint64_t x = states[c];
  const uint64_t lo = (uint64_t)c * chunk;
  const uint64_t hi = min(lo + chunk, n);
  uint64_t i = lo;
  for (; i + 16 <= hi; i += 16) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        v |= (uint32_t)((x >> 24) & 0xFF) << (8 * b);
      }
      w[j] = v;
    }
    *reinterpret_cast<uint4*>(buf + i) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  for (; i < hi; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    buf[i] = (uint8_t)(x >> 24);
  }
}

}  // namespace yamd

// Launch wrappers (host side, called from scanner.cpp).
namespace yamd {

// t0 / t1 (timing): events stamped with the kernel's own start and end
// (hipExtLaunchKernel), so the measured duration is the kernel's -- not the
// gaps of separate markers around it on the stream.
#define YAMD_LAUNCH_SCAN(K)                                                                      \
  do {                                                                                           \
    if (t0 != nullptr || t1 != nullptr)                                                          \
      hipExtLaunchKernelGGL(K, dim3(grid), dim3(kWGThreads), (uint32_t)lds, s, t0, t1, 0u, p);   \
    else                                                                                         \
      hipLaunchKernelGGL(K, dim3(grid), dim3(kWGThreads), lds, s, p);                            \
  } while (0)
hipError_t launch_scan(const ScanParams& p, int grid, hipStream_t s, int mode, hipEvent_t t0,
                       hipEvent_t t1) {
  const size_t lds = kScanLdsBytes;
  switch (YAMD_DIAG ? mode : 0) {
#if YAMD_DIAG   // profiling ablations (tools/ablate.py): diagnostic builds only
    case 1: YAMD_LAUNCH_SCAN(scan_segments_kernel<1>); break;
    case 2: YAMD_LAUNCH_SCAN(scan_segments_kernel<2>); break;
    case 3: YAMD_LAUNCH_SCAN(scan_segments_kernel<3>); break;
    case 4: YAMD_LAUNCH_SCAN(scan_segments_kernel<4>); break;
    case 5: YAMD_LAUNCH_SCAN(scan_segments_kernel<5>); break;
    case 6: YAMD_LAUNCH_SCAN(scan_segments_kernel<6>); break;
    case 7: YAMD_LAUNCH_SCAN(scan_segments_kernel<7>); break;
    case 8: YAMD_LAUNCH_SCAN(scan_segments_kernel<8>); break;
    case 9: YAMD_LAUNCH_SCAN(scan_segments_kernel<9>); break;
    case 10: YAMD_LAUNCH_SCAN(scan_segments_kernel<10>); break;
    case 11: YAMD_LAUNCH_SCAN(scan_segments_kernel<11>); break;
    case 12: YAMD_LAUNCH_SCAN(scan_segments_kernel<12>); break;
    case 13: YAMD_LAUNCH_SCAN(scan_segments_kernel<13>); break;
    case 24: YAMD_LAUNCH_SCAN(scan_segments_kernel<24>); break;
    case 25: YAMD_LAUNCH_SCAN(scan_segments_kernel<25>); break;
    case 101: case 102: case 103: case 104: {
      // the ablations of the byte-key variant the product would run (even
      // filters plain only; others: the pair filter)
      if (p.n_byte_keys == 0) return hipErrorInvalidValue;
      const int base = p.filter_mode == kFilterEven ? (p.kx_next ? kModeByteKeysNextEven : kModeByteKeysEven)
                                                    : (p.kx_next ? kModeByteKeysNext : kModeByteKeys);
#define YAMD_ABL(A, V)                                                                             \
  if (mode == 100 + A && base == V)                                                                \
    YAMD_LAUNCH_SCAN(scan_segments_kernel<100 * A + V>);
#define YAMD_ABL4(A) YAMD_ABL(A, kModeByteKeys) YAMD_ABL(A, kModeByteKeysNext) YAMD_ABL(A, kModeByteKeysEven) YAMD_ABL(A, kModeByteKeysNextEven)
      YAMD_ABL4(1) YAMD_ABL4(2) YAMD_ABL4(3) YAMD_ABL4(4)
#undef YAMD_ABL4
#undef YAMD_ABL
      break;
    }
#endif
    default:
      if (p.n_byte_keys != 0) {
        const int m = (p.kx_next != 0 ? 2 : 0) + (p.filter_mode == kFilterEven       ? 1
                                                  : p.filter_mode == kFilterEvenHash ? 3
                                                                                     : 0) * 4;
#define YAMD_BK_CASES(D)                                                                          \
  switch (m) {                                                                                    \
    case 0: YAMD_LAUNCH_SCAN(scan_segments_kernel<D + kModeByteKeys>); break;                     \
    case 2: YAMD_LAUNCH_SCAN(scan_segments_kernel<D + kModeByteKeysNext>); break;                 \
    case 4: YAMD_LAUNCH_SCAN(scan_segments_kernel<D + kModeByteKeysEven>); break;                 \
    case 6: YAMD_LAUNCH_SCAN(scan_segments_kernel<D + kModeByteKeysNextEven>); break;             \
    case 12: YAMD_LAUNCH_SCAN(scan_segments_kernel<D + kModeByteKeysEvenHash>); break;            \
    default: YAMD_LAUNCH_SCAN(scan_segments_kernel<D + kModeByteKeysNextEvenHash>); break;        \
  }
        if (p.drop_dead != 0u && p.kp_on != 0u) {
          YAMD_BK_CASES(kDropPlanModes)
        } else if (p.drop_dead != 0u && p.kd_bguard != 0u) {
          YAMD_BK_CASES(kDropBgModes)
        } else if (p.drop_dead != 0u) {
          YAMD_BK_CASES(kDropModes)
        } else {
          YAMD_BK_CASES(0)
        }
#undef YAMD_BK_CASES
      } else if (p.filter_mode == kFilterEven)
        YAMD_LAUNCH_SCAN(scan_segments_kernel<kModeEven>);
      else if (p.filter_mode == kFilterEvenHash)
        YAMD_LAUNCH_SCAN(scan_segments_kernel<kModeEvenHash>);
      else
        YAMD_LAUNCH_SCAN(scan_segments_kernel<0>);
      break;
  }
  return hipGetLastError();
}
#undef YAMD_LAUNCH_SCAN

hipError_t launch_compact(const ScanParams& p, uint64_t* seg_offset, uint64_t* summary,
                          uint64_t* positions, bool scatter, hipStream_t s) {
  if (!scatter) {
    hipLaunchKernelGGL(seg_offsets_kernel, dim3(1), dim3(1024), 0, s, p.seg_count, p.n_segments,
                       p.seg_cap, seg_offset, summary);
    // verified-only scans: the offsets and total of the segments' full streams
    if (p.drop_dead != 0u)
      hipLaunchKernelGGL(seg_offsets_kernel, dim3(1), dim3(1024), 0, s, (const uint32_t*)p.seg_full,
                         p.n_segments, 0xFFFFFFFFu, p.seg_full_offset, summary + 2);
  } else {
    // sparse segments (the default capacity, no rerun at exact offsets: at
    // most one candidate per 256 bytes) take two waves each, dense ones
    // kScatterWaves (a 4 GiB block: 8,192 instead of 32,768 waves)
    if (p.seg_base == nullptr && p.seg_cap <= p.seg_bytes / 256)
      hipLaunchKernelGGL(seg_scatter_kernel<2>, dim3(p.n_segments), dim3(2 * kWave), 0, s, p,
                         (const uint64_t*)seg_offset, positions);
    else
      hipLaunchKernelGGL(seg_scatter_kernel<kScatterWaves>, dim3(p.n_segments), dim3(kScatterWaves * kWave),
                         0, s, p, (const uint64_t*)seg_offset, positions);
  }
  return hipGetLastError();
}

// Exclusive offsets of n counts, the total at offsets[n] and in summary[0]
// (pre-verification's live lists).
hipError_t launch_counts_offsets(const uint32_t* counts, uint32_t n, uint64_t* offsets, uint64_t* summary,
                                 hipStream_t s) {
  hipLaunchKernelGGL(seg_offsets_kernel, dim3(1), dim3(1024), 0, s, counts, n, 0xFFFFFFFFu, offsets, summary);
  return hipGetLastError();
}

hipError_t launch_xorshift(uint8_t* buf, uint64_t n, const uint64_t* states, uint32_t n_chunks,
                           uint32_t chunk, hipStream_t s) {
  hipLaunchKernelGGL(xorshift_fill_kernel, dim3((n_chunks + 255) / 256), dim3(256), 0, s, buf, n,
                     states, n_chunks, chunk);
  return hipGetLastError();
}

hipError_t configure_scan_kernel() {
  const int lds = (int)kScanLdsBytes;
  hipError_t e = hipSuccess;
  for (const void* k : {(const void*)scan_segments_kernel<0>,
                        (const void*)scan_segments_kernel<kModeByteKeys>,
                        (const void*)scan_segments_kernel<kModeByteKeysNext>,
                        (const void*)scan_segments_kernel<kModeEven>,
                        (const void*)scan_segments_kernel<kModeEvenHash>,
                        (const void*)scan_segments_kernel<kModeByteKeysEven>,
                        (const void*)scan_segments_kernel<kModeByteKeysEvenHash>,
                        (const void*)scan_segments_kernel<kModeByteKeysNextEven>,
                        (const void*)scan_segments_kernel<kModeByteKeysNextEvenHash>,
                        (const void*)scan_segments_kernel<kDropModes + kModeByteKeys>,
                        (const void*)scan_segments_kernel<kDropModes + kModeByteKeysNext>,
                        (const void*)scan_segments_kernel<kDropModes + kModeByteKeysEven>,
                        (const void*)scan_segments_kernel<kDropModes + kModeByteKeysEvenHash>,
                        (const void*)scan_segments_kernel<kDropModes + kModeByteKeysNextEven>,
                        (const void*)scan_segments_kernel<kDropModes + kModeByteKeysNextEvenHash>,
                        (const void*)scan_segments_kernel<kDropBgModes + kModeByteKeys>,
                        (const void*)scan_segments_kernel<kDropBgModes + kModeByteKeysNext>,
                        (const void*)scan_segments_kernel<kDropBgModes + kModeByteKeysEven>,
                        (const void*)scan_segments_kernel<kDropBgModes + kModeByteKeysEvenHash>,
                        (const void*)scan_segments_kernel<kDropBgModes + kModeByteKeysNextEven>,
                        (const void*)scan_segments_kernel<kDropBgModes + kModeByteKeysNextEvenHash>,
                        (const void*)scan_segments_kernel<kDropPlanModes + kModeByteKeys>,
                        (const void*)scan_segments_kernel<kDropPlanModes + kModeByteKeysNext>,
                        (const void*)scan_segments_kernel<kDropPlanModes + kModeByteKeysEven>,
                        (const void*)scan_segments_kernel<kDropPlanModes + kModeByteKeysEvenHash>,
                        (const void*)scan_segments_kernel<kDropPlanModes + kModeByteKeysNextEven>,
                        (const void*)scan_segments_kernel<kDropPlanModes + kModeByteKeysNextEvenHash>,
#if YAMD_DIAG
                        (const void*)scan_segments_kernel<1>,
                        (const void*)scan_segments_kernel<2>, (const void*)scan_segments_kernel<3>,
                        (const void*)scan_segments_kernel<4>, (const void*)scan_segments_kernel<5>,
                        (const void*)scan_segments_kernel<6>, (const void*)scan_segments_kernel<7>,
                        (const void*)scan_segments_kernel<8>, (const void*)scan_segments_kernel<9>,
                        (const void*)scan_segments_kernel<10>, (const void*)scan_segments_kernel<11>,
                        (const void*)scan_segments_kernel<12>, (const void*)scan_segments_kernel<13>,
                        (const void*)scan_segments_kernel<24>, (const void*)scan_segments_kernel<25>,
#define YAMD_ABL_K(A) (const void*)scan_segments_kernel<100 * A + kModeByteKeys>,                  \
                      (const void*)scan_segments_kernel<100 * A + kModeByteKeysNext>,              \
                      (const void*)scan_segments_kernel<100 * A + kModeByteKeysEven>,              \
                      (const void*)scan_segments_kernel<100 * A + kModeByteKeysNextEven>,
                        YAMD_ABL_K(1) YAMD_ABL_K(2) YAMD_ABL_K(3) YAMD_ABL_K(4)
#undef YAMD_ABL_K
#endif
                       }) {
    hipError_t r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (r != hipSuccess) e = r;
  }
  return e;
}

}  // namespace yamd
