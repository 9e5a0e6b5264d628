// Internal definitions shared by the host flattening code and the gfx950
// kernels.  Nothing here is part of the C ABI (include/yara_amd.h).
#pragma once

#include <stdint.h>
#include <stdlib.h>

#include <hip/hip_runtime.h>

// Diagnostic builds (make -C yara_amd/csrc diag -> yara_amd/_diag/libyara_amd.so,
// used by tools/ only): the scan kernel's profiling ablations
// (yr_amd__diag_kernel_mode) and the A/B environment switches.  The product
// library instantiates only the product kernels and reads none of the switches.
#ifndef YAMD_DIAG
#define YAMD_DIAG 0
#endif

namespace yamd {

// An A/B experiment switch (tools/README.md): null in the product library.
inline const char* diag_env(const char* name) { return YAMD_DIAG ? getenv(name) : nullptr; }

// ---------------------------------------------------------------------------
// Geometry of the scan kernel (gfx950: wave64, 160 KiB LDS per CU).
//
// A TILE is what one wave loads per step: 64 lanes x 16 B = 1 KiB, one
// coalesced buffer_load_dwordx4 per lane.  A SEGMENT is the unit of work a
// wave takes from the grid-stride loop and the unit of ordered output: its
// candidates are written, ascending, into its own output slot range.
// ---------------------------------------------------------------------------
constexpr int kWave = 64;
constexpr int kBytesPerLane = 16;
constexpr int kTile = kWave * kBytesPerLane;        // 1024 B
constexpr uint32_t kSegment = 1u << 20;   // max segment: 1 MiB (ring entries hold offset/16 in 16 bits)
constexpr uint32_t kSegmentTarget = kSegment;   // preferred segment size (scanner.cpp)
constexpr uint32_t kMaxByteKeys = 4;   // 1-byte keys tested in stage 1 (more: filter)
constexpr uint32_t kMaxPairKeys = 4;   // even filters: 2-byte keys tested as aligned half-words
constexpr int kWavesPerWG = 16;
constexpr int kWGThreads = kWave * kWavesPerWG;     // 1024

// LDS window filter: 2^20 bits = 128 KiB over the 3-byte windows (filter_probe).
constexpr int kFilterLog2Bits = 20;
constexpr uint32_t kFilterWords = 1u << (kFilterLog2Bits - 5);   // 32768
constexpr uint32_t kFilterBytes = kFilterWords * 4;              // 131072

// Per-wave LDS ring of filter hits awaiting the exact check: one 24-byte entry
// per (tile, lane) with hits = the lane's 20 bytes of window context + mask;
// then per wave a pending list of 64 {window, offset} pairs (kernels.hip).
constexpr uint32_t kQueueCap = 64;
constexpr uint32_t kQueueEntryWords = 6;
constexpr uint32_t kQueueBytes = kWavesPerWG * kQueueCap * kQueueEntryWords * 4;   // 24 KiB
constexpr uint32_t kPendBytes = kWavesPerWG * kWave * 8;                          // 8 KiB
constexpr uint32_t kScanLdsBytes = kFilterBytes + kQueueBytes + kPendBytes;       // 160 KiB

// Pair filter over 3-byte windows: one 8-byte block serves the windows ending
// at two adjacent positions.  With a | b << 8 | c << 16 | d << 24 the four
// bytes around a pair (positions of c and d), both windows (a,b,c) and
// (b,c,d) contain b and c, and the block is chosen by b[2..7] and c alone;
// each window then tests one bit of the block's low word and one of its high
// word, picked by the bits of that window not in the block index (10 each):
//   block = x[10..23]           device byte address (x >> 7) & 0x1FFF8
//   left  (a,b,c): lo x[0..4]  = a[0..4],  hi x[5..9]  = a[5..7] b[0..1]
//   right (b,c,d): lo x[24..28] = d[0..4], hi d[5..7] b[0..1]
// Every key window is inserted in both roles (a window may end at either
// position of a pair), so a block holds ~2x the keys of a one-window block
// (config C: 0.39% of random positions pass instead of 0.15%), but one
// ds_read_b64 now serves two positions: the LDS bank conflicts of these
// random reads were the kernel's bound.
// Even-position filter (kFilterEven, rule sets whose keys are all 4 bytes):
// the left role alone, tested at the even positions only (half of stage 1's
// work).  A 4-byte key ending at an even position has its last 3 bytes as the
// window there; one ending at an odd position k + 1 has its first 3 bytes as
// the window ending at k.  Both are inserted in the left role, so a pass at
// even k makes k and k + 1 filter hits; the exact stages are unchanged.
constexpr uint32_t kFilterPair = 0;
constexpr uint32_t kFilterEven = 1;
// kFilterEvenHash: the even-position filter with its block picked by a
// multiplicative hash of all three bytes (x * K, bits 18..31: one
// v_mul_u32_u24 more per test); the bits by the raw fields as in the left
// role.  Sets of many similar keys crowd a few plain blocks (config E's nocase
// variants share their middle bytes: 0.30 % of random windows pass the plain
// filter, 0.18 % the hashed one); the host picks the form whose blocks pass
// fewer random windows (tables.cpp).
constexpr uint32_t kFilterEvenHash = 2;
constexpr uint32_t kEvenHashK = 0xEBCA77u;
struct FilterProbe {
  uint32_t block;  // index into the kFilterWords / 2 blocks; words 2*block, 2*block+1
  uint32_t b_lo, b_hi;
};
// window w3 = p | q << 8 | r << 16 in the left role (p, q, r) = (a, b, c)
__host__ __device__ inline FilterProbe filter_probe_left(uint32_t w3) {
  const uint32_t x = w3 & 0xFFFFFFu;
  return FilterProbe{x >> 10, x & 31u, (x >> 5) & 31u};
}
// a window of the even-position filter (kFilterEven / kFilterEvenHash)
__host__ __device__ inline FilterProbe filter_probe_even(uint32_t w3, bool hashed) {
  const uint32_t x = w3 & 0xFFFFFFu;
  const uint32_t block = hashed ? (x * kEvenHashK) >> 18 : x >> 10;   // (x, K < 2^24)
  return FilterProbe{block, x & 31u, (x >> 5) & 31u};
}
// the same window in the right role (p, q, r) = (b, c, d)
__host__ __device__ inline FilterProbe filter_probe_right(uint32_t w3) {
  const uint32_t x = w3 & 0xFFFFFFu;
  return FilterProbe{x >> 2 & 0x3FFFu, (x >> 16) & 31u, ((x >> 21) & 7u) | ((x & 3u) << 3)};
}

// Exact key sets (second stage), one uint32 array in HBM:
//   [0, 8)        1-byte keys: 256-bit bitmap
//   [8, 2056)     2-byte keys: 65536-bit bitmap
//   t3, t4        3- and 4-byte keys: two-choice bucketed hash tables, 4 keys
//                 per 16-byte bucket; a lookup loads both candidate buckets
//                 (two independent dwordx4 loads: one round trip, no probe
//                 chains).  t3 stores key | 1 << 24, t4 stores the key; 0 marks
//                 an empty slot (a 4-byte key of 0 is kept in a flag).
// Keys are little endian: the first byte of the key in bits 0..7.
//   [2056, +32768) first-level word filter of the 3- and 4-byte keys (below)
constexpr uint32_t kExactBm1 = 0;
constexpr uint32_t kExactBm2 = 8;
constexpr uint32_t kExactFl = 8 + 2048;
constexpr uint32_t kExactFlLog2 = 15;
constexpr uint32_t kExactFlWords = 1u << kExactFlLog2;
constexpr uint32_t kExactHeadWords = kExactFl + kExactFlWords;
constexpr uint32_t kExactZero4 = 1u;   // flag: the 4-byte key 0x00000000 exists

// First level of the exact check (one dword = one cache line per filter hit
// instead of four 16-byte buckets): the word is chosen by the last 3 bytes of
// the position's window; a 3-byte key sets one of its bits 0..15 (picked by
// the same 3 bytes), a 4-byte key one of bits 16..31 (picked by all 4).  A
// clear bit proves "no 3-/4-byte key ends here"; a set one sends the position
// to the bucket tables.  w4 = the 4 bytes ending at the position.
// The hashes are 24 x 24-bit products (low 32 bits), so the device uses the
// full-rate v_mul_u32_u24 rather than the quarter-rate v_mul_lo_u32; the
// 4-byte bit folds the window's first byte into the top byte of the other 3.
// (Both bits over all 32 from the high halves of 24-bit products -- 6 instead
// of 12 instructions per deferred hit -- measured config C's kernel 3 % slower
// in one-process A/B, profiles/r04_ab_inproc.json.)
__host__ __device__ inline uint32_t fl_mul24(uint32_t a, uint32_t b) {
  return (a & 0xFFFFFFu) * (b & 0xFFFFFFu);
}
__host__ __device__ inline uint32_t fl_word(uint32_t w4) {
  return fl_mul24(w4 >> 8, 0x9E3779u) >> (32 - kExactFlLog2);
}
// 3-byte keys in bits 0..15, 4-byte keys in 16..31
__host__ __device__ inline uint32_t fl_bit3(uint32_t w4) { return fl_mul24(w4 >> 8, 0xEBCA77u) >> 28; }
__host__ __device__ inline uint32_t fl_bit4(uint32_t w4) {
  return 16u + (fl_mul24((w4 >> 8) ^ (w4 << 16), 0xB2AE35u) >> 28);
}

__host__ __device__ inline uint32_t bucket_hash1(uint32_t key) {
  uint32_t h = key * 0x9E3779B1u;
  return h ^ (h >> 16);
}
__host__ __device__ inline uint32_t bucket_hash2(uint32_t key) {
  uint32_t h = (key ^ 0x5BD1E995u) * 0x85EBCA77u;
  return h ^ (h >> 13);
}

// Accepting trie nodes by string, for the pre-verification kernels (one
// uint32 array): [0, 256) head of the 1-byte node b (0 = none), [256, 65792)
// head of the 2-byte node (little endian), then two-choice bucketed tables of
// the 3- and 4-byte nodes, 2 entries {key, head} per 16-byte bucket (3-byte
// keys carry 1 << 24; 0 = empty; the 4-byte node 0x00000000 sits in word
// kNodeZero4).  head = M[slot], the 1-based pool index of the node's list.
constexpr uint32_t kNodeL1 = 0;
constexpr uint32_t kNodeL2 = 256;
constexpr uint32_t kNodeZero4 = 256 + 65536;
constexpr uint32_t kNodeHeadWords = kNodeZero4 + 4;   // (keeps the buckets 16-B aligned)

// The class of a certain candidate (kernels.hip key_class, decided in the
// compaction; ScanParams::dead holds it per candidate): 0 = undecided, 1 = no
// call of its list can have an effect, 2 | k << 2 = every call of 1-byte key
// k's list is kept (ScanParams::kd_n / kd_head).  The scan keeps five bytes
// next to a certain candidate's key: four in ScanParams::seg_x, and its
// segment output entry (offset below 2^20, the bits of its pending entry)
// holds the fifth byte in bits kOutByteShift.., the key's place among the five
// + 2 (1: just before them; 0: not a certain candidate) in bits
// kOutKeyShift.., and with ScanParams::kx_deep kOutDeep: the byte before the
// key is one of key 0's exclusions (kd_x0 / kd_x1).
constexpr uint32_t kOutByteShift = 20;
constexpr uint32_t kOutKeyShift = 28;
constexpr uint32_t kOutDeep = 0x80000000u;
constexpr uint32_t kOutOffsetMask = (1u << 20) - 1u;
constexpr uint32_t kClassDead = 1u;
constexpr uint32_t kClassKept = 2u;
constexpr uint32_t kClassFetch = 0xFFu;   // (verified-only scans) undecided from the scan's
                                          // eight bytes: the compaction reads the input
constexpr uint32_t kOutPlaceScanClass = 7u;   // key place of an entry carrying its class
// ScanParams::kc: 32 words of key class records (8 per key), then the plan of
// the one-plan drop instance (scanner.cpp key_plan): info, the one compared
// byte's value replicated to four bytes, its shift in byte_test24's mask
constexpr uint32_t kKcPlan = 32;
constexpr uint32_t kKcWords = 36;

struct ScanParams {
  const uint8_t* data;      // block base in HBM (16-byte aligned)
  uint64_t block_size;      // bytes in the block
  uint64_t byte_begin;      // first byte of this launch (multiple of 16)
  uint64_t byte_end;        // one past the last byte
  const uint32_t* filter;   // kFilterWords words
  const uint32_t* exact;    // exact key sets (layout above)
  uint32_t t3_off, t3_mask; // word offset / bucket-count mask of the 3-byte table
  uint32_t t4_off, t4_mask; // same for the 4-byte table
  uint32_t exact_flags;     // kExactZero4
  uint32_t len_mask;        // bit L set iff keys of length L exist
  uint32_t n_segments;
  uint32_t seg_bytes;       // bytes per segment (multiple of kTile)
  uint32_t seg_cap;         // output capacity (entries) per segment
  uint32_t* seg_count;      // [n_segments] candidates found (may exceed cap)
  uint32_t* seg_out;        // [n_segments * seg_cap] byte offset within segment
  const uint64_t* seg_base; // null: segment s writes at seg_out + s * seg_cap; else at
                            // seg_out + seg_base[s] (exact-size rerun after an overflow)
  uint32_t byte_keys;       // FlatTables::byte_keys / n_byte_keys (stage-1 byte test)
  uint32_t n_byte_keys;
  // Per 1-byte key k: the guard that decides every call of the key's match
  // list from the bytes next to it (scanner.cpp key_dead_guards): m, v and info
  // = valid | has-exclusions << 1 | kept-list << 2 | region start relative to the key byte
  // (int8) << 8 | span << 16 | last tested byte of the 4 << 20 | region end
  // relative to the position (int8) << 24; info 0 = none
  uint32_t kd_m[4], kd_v[4], kd_info[4];
  // with info bit 1: the bytes before the key (up to 8, repeated to fill) after
  // which a deeper state ends at the key -- such candidates are not decided
  uint32_t kd_x0[4], kd_x1[4];
  // with info bit 2 ("kept" keys: every call of the list is kept whatever the
  // bytes): the list's length and head, and the smallest position at which
  // every call is made (the largest backtrack, scanner.c:107)
  uint32_t kd_n[4], kd_head[4], kd_min_pos[4];
  // with info bit 3 (guard-decided keys): a backward guard too -- the bytes
  // before the key that the call's backward program tests first: mask / value
  // (shifted so that their lowest tested byte is byte 0) in fields 6 and 7 of
  // the key's record in kc (below), and in kd_min_pos (unused by such keys)
  // the first tested byte relative to the key byte (int8) | last tested byte
  // << 12 (guards at one position only)
  uint32_t* seg_x;          // null, or beside seg_out: a certain candidate's first four
                            // bytes (lane bytes s .. s + 3, s = min(key + kx_end - 3, 11))
  uint32_t kx_end;          // 2..4 (scanner.cpp key_classes)
  uint32_t kx_deep;         // 1: the scan tests the byte before the key (one 1-byte key)
  uint32_t kx_next;         // 1: guard-decided keys -- the byte-key kernel that keeps the
                            // next lane's first two bytes in each ring entry (kernels.hip)
  uint8_t* dead;            // null, or per output candidate its class (key_class;
                            // written by the compaction), and
  uint32_t* live;           // per segment s, in [seg_offset[s], + live_count[s]): the indices
                            // of its other candidates (any order)
  uint32_t* live_count;     // [n_segments]
  uint32_t filter_mode;     // kFilterPair / kFilterEven / kFilterEvenHash (FlatTables)
  uint32_t pair_keys[2];    // even filters: FlatTables::pair_keys / n_pair_keys (16-bit
  uint32_t n_pair_keys;     // test of the 2-byte keys ending at odd positions)
  uint32_t* seg_next;       // null: wave w takes segments w, w + waves, ...; else each wave
                            // takes its first segment by index and the next ones from this
                            // counter (initialised to the launch's wave count)
  // Verified-only scans (yr_amd_scanner_set_verified_only; byte-key kernels
  // with candidate classes): the scan decides each certain candidate's class
  // from eight bytes around its key (kernels.hip resolve_pending) and leaves
  // the dead ones out of the output.  Output entries of certain candidates
  // then carry the class code in bits kOutByteShift.. (kClassFetch: let the
  // compaction read the input) with key place 7, seg_x holds each output
  // candidate's index in the segment's FULL stream, seg_full[s] the length of
  // that stream, and the compaction writes the full stream's global index of
  // every output candidate into cand_index (only if some candidate was left
  // out: seg_full_offset[n_segments] != the output total).
  uint32_t drop_dead;
  uint32_t kd_bguard;       // some key has a backward guard (info bit 3)
  const uint32_t* kc;       // [32]: key k's class record (kd_info, kd_m, kd_v, kd_x0, kd_x1,
                            // kd_min_pos, kd_bm, kd_bv) at [8k, 8k + 8) -- the scan kernel reads it
                            // into one VGPR and fetches fields by lane permutes
  uint32_t* seg_full;
  uint64_t* seg_full_offset;   // [n_segments + 1], written by the offsets kernel
  uint32_t* cand_index;
  // The one-plan drop instance (kernels.hip kDropPlanModes; scanner.cpp
  // key_plan): every 1-byte key's class is the same forward guard once the
  // test of the key byte itself is left out (rx: both keys test the byte after
  // them against 0xC3), so the drain decides all certain candidates of an
  // entry at once, in straight-line code -- not per key from the records.  The
  // plan's words follow the records in kc (kKcPlan..): read by scalar loads in
  // each drain, so they hold no SGPRs across the tile loop.
  uint32_t kp_on;
};

}  // namespace yamd
