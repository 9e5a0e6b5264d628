// Device data of the on-device literal pre-verification (verify.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace yamd {

// YR_STRING.flags bits (libyara/include/yara/types.h:66-88).
constexpr uint32_t kStrNoCase = 0x04;
constexpr uint32_t kStrAscii = 0x08;
constexpr uint32_t kStrWide = 0x10;
constexpr uint32_t kStrFullWord = 0x80;
constexpr uint32_t kStrLiteral = 0x400;
constexpr uint32_t kStrFitsInAtom = 0x800;
constexpr uint32_t kStrFixedOffset = 0x8000;
constexpr uint32_t kStrXor = 0x80000;
// literal flags whose comparison is not restated on the device: such calls
// are always handed to the host (base64 / base64wide)
constexpr uint32_t kStrUnmodelled = 0x200000 | 0x400000;

constexpr uint32_t kStrFastRegexp = 0x40;
constexpr uint32_t kStrDotAll = 0x20000;
// DevPoolRec.flags only (above every STRING_FLAGS_* bit, types.h:66-88): the
// entry's yr_re_exec forward program provably cannot fail with
// ERROR_TOO_MANY_RE_FIBERS (scanner.cpp re_fiber_safe), so a failing backward
// guard decides the call without running the forward search first
constexpr uint32_t kPoolFwdFiberSafe = 0x80000000u;
constexpr uint32_t kStrBase64Any = 0x200000 | 0x400000;

// Fast-exec RE programs (hex strings) of one pool entry: forward code at
// re_code[fwd_off, +fwd_len), backward code likewise; fwd_len == 0 = none.
struct DevRe {
  uint32_t fwd_off, fwd_len, bwd_off, bwd_len;
};

// re.c opcodes of the fast executor (libyara/include/yara/re.h:65-92).
constexpr uint8_t kReAny = 0xA0, kReLiteral = 0xA2, kReMaskedLiteral = 0xA4, kReMatch = 0xAD,
                  kReNotLiteral = 0xAE, kReMaskedNotLiteral = 0xAF, kReRepeatAnyUngreedy = 0xB5;
constexpr int kReScanLimit = 4096;   // YR_RE_SCAN_LIMIT (limits.h:163)

// A necessary condition of a fast-exec program matching, computed on the host
// from its opcodes (scanner.cpp fast_guard): with x_b the b-th input byte the
// program reads (forwards x_b = data[offset + b], backwards data[offset - 1 -
// b]), some j in [0, span] has (x_{base + j + t} & m_t) == v_t for t = 0..3
// (m_t, v_t = byte t of m, v; forwards in program order, backwards in memory
// order, i.e. byte 3 - t).  The positions are 4 consecutive bytes the program
// must consume at a fixed distance (span 0: its first run of literal / masked /
// any opcodes), or right after its first REPEAT_ANY {min, max} (base = the
// run before it + min, span = max - min).  m == 0: no guard.
struct DevGuard {
  uint32_t m, v;
};

// One pool entry (YR_AC_MATCH, types.h:324-344) with everything a verify call
// reads about it -- list link, backtrack, its YR_STRING's fields, its regexp
// programs and their guards -- in one 64-byte record, so walking a list costs
// one memory round trip per entry (four independent 16-byte loads).
struct DevPoolRec {
  uint32_t next;          // 1-based pool index of ac_match_pool[k].next, 0 = end
  uint16_t backtrack;     // YR_AC_MATCH.backtrack (uint16_t, types.h:330)
  uint8_t fguard_bs;      // forward guard: base | span << 4 (DevGuard)
  uint8_t bguard_bs;      // backward guard
  uint32_t flags;         // YR_STRING.flags
  uint32_t length;        // YR_STRING.length
  int64_t fixed_offset;   // YR_STRING.fixed_offset
  uint64_t bytes_off;     // YR_STRING.string in the byte blob
  DevRe re;               // regexp programs (fwd_len 0: none)
  DevGuard fguard, bguard;
};
static_assert(sizeof(DevPoolRec) == 64, "pool record layout");

// Same layout as yr_amd_verify_rec (include/yara_amd.h).
struct VerifyRec {
  uint64_t offset;
  uint32_t pool_index;
  uint32_t candidate;
};

struct VerifyParams {
  const uint8_t* data;        // block in HBM (position 0; only [win_lo, win_hi) is read)
  uint64_t size;              // block size
  uint64_t win_lo, win_hi;    // the bytes of the block present in HBM (yr_amd_scan_window)
  uint64_t data_base;         // YR_MEMORY_BLOCK.base (fixed-offset strings)
  const uint64_t* positions;  // ascending candidates (unused when all)
  const uint8_t* dead;        // null, or per candidate 1 = the scan proved no call of its
                              // list can have an effect (ScanParams::dead), and
  const uint32_t* live;       // per scan segment s: its other candidates' indices in
                              // [live_first[s], + live_count[s]) (ScanParams::live)
  const uint32_t* live_count; // [live_segs]
  const uint64_t* live_first; // [live_segs] the segments' first candidate
  uint32_t live_segs;
  uint64_t* live_off;         // [live_segs + 1] workspace: the lists' offsets in live_dense, total
  uint32_t* live_dense;       // [count] workspace: the lists concatenated
  int direct;                 // pass 1 as a grid of one wave per group without LDS
                              // (verify_write_kernel: records in most groups, the "kept"
                              // 1-byte keys; lists of at most 31 entries, no profiling)
                              // instead of persistent waves
  const uint32_t* cand_index; // null, or per candidate its index in the scan's full stream
                              // (verified-only scans that left candidates out): the
                              // records' candidate field
  uint32_t kd_n[4], kd_head[4];   // the "kept" keys' list lengths and heads (ScanParams)
  // the first kKeptDirect entries of each "kept" key's list: 0-based pool index
  // and backtrack (pass 1 writes such a candidate's records without the pool)
  uint32_t kd_idx[4][4], kd_bt[4][4];
  uint64_t count;             // candidates (size + 1 when all)
  int all;                    // every position of a range is a candidate:
  uint64_t all_first;         //   i = all_first + c
  const uint32_t* nodes;      // accepting trie nodes by string (internal.h kNode*)
  uint32_t n3_off, n3_mask, n4_off, n4_mask;
  uint32_t root_head;         // ac_match_table[0]
  const DevPoolRec* pool;     // per pool entry
  const uint8_t* str_bytes;
  const uint8_t* lowercase;   // the host's yr_lowercase[256]
  int re_on;                  // regexp programs attached (else every regexp call is kept)
  int profile;                // yr_amd_tables_set_profiling: dropped calls that stock
                              // libyara's profiling counts come out as count-only records
  const uint8_t* re_code;
  uint32_t* counts;           // [count] records per candidate (pass 0)
  uint32_t* keep;             // [count] pass 0's decisions for pass 1: bit t = the t-th
                              // entry of the candidate's list is kept (t < 31); bit 31 =
                              // the list is longer, pass 1 decides again
  uint32_t* heads;            // [count] the candidate's match-list head M[state] (pass 0)
  uint64_t* block_off;        // [verify_groups(count) + 1] pass 0: records per group of
                              // kGroup candidates; then (launch_block_offsets) exclusive
                              // offsets within the group's chunk of kChunkGroups
  uint64_t* chunk_off;        // [verify_chunks(count) + 1] the chunks' exclusive offsets, total
  VerifyRec* out;             // records (pass 1)
  uint64_t out_cap;           // records that fit in out; pass 1 drops the rest (the
                              // host re-runs it when the total turns out larger)
  uint64_t first;             // pass 0: the launch's first candidate (launch_verify
                              // slices the stream: a dispatch holds < 2^32 work-items)
};

hipError_t launch_verify(const VerifyParams& p, int pass, hipStream_t s);
// Pass 0 over the scan's live lists (p.live; block_off zeroed): the dead
// candidates keep nothing and are never read.
hipError_t launch_verify_live(const VerifyParams& p, uint64_t* summary, hipStream_t s);
// The "kept" keys' list lengths (the class byte's key index): their records
// count into the group totals without pass 0.
constexpr uint32_t kKeptDirect = 4;
struct KeptLists {
  uint32_t n[4];
};
hipError_t launch_block_offsets(uint64_t* block_off, uint64_t* chunk_off, uint64_t count,
                                uint64_t* total, const uint8_t* cls, const KeptLists& kept,
                                hipStream_t s);
constexpr uint64_t kGroup = 64;           // candidates per group (one wave)
constexpr uint64_t kChunkGroups = 256;    // groups per chunk of the offsets scan (4 threads each)
uint64_t verify_groups(uint64_t count);
uint64_t verify_chunks(uint64_t count);

}  // namespace yamd
