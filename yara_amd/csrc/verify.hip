// gfx950 kernels of the on-device pre-verification.
//
// Input: the candidate stream of a block scan (ascending positions i with
// ac_match_table[state_i] != 0).  For every candidate the reference loop
// (libyara/scanner.c:98-122, :144-163) calls
//     yr_scan_verify_match(ctx, m, data, size, base, i - m->backtrack)
// for each entry m of state_i's match list with backtrack <= i.  For a literal
// string (STRING_FLAGS_LITERAL) that call is a pure function of the bytes
// until the comparison succeeds: yr_scan_verify_match (scan.c:992-1089) only
// returns early, and _yr_scan_verify_literal_match (scan.c:887-990) returns
// ERROR_SUCCESS without touching the scan context when forward_matches == 0.
// These kernels evaluate exactly that comparison on the GPU and emit the
// calls that can have an effect -- every call on a non-literal string (regex /
// hex with jumps, unless its fast-exec program provably cannot match: see
// fast_re_reachable), and every literal call whose comparison succeeds -- as
// {offset, pool index} records in the reference's call order.  The host
// replays the records into the unmodified yr_scan_verify_match, so the final
// match set is unchanged while the host no longer walks lists, compares bytes
// or runs re.c for the (vast majority of) candidates that are atom hits only.
//
// Work per candidate (one lane each): recompute state_i by the reference
// transition rule from max(0, i - 4) (the trie is at most 4 deep, limits.h:68),
// walk the pool list, compare.  Candidates are ~0.015% of positions (config
// C): this is latency-bound pointer chasing in L2, microseconds per block, so
// the kernels are simple two-pass (count, exclusive scan, write).
#include <mutex>
#include <vector>

#include "internal.h"
#include "re_program.h"
#include "verify.h"

namespace yamd {

// The match-list head of the walk's state at candidate position i
// (libyara/scanner.c:98, :144: ac_match_table[state]).  The trie is at most 4
// deep (limits.h:68), so the state after data[0..i) is the longest suffix of
// data[i-4..i) that is a trie node; at a candidate that node accepts, and so
// it is the longest ACCEPTING suffix (acceptance is monotone along suffixes,
// tables.cpp).  The four suffixes are looked up in the accepting-node tables
// (internal.h kNode*) with independent loads -- one memory round trip instead
// of four dependent transitions (scanner.c:124-141).  No accepting suffix:
// the root (a root-accepting rule set, every position a candidate).
__device__ __forceinline__ bool node_bucket_get(const uint4& b, uint32_t key, uint32_t& head) {
  if (b.x == key) { head = b.y; return true; }
  if (b.z == key) { head = b.w; return true; }
  return false;
}
#ifndef YAMD_VERIFY_DIAG
#define YAMD_VERIFY_DIAG 0   // profiling builds only: 1 = decide nothing, 2 = no regex decisions,
                             // 3 = positions only, 4 = + list heads, 5 = 4 with the data
                             // read only, 6 = 4 without the data read
#endif

// The 8 block bytes [a, a + 8) around a candidate that node_head loads anyway
// (a = (i - 4) & ~3: at least the 4 bytes before i and byte i itself), kept
// for the guards (guard_ok): most calls of a dense rule set are decided by a
// guard whose tested bytes lie there, with no further memory access.
struct Near {
  uint64_t a;   // block position of byte 0; kNoNear: not loaded
  uint64_t v;   // the 8 bytes, little endian
};
constexpr uint64_t kNoNear = ~0ull;

__device__ __forceinline__ uint32_t node_head(const VerifyParams& p, uint64_t i, Near& near) {
  const uint32_t n = i < 4 ? (uint32_t)i : 4u;
  uint32_t w = 0;   // data[i-n .. i), oldest byte lowest, at the top (bytes i-4.. i-1)
  const uint64_t a = (i - 4) & ~3ull;   // p.data is 16-byte aligned
  near.a = kNoNear;
  if (i >= 4 && a >= p.win_lo && a + 8 <= p.win_hi) {
    // one 8-byte load (4 byte loads per lane cost 2-3x the time: the random
    // reads of the candidates' neighbourhoods are the count pass's largest item)
    const uint2 v = *reinterpret_cast<const uint2*>(p.data + a);
    near.a = a;
    near.v = (uint64_t)v.x | ((uint64_t)v.y << 32);
    w = __builtin_amdgcn_alignbyte(v.y, v.x, (uint32_t)(i - 4 - a));
  } else {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
      if (j < n) w |= (uint32_t)p.data[i - n + j] << (8 * (4 - n + j));
  }
#if YAMD_VERIFY_DIAG == 5
  return w | 1u;   // profiling: the data read only
#elif YAMD_VERIFY_DIAG == 6
  w = (uint32_t)i * 2654435761u;   // profiling: the probes without the data read
#endif
  const uint32_t k1 = w >> 24, k2 = w >> 16, k3 = (w >> 8) | (1u << 24), k4 = w;
  const uint32_t* __restrict__ t = p.nodes;
  const uint32_t h1 = n >= 1 ? t[kNodeL1 + k1] : 0u;
  const uint32_t h2 = n >= 2 ? t[kNodeL2 + k2] : 0u;
  uint4 a3 = make_uint4(0, 0, 0, 0), b3 = a3, a4 = a3, b4 = a3;
  if (n >= 3) {
    a3 = *reinterpret_cast<const uint4*>(t + p.n3_off + (bucket_hash1(k3) & p.n3_mask) * 4);
    b3 = *reinterpret_cast<const uint4*>(t + p.n3_off + (bucket_hash2(k3) & p.n3_mask) * 4);
  }
  if (n >= 4 && k4 != 0) {
    a4 = *reinterpret_cast<const uint4*>(t + p.n4_off + (bucket_hash1(k4) & p.n4_mask) * 4);
    b4 = *reinterpret_cast<const uint4*>(t + p.n4_off + (bucket_hash2(k4) & p.n4_mask) * 4);
  }
  uint32_t head;
  if (n >= 4) {
    if (k4 == 0) {
      if (t[kNodeZero4]) return t[kNodeZero4];
    } else if (node_bucket_get(a4, k4, head) || node_bucket_get(b4, k4, head)) {
      return head;
    }
  }
  if (n >= 3 && (node_bucket_get(a3, k3, head) || node_bucket_get(b3, k3, head))) return head;
  if (h2) return h2;
  if (h1) return h1;
  return p.root_head;
}

// yr_re_fast_exec (re.c:2150-2391) as a reachability question: is MATCH
// reachable from bytes_matched = 0?  The reference runs the linear program
// over a list of input positions; here a depth-first search over the choices
// of RE_OPCODE_REPEAT_ANY_UNGREEDY (b -> b + min unconditionally, b + j for
// min < j <= max while b + j < max_bytes_matched) with every consuming opcode
// requiring b < max_bytes_matched.  "Exists a path" semantics, i.e. a superset
// of what the reference's de-duplicating list reaches; out of stack or step
// budget -> true (keep the call).
// The input bytes a fast program can touch first, staged in LDS: the search
// reads them one at a time, each read depending on the previous one's outcome,
// so reading them from HBM would cost one memory round trip per byte.  One
// window per lane: 48 bytes from three aligned 16-byte loads (issued together),
// covering the 32 bytes after (forward) or before (backward) the start; reads
// outside it, or any read when the window would leave the block, go to memory.
constexpr int kWinBytes = 48;
#ifndef YAMD_STAGE_STR
#define YAMD_STAGE_STR 1
#endif
constexpr uint32_t kCodeBytes = 48;   // (stage_code, stage_str: a second buffer per lane)
constexpr uint32_t kNoLds = 0xFFFFFFFFu;
struct ByteWindow {
  const uint8_t* lo;   // block address of window byte 0 (null: no window)
  uint32_t lds;        // LDS byte address of this lane's window
};
__device__ __forceinline__ ByteWindow stage_window(const VerifyParams& p, const uint8_t* start,
                                                   bool backwards, uint32_t lds) {
  const uint8_t* s = backwards ? start - 32 : start;
  const uint8_t* lo = reinterpret_cast<const uint8_t*>((uintptr_t)s & ~(uintptr_t)15);
  if (lds == 0xFFFFFFFFu || lo < p.data + p.win_lo || lo + kWinBytes > p.data + p.win_hi)
    return {nullptr, lds};
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* g = reinterpret_cast<const u32x4*>(lo);
  const u32x4 a = g[0], b = g[1], c = g[2];
  typedef __attribute__((address_space(3))) u32x4 lds_u4;
  reinterpret_cast<lds_u4*>((uintptr_t)lds)[0] = a;
  reinterpret_cast<lds_u4*>((uintptr_t)lds)[1] = b;
  reinterpret_cast<lds_u4*>((uintptr_t)lds)[2] = c;
  return {lo, lds};
}
__device__ __forceinline__ uint8_t window_byte(const ByteWindow& w, const uint8_t* at) {
  if (w.lo != nullptr && at >= w.lo && at < w.lo + kWinBytes)
    return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(
        (uintptr_t)(w.lds + (uint32_t)(at - w.lo)));
  return *at;
}

// The input bytes of one regexp direction through the staged window with
// 32-bit offsets: byte b (0, 1, ... away from the call's offset, backwards
// or forwards) is window byte rel0 + b (forwards) or rel0 - 1 - b
// (backwards); outside the window it is read from memory.  (window_byte's
// 64-bit pointer compares cost several VOP3 instructions per byte.)
struct DirWindow {
  int32_t rel0;   // window index of input[0]
  uint32_t lds;
  const uint8_t* input;
  bool backwards;
  __device__ DirWindow(const ByteWindow& w, const uint8_t* in, bool bw)
      : rel0(w.lo != nullptr ? (int32_t)(in - w.lo) : -(1 << 30)), lds(w.lds), input(in),
        backwards(bw) {}
  __device__ uint8_t operator()(int b) const {
    const int32_t k = backwards ? rel0 - 1 - b : rel0 + b;
    if ((uint32_t)k < (uint32_t)kWinBytes)
      return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(
          (uintptr_t)(lds + (uint32_t)k));
    return backwards ? input[-1 - b] : input[b];
  }
};

// A literal's string bytes for the comparisons below: its first bytes staged
// like the input window -- three aligned 16-byte loads into this lane's code
// buffer (a literal call stages no regexp code), issued with the window's --
// so a comparison that runs past the atom's bytes costs no dependent load per
// character.  (The string blob carries kCodeBytes of padding: the aligned
// loads never leave it.)
struct StrBytes {
  const uint8_t* s;
  uint32_t lds;   // LDS address of string byte 0 (kNoLds: none staged)
  uint32_t n;     // bytes staged from s on
};
__device__ __forceinline__ StrBytes stage_str(const uint8_t* s, uint32_t buf) {
  if (buf == kNoLds) return {s, kNoLds, 0u};
  const uintptr_t a = (uintptr_t)s, lo = a & ~(uintptr_t)15;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* g = reinterpret_cast<const u32x4*>(lo);
  const u32x4 c0 = g[0], c1 = g[1], c2 = g[2];
  typedef __attribute__((address_space(3))) u32x4 lds_u4;
  lds_u4* d = reinterpret_cast<lds_u4*>((uintptr_t)buf);
  d[0] = c0;
  d[1] = c1;
  d[2] = c2;
  const uint32_t head = (uint32_t)(a - lo);
  return {s, buf + head, kCodeBytes - head};
}
__device__ __forceinline__ uint8_t str_byte(const StrBytes& t, uint32_t i) {
  if (i < t.n)
    return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>((uintptr_t)(t.lds + i));
  return t.s[i];
}

// _yr_scan_compare / _yr_scan_icompare (scan.c:142-179): forward match length
// of the ascii form, 0 if none.
__device__ bool cmp_ascii(const uint8_t* d, uint64_t avail, const StrBytes& s, uint32_t n,
                          const uint8_t* lower, const ByteWindow& w) {
  if (avail < n) return false;
  if (lower == nullptr) {
    for (uint32_t i = 0; i < n; ++i)
      if (window_byte(w, d + i) != str_byte(s, i)) return false;
  } else {
    for (uint32_t i = 0; i < n; ++i)
      if (lower[window_byte(w, d + i)] != lower[str_byte(s, i)]) return false;
  }
  return true;
}

// _yr_scan_wcompare / _yr_scan_wicompare (scan.c:181-255): the wide form
// (every character followed by 0x00).
__device__ bool cmp_wide(const uint8_t* d, uint64_t avail, const StrBytes& s, uint32_t n,
                         const uint8_t* lower, const ByteWindow& w) {
  if (avail < 2ull * n) return false;
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t a = window_byte(w, d + 2 * i), b = str_byte(s, i);
    if ((lower == nullptr ? a != b : lower[a] != lower[b]) || window_byte(w, d + 2 * i + 1) != 0)
      return false;
  }
  return true;
}

// _yr_scan_xor_compare (scan.c:62-101) and _yr_scan_xor_wcompare (:103-140):
// key k = data[0] ^ string[0], then every byte (and, wide, every 0x00 ^ k).
__device__ bool cmp_xor(const uint8_t* d, uint64_t avail, const StrBytes& s, uint32_t n, bool wide,
                        const ByteWindow& w) {
  if (avail < (wide ? 2ull * n : (uint64_t)n)) return false;
  if (n == 0) return false;   // both reference loops yield 0 for an empty string
  const uint8_t k = window_byte(w, d) ^ str_byte(s, 0);
  for (uint32_t i = 0; i < n; ++i) {
    if (wide) {
      if (window_byte(w, d + 2 * i) != (uint8_t)(str_byte(s, i) ^ k) ||
          (uint8_t)(window_byte(w, d + 2 * i + 1) ^ k) != 0)
        return false;
    } else if (window_byte(w, d + i) != (uint8_t)(str_byte(s, i) ^ k)) {
      return false;
    }
  }
  return true;
}


// Regexp code, read either from the blob in global memory or from this lane's
// LDS copy (stage_code): typed LDS reads (ds_read_u8) rather than flat ones,
// whose waits also cover every outstanding global load.
struct GlobalCode {
  const uint8_t* __restrict__ p;
  __device__ uint8_t operator[](uint32_t i) const { return p[i]; }
};
struct LdsCode {
  uint32_t a;   // LDS byte address
  __device__ uint8_t operator[](uint32_t i) const {
    return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>((uintptr_t)(a + i));
  }
};

template <class Code>
__device__ bool fast_re_reachable(const Code code, uint32_t len,
                                  const uint8_t* __restrict__ input, uint64_t avail,
                                  bool backwards, const ByteWindow& win) {
  constexpr int kMaxChoices = 8;
  struct Choice {
    uint32_t ip;
    int b, j, jmax;
  } st[kMaxChoices];
  int sp = 0;
  const int maxb = (int)min<uint64_t>(avail, (uint64_t)kReScanLimit);
  uint32_t ip = 0;
  int b = 0;
  for (int budget = 0; budget < 8192; ++budget) {
    if (ip >= len) return true;
    const uint8_t op = code[ip];
    if (op == kReMatch) return true;
    bool ok = false;
    if (b < maxb) {
      const uint8_t c = window_byte(win, backwards ? input - 1 - b : input + b);
      switch (op) {
        case kReAny: ok = true; ip += 1; break;
        case kReLiteral: ok = c == code[ip + 1]; ip += 2; break;
        case kReNotLiteral: ok = c != code[ip + 1]; ip += 2; break;
        case kReMaskedLiteral: ok = (c & code[ip + 2]) == code[ip + 1]; ip += 3; break;
        case kReMaskedNotLiteral: ok = (c & code[ip + 2]) != code[ip + 1]; ip += 3; break;
        case kReRepeatAnyUngreedy: {
          const int mn = code[ip + 1] | (code[ip + 2] << 8);
          const int mx = code[ip + 3] | (code[ip + 4] << 8);
          ip += 5;
          const int jmax = min(mx, maxb - 1 - b);
          if (mn + 1 <= jmax) {
            if (sp == kMaxChoices) return true;
            st[sp++] = Choice{ip, b, mn + 1, jmax};
          }
          b += mn;
          continue;   // position advanced by min, unconditionally
        }
        default: return true;   // not a fast program
      }
      if (ok) {
        b += 1;
        continue;
      }
    }
    // dead position: resume the most recent open choice
    if (sp == 0) return false;
    Choice& t = st[sp - 1];
    ip = t.ip;
    b = t.b + t.j;
    if (++t.j > t.jmax) --sp;
  }
  return true;
}

// The same question in the oracle's set form (oracle/ac_oracle.c
// fast_re_reachable): the set of bytes_matched values reachable before each
// opcode, kept as a 64-bit window m over [base, base + 64).  A consuming
// opcode tests the bytes of every live element (b < max_bytes_matched) --
// independent LDS reads, no choice stack -- and a REPEAT_ANY {min, max} maps
// b -> b + min and b + j (min < j <= max, b + j < max_bytes_matched).
// Returns 0 = no path reaches MATCH, 1 = some path does, 2 = the set would
// leave the window or come near YR_RE_SCAN_LIMIT, or an opcode outside the
// fast set: the caller then runs the depth-first search, whose answer this
// form equals wherever it answers.
template <class Code>
__device__ int fast_re_set(const Code code, uint32_t len, const uint8_t* __restrict__ input,
                           uint64_t avail, bool backwards, const ByteWindow& win) {
  const int maxb = (int)min<uint64_t>(avail, (uint64_t)kReScanLimit);
  const DirWindow in(win, input, backwards);
  int base = 0;
  uint64_t m = 1;
  uint32_t ip = 0;
  // Lanes interpret different programs, so the opcode kinds differ across the
  // wave: every byte test is one branch-free form, (c & mask) == val, negated
  // for the NOT forms, and the operand bytes are read together with the
  // opcode (independent LDS reads; the blob and the staging buffer are padded).
  while (ip < len) {
    const uint8_t op = code[ip], b1 = code[ip + 1], b2 = code[ip + 2];
    if (op == kReMatch) return m != 0 ? 1 : 0;
    const int lim = maxb - base;   // bits i < lim are live (b < max_bytes_matched)
    const uint64_t live = lim >= 64 ? m : (lim <= 0 ? 0ull : m & ((1ull << lim) - 1));
    if (live == 0) return 0;
    if (op == kReRepeatAnyUngreedy) {
      const int mn = b1 | (b2 << 8);
      const int mx = code[ip + 3] | (code[ip + 4] << 8);
      const int lo = __builtin_ctzll(live), hi = 63 - __builtin_clzll(live);
      const int span = hi - lo + (mx - mn);
      const int nb = base + lo + mn;
      if (span > 63 || nb + span >= kReScanLimit) return 2;
      // t | t << 1 | ... | t << (mx - mn), by doubling
      uint64_t acc = live >> lo;
      const int r = mx - mn + 1;   // copies
      int have = 1;
      while (2 * have <= r) {
        acc |= acc << have;
        have *= 2;
      }
      if (have < r) acc |= acc << (r - have);
      const int lim2 = maxb - nb;
      acc &= lim2 >= 64 ? ~0ull : (lim2 <= 0 ? 0ull : (1ull << lim2) - 1);
      m = acc;
      base = nb;
      ip += 5;
      continue;
    }
    uint32_t mask, val, sz;
    bool neg = false;
    switch (op) {
      case kReAny: mask = 0; val = 0; sz = 1; break;
      case kReLiteral: mask = 0xFF; val = b1; sz = 2; break;
      case kReNotLiteral: mask = 0xFF; val = b1; sz = 2; neg = true; break;
      case kReMaskedLiteral: mask = b2; val = b1; sz = 3; break;
      case kReMaskedNotLiteral: mask = b2; val = b1; sz = 3; neg = true; break;
      default: return 2;
    }
    uint64_t res = 0, x = live;
    while (x) {   // live positions, four at a time (independent LDS reads)
      const int i = __builtin_ctzll(x);
      const int bb = base + i;
      uint32_t pass = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int iq = i + q;   // only live positions are read (never past the block)
        if (iq < 64 && ((x >> iq) & 1u)) {
          const uint8_t c = in(bb + q);
          pass |= (uint32_t)((((uint32_t)c & mask) == val) != neg) << q;
        }
      }
      res |= ((uint64_t)pass << i) & x;
      x &= i + 4 >= 64 ? 0ull : ~0ull << (i + 4);
    }
    if (res == 0) return 0;
    m = res;
    base += 1;
    ip += sz;
  }
  return 1;
}

// A fast program is interpreted one opcode at a time, each step depending on
// the previous one's position in the code: read from memory that is one L2
// round trip per opcode.  Programs that fit are staged first -- three
// independent 16-byte loads into this lane's kCodeBytes of LDS -- and
// interpreted from there.  (The code blob is allocated with kCodeBytes of
// padding, so the aligned loads never leave it.)
__device__ __forceinline__ uint32_t stage_code(const uint8_t* code, uint32_t len, uint32_t buf) {
  const uintptr_t a = (uintptr_t)code, lo = a & ~(uintptr_t)15;
  const uint32_t head = (uint32_t)(a - lo);
  if (buf == kNoLds || head + len > kCodeBytes) return kNoLds;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* g = reinterpret_cast<const u32x4*>(lo);
  const u32x4 c0 = g[0], c1 = g[1], c2 = g[2];
  typedef __attribute__((address_space(3))) u32x4 lds_u4;
  lds_u4* d = reinterpret_cast<lds_u4*>((uintptr_t)buf);
  d[0] = c0;
  d[1] = c1;
  d[2] = c2;
  return buf + head;
}

// scan.c:778-880 for a fast-exec string: the forward program from the call's
// offset, then (if it matched) the backward one.
template <class Code>
__device__ __forceinline__ bool fast_re_call(const VerifyParams& p, const DevRe& r, Code fwd,
                                             Code bwd, const uint8_t* d, uint64_t offset,
                                             uint32_t lds) {
  if (YAMD_VERIFY_DIAG == 8) {   // profiling: the staging loads without interpretation
    const ByteWindow w = stage_window(p, d, false, lds);
    return (window_byte(w, d) ^ fwd[0]) == 0x5Au;
  }
  if (r.fwd_len == 1)   // forward program = MATCH: forward_matches = 0
    return r.bwd_len > 0 &&
           fast_re_decide(bwd, r.bwd_len, d, offset, true, stage_window(p, d, true, lds));
  if (!fast_re_decide(fwd, r.fwd_len, d, p.size - offset, false, stage_window(p, d, false, lds)))
    return false;
  if (r.bwd_len > 0 &&
      !fast_re_decide(bwd, r.bwd_len, d, offset, true, stage_window(p, d, true, lds)))
    return false;
  return true;
}

template <class Code>
__device__ __forceinline__ bool fast_re_decide(const Code code, uint32_t len,
                                               const uint8_t* input, uint64_t avail,
                                               bool backwards, const ByteWindow& win) {
  const int v = fast_re_set(code, len, input, avail, backwards, win);
  return v == 2 ? fast_re_reachable(code, len, input, avail, backwards, win) : v == 1;
}

// yr_re_exec (re.c:1693-2072) as a reachability question: can some path from
// the program's start reach RE_OPCODE_MATCH?  Every opcode is modelled with the
// reference's own semantics: character tests (LITERAL with the host's case
// folding, NOT / MASKED literals, CLASS with yr_altercase, ANY, and \w \W \s
// \S \d \D, all locale-free in libyara: yr_isalnum, strutils.c:240-244), the
// prolog of every consuming opcode (bytes_matched < max_bytes_matched, zero
// high byte for wide input, re.c:1729-1737), REPEAT_ANY ranges with every
// repeated character passing ANY's test (re.c:1810-1821, :1584-1641),
// counted REPEAT_START / REPEAT_END loops with the fiber's counter stack
// (re.c:1533-1582), the zero-width \b \B ^ $ assertions (re.c:1937-1981),
// both branches of SPLIT and JUMP.  A reference fiber's path is one of the
// search's paths, and every path the search takes is one a fiber can take --
// except where the reference kills a fiber for re-executing a SPLIT inside one
// synchronisation (re.c:1482-1495; only loops that can match empty strings)
// -- so "no path" proves forward_matches == -1 and "a path" is exact up to
// that case.  Depth-first with an explicit choice stack (each choice keeps the
// counter stack).  Stack or step budget exhausted, deeper loop nesting than
// kReCounters, or code this search does not know -> kPathUnknown, and the
// caller keeps the call outright.  The budget (1000 steps) is below
// RE_MAX_FIBERS (1024, limits.h:168): every live reference fiber is a
// distinct reachable state, each visited by this search before it can answer
// "no path", so an exec that would fail with ERROR_TOO_MANY_RE_FIBERS
// (re.c:1228-1229, a scan error the host must still see) always exhausts it.
constexpr int kPathDead = 0, kPathMatch = 1, kPathUnknown = 2;
constexpr int kReGeneralBudget = 1000;
constexpr int kReCounters = 4;
__device__ __forceinline__ bool re_is_word(const uint8_t* ch, int cs) {   // re.c:114-122
  const uint8_t c = ch[0];
  const bool w = (c >= 0x30 && c <= 0x39) || (c >= 0x41 && c <= 0x5a) || (c >= 0x61 && c <= 0x7a) ||
                 c == '_';
  return cs == 2 ? (w && ch[1] == 0) : w;
}
__device__ int general_re_reachable(const uint8_t* __restrict__ code, uint32_t len,
                                     const uint8_t* __restrict__ input, uint64_t fwd_size,
                                     uint64_t bwd_size, bool backwards, bool wide, bool nocase,
                                     bool dotall, const uint8_t* __restrict__ lower) {
  constexpr int kMaxChoices = 16;
  struct Choice {
    int32_t ip;
    int16_t b, j, jmax;
    int8_t step, sp;
    uint16_t cnt[kReCounters];
  } st[kMaxChoices];
  int csp = 0;
  const int cs = wide ? 2 : 1;
  int maxb = (int)min<uint64_t>(backwards ? bwd_size : fwd_size, (uint64_t)kReScanLimit);
  maxb -= maxb % cs;
  int32_t ip = 0;
  int b = 0, sp = -1;
  uint16_t cnt[kReCounters] = {0, 0, 0, 0};
  // the character bytes_matched = bb reads (forward: input[bb]; backward: the
  // character ending at input - bb)
  auto at = [&](int bb) { return backwards ? input - cs - bb : input + bb; };
  auto push = [&](int32_t cip, int cb, int j, int jmax, int step) -> bool {
    if (csp == kMaxChoices) return false;
    Choice& c = st[csp++];
    c.ip = cip;
    c.b = (int16_t)cb;
    c.j = (int16_t)j;
    c.jmax = (int16_t)jmax;
    c.step = (int8_t)step;
    c.sp = (int8_t)sp;
#pragma unroll
    for (int q = 0; q < kReCounters; ++q) c.cnt[q] = cnt[q];
    return true;
  };
  for (int budget = 0; budget < kReGeneralBudget; ++budget) {
    if (ip < 0 || (uint32_t)ip >= len) return kPathUnknown;
    const uint8_t op = code[ip];
    bool dead = false;
    switch (op) {
      case kOpMatch:
        return kPathMatch;
      case kOpJump:
        ip += re_i16(code + ip + 1);
        continue;
      case kOpSplitA:
      case kOpSplitB:
        if (!push(ip + re_i16(code + ip + 2), b, 0, 0, 0)) return kPathUnknown;
        ip += 4;
        continue;
      case kOpRepeatStartGreedy:
      case kOpRepeatStartUngreedy:   // re.c:1533-1553
        if (re_u16(code + ip + 1) == 0 && !push(ip + re_i32(code + ip + 5), b, 0, 0, 0))
          return kPathUnknown;   // min == 0: the loop may be skipped (no counter)
        if (sp + 1 >= kReCounters) return kPathUnknown;
        cnt[++sp] = 0;
        ip += 9;
        continue;
      case kOpRepeatEndGreedy:
      case kOpRepeatEndUngreedy: {   // re.c:1555-1582
        if (sp < 0) return kPathUnknown;
        const int mn = re_u16(code + ip + 1), mx = re_u16(code + ip + 3);
        ++cnt[sp];
        if (cnt[sp] < mn) {
          ip += re_i32(code + ip + 5);
          continue;
        }
        if (cnt[sp] < mx && !push(ip + re_i32(code + ip + 5), b, 0, 0, 0)) return kPathUnknown;
        --sp;   // leave the loop
        ip += 9;
        continue;
      }
      case kOpWordBoundary:
      case kOpNonWordBoundary: {   // re.c:1937-1965
        bool m;
        if (b == 0 && bwd_size < (uint64_t)cs) {
          m = true;
        } else if (b >= maxb) {
          m = true;
        } else {
          const uint8_t* cur = at(b);
          m = re_is_word(cur, cs) != re_is_word(backwards ? cur + cs : cur - cs, cs);
        }
        if (op == kOpNonWordBoundary) m = !m;
        dead = !m;
        ip += 1;
        break;
      }
      case kOpMatchAtStart:   // re.c:1967-1974
        dead = backwards ? bwd_size > (uint64_t)b : (bwd_size > 0 || b != 0);
        ip += 1;
        break;
      case kOpMatchAtEnd:     // re.c:1976-1981
        dead = backwards || fwd_size > (uint64_t)b;
        ip += 1;
        break;
      case kOpRepeatAnyGreedy:
      case kOpRepeatAnyUngreedy: {   // re.c:1810-1821 + the rc spin of :1584-1641
        const int mn = re_u16(code + ip + 1), mx = re_u16(code + ip + 3);
        int k = 0;   // consecutive characters from b that pass the prolog and ANY
        while (k < mx) {
          const int bb = b + k * cs;
          if (bb >= maxb) break;
          const uint8_t* ch = at(bb);
          if ((wide && ch[1] != 0) || (!dotall && ch[0] == 0x0A)) break;
          ++k;
        }
        if (k < mn) {
          dead = true;
          break;
        }
        if (mn < k && !push(ip + 5, b, mn + 1, k, cs)) return kPathUnknown;
        b += mn * cs;
        ip += 5;
        continue;
      }
      default: {
        const uint32_t sz = re_op_size(op);
        if (sz == 0) return kPathUnknown;   // not a program this search knows
        if (b >= maxb) {
          dead = true;
          break;
        }
        const uint8_t* ch = at(b);
        if (wide && ch[1] != 0) {
          dead = true;
          break;
        }
        const uint8_t c = ch[0];
        bool ok = true;
        switch (op) {
          case kOpAny: ok = dotall || c != 0x0A; break;
          case kOpLiteral: ok = nocase ? lower[c] == lower[code[ip + 1]] : c == code[ip + 1]; break;
          case kOpNotLiteral: ok = c != code[ip + 1]; break;
          case kOpMaskedLiteral: ok = (c & code[ip + 2]) == code[ip + 1]; break;
          case kOpMaskedNotLiteral: ok = (c & code[ip + 2]) != code[ip + 1]; break;
          case kOpClass: {   // re.c:97-112 with yr_altercase (libyara.c:249-256)
            const uint8_t* bm = code + ip + 2;
            bool in = (bm[c >> 3] >> (c & 7)) & 1;
            if (nocase) {
              const uint8_t a = (c >= 'a' && c <= 'z') ? c - 32 : (c >= 'A' && c <= 'Z') ? c + 32 : c;
              in = in || ((bm[a >> 3] >> (a & 7)) & 1);
            }
            ok = code[ip + 1] ? !in : in;
            break;
          }
          case kOpWordChar: ok = re_is_word(ch, cs); break;
          case kOpNonWordChar: ok = !re_is_word(ch, cs); break;
          case kOpSpace:
          case kOpNonSpace: {   // re.c:1897-1921
            const bool sp_ = c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f';
            ok = op == kOpSpace ? sp_ : !sp_;
            break;
          }
          case kOpDigit: ok = c >= '0' && c <= '9'; break;    // isdigit, re.c:1923-1935
          case kOpNonDigit: ok = !(c >= '0' && c <= '9'); break;
          default: break;
        }
        if (!ok) {
          dead = true;
          break;
        }
        b += cs;
        ip += (int32_t)sz;
        continue;
      }
    }
    if (!dead) continue;
    if (csp == 0) return kPathDead;
    Choice& t = st[csp - 1];
    ip = t.ip;
    b = t.b + t.j * t.step;
    sp = t.sp;
#pragma unroll
    for (int q = 0; q < kReCounters; ++q) cnt[q] = t.cnt[q];
    if (++t.j > t.jmax) --csp;
  }
  return kPathUnknown;
}


// A program's guard (verify.h DevGuard; scanner.cpp fast_guard / general_guard)
// against the input: false only if no j in [0, span] passes, i.e. the program
// cannot reach MATCH.  Bytes not all
// in the block or the staged window: true (the interpreter decides).  The
// guard's 4 + span bytes come from four LDS dwords of the staged window and
// byte shifts; every j is one AND and one compare.
__device__ bool guard_ok(const VerifyParams& p, const uint8_t* d, uint64_t offset, bool backwards,
                         uint32_t bs, DevGuard g, uint32_t lds, const Near& near) {
  const uint32_t base = bs & 15u, span = bs >> 4, L = base + span + 4;
  if (backwards ? offset < L : p.size - offset < L) return true;
  const ByteWindow w = stage_window(p, d, backwards, lds);
  if (w.lo == nullptr) return true;
  const int32_t rel0 = (int32_t)(d - w.lo);
  // lowest window byte of the guard's region: forwards x_base, backwards
  // x_{base + span + 3}; the region is inside the window (base + span + 4 <= 27
  // bytes from the start, the window covers 32 from it)
  const uint32_t a = w.lds + (uint32_t)(backwards ? rel0 - (int32_t)L : rel0 + (int32_t)base);
  const uint32_t a0 = a & ~3u, sh = a & 3u;
  typedef const __attribute__((address_space(3))) uint32_t lds_u32;
  const uint32_t d0 = *reinterpret_cast<lds_u32*>((uintptr_t)a0);
  const uint32_t d1 = *reinterpret_cast<lds_u32*>((uintptr_t)(a0 + 4));
  const uint32_t d2 = *reinterpret_cast<lds_u32*>((uintptr_t)(a0 + 8));
  const uint32_t d3 = *reinterpret_cast<lds_u32*>((uintptr_t)(a0 + 12));
  const uint32_t W[3] = {__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                         __builtin_amdgcn_alignbyte(d3, d2, sh)};
  bool hit = false;
#pragma unroll
  for (uint32_t q = 0; q <= 8; ++q) {
    // region bytes q .. q + 3 (forwards j = q, backwards j = span - q)
    const uint32_t r = (q & 3) == 0 ? W[q >> 2] : __builtin_amdgcn_alignbyte(W[(q >> 2) + 1], W[q >> 2], q & 3);
    hit |= q <= span && (r & g.m) == g.v;
  }
  return hit;
}

// _yr_scan_verify_re_match (scan.c:778-880) for FAST ascii hex strings: the
// forward program from `offset` must reach MATCH (else forward_matches == -1:
// return), a zero-length forward match needs a backward program, and with a
// backward program its MATCHes are the only way to _yr_scan_match_callback.
__device__ bool re_call_matters(const VerifyParams& p, const DevPoolRec& e, uint32_t flags,
                                uint64_t offset, uint32_t lds, uint32_t codebuf, const Near& near) {
  if (YAMD_VERIFY_DIAG == 2) return true;
  if (!p.re_on) return true;
  const DevRe r = e.re;
  if (r.fwd_len == 0) return true;
  const uint8_t* d = p.data + offset;
  const uint8_t* fwd = p.re_code + r.fwd_off;
  const uint8_t* bwd = p.re_code + r.bwd_off;
  if (flags & kStrFastRegexp) {
    if (!(flags & kStrAscii) || (flags & (kStrWide | kStrBase64Any))) return true;
    // the guards first: most calls are atom hits whose next bytes already
    // rule the program out (no code staging, no interpretation)
    if (e.fguard.m != 0 && !guard_ok(p, d, offset, false, e.fguard_bs, e.fguard, lds, near)) return false;
    if (r.bwd_len > 0 && e.bguard.m != 0 &&
        !guard_ok(p, d, offset, true, e.bguard_bs, e.bguard, lds, near))
      return false;
    // forward and backward programs are contiguous in the blob (the shim and
    // yarc.cpp lay them out so): stage both at once when they fit
    if (r.bwd_len == 0 || r.bwd_off == r.fwd_off + r.fwd_len) {
      const uint32_t at = stage_code(fwd, r.fwd_len + r.bwd_len, codebuf);
      if (at != kNoLds)
        return fast_re_call(p, r, LdsCode{at}, LdsCode{at + r.fwd_len}, d, offset, lds);
    }
    return fast_re_call(p, r, GlobalCode{fwd}, GlobalCode{bwd}, d, offset, lds);
  }
  // yr_re_exec strings: the ascii attempt runs for ASCII / base64 strings, the
  // wide one (flags | RE_FLAGS_WIDE) for WIDE non-base64 strings when the
  // ascii one found nothing; the backward program runs with the flags of the
  // attempt that matched.  Keep iff some attempt can match both ways.
  const bool nocase = flags & kStrNoCase, dotall = flags & kStrDotAll;
  const bool try_ascii = flags & (kStrAscii | kStrBase64Any);
  const bool try_wide = (flags & kStrWide) && !(flags & kStrBase64Any);
  // A forward "match" here may be a reference miss, after which the wide
  // attempt runs: both branches are covered by trying every attempt.
  // The guards (host-compiled, scanner.cpp general_guard) hold for the ascii
  // attempt: a failing one proves that attempt dead in that direction without
  // running the search (and without any fiber to run out of).
  for (int w = 0; w < 2; ++w) {
    if (w == 0 ? !try_ascii : !try_wide) continue;
    if (w == 0 && e.fguard.m != 0 && !guard_ok(p, d, offset, false, e.fguard_bs, e.fguard, lds, near))
      continue;
    // a forward run that cannot fail (kPoolFwdFiberSafe) leaves the backward
    // guard to decide first: no forward search for a call it rules out
    if (w == 0 && (e.flags & kPoolFwdFiberSafe) && r.bwd_len > 0 && e.bguard.m != 0 &&
        !guard_ok(p, d, offset, true, e.bguard_bs, e.bguard, lds, near))
      continue;
    const int f = general_re_reachable(fwd, r.fwd_len, d, p.size - offset, offset, false, w == 1,
                                       nocase, dotall, p.lowercase);
    if (f == kPathUnknown) return true;
    if (f == kPathDead) continue;
    if (r.bwd_len == 0) return true;
    if (w == 0 && e.bguard.m != 0 && !guard_ok(p, d, offset, true, e.bguard_bs, e.bguard, lds, near))
      continue;
    const int b = general_re_reachable(bwd, r.bwd_len, d, p.size - offset, offset, true, w == 1,
                                       nocase, dotall, p.lowercase);
    if (b != kPathDead) return true;
  }
  return false;
}

// Does yr_scan_verify_match(ctx, &pool[k], data, size, base, offset) possibly
// have an effect?  false only where the reference provably returns without
// touching the context.
__device__ bool call_matters(const VerifyParams& p, const DevPoolRec& st, uint64_t offset,
                             uint32_t lds, uint32_t codebuf, const Near& near) {
  if (YAMD_VERIFY_DIAG == 1) return false;
  // scan.c:1013: data_size - offset <= 0 (size_t) <=> offset == size
  if (offset >= p.size) return false;
  // scan.c:1023-1025
  if ((st.flags & kStrFixedOffset) && st.fixed_offset != (int64_t)(p.data_base + offset))
    return false;
  if ((st.flags & (kStrLiteral | kStrFitsInAtom)) == (kStrLiteral | kStrFitsInAtom) &&
      !(st.flags & (kStrUnmodelled | kStrFullWord)))
    return st.backtrack != 0;   // scan.c:907-915: decided without reading data
  // Every byte the call may read lies in [offset - YR_RE_SCAN_LIMIT, offset +
  // max(YR_RE_SCAN_LIMIT, 2 * length + 2)) (regexp scans are limited to
  // YR_RE_SCAN_LIMIT each way, re.c:1753-1760, :2172-2174; a wide literal compares 2 * length
  // bytes and its FULL_WORD test reads the two after them, scan.c:680-682).  A shard holding only [win_lo, win_hi) of the block keeps a call
  // whose bytes are not all there (a shard sized with the tables' verify halo,
  // yr_amd_tables_info, never does).
  if (p.win_lo != 0 || p.win_hi != p.size) {
    const uint64_t need_lo = offset - min<uint64_t>(offset, (uint64_t)kReScanLimit);
    const uint64_t need_hi =
        min<uint64_t>(p.size, offset + max<uint64_t>((uint64_t)kReScanLimit, 2ull * st.length + 2));
    if (need_lo < p.win_lo || need_hi > p.win_hi) return true;
  }
  if (!(st.flags & kStrLiteral)) return re_call_matters(p, st, st.flags, offset, lds, codebuf, near);
  if (st.flags & kStrUnmodelled) return true;            // conservative
  // _yr_scan_verify_literal_match, scan.c:907-972
  const uint8_t* d = p.data + offset;
  const uint64_t avail = p.size - offset;
  const uint8_t* sp = p.str_bytes + st.bytes_off;
  const uint32_t n = st.length;
  uint64_t fm = 0;   // forward_matches
  ByteWindow w = {nullptr, lds};
  if (st.flags & kStrFitsInAtom) {
    fm = st.backtrack;   // scan.c:912-915
  } else {
    // the compared bytes from LDS (one round trip of 16-byte loads) instead of
    // one dependent byte load per character
    w = stage_window(p, d, false, lds);
    const StrBytes s = YAMD_STAGE_STR ? stage_str(sp, codebuf) : StrBytes{sp, kNoLds, 0u};
    const uint8_t* lower = (st.flags & kStrNoCase) ? p.lowercase : nullptr;
    if ((st.flags & kStrAscii) && cmp_ascii(d, avail, s, n, lower, w)) fm = n;
    if (fm == 0 && (st.flags & kStrWide) && cmp_wide(d, avail, s, n, lower, w)) fm = 2ull * n;
    if (fm == 0 && !(st.flags & kStrNoCase) && (st.flags & kStrXor)) {
      if ((st.flags & kStrWide) && cmp_xor(d, avail, s, n, true, w)) fm = 2ull * n;
      if (fm == 0 && cmp_xor(d, avail, s, n, false, w)) fm = n;
    }
  }
  if (fm == 0) return false;   // scan.c:974-975
  if (!(st.flags & kStrFullWord)) return true;
  // _yr_scan_match_callback's FULL_WORD test (scan.c:672-694): the match is
  // dropped when an alphanumeric character (yr_isalnum) touches it -- for the
  // wide form, an alphanumeric followed by 0x00
  auto at = [&](uint64_t k) { return window_byte(w, p.data + k); };
  auto alnum = [](uint8_t c) {
    return (c >= 0x30 && c <= 0x39) || (c >= 0x41 && c <= 0x5a) || (c >= 0x61 && c <= 0x7a);
  };
  if (fm == 2ull * n) {   // RE_FLAGS_WIDE (scan.c:977-978)
    if (offset >= 2 && at(offset - 1) == 0 && alnum(at(offset - 2))) return false;
    if (offset + fm + 1 < p.size && at(offset + fm + 1) == 0 && alnum(at(offset + fm)))
      return false;
  } else {
    if (offset >= 1 && alnum(at(offset - 1))) return false;
    if (offset + fm < p.size && alnum(at(offset + fm))) return false;
  }
  return true;
}

// One candidate: PASS 0 decides every call of its list, counts the records and
// keeps the decisions (keep mask + state); PASS 1 writes the records from `o`
// on -- from the keep mask, without deciding again, except for lists longer
// than 31 entries.
constexpr uint32_t kKeepOverflow = 1u << 31;
constexpr uint32_t kRecCountOnly = 0x80000000u;   // include/yara_amd.h YR_AMD_REC_COUNT_ONLY
template <int PASS, bool kLean = false>
__device__ __forceinline__ void verify_one(const VerifyParams& p, uint64_t c, uint32_t lds,
                                           uint32_t codebuf, uint32_t keep, uint32_t head,
                                           uint64_t o, uint32_t& count) {
  if (!PASS && p.dead != nullptr && (p.dead[c] & kClassDead)) {
    // the scan's drain already ran this candidate's one guard on the bytes it
    // held (kernels.hip key_class): nothing to read
    p.keep[c] = 0;
    count = 0;
    return;
  }
  const uint64_t i = p.all ? p.all_first + c : p.positions[c];
  if (!PASS && YAMD_VERIFY_DIAG == 3) {   // profiling: candidate positions only
    p.counts[c] = 0; p.keep[c] = 0; p.heads[c] = (uint32_t)i; count = 0; return;
  }
  Near near;
  near.a = kNoNear;
  if (!PASS) head = node_head(p, i, near);
  if (!PASS && YAMD_VERIFY_DIAG >= 4) {   // profiling: + the state's list head
    p.counts[c] = 0; p.keep[c] = 0; p.heads[c] = head; count = 0; return;
  }
  // profiling: pass 1 decides again (the keep mask does not tell count-only
  // records from kept ones)
  // (kLean: a write pass without LDS -- only for tables whose lists fit the
  // keep mask, without profiling: it never decides)
  const bool decide = !kLean && (!PASS || (keep & kKeepOverflow) || p.profile);
  uint32_t n = 0, t = 0, mask = 0;
  // scanner.c:105-121: the list of state_i in pool order
  for (uint32_t k = head; k != 0; ++t) {
    const DevPoolRec e = p.pool[k - 1];
    const uint32_t bt = e.backtrack;
    bool kept, count_only = false;
    if (decide) {
      kept = bt <= i && call_matters(p, e, i - bt, lds, codebuf, near);
      // YR_PROFILING_ENABLED: yr_scan_verify_match counts atom_matches for
      // every call past its early returns (scan.c:1013-1027, :1083), effect or
      // not -- a dropped call past them becomes a count-only record, which the
      // host counts without verifying (its temp-disabled / fast-mode tests
      // are host state, applied at replay time, in the call order)
      if (p.profile && !kept && bt <= i)
        count_only = i - bt < p.size &&
                     (!(e.flags & kStrFixedOffset) ||
                      e.fixed_offset == (int64_t)(p.data_base + (i - bt)));
    } else {
      kept = t < 31 && ((keep >> t) & 1u);
    }
    const uint32_t kk = k;
    k = e.next;
    if (!kept && !count_only) continue;
    if (PASS) {
      VerifyRec r;
      r.offset = i - bt;
      r.pool_index = (kk - 1) | (count_only ? kRecCountOnly : 0u);
      r.candidate = p.cand_index != nullptr ? p.cand_index[c] : (uint32_t)c;
      if (o < p.out_cap) p.out[o] = r;
      ++o;
    } else if (t < 31) {
      mask |= 1u << t;
    }
    ++n;
  }
  if (!PASS) {
    // pass 1 reads counts and heads only where keep != 0: most candidates of
    // a dense rule set keep nothing and write 4 bytes here instead of 12
    p.keep[c] = n == 0 ? 0u : (t > 31 || p.profile ? kKeepOverflow : mask);
    if (n != 0) {
      p.counts[c] = n;
      p.heads[c] = head;
    }
  }
  count = n;
}

// Candidates are decided in groups of 64, one wave each: block_off[g] = the
// group's record count, then (launch_block_offsets) its exclusive offset
// within its chunk of kChunkGroups groups, chunk_off[] the chunks' offsets --
// no barrier anywhere, so a wave never waits for another's longest list.
__device__ __forceinline__ uint64_t group_offset(const VerifyParams& p, uint64_t g) {
  return p.chunk_off[g / kChunkGroups] + p.block_off[g];
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_exclusive(uint32_t v) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += u;
  }
  return inc - v;
}
// The exclusive prefix of the lanes' record counts; when every lane has the
// same count (the dense "kept" keys' groups: one record per candidate) it is
// lane * n, with no cross-lane scan (six dependent ds_bpermute round trips).
__device__ __forceinline__ uint32_t records_before(uint32_t n) {
  const uint32_t n0 = __builtin_amdgcn_readfirstlane(n);
  if (__ballot(n != n0) == 0) return (threadIdx.x & 63u) * n0;
  return wave_exclusive(n);
}
__device__ __forceinline__ uint32_t wave_in_block() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// One of four wave-uniform values (kernel arguments, in SGPRs) by a per-lane
// index: two selects.  Indexing the argument arrays by a lane's key instead
// made the compiler copy them to scratch or re-load them from the kernel
// argument segment -- a dependent memory round trip per record.
__device__ __forceinline__ uint32_t pick4(uint32_t k, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  const uint32_t lo = (k & 1u) ? a1 : a0, hi = (k & 1u) ? a3 : a2;
  return (k & 2u) ? hi : lo;
}
#define YAMD_PICK4(k, A) pick4((k), A[0], A[1], A[2], A[3])
#define YAMD_PICK4T(k, A, t) pick4((k), A[0][t], A[1][t], A[2][t], A[3][t])

// Pass 1 of one group with records (o = its first record's index).
__device__ __forceinline__ void verify_group(const VerifyParams& p, uint64_t g, uint64_t o,
                                             uint32_t lds, uint32_t codebuf) {
  const uint64_t c = g * kGroup + (threadIdx.x & 63u);
  // the scan's class (kernels.hip key_class): dead -- nothing; kept -- every
  // call of the key's list; else pass 0's decisions
  const uint32_t cls = c < p.count && p.dead != nullptr ? p.dead[c] : 0u;
  uint32_t keep = 0, n = 0, head = 0;
  if (cls & kClassKept) {
    n = YAMD_PICK4((cls >> 2) & 3u, p.kd_n);
    keep = (1u << n) - 1u;
    head = YAMD_PICK4((cls >> 2) & 3u, p.kd_head);
  } else if (c < p.count && !(cls & kClassDead)) {
    keep = p.keep[c];
    if (keep != 0) {
      n = p.counts[c];
      head = p.heads[c];
    }
  }
  const uint32_t pre = records_before(n);
  if ((cls & kClassKept) && n <= kKeptDirect) {
    // every call of the key's list, from the key's own list copy: no pool
    // records, no list walk (the dense "kept" keys' candidates)
    const uint32_t k = (cls >> 2) & 3u;
    const uint64_t i = p.positions[c];
    const uint64_t at = o + pre;
#pragma unroll
    for (uint32_t t = 0; t < kKeptDirect; ++t) {
      if (t >= n) break;
      VerifyRec r;
      r.offset = i - YAMD_PICK4T(k, p.kd_bt, t);
      r.pool_index = YAMD_PICK4T(k, p.kd_idx, t);
      r.candidate = p.cand_index != nullptr ? p.cand_index[c] : (uint32_t)c;
      if (at + t < p.out_cap) p.out[at + t] = r;
    }
  } else if (keep != 0) {
    verify_one<1>(p, c, lds, codebuf, keep, head, o + pre, n);
  }
}

// The write pass as a grid covering every group, kWriteGroups groups per wave
// (p.first: the launch's first group) -- for tables whose groups mostly have
// records (the "kept" 1-byte keys: every candidate a record), where the
// persistent waves of verify_kernel<1> take their groups one after another.
// No LDS (every decision is pass 0's: VerifyParams::direct is set only where
// lists fit the keep mask and without profiling), and every load the wave's
// groups need -- offsets, classes, positions, pass 0's keep masks -- issued
// together: one memory round trip before their records are written
// (short, 16.8 M records: 234 us with one group per wave and LDS, 157 us
// without LDS, gpurun r5h6 / r5h7).
// groups per wave (verify_write_kernel; 2 against 4 and 8: short's pre-
// verification 4 % faster, fuzz3's 5 %, in one process, gpurun r5h22 / r5h23)
constexpr uint32_t kWriteGroups = 2;
__global__ __launch_bounds__(256) void verify_write_kernel(VerifyParams p) {
  const uint64_t groups = (p.count + kGroup - 1) / kGroup;
  const uint64_t g0 = p.first + ((uint64_t)blockIdx.x * (blockDim.x / 64) + wave_in_block()) * kWriteGroups;
  if (g0 >= groups) return;
  // kWriteGroups groups per wave, every load of all of them issued first
  uint64_t o[kWriteGroups + 1], i[kWriteGroups];
  uint32_t cls[kWriteGroups];
  // (indices clamped rather than loads predicated: no branch between the
  // loads, so they all go out before the first wait -- the predicated form
  // compiled to one dependent round trip per group offset)
#pragma unroll
  for (uint32_t q = 0; q <= kWriteGroups; ++q) o[q] = group_offset(p, min(g0 + q, groups));
#pragma unroll
  for (uint32_t q = 0; q < kWriteGroups; ++q) {
    const uint64_t c = min((g0 + q) * kGroup + (threadIdx.x & 63u), p.count - 1);
    cls[q] = p.dead != nullptr ? p.dead[c] : 0u;
    i[q] = p.positions[c];
  }
#pragma unroll
  for (uint32_t q = 0; q < kWriteGroups; ++q) {
    const uint64_t g = g0 + q;
    if (g >= groups || o[q + 1] == o[q]) continue;   // (wave-uniform)
    const uint64_t c = g * kGroup + (threadIdx.x & 63u);
    if (c >= p.count) cls[q] = 0u;   // (past the stream: no records)
    uint32_t keep = 0, n = 0, head = 0;
    const uint32_t k = (cls[q] >> 2) & 3u;
    if (cls[q] & kClassKept) {
      n = YAMD_PICK4(k, p.kd_n);
      keep = (1u << n) - 1u;
      head = YAMD_PICK4(k, p.kd_head);
    } else if (c < p.count && !(cls[q] & kClassDead)) {
      keep = p.keep[c];   // (pass 0 wrote it for live candidates only)
      if (keep != 0) {
        n = p.counts[c];
        head = p.heads[c];
      }
    }
    const uint32_t pre = records_before(n);
    if ((cls[q] & kClassKept) && n <= kKeptDirect) {
      const uint64_t at = o[q] + pre;
      const uint32_t cand = p.cand_index != nullptr ? p.cand_index[c] : (uint32_t)c;
#pragma unroll
      for (uint32_t t = 0; t < kKeptDirect; ++t) {
        if (t >= n) break;
        VerifyRec r;
        r.offset = i[q] - YAMD_PICK4T(k, p.kd_bt, t);
        r.pool_index = YAMD_PICK4T(k, p.kd_idx, t);
        r.candidate = cand;
        // (non-temporal: the records leave for the host, nothing on the GPU
        // reads them back -- 5 % of short's / fuzz3's pre-verification)
        if (at + t < p.out_cap) {
          typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 q4 = {(uint32_t)r.offset, (uint32_t)(r.offset >> 32), r.pool_index, r.candidate};
          __builtin_nontemporal_store(q4, reinterpret_cast<u32x4*>(p.out + at + t));
        }
      }
    } else if (keep != 0) {
      verify_one<1, true>(p, c, 0u, 0u, keep, head, o[q] + pre, n);
    }
  }
}

// PASS 0: one candidate per lane; each wave's record count goes to its group.
// PASS 1: persistent waves over the groups, 64 tested at once for records;
// the groups with some scan their candidates' counts and write the records
// from the group's offset on.
template <int PASS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void verify_kernel(
    VerifyParams p) {   // (5 waves per SIMD: the LDS allows them, and pass 1 fits 96 VGPRs)
  __shared__ __attribute__((aligned(16))) uint8_t win[256 * kWinBytes];
  __shared__ __attribute__((aligned(16))) uint8_t code[256 * kCodeBytes];
  // (the low 32 bits of a flat LDS address are the LDS offset)
  const uint32_t lds = (uint32_t)(uintptr_t)(win + threadIdx.x * kWinBytes);
  const uint32_t codebuf = (uint32_t)(uintptr_t)(code + threadIdx.x * kCodeBytes);
  const uint64_t groups = (p.count + kGroup - 1) / kGroup;
  if (PASS == 0) {
    const uint64_t c = p.first + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t n = 0;
    if (c < p.count) verify_one<0>(p, c, lds, codebuf, 0, 0, 0, n);
    const uint32_t sum = wave_sum(n);
    if ((threadIdx.x & 63u) == 0 && c / kGroup < groups) p.block_off[c / kGroup] = sum;
    return;
  }

  // wave w takes groups w, w + waves, ...; it tests 64 of them for records at
  // once (one lane each: a group without records reads nothing more -- most of
  // a dense rule set's, e.g. rx: 539 records from 525,000 groups), then runs
  // the groups that have some
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t g0 = (uint64_t)blockIdx.x * (blockDim.x / 64) + wave_in_block(); g0 < groups;
       g0 += waves * 64) {
    const uint64_t gl = g0 + lane * waves;
    const bool has = gl < groups && group_offset(p, gl + 1) != group_offset(p, gl);
    // (the group's offset loaded again, wave-uniform: a VGPR pair held across
    // the loop costs the kernel a wave per SIMD)
    for (uint64_t m = __ballot(has); m != 0; m &= m - 1) {
      const uint64_t g = g0 + (uint64_t)__builtin_ctzll(m) * waves;
      verify_group(p, g, group_offset(p, g), lds, codebuf);
    }
  }
}

// The scan segments' live lists concatenated (live_off: their offsets, from
// launch_counts_offsets): one wave per segment, persistent over the segments.
// Each wave also zeroes the record counts of the groups its segment's
// candidates fall in (verify_live_kernel adds to them; a group shared by two
// segments is zeroed by both, before either adds) -- no separate memset.
__global__ __launch_bounds__(256) void live_gather_kernel(VerifyParams p) {
  const uint32_t waves = gridDim.x * (blockDim.x / 64), lane = threadIdx.x & 63u;
  const uint64_t groups = (p.count + kGroup - 1) / kGroup;
  for (uint32_t seg = blockIdx.x * (blockDim.x / 64) + wave_in_block(); seg < p.live_segs; seg += waves) {
    const uint32_t n = p.live_count[seg];
    const uint32_t* src = p.live + p.live_first[seg];
    uint32_t* dst = p.live_dense + p.live_off[seg];
    for (uint32_t h = lane; h < n; h += 64) dst[h] = src[h];
    const uint64_t c0 = p.live_first[seg], c1 = min(p.live_first[seg + 1], p.count);
    if (c1 > c0)
      for (uint64_t g = c0 / kGroup + lane; g <= (c1 - 1) / kGroup; g += 64) p.block_off[g] = 0;
    if (seg == p.live_segs - 1 && lane == 0) p.block_off[groups] = 0;   // (past the last group)
  }
}

// Pass 0 over the concatenated live lists (persistent blocks): each live
// candidate decided as verify_kernel<0> does, its record count added to its
// group's.
__global__ __launch_bounds__(256) void verify_live_kernel(VerifyParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t win[256 * kWinBytes];
  __shared__ __attribute__((aligned(16))) uint8_t code[256 * kCodeBytes];
  const uint32_t lds = (uint32_t)(uintptr_t)(win + threadIdx.x * kWinBytes);
  const uint32_t codebuf = (uint32_t)(uintptr_t)(code + threadIdx.x * kCodeBytes);
  const uint64_t n_live = p.live_off[p.live_segs];
  for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n_live;
       h += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = p.live_dense[h];
    uint32_t n = 0;
    verify_one<0>(p, c, lds, codebuf, 0, 0, 0, n);
    if (n != 0) atomicAdd(reinterpret_cast<unsigned long long*>(p.block_off + c / kGroup),
                          (unsigned long long)n);
  }
}

// Offsets, step 1: one 1024-thread block per chunk of kChunkGroups groups,
// four threads per group (16 candidates each: one 16-byte load of their
// classes) -- the chunk's exclusive scan in place (entry `groups`, past the
// last group, counts 0) and its total into chunk_off[chunk].  (One thread per
// group, 1024 groups a block, was latency-bound: short's 263 k groups in
// 15 us, 1.3 TB/s.)
__global__ __launch_bounds__(1024) void group_scan_kernel(uint64_t* block_off, uint64_t groups,
                                                          uint64_t* chunk_off, const uint8_t* cls,
                                                          uint64_t count, KeptLists kept) {
  static_assert(kChunkGroups * 4 == 1024, "four threads per group, one block per chunk");
  __shared__ uint64_t wsum[16];
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6, q = threadIdx.x & 3u;
  const uint64_t i = (uint64_t)blockIdx.x * kChunkGroups + (threadIdx.x >> 2);
  uint64_t v = q == 0 && i < groups ? block_off[i] : 0;
  if (cls != nullptr && i < groups) {
    // + the records of the group's "kept" candidates (their calls are the
    // key's whole list; pass 0 never saw them)
    const uint64_t c0 = i * kGroup + 16u * q, c1 = min(c0 + 16u, count);
    auto add = [&](uint32_t word) {   // four class bytes
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t x = (word >> (8 * b)) & 0xFFu;
        v += (x & kClassKept) ? YAMD_PICK4((x >> 2) & 3u, kept.n) : 0u;
      }
    };
    if (c1 > c0 && c1 - c0 == 16u) {   // a whole quarter: one 16-byte load
      const uint4 u = *reinterpret_cast<const uint4*>(cls + c0);
      add(u.x);
      add(u.y);
      add(u.z);
      add(u.w);
    } else {
      for (uint64_t c = c0; c < c1; ++c) add(cls[c]);
    }
  }
  // the group's total in its four lanes; one contribution per group to the scan
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  const uint64_t gv = q == 0 ? v : 0;
  uint64_t inc = gv;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t u = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += u;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  if (w == 0) {
    const uint64_t x = lane < 16 ? wsum[lane] : 0;
    uint64_t y = x;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const uint64_t u = __shfl_up(y, d, 64);
      if (lane >= (uint32_t)d) y += u;
    }
    if (lane < 16) wsum[lane] = y - x;
    if (lane == 15) chunk_off[blockIdx.x] = y;
  }
  __syncthreads();
  if (q == 0 && i <= groups) block_off[i] = wsum[w] + inc - gv;
}

// Offsets, step 2 (one workgroup): exclusive scan, in place, of the chunk
// totals, and their sum (into chunk_off[n] and *total).
__global__ __launch_bounds__(1024) void block_offsets_kernel(uint64_t* block_off, uint64_t n_blocks,
                                                             uint64_t* total) {
  __shared__ uint64_t part[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t per = (n_blocks + 1023) / 1024;
  const uint64_t lo = min(t * per, n_blocks), hi = min(lo + per, n_blocks);
  uint64_t s = 0;
#pragma unroll 16
  for (uint64_t i = lo; i < hi; ++i) s += block_off[i];
  part[t] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    const uint64_t v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = part[t] - s;
#pragma unroll 16
  for (uint64_t i = lo; i < hi; ++i) {
    const uint64_t c = block_off[i];
    block_off[i] = run;
    run += c;
  }
  if (t == 1023) {
    block_off[n_blocks] = part[1023];
    *total = part[1023];
  }
}

// Grid of the persistent kernels: as many 256-thread blocks as the device
// keeps resident (a second wave of blocks would finish late).
// (Queried once per kernel and device: the occupancy query costs microseconds
// of host time between launches that the GPU would spend idle.)
static uint32_t resident_blocks(const void* kernel) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  struct Entry { const void* k; int dev; uint32_t n; };
  static std::mutex mu;
  static std::vector<Entry> cache;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (const Entry& e : cache)
      if (e.k == kernel && e.dev == dev) return e.n;
  }
  int cus = 0, per = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess)
    return 256;
  const uint32_t n = (uint32_t)std::max(1, cus * std::max(1, per));
  std::lock_guard<std::mutex> lk(mu);
  cache.push_back(Entry{kernel, dev, n});
  return n;
}

hipError_t launch_verify(const VerifyParams& p, int pass, hipStream_t s) {
  if (p.count == 0) return hipSuccess;
  if (pass == 0) {
    // one thread per candidate, in slices of 2^31: an AQL dispatch's grid size
    // is a 32-bit count of work-items, so 2^32 candidates (the largest stream
    // yr_amd_verify_device accepts) do not fit one launch.  (Slices are whole
    // groups: kGroup divides 2^31.)
    constexpr uint64_t kSlice = 1ull << 31;
    static_assert(kSlice % kGroup == 0, "slices of whole groups");
    VerifyParams q = p;
    for (q.first = 0; q.first < p.count; q.first += kSlice) {
      const uint64_t n = std::min<uint64_t>(p.count - q.first, kSlice);
      hipLaunchKernelGGL(verify_kernel<0>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, q);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  } else if (p.direct) {
    // kWriteGroups groups per wave, in slices of 2^31 work-items per dispatch
    constexpr uint64_t kSliceGroups = (1ull << 31) / kGroup;
    const uint64_t groups = verify_groups(p.count);
    VerifyParams q = p;
    for (q.first = 0; q.first < groups; q.first += kSliceGroups) {
      const uint64_t n = std::min<uint64_t>(groups - q.first, kSliceGroups);
      const uint64_t waves = (n + kWriteGroups - 1) / kWriteGroups;
      hipLaunchKernelGGL(verify_write_kernel, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, s, q);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  } else {
    const uint64_t waves = verify_groups(p.count);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(
        (waves + 3) / 4, resident_blocks((const void*)verify_kernel<1>));
    hipLaunchKernelGGL(verify_kernel<1>, dim3(blocks), dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

hipError_t launch_counts_offsets(const uint32_t* counts, uint32_t n, uint64_t* offsets, uint64_t* summary,
                                 hipStream_t s);   // (kernels.hip)
hipError_t launch_verify_live(const VerifyParams& p, uint64_t* summary, hipStream_t s) {
  if (p.count == 0) return hipSuccess;
  if (p.live_segs == 0)   // (no segments: nothing to gather, the counts zeroed here)
    return hipMemsetAsync(p.block_off, 0, (verify_groups(p.count) + 1) * sizeof(uint64_t), s);
  hipError_t e = launch_counts_offsets(p.live_count, p.live_segs, p.live_off, summary, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(live_gather_kernel, dim3((p.live_segs + 3) / 4), dim3(256), 0, s, p);
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(
      (p.count + 255) / 256, resident_blocks((const void*)verify_live_kernel));
  hipLaunchKernelGGL(verify_live_kernel, dim3(blocks), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_block_offsets(uint64_t* block_off, uint64_t* chunk_off, uint64_t count,
                                uint64_t* total, const uint8_t* cls, const KeptLists& kept,
                                hipStream_t s) {
  const uint64_t groups = verify_groups(count);
  if (groups == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), s);
  const uint64_t chunks = verify_chunks(count);
  hipLaunchKernelGGL(group_scan_kernel, dim3((uint32_t)chunks), dim3(1024), 0, s, block_off, groups,
                     chunk_off, cls, count, kept);
  hipLaunchKernelGGL(block_offsets_kernel, dim3(1), dim3(1024), 0, s, chunk_off, chunks, total);
  return hipGetLastError();
}

uint64_t verify_groups(uint64_t count) { return (count + kGroup - 1) / kGroup; }
uint64_t verify_chunks(uint64_t count) { return (verify_groups(count) + 1 + kChunkGroups - 1) / kChunkGroups; }

}  // namespace yamd
