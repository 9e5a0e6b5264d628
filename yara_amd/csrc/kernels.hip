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
//   stage 1 (every byte, LDS):  a split-block Bloom filter (2^20 bits) over
//             the 3-byte window ending at the byte (internal.h filter_probe).
//             128 KiB, staged once per workgroup; one ds_read_b64 per input
//             byte.  Superset of the keys (config C: 0.15% of positions pass).
//   stage 2 (filter hits):  hits are appended in position order to a per-wave
//             LDS ring; full batches of 64 are checked exactly against the key
//             sets (bitmaps / bucketed cuckoo tables in HBM/L2), and survivors
//             are compacted with a wave ballot + mbcnt into the segment's output.
//
// Memory: the input is streamed once, 16 B per lane (1 KiB per wave per step),
// tile t+1 in flight while tile t is filtered.  Roofline: HBM read bandwidth
// (1 algorithmic byte per input byte).
#include "internal.h"

namespace yamd {

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
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

// Exact test of one position `pos` of the block: does a key of length
// L <= min(4, pos) equal the last L bytes before it?  w4 = those 4 bytes,
// little endian (oldest lowest; zeros before the block start).  Every load
// (bitmap words, both candidate buckets of each table) is independent: one
// round trip.
__device__ __forceinline__ bool exact_check(uint32_t w4, uint64_t pos, const ScanParams& p) {
  const uint32_t* __restrict__ ex = p.exact;
  bool hit = false;
  const uint32_t lm = p.len_mask;
  if ((lm & 2u) && pos >= 1) {
    const uint32_t k = w4 >> 24;
    hit |= (ex[kExactBm1 + (k >> 5)] >> (k & 31)) & 1u;
  }
  if ((lm & 4u) && pos >= 2) {
    const uint32_t k = w4 >> 16;
    hit |= (ex[kExactBm2 + (k >> 5)] >> (k & 31)) & 1u;
  }
  if ((lm & 8u) && pos >= 3) {
    const uint32_t k = (w4 >> 8) | (1u << 24);
    const uint4 a = *reinterpret_cast<const uint4*>(ex + p.t3_off + (bucket_hash1(k) & p.t3_mask) * 4);
    const uint4 b = *reinterpret_cast<const uint4*>(ex + p.t3_off + (bucket_hash2(k) & p.t3_mask) * 4);
    hit |= a.x == k || a.y == k || a.z == k || a.w == k || b.x == k || b.y == k || b.z == k || b.w == k;
  }
  if ((lm & 16u) && pos >= 4) {
    const uint32_t k = w4;
    if (k == 0) {
      hit |= (p.exact_flags & kExactZero4) != 0;
    } else {
      const uint4 a = *reinterpret_cast<const uint4*>(ex + p.t4_off + (bucket_hash1(k) & p.t4_mask) * 4);
      const uint4 b = *reinterpret_cast<const uint4*>(ex + p.t4_off + (bucket_hash2(k) & p.t4_mask) * 4);
      hit |= a.x == k || a.y == k || a.z == k || a.w == k || b.x == k || b.y == k || b.z == k || b.w == k;
    }
  }
  return hit;
}

// The 4 bytes ending at lane byte j (0..15) from the lane's window context
// C[0] = the 4 bytes before the lane, C[1..4] = its 16 bytes.
__device__ __forceinline__ uint32_t window4(const uint32_t (&C)[5], uint32_t j) {
  const uint32_t o = j + 1, i = o >> 2;
  uint32_t lo = C[0], hi = C[1];
  if (i == 1) { lo = C[1]; hi = C[2]; }
  if (i == 2) { lo = C[2]; hi = C[3]; }
  if (i == 3) { lo = C[3]; hi = C[4]; }
  if (i == 4) { lo = C[4]; hi = 0u; }
  return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
}

// Lane byte (0..15) of bit b of a tile hit mask: bit 8n + r <=> byte 4n + r.
__device__ __forceinline__ uint32_t mask_position(uint32_t b) { return ((b >> 3) << 2) | (b & 3u); }

// Per-wave LDS ring of filter hits awaiting the exact check.  One entry (32-byte
// slot, 24 bytes written) per (tile, lane) with at least one hit: the lane's
// window context (4 bytes before it + its 16 bytes) and (lane byte offset in
// segment / 16) | (16-bit hit mask, bit j = lane byte j) << 16.  Entries are appended in lane order, so ring order
// is ascending position order.  The exact check then needs no global load
// of the input, only the hash-table probes.
struct WaveQueue {
  uint32_t* ring;   // kQueueCap entries of kQueueEntryWords dwords
  uint32_t head;    // wave-uniform counters (monotonic)
  uint32_t tail;
};

// Exact-check the hits of up to 64 ring entries and append the survivors, in
// order, to the segment's output.
template <int MODE>
__device__ __forceinline__ void drain(const ScanParams& p, WaveQueue& q, uint32_t lane,
                                      uint64_t seg_start, uint32_t* out, uint32_t& found) {
  const uint32_t n = min(q.tail - q.head, (uint32_t)kWave);
  if constexpr (MODE == 7) {   // ablation: ring appends only, entries dropped
    q.head += n;
    return;
  }
  if constexpr (MODE == 8)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   // ring in global memory
  else
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  uint32_t keep = 0, off0 = 0;
  if (lane < n) {
    const uint32_t* ent = q.ring + ((q.head + lane) % kQueueCap) * kQueueEntryWords;
    const uint4 a = *reinterpret_cast<const uint4*>(ent);
    const uint2 b = *reinterpret_cast<const uint2*>(ent + 4);
    const uint32_t C[5] = {a.x, a.y, a.z, a.w, b.x};
    off0 = (b.y & 0xFFFFu) * kBytesPerLane;
    uint32_t m = b.y >> 16;   // 16-bit mask, bit j = lane byte j
    while (m) {
      const uint32_t j = (uint32_t)__builtin_ctz(m);
      m &= m - 1;
      const bool hit = MODE == 1 ? ((off0 + j) & 1023u) == 7u
                                 : exact_check(window4(C, j), seg_start + off0 + j + 1, p);
      keep |= (uint32_t)hit << j;
    }
  }
  const uint32_t c = __popc(keep);
  const uint32_t incl = wave_inclusive_scan(c);
  uint32_t idx = found + incl - c;
  while (keep) {
    const uint32_t j = (uint32_t)__builtin_ctz(keep);
    keep &= keep - 1;
    if (idx < p.seg_cap) out[idx] = off0 + j;
    ++idx;
  }
  found += __builtin_amdgcn_readlane(incl, kWave - 1);
  q.head += n;
}

// A tile entirely inside the block: one 16-byte non-temporal load per lane
// (read-once stream; keeps the exact tables' L2 lines).
__device__ __forceinline__ uint4 load_tile_full(const uint8_t* base, uint32_t tile_off, uint32_t lane) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(
      reinterpret_cast<const u32x4*>(base + tile_off + lane * kBytesPerLane));
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
  uint32_t carry;   // the 4 bytes before the current tile (lane 0's window head)
};

// One 1 KiB tile: stage-1 filter over its 1024 byte positions, then the ordered
// append of the hits to the wave ring.  TAIL: the segment's last, partial tile
// (positions past seg_len are masked off).
template <int MODE, bool TAIL>
__device__ __forceinline__ void tile_step(const ScanParams& p, WaveQueue& q, SegState& st,
                                          uint4 cur, uint32_t tile_off, uint32_t lane) {
  // previous lane's last dword (lane 0: the previous tile's / the halo)
  const uint32_t S0 = __builtin_amdgcn_update_dpp(st.carry, cur.w, 0x138, 0xF, 0xF, false);  // wave_shr:1
  st.carry = __builtin_amdgcn_readlane(cur.w, kWave - 1);
  const uint32_t S[6] = {S0, cur.x, cur.y, cur.z, cur.w, 0u};

  // Phase A: the 16 windows of this lane and their 16 filter-block reads.
  uint32_t xs[kBytesPerLane];
  uint2 ws[kBytesPerLane];
#pragma unroll
  for (int k = 0; k < kBytesPerLane; ++k) {
    // low 24 bits = bytes k-2, k-1, k of this lane (stream offset k + 2)
    const int o = k + 2;
    xs[k] = (o & 3) == 0   ? S[o >> 2]
            : (o & 3) == 1 ? S[o >> 2] >> 8
                           : __builtin_amdgcn_alignbyte(S[(o >> 2) + 1], S[o >> 2], o & 3);
    if constexpr (MODE != 3) {
      const uint32_t x = xs[k];
      uint32_t addr = (x >> 7) & (kFilterBytes - 8);   // block x[10..23], 8 B each
      if constexpr (MODE == 4) addr = ((lane & 31u) * 8u + (uint32_t)k * 256u) & (kFilterBytes - 8);
      if constexpr (MODE == 5) {
        ws[k] = make_uint2(addr ^ x, addr + x);
      } else {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x2*>(
            (uintptr_t)addr);   // filter sits at LDS offset 0: no base add
        ws[k] = make_uint2(v.x, v.y);
      }
    }
  }
  // Phase B: split-block test, bit x[0..4] of the lo word and bit x[5..9] of
  // the hi word (the shifter reads only the low 5 bits of the amount).  The
  // AND of the two shifted words is written by one SDWA v_and straight into
  // byte n of accumulator r (k = 4n + r), so bit 0 of that byte is position
  // k's result and no separate accumulate instruction is needed; bits 1..7
  // of each byte are don't-care and masked off once per tile below.
  uint32_t acc[4];   // every byte is written below: no initial value needed
#pragma unroll
  for (int k = 0; k < kBytesPerLane; ++k) {
    if constexpr (MODE == 3) {
      acc[k & 3] ^= xs[k];
    } else if constexpr (MODE == 6) {
      acc[k & 3] ^= ws[k].x ^ ws[k].y;
    } else {
      const uint32_t x = xs[k];
      const uint32_t u = ws[k].x >> (x & 31u), v = ws[k].y >> ((x >> 5) & 31u);
      switch (k >> 2) {
        case 0: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                    : "+v"(acc[k & 3]) : "v"(u), "v"(v)); break;
        case 1: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                    : "+v"(acc[k & 3]) : "v"(u), "v"(v)); break;
        case 2: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                    : "+v"(acc[k & 3]) : "v"(u), "v"(v)); break;
        default: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
                     : "+v"(acc[k & 3]) : "v"(u), "v"(v)); break;
      }
    }
  }
  if constexpr (MODE >= 2 && MODE <= 6) {
    asm volatile("" ::"v"(acc[0] ^ acc[1] ^ acc[2] ^ acc[3]));
    return;
  }
  // hit mask: bit 8n + r <=> position 4n + r of the lane (mask_position())
  uint32_t mask = (acc[0] & 0x01010101u) | ((acc[1] & 0x01010101u) << 1) |
                  ((acc[2] & 0x01010101u) << 2) | ((acc[3] & 0x01010101u) << 3);
  const uint32_t lane_off = tile_off + lane * kBytesPerLane;
  if constexpr (TAIL) {
    if (lane_off + kBytesPerLane > st.seg_len) {
      const uint32_t lim = lane_off >= st.seg_len ? 0u : st.seg_len - lane_off;
      uint32_t keep = 0;
      for (uint32_t j = 0; j < lim; ++j) keep |= 1u << (((j >> 2) << 3) | (j & 3u));
      mask &= keep;
    }
  }
  const uint64_t any = __ballot(mask != 0);
  if (any != 0) {
    const uint32_t n = (uint32_t)__popcll(any);
    if (q.tail - q.head + n > kQueueCap) drain<MODE>(p, q, lane, st.seg_start, st.out, st.found);
    if (mask != 0) {
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(any >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)any, 0u));
      uint32_t* ent = q.ring + ((q.tail + below) % kQueueCap) * kQueueEntryWords;
      // 24-byte entry (b128 + b64: 19 LDS transfer cycles instead of 26):
      // context, then (lane index in segment) | (16-bit mask) << 16; the mask's
      // nibbles (bit 8n + r) are packed: t = m | m >> 4 has them in bytes 0, 2
      const uint32_t t = mask | (mask >> 4);
      const uint32_t m16 = __builtin_amdgcn_perm(0u, t, 0x0c0c0200u);   // bytes 0, 2
      *reinterpret_cast<uint4*>(ent) = make_uint4(S[0], S[1], S[2], S[3]);
      *reinterpret_cast<uint2*>(ent + 4) = make_uint2(S[4], (lane_off / kBytesPerLane) | (m16 << 16));
    }
    q.tail += n;
  }
}

// Stream one segment [seg_start, seg_start + seg_len) of the block: full tiles
// in the main loop (unmasked, the next tile's loads in flight), then the
// partial tail tile if any.
// MODE: 0 = the product kernel.  Others are profiling ablations only (their
// output is wrong by construction): 1 = no exact check, 2 = stage 1 only
// (no queue), 3 = input streaming only (no filter), 4 = stage 1 with
// bank-conflict-free LDS addresses, 5 = stage 1 VALU without the LDS reads,
// 6 = stage 1 addresses + LDS reads without the bit tests, 7 = stage 1 +
// ring appends, drains drop the entries, 8 = product with the hit rings in
// global memory (L2) instead of LDS.
template <int MODE>
__device__ void scan_segment(const ScanParams& p, WaveQueue& q, uint32_t seg, uint32_t lane) {
  SegState st;
  st.seg_start = p.byte_begin + (uint64_t)seg * p.seg_bytes;
  const uint64_t seg_end = min(st.seg_start + p.seg_bytes, p.byte_end);
  st.seg_len = (uint32_t)(seg_end - st.seg_start);
  st.out = p.seg_out + (p.seg_base ? p.seg_base[seg] : (size_t)seg * p.seg_cap);
  st.found = 0;
  const uint64_t avail = p.block_size - st.seg_start;
  const uint8_t* base = p.data + st.seg_start;

  // 4 bytes before the segment (warm-up halo); zeros before the block start.
  st.carry = st.seg_start >= 4 ? *reinterpret_cast<const uint32_t*>(base - 4) : 0u;
  q.head = q.tail = 0;

  const uint32_t n_full = st.seg_len / kTile;            // tiles needing no mask / bounds
  const uint32_t n_all = (st.seg_len + kTile - 1) / kTile;
  // the next tile's loads in flight while this one is filtered
  auto fetch = [&](uint32_t t) {
    return t < n_full ? load_tile_full(base, t * kTile, lane)
                      : (t < n_all ? load_tile(base, t * kTile, lane, avail) : make_uint4(0, 0, 0, 0));
  };
  uint4 cur = fetch(0);
  for (uint32_t t = 0; t < n_full; ++t) {
    const uint4 nxt = fetch(t + 1);
    tile_step<MODE, false>(p, q, st, cur, t * kTile, lane);
    cur = nxt;
  }
  if (n_all > n_full) tile_step<MODE, true>(p, q, st, cur, n_full * kTile, lane);
  while (q.tail != q.head) drain<MODE>(p, q, lane, st.seg_start, st.out, st.found);
  if (lane == 0) p.seg_count[seg] = st.found;
}

template <int MODE>
__global__ __launch_bounds__(kWGThreads, 1) void scan_segments_kernel(ScanParams p) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  uint32_t* filt = lds;
  {
    const uint4* src = reinterpret_cast<const uint4*>(p.filter);
    uint4* dst = reinterpret_cast<uint4*>(filt);
    for (uint32_t i = threadIdx.x; i < kFilterWords / 4; i += blockDim.x) dst[i] = src[i];
  }
  __syncthreads();
  const uint32_t lane = lane_id();
  // wave index, provably wave-uniform: everything derived from it (segment
  // bounds, loop counts, ring base) stays in SGPRs with scalar branches
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  WaveQueue q;
  if constexpr (MODE == 8)
    q.ring = p.gring + ((size_t)blockIdx.x * kWavesPerWG + wid) * kQueueCap * kQueueEntryWords;
  else
    q.ring = lds + kFilterWords + wid * kQueueCap * kQueueEntryWords;
  const uint32_t total_waves = gridDim.x * kWavesPerWG;
  for (uint32_t seg = blockIdx.x * kWavesPerWG + wid; seg < p.n_segments; seg += total_waves) {
    scan_segment<MODE>(p, q, seg, lane);
  }
}

// ---------------------------------------------------------------------------
// Candidate compaction: per-segment counts -> offsets (one workgroup), then a
// scatter of every segment's ascending entries into one ascending uint64 array.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void seg_offsets_kernel(const uint32_t* seg_count, uint32_t n,
                                                           uint32_t cap, uint64_t* seg_offset,
                                                           uint64_t* summary) {
  __shared__ uint64_t part[1024];
  __shared__ uint32_t pmax[1024];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t lo = min(t * per, n), hi = min(lo + per, n);
  uint64_t s = 0;
  uint32_t mx = 0;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t c = seg_count[i];
    s += min(c, cap);
    mx = max(mx, c);
  }
  part[t] = s;
  pmax[t] = mx;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    uint64_t v = t >= d ? part[t - d] : 0;
    uint32_t m = t >= d ? pmax[t - d] : 0;
    __syncthreads();
    part[t] += v;
    pmax[t] = max(pmax[t], m);
    __syncthreads();
  }
  uint64_t run = part[t] - s;
  for (uint32_t i = lo; i < hi; ++i) {
    seg_offset[i] = run;
    run += min(seg_count[i], cap);
  }
  if (t == 1023) {
    summary[0] = part[1023];   // total entries written
    summary[1] = pmax[1023];   // max per-segment count (overflow if > cap)
  }
}

__global__ __launch_bounds__(256) void seg_scatter_kernel(const uint32_t* seg_count,
                                                          const uint32_t* seg_out,
                                                          const uint64_t* seg_base,
                                                          const uint64_t* seg_offset, uint32_t cap,
                                                          uint64_t byte_begin, uint32_t seg_bytes,
                                                          uint64_t* positions) {
  const uint32_t seg = blockIdx.x;
  const uint32_t c = min(seg_count[seg], cap);
  const uint64_t base = byte_begin + (uint64_t)seg * seg_bytes + 1;  // position = byte + 1
  const uint32_t* src = seg_out + (seg_base ? seg_base[seg] : (size_t)seg * cap);
  uint64_t* dst = positions + seg_offset[seg];
  for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) dst[i] = base + src[i];
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

hipError_t launch_scan(const ScanParams& p, int grid, hipStream_t s, int mode) {
  const size_t lds = kScanLdsBytes;
  switch (mode) {
    case 1: hipLaunchKernelGGL(scan_segments_kernel<1>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
    case 2: hipLaunchKernelGGL(scan_segments_kernel<2>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
    case 3: hipLaunchKernelGGL(scan_segments_kernel<3>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
    case 4: hipLaunchKernelGGL(scan_segments_kernel<4>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
    case 5: hipLaunchKernelGGL(scan_segments_kernel<5>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
    case 6: hipLaunchKernelGGL(scan_segments_kernel<6>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
    case 7: hipLaunchKernelGGL(scan_segments_kernel<7>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
    case 8: hipLaunchKernelGGL(scan_segments_kernel<8>, dim3(grid), dim3(kWGThreads), kFilterBytes, s, p); break;
    default: hipLaunchKernelGGL(scan_segments_kernel<0>, dim3(grid), dim3(kWGThreads), lds, s, p); break;
  }
  return hipGetLastError();
}

hipError_t launch_compact(const ScanParams& p, uint64_t* seg_offset, uint64_t* summary,
                          uint64_t* positions, bool scatter, hipStream_t s) {
  if (!scatter) {
    hipLaunchKernelGGL(seg_offsets_kernel, dim3(1), dim3(1024), 0, s, p.seg_count, p.n_segments,
                       p.seg_cap, seg_offset, summary);
  } else {
    hipLaunchKernelGGL(seg_scatter_kernel, dim3(p.n_segments), dim3(256), 0, s, p.seg_count,
                       p.seg_out, p.seg_base, seg_offset, p.seg_cap, p.byte_begin, p.seg_bytes,
                       positions);
  }
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
  for (const void* k : {(const void*)scan_segments_kernel<0>, (const void*)scan_segments_kernel<1>,
                        (const void*)scan_segments_kernel<2>, (const void*)scan_segments_kernel<3>,
                        (const void*)scan_segments_kernel<4>, (const void*)scan_segments_kernel<5>,
                        (const void*)scan_segments_kernel<6>, (const void*)scan_segments_kernel<7>,
                        (const void*)scan_segments_kernel<8>}) {
    hipError_t r = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (r != hipSuccess) e = r;
  }
  return e;
}

}  // namespace yamd
