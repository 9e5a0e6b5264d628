// Internal definitions shared by the host flattening code and the gfx950
// kernels.  Nothing here is part of the C ABI (include/yara_amd.h).
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>

namespace yamd {

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
constexpr int kSegTiles = 64;
constexpr uint32_t kSegment = kTile * kSegTiles;    // 64 KiB
constexpr int kWavesPerWG = 16;
constexpr int kWGThreads = kWave * kWavesPerWG;     // 1024

// LDS window filter: 2^20 bits = 128 KiB, one bit per hashed 3-byte window.
constexpr int kFilterLog2Bits = 20;
constexpr uint32_t kFilterWords = 1u << (kFilterLog2Bits - 5);   // 32768
constexpr uint32_t kFilterBytes = kFilterWords * 4;              // 131072

// Per-wave LDS ring of filter hits awaiting the exact check.
constexpr uint32_t kQueueCap = 256;

constexpr uint32_t kHashK = 0x9E3779u;  // 24-bit odd multiplier

// Blocked-Bloom filter hash of a 3-byte window: one 32-bit filter word and two
// bit positions inside it (k = 2 in one word: one LDS read per position).
// w3 holds the window in its low 24 bits (little endian, oldest byte lowest);
// any upper byte is ignored.  On gfx950 the two halves of the 48-bit product
// are v_mul_u32_u24 and v_mul_hi_u32_u24 (full rate).
struct FilterProbe {
  uint32_t word;  // index into the kFilterWords-word filter
  uint32_t b1, b2;
};
__host__ __device__ inline FilterProbe filter_probe(uint32_t w3) {
  const uint32_t x = w3 & 0xFFFFFFu;
  const uint32_t lo = x * kHashK;
  const uint32_t hi = (uint32_t)(((uint64_t)x * kHashK) >> 32);
  return FilterProbe{hi & (kFilterWords - 1), lo >> 27, (lo >> 22) & 31u};
}

// Exact table: open addressing, linear probing, 64-bit slots
//   slot = (1 << 63) | (len << 32) | key,  0 = empty
// key = the last `len` bytes before the position, little endian.
__host__ __device__ inline uint64_t exact_entry(uint32_t key, uint32_t len) {
  return (1ull << 63) | ((uint64_t)len << 32) | key;
}
__host__ __device__ inline uint32_t exact_hash(uint32_t key, uint32_t len) {
  uint32_t h = key * 0x85EBCA6Bu ^ (len * 0xC2B2AE35u);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 13;
  return h;
}

struct ScanParams {
  const uint8_t* data;      // block base in HBM (16-byte aligned)
  uint64_t block_size;      // bytes in the block
  uint64_t byte_begin;      // first byte of this launch (multiple of 16)
  uint64_t byte_end;        // one past the last byte
  const uint32_t* filter;   // kFilterWords words
  const uint64_t* exact;    // exact_slots entries
  uint32_t exact_mask;      // exact_slots - 1
  uint32_t len_mask;        // bit L set iff keys of length L exist
  uint32_t n_segments;
  uint32_t seg_bytes;       // bytes per segment (multiple of kTile)
  uint32_t seg_cap;         // output capacity (entries) per segment
  uint32_t* seg_count;      // [n_segments] candidates found (may exceed cap)
  uint32_t* seg_out;        // [n_segments * seg_cap] byte offset within segment
};

}  // namespace yamd
