// Device trace of the reference walk (yr_amd_trace_walk, include/yara_amd.h):
// the analogue of libyara/scanner.c:83-96's YR_DEBUG_VERBOSITY == 2 output.
//
// One lane per block position i: the walk's state after bytes [0, i) is the
// state reached from the root over the last <= 4 of them (the trie is at most
// YR_MAX_ATOM_LENGTH deep), each byte taken with the reference's transition
// rule -- the slot check and the failure links of the untouched transition
// table (scanner.c:123-141).  Nothing here shares code with the scan kernel's
// filter path, so the trace is an independent device-side check of it.
//
// Two passes over the positions: counts per 256-position block, then the rows
// written at the blocks' offsets (the host turns counts into offsets; this is a
// debugging path for small blocks, not a hot one).
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/yara_amd.h"

namespace yamd {

namespace {

constexpr int kTraceThreads = 256;
constexpr uint32_t kMaxDepth = 4;   // YR_MAX_ATOM_LENGTH (limits.h)

__device__ __forceinline__ uint32_t walk_state(const uint32_t* T, const uint8_t* data,
                                               uint64_t i) {
  uint32_t state = 0;
  for (uint64_t j = i > kMaxDepth ? i - kMaxDepth : 0; j < i; ++j) {
    const uint32_t index = (uint32_t)data[j] + 1u;
    uint32_t t = T[state + index];
    while ((t & 0x1FFu) != index) {   // YR_AC_INVALID_TRANSITION
      if (state != 0u) {
        state = T[state] >> 9;        // YR_AC_NEXT_STATE of the failure link
        t = T[state + index];
      } else {
        t = 0u;
        break;
      }
    }
    state = t >> 9;
  }
  return state;
}

__global__ __launch_bounds__(kTraceThreads) void trace_count_kernel(const uint32_t* T,
                                                                   const uint8_t* data,
                                                                   uint64_t n_pos,
                                                                   uint32_t* block_count) {
  const uint64_t i = (uint64_t)blockIdx.x * kTraceThreads + threadIdx.x;
  const bool row = i < n_pos && walk_state(T, data, i) != 0u;
  const int c = __syncthreads_count(row);
  if (threadIdx.x == 0) block_count[blockIdx.x] = (uint32_t)c;
}

__global__ __launch_bounds__(kTraceThreads) void trace_write_kernel(
    const uint32_t* T, const uint32_t* M, const uint8_t* data, uint64_t n_pos,
    const uint64_t* block_offset, yr_amd_trace_rec* out, uint64_t cap) {
  __shared__ uint32_t wave_base[kTraceThreads / 64];
  const uint64_t i = (uint64_t)blockIdx.x * kTraceThreads + threadIdx.x;
  const uint32_t state = i < n_pos ? walk_state(T, data, i) : 0u;
  const bool row = state != 0u;
  const uint64_t ballot = __ballot(row);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(ballot >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)ballot, 0u));
  if (lane == 0) wave_base[wave] = (uint32_t)__popcll(ballot);
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < wave; ++w) before += wave_base[w];
  if (row) {
    const uint64_t k = block_offset[blockIdx.x] + before + below;
    if (k < cap) {
      yr_amd_trace_rec r;
      r.position = i;
      r.state = state;
      r.match = M[state];
      out[k] = r;
    }
  }
}

}  // namespace

hipError_t launch_trace_count(const uint32_t* T, const uint8_t* data, uint64_t n_pos,
                              uint32_t* block_count, uint32_t n_blocks, hipStream_t s) {
  hipLaunchKernelGGL(trace_count_kernel, dim3(n_blocks), dim3(kTraceThreads), 0, s, T, data, n_pos,
                     block_count);
  return hipGetLastError();
}

hipError_t launch_trace_write(const uint32_t* T, const uint32_t* M, const uint8_t* data,
                              uint64_t n_pos, const uint64_t* block_offset,
                              yr_amd_trace_rec* out, uint64_t cap, uint32_t n_blocks,
                              hipStream_t s) {
  hipLaunchKernelGGL(trace_write_kernel, dim3(n_blocks), dim3(kTraceThreads), 0, s, T, M, data,
                     n_pos, block_offset, out, cap);
  return hipGetLastError();
}

}  // namespace yamd
