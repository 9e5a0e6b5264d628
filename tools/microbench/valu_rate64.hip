// Issue rate of the 64-bit shift forms (gfx950) against the 32-bit VOP2
// shift: can one v_lshrrev_b64 produce the shifted values of two 32-bit
// registers at the cost of one instruction?  8 independent chains per lane,
// 1024-thread workgroups.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t iters, uint32_t seed) {
  uint64_t a[8];
  uint32_t b[8];
  for (int i = 0; i < 8; ++i) {
    a[i] = (uint64_t)seed * (threadIdx.x + 1 + i * 7919) * 0x9E3779B97F4A7C15ull;
    b[i] = seed * (threadIdx.x + 3 + i * 31);
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == 0)  // v_lshrrev_b64 by a register amount
          asm("v_lshrrev_b64 %0, %1, %0" : "+v"(a[i]) : "v"(b[(i + 1) & 7]));
        if constexpr (OP == 1)  // v_lshrrev_b64 by an inline constant
          asm("v_lshrrev_b64 %0, 5, %0" : "+v"(a[i]));
        if constexpr (OP == 2)  // v_lshrrev_b32 (VOP2), for reference
          asm("v_lshrrev_b32 %0, %1, %0" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
        if constexpr (OP == 3)  // v_lshlrev_b64 by a constant
          asm("v_lshlrev_b64 %0, 3, %0" : "+v"(a[i]));
        if constexpr (OP == 4)  // v_lshl_add_u64
          asm("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
        if constexpr (OP == 5)  // v_mov_b32_dpp wave_shr:1
          asm("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(b[i]) : "v"(b[(i + 1) & 7]));
        if constexpr (OP == 6)  // v_bfe_u32 with constant offset/width
          asm("v_bfe_u32 %0, %0, 10, 14" : "+v"(b[i]));
        if constexpr (OP == 7)  // v_and_b32 with a literal
          asm("v_and_b32 %0, 0x1fff8, %0" : "+v"(b[i]));
        if constexpr (OP == 8)  // v_alignbit_b32 with a register amount
          asm("v_alignbit_b32 %0, %1, %0, %2" : "+v"(b[i]) : "v"(b[(i + 1) & 7]), "v"(b[(i + 2) & 7]));
        if constexpr (OP == 9)  // v_pk_mov_b32 (two dwords)
          asm("v_pk_mov_b32 %0, %1, %0 op_sel:[1,0]" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
      }
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= (uint32_t)a[i] ^ (uint32_t)(a[i] >> 32) ^ b[i];
  if (s == 0x12345678) out[0] = s;
}

template <int OP>
double run(uint32_t* out, int grid, uint32_t iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(1024), 0, 0, out, iters, 3u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(1024), 0, 0, out, iters, 3u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  uint32_t* out;
  hipMalloc(&out, 4);
  int cus;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint32_t iters = 4096;
  const char* names[] = {"lshrrev_b64_v", "lshrrev_b64_k", "lshrrev_b32", "lshlrev_b64_k", "lshl_add_u64",
                         "mov_dpp_wshr", "bfe_k", "and_literal", "alignbit_v", "pk_mov_b32"};
  for (int g : {cus, 2 * cus}) {
    double ms[10] = {run<0>(out, g, iters), run<1>(out, g, iters), run<2>(out, g, iters),
                     run<3>(out, g, iters), run<4>(out, g, iters), run<5>(out, g, iters),
                     run<6>(out, g, iters), run<7>(out, g, iters), run<8>(out, g, iters),
                     run<9>(out, g, iters)};
    for (int o = 0; o < 10; ++o) {
      double winstr = (double)g * 16 * iters * 64;
      printf("grid %d  %-15s %8.3f ms  %.3f wave-instr/clk/CU @2.4GHz\n", g, names[o], ms[o],
             winstr / (ms[o] * 1e-3) / cus / 2.4e9);
    }
  }
  return 0;
}
