// VALU issue-rate microbenchmark on gfx950: per-op throughput with 8
// independent chains per lane, 1024-thread workgroups, 1 WG/CU or more.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t iters, uint32_t seed) {
  uint32_t a[8];
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1 + i * 7919);
  const uint32_t c = seed | 1;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (OP == 0) a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) & 7], 1);  // alignbit
        if constexpr (OP == 1) a[i] = (a[i] & 0xFFFFFF) * 0x9E3779u ^ c;                     // mul_u24 (+xor)
        if constexpr (OP == 2) a[i] = (uint32_t)(((uint64_t)(a[i] & 0xFFFFFF) * 0x9E3779u) >> 32) + c; // mul_hi_u24 (+add)
        if constexpr (OP == 3) a[i] = (a[i] >> (a[(i + 3) & 7] & 31)) ^ c;                   // lshr + xor
        if constexpr (OP == 4) a[i] = a[i] + c;                                               // add
        if constexpr (OP == 5) a[i] = __builtin_amdgcn_alignbyte(a[i], a[(i + 1) & 7], 1);  // alignbyte
        if constexpr (OP == 6) a[i] = __builtin_amdgcn_perm(a[i], a[(i + 1) & 7], 0x06050403u);  // perm
        if constexpr (OP == 7) a[i] = __builtin_amdgcn_ubfe(a[(i + 1) & 7], a[i], 1) ^ a[i];       // bfe + xor
        if constexpr (OP == 8) a[i] = ((a[i] >> 7) ^ (a[(i + 1) & 7] << 2)) & 0x1FFFCu;            // lshr,lshl,bitop3
        if constexpr (OP == 9) a[i] = (a[(i + 1) & 7] << (i + 1)) | a[i];                          // lshl_or
        if constexpr (OP == 10)  // v_and_b32_sdwa into byte 1, preserving the rest
          asm("v_and_b32_sdwa %0, %1, %2 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
              : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
        if constexpr (OP == 11)  // v_lshrrev_b32_sdwa, amount = byte 1 of a register
          asm("v_lshrrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
              : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
        if constexpr (OP == 12)  // packed 16-bit shift: two shifts per lane
          asm("v_pk_lshrrev_b16 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
        if constexpr (OP == 13)  // v_and_or_b32
          asm("v_and_or_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
        if constexpr (OP == 14)  // v_bitop3_b32 (a & b) | c
          asm("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xec" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
        if constexpr (OP == 15)  // v_lshl_or_b32 with a register shift amount
          asm("v_lshl_or_b32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]));
        if constexpr (OP == 16)  // v_lshrrev_b32 (VOP2) alone
          asm("v_lshrrev_b32 %0, %1, %0" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
      }
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s ^= a[i];
  if (s == 0x12345678) out[0] = s;
}

template <int OP>
double run(uint32_t* out, int grid, uint32_t iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(1024), 0, 0, out, iters, 3u);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(1024), 0, 0, out, iters, 3u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  uint32_t* out; hipMalloc(&out, 4);
  int cus; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint32_t iters = 4096;
  const char* names[] = {"alignbit", "mul_u24+xor", "mul_hi_u24+add", "lshr+xor", "add", "alignbyte", "perm", "bfe+xor", "lshr,lshl,bitop3", "lshl_or", "and_sdwa_byte", "lshr_sdwa_src",
                         "pk_lshrrev_b16", "and_or", "bitop3", "lshl_or_vvv", "lshrrev_vop2"};
  for (int g : {cus, 2 * cus}) {
    double ms[17] = {run<0>(out, g, iters), run<1>(out, g, iters), run<2>(out, g, iters),
                    run<3>(out, g, iters), run<4>(out, g, iters), run<5>(out, g, iters),
                    run<6>(out, g, iters), run<7>(out, g, iters), run<8>(out, g, iters),
                    run<9>(out, g, iters), run<10>(out, g, iters), run<11>(out, g, iters),
                    run<12>(out, g, iters), run<13>(out, g, iters), run<14>(out, g, iters),
                    run<15>(out, g, iters), run<16>(out, g, iters)};
    for (int o = 0; o < 17; ++o) {
      // wave-instructions executed per chain-step
      const double nops[17] = {1, 2, 2, 2, 1, 1, 1, 2, 3, 1, 1, 1, 1, 1, 1, 1, 1};
      double ops = nops[o];
      double winstr = (double)g * 16 * iters * 64 * ops;
      printf("grid %d  %-15s %8.3f ms  %.3f wave-instr/clk/CU @2.4GHz  (%.1f G lane-op/s/CU)\n", g,
             names[o], ms[o], winstr / (ms[o] * 1e-3) / cus / 2.4e9, winstr * 64 / (ms[o] * 1e-3) / cus / 1e9);
    }
  }
  return 0;
}
