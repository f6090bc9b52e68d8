// ubench.hip — issue cost of single VALU instructions on gfx950 (diagnostic, tools/ubench.py).
// Each wave runs ITERS x 8 independent copies of one instruction (8 separate destination registers,
// so throughput, not latency, is measured) between two s_memtime stamps; cycles per instruction =
// delta / (ITERS * 8).  Launched with 1 or 2 waves per SIMD; the s_memrealtime (100 MHz) delta gives
// the wall time, so the SIMD's aggregate issue rate at 2 waves is comparable with 1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BODY8(INS)                                                                                     \
  asm volatile(INS " %0, %8, %9\n\t" INS " %1, %8, %9\n\t" INS " %2, %8, %9\n\t" INS " %3, %8, %9\n\t" \
               INS " %4, %8, %9\n\t" INS " %5, %8, %9\n\t" INS " %6, %8, %9\n\t" INS " %7, %8, %9"      \
               : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)        \
               : "v"(a), "v"(b))

template <int OP>
__global__ void __launch_bounds__(512) ubench_kernel(int iters, uint32_t seed, long long* cyc, uint32_t* sink) {
  uint32_t r0 = seed ^ threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, r6 = r0 + 6,
           r7 = r0 + 7;
  uint32_t a = seed * 3u + threadIdx.x, b = seed * 7u + 1u;
  const long long t0 = __builtin_amdgcn_s_memtime();
  const long long r0t = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) BODY8("v_add_u32");
    if constexpr (OP == 1) BODY8("v_mul_lo_u32");
    if constexpr (OP == 2) BODY8("v_mul_hi_u32");
    if constexpr (OP == 3) BODY8("v_fmac_f32");
    if constexpr (OP == 4) BODY8("v_xor_b32");
    if constexpr (OP == 5) {   // v_mad_u64_u32 d[2], null, a, b, 0 : 64-bit destination pairs
      uint64_t q0 = r0, q1 = r1, q2 = r2, q3 = r3;
      uint64_t c0, c1, c2, c3;    // carry-out SGPR pairs (unused)
      asm volatile("v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\t"
                   "v_mad_u64_u32 %2, %6, %8, %9, %2\n\tv_mad_u64_u32 %3, %7, %8, %9, %3\n\t"
                   "v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\t"
                   "v_mad_u64_u32 %2, %6, %8, %9, %2\n\tv_mad_u64_u32 %3, %7, %8, %9, %3"
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
                   : "v"(a), "v"(b));
      r0 = (uint32_t)q0; r1 = (uint32_t)q1; r2 = (uint32_t)q2; r3 = (uint32_t)q3;
    }
    if constexpr (OP == 6) {   // v_exp_f32 (1 source)
      asm volatile("v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"
                   "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
    }
    if constexpr (OP == 7) {   // v_pk_fma_f32 on 64-bit pairs
      uint64_t q0 = r0, q1 = r1, q2 = r2, q3 = r3;
      const uint64_t ab = ((uint64_t)b << 32) | a;
      asm volatile("v_pk_fma_f32 %0, %4, %4, %0\n\tv_pk_fma_f32 %1, %4, %4, %1\n\t"
                   "v_pk_fma_f32 %2, %4, %4, %2\n\tv_pk_fma_f32 %3, %4, %4, %3\n\t"
                   "v_pk_fma_f32 %0, %4, %4, %0\n\tv_pk_fma_f32 %1, %4, %4, %1\n\t"
                   "v_pk_fma_f32 %2, %4, %4, %2\n\tv_pk_fma_f32 %3, %4, %4, %3"
                   : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(ab));
      r0 = (uint32_t)q0; r1 = (uint32_t)q1; r2 = (uint32_t)q2; r3 = (uint32_t)q3;
    }
    if constexpr (OP == 8) BODY8("v_mul_u32_u24");
    if constexpr (OP == 10) {   // v_fmac_f32, 64 per iteration: the loop branch amortised 8x further
#pragma unroll
      for (int u = 0; u < 8; ++u) BODY8("v_fmac_f32");
    }
    if constexpr (OP == 11) {   // v_exp_f32, 64 per iteration
#pragma unroll
      for (int u = 0; u < 8; ++u)
        asm volatile("v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"
                     "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7"
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
    }
    if constexpr (OP == 13) {   // v_pk_fma_f32, 64 per iteration
      uint64_t q0 = r0, q1 = r1, q2 = r2, q3 = r3;
      const uint64_t ab = ((uint64_t)b << 32) | a;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        asm volatile("v_pk_fma_f32 %0, %4, %4, %0\n\tv_pk_fma_f32 %1, %4, %4, %1\n\t"
                     "v_pk_fma_f32 %2, %4, %4, %2\n\tv_pk_fma_f32 %3, %4, %4, %3\n\t"
                     "v_pk_fma_f32 %0, %4, %4, %0\n\tv_pk_fma_f32 %1, %4, %4, %1\n\t"
                     "v_pk_fma_f32 %2, %4, %4, %2\n\tv_pk_fma_f32 %3, %4, %4, %3"
                     : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3) : "v"(ab));
      r0 = (uint32_t)q0; r1 = (uint32_t)q1; r2 = (uint32_t)q2; r3 = (uint32_t)q3;
    }
    if constexpr (OP == 14) {   // v_cvt_pk_bf16_f32, 64 per iteration
#pragma unroll
      for (int u = 0; u < 8; ++u) BODY8("v_cvt_pk_bf16_f32");
    }
    if constexpr (OP == 15) {   // v_accvgpr_read_b32, 64 per iteration (8 AGPRs written once)
      asm volatile("v_accvgpr_write_b32 a0, %0\n\tv_accvgpr_write_b32 a1, %0\n\tv_accvgpr_write_b32 a2, %0\n\t"
                   "v_accvgpr_write_b32 a3, %0\n\tv_accvgpr_write_b32 a4, %0\n\tv_accvgpr_write_b32 a5, %0\n\t"
                   "v_accvgpr_write_b32 a6, %0\n\tv_accvgpr_write_b32 a7, %0\n\ts_nop 2" ::"v"(a) : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7");
#pragma unroll
      for (int u = 0; u < 8; ++u)
        asm volatile("v_accvgpr_read_b32 %0, a0\n\tv_accvgpr_read_b32 %1, a1\n\tv_accvgpr_read_b32 %2, a2\n\t"
                     "v_accvgpr_read_b32 %3, a3\n\tv_accvgpr_read_b32 %4, a4\n\tv_accvgpr_read_b32 %5, a5\n\t"
                     "v_accvgpr_read_b32 %6, a6\n\tv_accvgpr_read_b32 %7, a7"
                     : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3), "=v"(r4), "=v"(r5), "=v"(r6), "=v"(r7));
    }
    if constexpr (OP == 12) {   // v_mad_u64_u32, 64 per iteration (4 chains x 2 per BODY)
      uint64_t q0 = r0, q1 = r1, q2 = r2, q3 = r3;
      uint64_t c0, c1, c2, c3;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        asm volatile("v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\t"
                     "v_mad_u64_u32 %2, %6, %8, %9, %2\n\tv_mad_u64_u32 %3, %7, %8, %9, %3\n\t"
                     "v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %1, %5, %8, %9, %1\n\t"
                     "v_mad_u64_u32 %2, %6, %8, %9, %2\n\tv_mad_u64_u32 %3, %7, %8, %9, %3"
                     : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
                     : "v"(a), "v"(b));
      r0 = (uint32_t)q0; r1 = (uint32_t)q1; r2 = (uint32_t)q2; r3 = (uint32_t)q3;
    }
    if constexpr (OP == 9) {   // v_rcp_f32 (1 source)
      asm volatile("v_rcp_f32 %0, %0\n\tv_rcp_f32 %1, %1\n\tv_rcp_f32 %2, %2\n\tv_rcp_f32 %3, %3\n\t"
                   "v_rcp_f32 %4, %4\n\tv_rcp_f32 %5, %5\n\tv_rcp_f32 %6, %6\n\tv_rcp_f32 %7, %7"
                   : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7));
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const long long r1t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x % 64 == 0) {     // [wave][2]: s_memtime ticks, s_memrealtime ticks (100 MHz)
    cyc[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = t1 - t0;
    cyc[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) + 1] = r1t - r0t;
  }
  sink[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
}

extern "C" int ubench(int op, int blocks, int threads, int iters, long long* cyc, uint32_t* sink) {
  const dim3 g(blocks), t(threads);
  switch (op) {
    case 0: hipLaunchKernelGGL(ubench_kernel<0>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 1: hipLaunchKernelGGL(ubench_kernel<1>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 2: hipLaunchKernelGGL(ubench_kernel<2>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 3: hipLaunchKernelGGL(ubench_kernel<3>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 4: hipLaunchKernelGGL(ubench_kernel<4>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 5: hipLaunchKernelGGL(ubench_kernel<5>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 6: hipLaunchKernelGGL(ubench_kernel<6>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 7: hipLaunchKernelGGL(ubench_kernel<7>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 8: hipLaunchKernelGGL(ubench_kernel<8>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 9: hipLaunchKernelGGL(ubench_kernel<9>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 10: hipLaunchKernelGGL(ubench_kernel<10>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 11: hipLaunchKernelGGL(ubench_kernel<11>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 12: hipLaunchKernelGGL(ubench_kernel<12>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 13: hipLaunchKernelGGL(ubench_kernel<13>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 14: hipLaunchKernelGGL(ubench_kernel<14>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    case 15: hipLaunchKernelGGL(ubench_kernel<15>, g, t, 0, 0, iters, 12345u, cyc, sink); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// LDS-DMA source pattern: a 256-row panel of a row-major [M][K] bf16 matrix streamed into a 5-deep LDS
// ring K-tile by K-tile (one s_waitcnt + one barrier per 32-deep K-tile, as the GEMM K-loops), with
//   PAT 0: each wave-instruction = 16 rows x 64 B (one K-tile's slice of each row: half a 128-B line)
//   PAT 1: each wave-instruction = 8 rows x 128 B (two K-tiles of each row: whole lines), issued for a
//          K-tile pair every second K-tile
// Same bytes, same instruction count; `rounds` passes over the same panel (L2-warm after the first).
template <int PAT>
__global__ void __launch_bounds__(256, 1) dma_kernel(const uint16_t* __restrict__ A, int K, int rounds, int panels,
                                                     long long* cyc) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[5 * 256 * 32];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint16_t* panel = A + (long)(blockIdx.x % panels) * 256 * K;   // panels < grid: L2-shared sources
  typedef __attribute__((address_space(3))) void lv;
  const uint32_t l0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lv*)lds);
  // raw buffer resource over the panel (gfx9 dword3 0x00020000), built from uniform values
  typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;
  const uint64_t pb = (uint64_t)(uintptr_t)panel;
  u32x4_t rsrc;
  rsrc[0] = __builtin_amdgcn_readfirstlane((uint32_t)pb);
  rsrc[1] = __builtin_amdgcn_readfirstlane((uint32_t)(pb >> 32) & 0xFFFFu);
  rsrc[2] = 0xFFFFFFFFu;
  rsrc[3] = 0x00020000u;
  asm volatile("s_nop 4" ::: "memory");
  const long long t0 = __builtin_amdgcn_s_memtime();
  const int nk = K / 32;
  for (int r = 0; r < rounds; ++r) {
    for (int kt = 0; kt < nk; ++kt) {
      const int slot = kt % 5;
      if (PAT == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = (wave * 4 + j) * 16 + (lane >> 2);
          const uint16_t* src = panel + (long)row * K + kt * 32 + (lane & 3) * 8;
          const uint32_t dst = l0 + 2u * (slot * 256 * 32 + (wave * 4 + j) * 16 * 32);
          asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(dst) : "memory");
        }
      } else if (PAT == 2) {      // PAT 0's rows through the buffer path (MUBUF ... lds)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = (wave * 4 + j) * 16 + (lane >> 2);
          const uint32_t voff = (uint32_t)(((long)row * K + kt * 32 + (lane & 3) * 8) * 2);
          const uint32_t dst = l0 + 2u * (slot * 256 * 32 + (wave * 4 + j) * 16 * 32);
          asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc),
                       "s"(dst) : "memory");
        }
      } else if (PAT == 3) {      // PAT 1's rows through the buffer path
        if ((kt & 1) == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int row = (wave * 8 + j) * 8 + (lane >> 3);
            const uint32_t voff = (uint32_t)(((long)row * K + kt * 32 + (lane & 7) * 8) * 2);
            const uint32_t dst = l0 + 2u * ((slot % 4) * 256 * 32 + (wave * 8 + j) * 8 * 64 % (256 * 32));
            asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff),
                         "s"(rsrc), "s"(dst) : "memory");
          }
        }
      } else if ((kt & 1) == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int row = (wave * 8 + j) * 8 + (lane >> 3);
          const uint16_t* src = panel + (long)row * K + kt * 32 + (lane & 7) * 8;
          const uint32_t dst = l0 + 2u * ((slot % 4) * 256 * 32 + (wave * 8 + j) * 8 * 64 % (256 * 32));
          asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(dst) : "memory");
        }
      }
      asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

extern "C" int ubench_dma(int pat, int blocks, const void* A, int K, int rounds, int panels, long long* cyc) {
  const uint16_t* a = (const uint16_t*)A;
  if (pat == 0) hipLaunchKernelGGL(dma_kernel<0>, dim3(blocks), dim3(256), 0, 0, a, K, rounds, panels, cyc);
  else if (pat == 1) hipLaunchKernelGGL(dma_kernel<1>, dim3(blocks), dim3(256), 0, 0, a, K, rounds, panels, cyc);
  else if (pat == 2) hipLaunchKernelGGL(dma_kernel<2>, dim3(blocks), dim3(256), 0, 0, a, K, rounds, panels, cyc);
  else hipLaunchKernelGGL(dma_kernel<3>, dim3(blocks), dim3(256), 0, 0, a, K, rounds, panels, cyc);
  return (int)hipGetLastError();
}
