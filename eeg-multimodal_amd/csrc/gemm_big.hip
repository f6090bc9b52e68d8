// gemm_big.hip — bf16 MFMA GEMMs for the token-sized projections (M = B*L rows): every BERT forward
// (x W^T + bias [+GELU / GELU']), input gradient (dY W [* act'] [+ residual]) and weight gradient
// (dY^T X over the tokens, split-K, with the bias row sums fused).
//
//   gemm4r  persistent 256x256, 4 waves of 128x128, whole-line K-tile pairs, rolling A fragments: every
//           full-tile bf16 GEMM with K % 64 == 0 (all of the bench step's forwards and input gradients);
//   gemm4p  the same persistent structure on 64-B half-line K-tiles: full tiles with other K;
//   gemm4w  non-persistent 4-wave 256x256: weight gradients (fp32 split-K slabs) and every other shape.
// Common structure (cdna_hip_programming.md §5): operands staged global -> LDS by asm LDS-DMA into XOR-
// swizzled images (conflict-free ds_read_b128 / ds_read_b64_tr_b16), accumulators pinned to AGPRs by
// asm MFMAs, counted vmcnt waits, XCD-aware tile order.  Edges (gemm4w): rows / cols beyond M / N are
// clamped to valid memory and never stored; K % 64 == 0.
// Retired in round 6 (superseded; git history 829c7a6): the 2-phase gemm_big_kernel, the 8-wave gemm8,
// the 256x128 two-workgroup gemm4h and the five-slot-ring gemm4q, with their timing probes.
#include <type_traits>

#include "common.h"
#include "eegfusion_internal.h"

namespace {

constexpr int TM = 256, TN = 256, BK = 64, NT = 512;
constexpr int TILE = TM * BK;                 // elements per operand tile (32 KB)
constexpr int LDC = TN + 8;                   // epilogue tile row stride (elements)
constexpr int LDS_ELEMS = TM * LDC;           // 135168 B >= 4 * TILE * 2 B

struct BigArgs {
  const bf16* A; const bf16* B; void* C; const float* bias; bf16* aux;
  long lda, ldb, ldc, ldaux;
  int M, N, K;
  float alpha, beta, epi_scale;
  int ksplit;            // >0: split-K slice length; C = fp32 slabs [blockIdx.y][M][N]
  float* rowsum_part;    // gemm4w RS only: [splits][M] sums over this split's K of each row of a k-major A
  long long* ts;         // diagnostics (eegf_gemm_big_timestamps): per-workgroup phase times, null = off
  int group_m;           // tile raster: 0 row-major, G > 0 groups of G row panels walked column by column
};
// groups of 4 row panels when the grid is at least 8 tile columns wide (the K = 768 forward / input-
// gradient GEMMs with N >= 2304: +2-4 %, profiles/r2r_group.log), row-major otherwise (N = 768: 3 tile
// columns, no gain)
int group_for(int N) { return (N + 255) / 256 >= 8 ? 4 : 0; }
// Logical tile t (after xcd_remap: consecutive t share an XCD) -> (tile row, tile column).  Grouped
// raster: G row panels x all column tiles per group, column-major inside the group, so the ~32 tiles
// an XCD runs at once touch G A-panels and ~32/G B-panels instead of ~3 A-panels and every B-panel.
DEV void tile_coords(const BigArgs& g, int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  if (g.group_m <= 0) {
    tm = t / tiles_n;
    tn = t % tiles_n;
    return;
  }
  const int per = g.group_m * tiles_n, grp = t / per, r = t % per;
  const int rows = min(g.group_m, tiles_m - grp * g.group_m);
  tm = grp * g.group_m + r % rows;
  tn = r / rows;
}
// Phase timestamps (100 MHz s_memrealtime) of one workgroup: 0 start, 1 prologue done, 2 K-loop done,
// 3 epilogue issued; slot 4 = the CU it ran on (8 int64 per workgroup) -- tools/gemm_phases.py turns them into per-phase times and dispatch gaps
#ifndef EEGF_DIAG
#define EEGF_DIAG 0
#endif
DEV void ts_mark(const BigArgs& g, int k) {
  if (EEGF_DIAG && g.ts && threadIdx.x == 0) {
    long long* p = g.ts + ((long)blockIdx.y * gridDim.x + blockIdx.x) * 8;
    p[k] = (long long)__builtin_amdgcn_s_memrealtime();
    if (k == 0) {                    // which CU: XCC id << 16 | HW_ID bits 8-15 (CU, SH, SE)
      uint32_t hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      p[4] = (long long)(((xcc & 15u) << 16) | ((hw >> 8) & 255u));
    }
  }
}
long long* g_ts_buf = nullptr;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glb_void;

DEV void glds16(const bf16* g, bf16* lds_base) { glds16_asm(g, lds_base); }   // common.h: why asm

DEV int swz_row(int r) { return (r >> 1) & 7; }
DEV int swz_k(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

// Row-major operand tile rows [r0, r0+256) x k [k0, k0+64): 4 glds per wave.
DEV void stage_rowmajor(bf16* dst, const bf16* src, long ld, int r0, int rmax, int k0, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int R0 = (wave * 4 + j) * 8;
    const int r = R0 + (lane >> 3);
    const int c = (lane & 7) ^ swz_row(r);
    const int gr = min(r0 + r, rmax - 1);
    glds16(src + (long)gr * ld + k0 + c * 8, dst + R0 * BK);
  }
}

// k-major operand tile k [k0, k0+64) x cols [c0, c0+256): 4 glds per wave.
DEV void stage_kmajor(bf16* dst, const bf16* src, long ld, int c0, int cmax, int k0, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int K0 = (wave * 4 + j) * 2;
    const int k = K0 + (lane >> 5);
    const int c = (lane & 31) ^ swz_k(k);
    const int col = min(c0 + c * 8, cmax - 8);
    glds16(src + (long)(k0 + k) * ld + col, dst + K0 * TN);
  }
}

DEV bf16x8 rd_row(const bf16* t, int r, int chunk) {
  return *(const bf16x8*)(t + r * BK + ((chunk ^ swz_row(r)) << 3));
}

// 8 k-values (k0+0..3, k0+4..7 of the lane's 16-group) of column c0 + (lane&15) from a k-major tile
DEV bf16x8 rd_col(const bf16* t, int k0, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;
  const int ch = col >> 3, off = col & 7;
  const int ka = k0 + q, kb = k0 + 4 + q;
  const bf16* a0 = t + ka * TN + (((ch ^ swz_k(ka)) << 3) | off);
  const bf16* a1 = t + kb * TN + (((ch ^ swz_k(kb)) << 3) | off);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// rd_col on a row-major [256][64] tile: 8 rows r0..r0+7 (lane group) of column c0 + (lane&15)
DEV bf16x8 rd_col_rm(const bf16* t, int r0, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int col = c0 + 4 * p;
  const int ch = col >> 3, off = col & 7;
  const int ra = r0 + q, rb = r0 + 4 + q;
  const bf16* a0 = t + ra * BK + (((ch ^ swz_row(ra)) << 3) | off);
  const bf16* a1 = t + rb * BK + (((ch ^ swz_row(rb)) << 3) | off);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

template <bool LOAD, int NTH = NT, int TNT = TN, bool BATCHED = false>
DEV void tile_io(bf16* lds, bf16* gp, long ld, int m0, int n0, int M, int N, int tid) {
  constexpr int LDCT = TNT + 8, CPR = TNT / 8;      // epilogue tile row stride, 16-B chunks per row
  constexpr int ITER = (TM * TNT / 8) / NTH;
  if (BATCHED && m0 + TM <= M && n0 + TNT <= N) {
    // interior tile: BATCH loads in flight before the first use.  The guarded loop below compiles
    // to load -> s_waitcnt vmcnt(0) -> ds_write per 16-B chunk, i.e. one full memory round trip per
    // chunk (16 per thread for the aux tile of the activation-product input gradient).  Batch sized
    // to the registers left free while the accumulators are live: 4 for the 8-wave and the
    // two-workgroup kernels, 8 for the 4-wave 256x256 kernel.  (Batching the final LDS -> global
    // store the same way measured no change: profiles/r2x_lib_ab.log.)
    constexpr int BATCH = (NTH >= 512 || TNT < TN) ? 4 : 8;
#pragma unroll
    for (int k0 = 0; k0 < ITER; k0 += BATCH) {
      u32x4 v[BATCH];
#pragma unroll
      for (int b = 0; b < BATCH; ++b) {
        const int c = tid + NTH * (k0 + b);
        const int r = c / CPR, cc = (c % CPR) * 8;
        v[b] = LOAD ? ld16(gp + (long)(m0 + r) * ld + n0 + cc) : ld16(lds + r * LDCT + cc);
      }
#pragma unroll
      for (int b = 0; b < BATCH; ++b) {
        const int c = tid + NTH * (k0 + b);
        const int r = c / CPR, cc = (c % CPR) * 8;
        if (LOAD) st16(lds + r * LDCT + cc, v[b]);
        else st16(gp + (long)(m0 + r) * ld + n0 + cc, v[b]);
      }
    }
    return;
  }
#pragma unroll 4
  for (int k = 0; k < (TM * TNT / 8) / NTH; ++k) {
    const int c = tid + NTH * k;
    const int r = c / CPR, cc = (c % CPR) * 8;
    const int m = m0 + r, n = n0 + cc;
    if (m >= M || n >= N) continue;
    bf16* g = gp + (long)m * ld + n;
    bf16* l = lds + r * LDCT + cc;
    if (n + 8 <= N) {
      if (LOAD) st16(l, ld16(g)); else st16(g, ld16(l));
    } else {
      for (int e = 0; e < 8 && n + e < N; ++e) { if (LOAD) l[e] = g[e]; else g[e] = l[e]; }
    }
  }
}

DEV void ld4(const bf16* p, float (&v)[4]) { const bf16x4 x = *(const bf16x4*)p; v[0] = (float)x[0]; v[1] = (float)x[1]; v[2] = (float)x[2]; v[3] = (float)x[3]; }
DEV void st4(bf16* p, const float (&v)[4]) { bf16x4 x; x[0] = (bf16)v[0]; x[1] = (bf16)v[1]; x[2] = (bf16)v[2]; x[3] = (bf16)v[3]; *(bf16x4*)p = x; }

// Shared epilogue of the 256x256 kernels: acc[i][j] holds rows wm*128 + 16i + (lane&15), columns
// wn*16NJ + 16j + 4*(lane>>4) + 0..3 of the block tile (m0, n0) (NJ = 4: 8 waves of 128x64, NJ = 8:
// 4 waves of 128x128); NTH threads.
template <int EPI, typename TO, int NJ = 4, int NTH = NT, int TNT = TN>
DEV void big_epilogue(const BigArgs& g, f32x4 (&acc)[8][NJ], bf16* lds, int m0, int n0, int tid, int lane, int wm,
                      int wn, int split = -1) {   // split: the split-K slab (-1: blockIdx.y)
  constexpr int WN = 16 * NJ;
  constexpr int LDC = TNT + 8;
  constexpr bool HAS_BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_TANH ||
                            EPI == EPI_BIAS_GELU_D;
  constexpr bool AUX_IN = EPI == EPI_DGELU || EPI == EPI_DRELU || EPI == EPI_DTANH || EPI == EPI_MUL_AUX;
  if constexpr (sizeof(TO) == 4) {
    // fp32 output (weight gradients): direct 16-B stores of 4 consecutive columns; split-K slabs
    float* Cf = (float*)g.C + (g.ksplit > 0 ? (long)(split >= 0 ? split : (int)blockIdx.y) * g.M * g.N : 0);
    const long ldc = g.ksplit > 0 ? g.N : g.ldc;
    const float beta = g.ksplit > 0 ? 0.f : g.beta;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wm * 128 + i * 16 + (lane & 15);
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = n0 + wn * WN + j * 16 + 4 * (lane >> 4);
        float* cp = Cf + (long)m * ldc + n;
        f32x4 v = acc[i][j] * g.alpha;
        if (n + 3 < g.N && ((uintptr_t)cp & 15) == 0) {
          if (beta != 0.f) v += beta * *(const f32x4*)cp;
          *(f32x4*)cp = v;
        } else {
          for (int r = 0; r < 4; ++r)
            if (n + r < g.N) cp[r] = v[r] + (beta != 0.f ? beta * cp[r] : 0.f);
        }
      }
    }
    return;
  } else {
  // LDS-staged bf16 epilogue: every global access is a full 16-B-per-lane row segment
  bf16* ct = lds;
  bf16* Cb = (bf16*)g.C;
  // the lane's bias values for all NJ column groups in one batch of 16-B loads (one wait): loaded per
  // column group inside the loop below, each group paid a full L2 round trip before its first use
  constexpr bool BIAS_PRE = HAS_BIAS && TNT == TN;   // the 256x128 kernel has no registers to spare
  f32x4 biasv[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    biasv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (BIAS_PRE) {
      const int n = n0 + wn * WN + j * 16 + 4 * (lane >> 4);
      if (n + 3 < g.N && ((uintptr_t)(g.bias + n) & 15) == 0) biasv[j] = *(const f32x4*)(g.bias + n);
      else
        for (int r = 0; r < 4; ++r) biasv[j][r] = (n + r < g.N) ? g.bias[n + r] : 0.f;
    }
  }
  if (AUX_IN || g.beta != 0.f) {
    // batched for the beta * C tile too: the guarded loop's per-chunk round trips cost the residual-
    // accumulating input gradients (beta = 1) ~50 us per launch (284 vs 233 us at beta = 0)
    tile_io<true, NTH, TNT, true>(ct, AUX_IN ? g.aux : Cb, AUX_IN ? g.ldaux : g.ldc, m0, n0, g.M, g.N, tid);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nl = wn * WN + j * 16 + 4 * (lane >> 4);
    float bias[4] = {biasv[j][0], biasv[j][1], biasv[j][2], biasv[j][3]};
    if (HAS_BIAS && !BIAS_PRE)
      for (int r = 0; r < 4; ++r) bias[r] = (n0 + nl + r < g.N) ? g.bias[n0 + nl + r] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16* lp = ct + (wm * 128 + i * 16 + (lane & 15)) * LDC + nl;
      float av[4] = {0.f, 0.f, 0.f, 0.f};
      if (AUX_IN || g.beta != 0.f) ld4(lp, av);
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = g.alpha * acc[i][j][r];
        if (EPI == EPI_BIAS) v += bias[r];
        else if (EPI == EPI_BIAS_GELU) v = g.aux ? v + bias[r] : v;      // no aux: GELU below (packed)
        else if (EPI == EPI_BIAS_RELU) v = relu_nan(v + bias[r]);
        else if (EPI == EPI_BIAS_TANH) v = tanhf(v + bias[r]);
        else if (EPI == EPI_DGELU) v *= gelu_grad(av[r]);
        else if (EPI == EPI_DRELU) v = av[r] > 0.f ? v * g.epi_scale : 0.f;
        else if (EPI == EPI_DTANH) v *= (1.f - av[r] * av[r]);
        else if (EPI == EPI_MUL_AUX) v *= av[r];
        else if (g.beta != 0.f) v += g.beta * av[r];         // EPI_NONE accumulate (beta * C)
        acc[i][j][r] = v;
        o[r] = v;
      }
      if (EPI == EPI_BIAS_GELU_D || (EPI == EPI_BIAS_GELU && !g.aux)) {
        // packed GELU on the 4 values: _D stores gelu' in this (aux) round and keeps gelu in acc
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const f32x2 x = {acc[i][j][2 * h2] + bias[2 * h2], acc[i][j][2 * h2 + 1] + bias[2 * h2 + 1]};
          f32x2 gl, gd;
          gelu2(x, gl, EPI == EPI_BIAS_GELU_D ? &gd : nullptr);
          acc[i][j][2 * h2] = gl.x;
          acc[i][j][2 * h2 + 1] = gl.y;
          o[2 * h2] = EPI == EPI_BIAS_GELU_D ? gd.x : gl.x;
          o[2 * h2 + 1] = EPI == EPI_BIAS_GELU_D ? gd.y : gl.y;
        }
      }
      st4(lp, o);
    }
  }
  __syncthreads();
  if ((EPI == EPI_BIAS_GELU && g.aux) || EPI == EPI_BIAS_GELU_D) {
    // store the pre-activation tile, then compute GELU while those stores drain (raw barriers: a
    // __syncthreads() here would wait for the stores); LDS reads of the tile are complete per
    // thread once its stores have issued
    tile_io<false, NTH, TNT>(ct, g.aux, g.ldaux, m0, n0, g.M, g.N, tid);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (EPI == EPI_BIAS_GELU) {
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            f32x2 gl;
            gelu2(f32x2{acc[i][j][2 * h2], acc[i][j][2 * h2 + 1]}, gl, nullptr);
            acc[i][j][2 * h2] = gl.x;
            acc[i][j][2 * h2 + 1] = gl.y;
          }
        }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        st4(ct + (wm * 128 + i * 16 + (lane & 15)) * LDC + wn * WN + j * 16 + 4 * (lane >> 4), o);
      }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  tile_io<false, NTH, TNT>(ct, Cb, g.ldc, m0, n0, g.M, g.N, tid);
  }
}

DEV void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// ---------------------------------------------------------------------------------------------
// 4-wave 256x256 kernel (hipBLASLt's MT256x256x64 geometry measured on this chip: 256 threads, one
// wave per SIMD): 2 x 2 waves of 128x128 (64 accumulators = 256 registers per lane, AGPR-backed),
// BK = 32 K-tiles in a 5-deep LDS ring (5 x 32 KB), K-tile t + 5 staged while t computes, the next
// K-tile's fragments read while the current one's 64 MFMAs run (8 groups of {2 ds_read_b128, 1 LDS-DMA,
// 8 MFMAs} pinned by sched_barriers), one counted vmcnt + one barrier per K-tile.  A, B K-contiguous.
// LDS image of an operand K-tile: [256 rows][32 k] bf16 = 64-B rows; 16-B chunk c of row r stored at
// chunk c ^ sw4(r), sw4(r) = 3 * ((r >> 3) & 1): conflict-free for the ds_read_b128 lane groups of a
// 16-row fragment read (lanes 16q + i read row i, chunk q).
#ifndef EEGF_W_NOP
#define EEGF_W_NOP 0
#endif
constexpr int BK4 = 32, NT4 = 256, SLOT4 = 2 * TM * BK4;   // elements per ring slot (A + B, 32 KB)
constexpr int NSLOT4 = 5;                                     // ring depth: 5 x 32 KB = the 160 KB of LDS
static_assert(NSLOT4 * SLOT4 >= TM * LDC, "the epilogue tile reuses the ring");
DEV void vm_wait_tiles(int n) {    // n younger K-tiles (8 LDS-DMAs each) may stay in flight
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
  }
}
DEV int sw4(int r) { return 3 * ((r >> 3) & 1); }
// MFMA with the accumulator pinned to AGPRs (256 of them hold the 64 accumulators): hipcc otherwise
// keeps MFMA accumulators in VGPRs and spills.  Volatile: program order is the issue order.
DEV void mma16_acc(f32x4& acc, bf16x8 b, bf16x8 a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
// the same MFMA with a VGPR accumulator (the weight-gradient row sums against a ones operand; every
// AGPR holds the tile).  Its D is read only after the K-loop's closing s_nop padding (isa_lint
// mfma_d_read checks both register files)
// s_nop 2 first: hipcc does not pad a VALU write of an asm MFMA's source (it rebuilt the ones operand
// with v_mov right before it: NaN row sums, isa_lint mfma_src_write)
DEV void mma16_vacc(f32x4& acc, bf16x8 b, bf16x8 a) {
  asm volatile("s_nop 2\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(b), "v"(a));
}
// first K-tile: the accumulator is DEFINED in AGPRs (srcC = 0), so no VGPR copy of it ever exists
DEV void mma16_acc0(f32x4& acc, bf16x8 b, bf16x8 a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(b), "v"(a));
}

// the two ds_read_b64_tr_b16 of rd_col at precomputed element offsets o0 / o1
DEV bf16x8 rd_col_off(const bf16* t, int o0, int o1) {
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(t + o0));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(t + o1));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// AKC / BKC: operand K-contiguous (row-major [rows][K] image, ds_read_b128 fragments) or k-major
// ([K][cols] in memory: [32 k][256 cols] image with the swz_k chunk swizzle of stage_kmajor,
// ds_read_b64_tr_b16 fragments: input-gradient B, weight-gradient A and B)
// RS (weight gradients, A = dY k-major): the same kernel also sums every A row over K (the bias
// gradient dY.sum(0) of the nn.Linear whose weight gradient this is): in workgroups of tile column 0,
// wave (wm, wn) sums its row blocks s = 4 wn .. 4 wn + 3 by one MFMA per block and K-tile against a
// ones operand, partials -> rowsum_part[split][M].  Spreading the blocks over the tile row's
// workgroups (at most 2 per wave for 3 tile columns) measured the same (profiles/r5zd_ab_summary.log).
template <bool AKC, bool BKC, int EPI, typename TO, bool RS = false>
__global__ void __launch_bounds__(NT4, 1) gemm4w_kernel(BigArgs g) {
  constexpr int LDS4 = NSLOT4 * SLOT4;
  static_assert(LDS4 * 2 <= 160 * 1024 && LDS4 >= TM * LDC, "LDS budget / epilogue tile");
  __shared__ __attribute__((aligned(16))) bf16 lds[LDS4];   // ring NSLOT4 x 32 KB | epilogue tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (g.N + TN - 1) / TN, tiles_m = (g.M + TM - 1) / TM, ntiles = tiles_m * tiles_n;
  // split-K (weight gradients): the (split, tile) pairs are numbered XCD-major over the whole grid, so
  // the tiles of one split -- which share that split's K-slices of A (across tile columns) and of B
  // (across tile rows) -- run side by side on one XCD and its L2 serves the re-reads.  Numbered per
  // split (blockIdx.y) instead, a split's tiles land on all 8 XCDs: L2 hit 0.27-0.34 and 3x the
  // algorithmic HBM bytes at 6-6.8 TB/s, i.e. HBM-bound (profiles/r2y_pmc_table.md)
  int t, split = 0;
  if (gridDim.y > 1) {
    const int tt = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    split = tt / ntiles;
    t = tt % ntiles;
  } else {
    t = xcd_remap(blockIdx.x, ntiles);
  }
  int tm, tn;
  tile_coords(g, t, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * TM, n0 = tn * TN;
  int kbeg = 0, kend = g.K;
  if (g.ksplit > 0) { kbeg = split * g.ksplit; kend = min(g.K, kbeg + g.ksplit); }
  const int nk = (kend - kbeg) / BK4;

  // staging: 8 LDS-DMAs per thread per K-tile (4 A + 4 B), each wave-instruction 16 rows x 64 B, in
  // the saddr form: uniform K-tile base (SGPRs, advanced per K-tile) + a per-lane 32-bit byte offset
  // fixed for the whole loop (row clamped to the matrix, swizzled chunk)
  //   K-contiguous part j: rows (4w + j) 16 + lane / 4, 16-B chunk (lane & 3) ^ sw4(row) of the 64 B;
  //   k-major part j: k-rows (4w + j) 2 + lane / 32, 16-B column chunk (lane & 31) ^ swz_k(k) of 512 B
  auto voff_of = [&](bool kc, int j, int c0, int cmax, long ld) -> uint32_t {
    if (kc) {
      const int r = (wave * 4 + j) * 16 + (lane >> 2);
      const int c = (lane & 3) ^ sw4(r);
      return (uint32_t)(((long)(min(c0 + r, cmax - 1) - c0) * ld + c * 8) * 2);
    }
    const int k = (wave * 4 + j) * 2 + (lane >> 5);
    const int c = (lane & 31) ^ swz_k(k);
    return (uint32_t)(((long)k * ld + min(c0 + c * 8, cmax - 8) - c0) * 2);
  };
  uint32_t voffA[4], voffB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    voffA[j] = voff_of(AKC, j, m0, g.M, g.lda);
    voffB[j] = voff_of(BKC, j, n0, g.N, g.ldb);
  }
  // uniform base of K-tile kt: K-contiguous advances 32 elements, k-major 32 rows
  const bf16* baseA = AKC ? g.A + (long)m0 * g.lda + kbeg : g.A + (long)kbeg * g.lda + m0;
  const bf16* baseB = BKC ? g.B + (long)n0 * g.ldb + kbeg : g.B + (long)kbeg * g.ldb + n0;
  const long stepA = AKC ? BK4 : (long)BK4 * g.lda;
  const long stepB = BKC ? BK4 : (long)BK4 * g.ldb;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(lds));
  // part j of a K-tile -> ring slot; NOP as gemm4p's (0 in the K-loop, whose bases are pinned to SGPRs
  // at the top of each K-tile, 3 in the prologue)
  auto stage_part = [&](const bf16* bA, const bf16* bB, int slot, int j, auto Nc) __attribute__((always_inline)) {
    constexpr int NOP = decltype(Nc)::value;
    const bool kc = j < 4 ? AKC : BKC;
    const uint32_t dst = lds0 + 2u * (slot * SLOT4 + (j < 4 ? 0 : TM * BK4) +
                                      (wave * 4 + (j & 3)) * (kc ? 16 * BK4 : 2 * TN));
    if (j < 4) glds16_asm_sa<NOP>(bA, voffA[j & 3], dst);
    else glds16_asm_sa<NOP>(bB, voffB[j & 3], dst);
  };
  using WNOP = std::integral_constant<int, EEGF_W_NOP>;
  using NOP3 = std::integral_constant<int, 3>;
  // fragment reads.  K-contiguous: rows r0 + (lane & 15) of a [256][32] image, chunk lane >> 4; the
  // swizzle of row r0 + 16s + i equals that of row i (r0 % 16 == 0): one per-lane offset +
  // immediates.  k-major: rd_col of k-rows 8 (lane >> 4) + .., columns r0 + 16s + (lane & 15), at
  // per-fragment offsets precomputed once (16 VGPRs per operand)
  const int fr = lane & 15, fq = lane >> 4;
  const int offA = (wm * 128 + fr) * BK4 + ((fq ^ sw4(fr)) << 3);
  const int offB = TM * BK4 + (wn * 128 + fr) * BK4 + ((fq ^ sw4(fr)) << 3);
  int tA0[8], tA1[8], tB0[8], tB1[8];
  auto col_offs = [&](int c0, int& o0, int& o1) {
    const int q = fr >> 2, p4 = fr & 3;
    const int col = c0 + 4 * p4, ch = col >> 3, off = col & 7;
    const int ka = 8 * fq + q, kb = ka + 4;
    o0 = ka * TN + (((ch ^ swz_k(ka)) << 3) | off);
    o1 = kb * TN + (((ch ^ swz_k(kb)) << 3) | off);
  };
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (!AKC) col_offs(wm * 128 + 16 * i, tA0[i], tA1[i]);
    if (!BKC) {
      col_offs(wn * 128 + 16 * i, tB0[i], tB1[i]);
      tB0[i] += TM * BK4;
      tB1[i] += TM * BK4;
    }
  }
  auto rdA = [&](const bf16* img, int i) {
    return AKC ? *(const bf16x8*)(img + offA + i * 16 * BK4) : rd_col_off(img, tA0[i], tA1[i]);
  };
  auto rdB = [&](const bf16* img, int i) {
    return BKC ? *(const bf16x8*)(img + offB + i * 16 * BK4) : rd_col_off(img, tB0[i], tB1[i]);
  };
  f32x4 acc[8][8];           // defined by the first K-tile's MFMAs (mma16_acc0)
  // RS: the row sums of the wave's 4 row blocks (s = 4 wn .. 4 wn + 3), one MFMA per block and K-tile
  // against a ones operand into a VGPR accumulator: D[i][j] = sum over the K-tile's 32 k of A row 16 s + j
  // for every i.  Summed on the VALU instead (16 VALU per fragment: 64 per K-tile beside 64 MFMAs) it
  // made the whole launch 12 % slower than the plain weight gradient (profiles/r5zb_ab.log: the
  // workgroups of tile column 0 are the critical path of a one-wave grid); 4 MFMAs are 6 % of the
  // K-tile.  Not bitwise the VALU order; deterministic.
  const bool do_rs = RS && tn == 0;
  f32x4 rsacc[4] = {};
  bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
  asm volatile("" : "+v"(ones));     // opaque: kept in 4 VGPRs instead of rebuilt before every use

  // prologue: K-tiles 0 .. NSLOT4-1 staged; 0 and 1 retired
  ts_mark(g, 0);
  for (int kt = 0; kt < NSLOT4; ++kt)
    if (kt < nk)
      for (int j = 0; j < 8; ++j) stage_part(baseA + kt * stepA, baseB + kt * stepB, kt, j, NOP3{});
  vm_wait_tiles(max(0, min(nk, NSLOT4) - 2));
  raw_barrier();
  bf16x8 fa[2][8], fb[2][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa[0][i] = rdA(lds, i);
    fb[0][i] = rdB(lds, i);
  }
  // K-tile 0's slot is restaged in the first K-tile: every wave's reads of it must be done
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  raw_barrier();
  ts_mark(g, 1);

  // one K-tile k (ring slot `slot`): fragments fa/fb[H] (read in the previous K-tile), the next
  // K-tile's (slot nslot) into [H ^ 1]; TAIL: near the end of K (fewer tiles left to read / stage)
  auto ktile = [&](auto Hc, int k, int slot, int nslot, auto Ic, auto Tc) __attribute__((always_inline)) {
    constexpr int H = decltype(Hc)::value;
    constexpr bool INIT = decltype(Ic)::value, TAIL = decltype(Tc)::value;
    const bool more = !TAIL || k + 1 < nk, st = !TAIL || k + NSLOT4 < nk;
    const bf16* nimg = lds + nslot * SLOT4;
    // uniform K-tile bases of the stage, moved to SGPRs here, 50+ instructions ahead of the first DMA
    // (left to hipcc they stay in VGPRs and each DMA is preceded by a v_readfirstlane pair)
    uint64_t sAu = (uint64_t)(uintptr_t)(baseA + (k + NSLOT4) * stepA);
    uint64_t sBu = (uint64_t)(uintptr_t)(baseB + (k + NSLOT4) * stepB);
    // (readfirstlane returns int: the low word is cast back to uint32_t, else it sign-extends into the
    // high word and bit 31 of an address corrupts bits 32..63 -- an illegal address, measured r4o)
    sAu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sAu >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sAu);
    sBu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sBu >> 32)) << 32) |
          (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sBu);
    asm volatile("" : "+s"(sAu), "+s"(sBu));
    const bf16* sA = (const bf16*)(uintptr_t)sAu;
    const bf16* sB = (const bf16*)(uintptr_t)sBu;
    auto mma = [&](int s, int jj) {
      if (INIT) mma16_acc0(acc[s][jj], fb[H][jj], fa[H][s]);
      else mma16_acc(acc[s][jj], fb[H][jj], fa[H][s]);
    };
    // next K-tile's fragment reads: one fa + one fb per 8-MFMA group
    auto rd_next = [&](int s, int jj) __attribute__((always_inline)) {
      if (!more) return;
      if (jj == 0) fa[H ^ 1][s] = rdA(nimg, s);
      if (jj == 1) fb[H ^ 1][s] = rdB(nimg, s);
    };
    // group s: the non-MFMA work sits in the shadows of the group's first MFMAs (staggering the four
    // waves' LDS-DMA over the group measured the same, profiles/r4zb_dma_position_prio_ab.log)
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      mma(s, 0);
      rd_next(s, 0);
      __builtin_amdgcn_sched_barrier(0);
      mma(s, 1);
      rd_next(s, 1);
      __builtin_amdgcn_sched_barrier(0);
      mma(s, 2);
      if (st) stage_part(sA, sB, slot, s, WNOP{});
      __builtin_amdgcn_sched_barrier(0);
      mma(s, 3);
      rd_next(s, 3);
      __builtin_amdgcn_sched_barrier(0);
      mma(s, 4);
      __builtin_amdgcn_sched_barrier(0);
      mma(s, 5);
      __builtin_amdgcn_sched_barrier(0);
      mma(s, 6);
      __builtin_amdgcn_sched_barrier(0);
      mma(s, 7);
      // RS: row sums of this K-tile's A rows 16 s .. 16 s + 15 (D column j = row 16 s + j)
      if constexpr (RS) {
        if (do_rs && (s >> 2) == wn) mma16_vacc(rsacc[s & 3], ones, fa[H][s]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // K-tile k + 2 retired (its fragments are read in the next K-tile); younger: k + 3 .. k + NSLOT4
    if (!TAIL) vm_wait_tiles(NSLOT4 - 2);
    else vm_wait_tiles(max(0, min(nk - 1, k + NSLOT4) - (k + 2)));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads of k + 1 done: its slot may be restaged
    raw_barrier();
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using F = std::false_type;
  using T = std::true_type;
  auto nxt = [](int sl) { return sl == NSLOT4 - 1 ? 0 : sl + 1; };
  int slot = 0;
  if (nk > NSLOT4) ktile(C0{}, 0, slot, nxt(slot), T{}, F{});
  else ktile(C0{}, 0, slot, nxt(slot), T{}, T{});
  slot = nxt(slot);
  int kt = 1;
  // steady state: every K-tile stages K-tile k + NSLOT4 and reads k + 1
  for (; kt + 1 + NSLOT4 < nk; kt += 2) {
    ktile(C1{}, kt, slot, nxt(slot), F{}, F{});
    slot = nxt(slot);
    ktile(C0{}, kt + 1, slot, nxt(slot), F{}, F{});
    slot = nxt(slot);
  }
  for (; kt < nk; kt += 2) {
    ktile(C1{}, kt, slot, nxt(slot), F{}, T{});
    slot = nxt(slot);
    if (kt + 1 < nk) {
      ktile(C0{}, kt + 1, slot, nxt(slot), F{}, T{});
      slot = nxt(slot);
    }
  }
  // the asm MFMAs are opaque to the hazard recognizer: cover the result latency before the first
  // accumulator read
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_waitcnt vmcnt(0)" ::: "memory");
  if (RS && do_rs) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {      // lanes 0..15 hold rows 16 (4 wn + j) + lane (every i the same sum)
      const int m = m0 + wm * 128 + 16 * (4 * wn + j) + lane;
      if (lane < 16 && m < g.M) g.rowsum_part[(long)split * g.M + m] = rsacc[j][0];
    }
  }
  __syncthreads();
  ts_mark(g, 2);
  big_epilogue<EPI, TO, 8, NT4>(g, acc, lds, m0, n0, tid, lane, wm, wn, split);
  ts_mark(g, 3);
}

// ---------------------------------------------------------------------------------------------
// Persistent 4-wave 256x256 bf16-output kernel: gemm4w's K-loop, one workgroup per CU looping over
// output tiles, with the next tile's first NSLOT4 K-tiles staged into the (then idle) LDS ring BEFORE
// the current tile's epilogue.  The non-persistent kernel pays, per tile, the HBM latency of its
// prologue and an epilogue during which the CU's MFMAs and loads idle (one workgroup per CU: the
// ring fills all of LDS); here the epilogue (bias / GELU / GELU' VALU and the output stores) runs
// under the next tile's operand fetch.  The epilogue is therefore written straight from the
// accumulators (8-B stores: every 128-B output line is filled by consecutive stores of one wave, so
// L2 merges them) and its inputs (bias, aux / C tiles) are read by asm loads issued before the
// prefetch, retired by one counted vmcnt: a compiler-visible load would make hipcc's waitcnt pass
// (blind to the asm LDS-DMA) wait for the prefetch too.  Full tiles only (M, N % 256 == 0).
// Tile order: round r of workgroup b takes logical tile r * grid + xcd_remap(b): each round an XCD
// runs a contiguous block of logical tiles, which tile_coords' grouped raster keeps on few A panels.
// the lane's 8 bias quads (columns n, n + 16, ... n + 112) in ONE asm statement that also retires them:
// the outputs exist only once the statement completes, so hipcc can neither read nor move them early
// (a compiler-visible load would instead make hipcc's waitcnt pass, blind to the asm LDS-DMA, wait for
// the next tile's prefetch at the first use)
DEV int g_odd(int lane) { return (lane >> 4) & 1; }
DEV void load_bias8(f32x4 (&b)[8], const float* p) {
  asm volatile(
      "global_load_dwordx4 %0, %8, off\n\tglobal_load_dwordx4 %1, %8, off offset:64\n\t"
      "global_load_dwordx4 %2, %8, off offset:128\n\tglobal_load_dwordx4 %3, %8, off offset:192\n\t"
      "global_load_dwordx4 %4, %8, off offset:256\n\tglobal_load_dwordx4 %5, %8, off offset:320\n\t"
      "global_load_dwordx4 %6, %8, off offset:384\n\tglobal_load_dwordx4 %7, %8, off offset:448\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]), "=&v"(b[4]), "=&v"(b[5]), "=&v"(b[6]), "=&v"(b[7])
      : "v"(p)
      : "memory");
}

// A bf16 input tile (the beta * C or the aux operand of an input-gradient epilogue) in the widened store
// layout: lane chunk (i, jp) = 16 B at row mrow + 16 i, column nst + 32 jp (see the store pairing below);
// all 32 loads in flight at once and retired by the statement's own vmcnt(0), which also covers the
// next tile's staging issued just before it.  One asm statement: hipcc can neither read nor copy the
// destination registers before the wait (a compiler-visible load would make its waitcnt pass, blind to
// the asm LDS-DMA, wait for everything anyway; separate load and wait statements let it move the
// registers in between)
DEV void load_tile16(uint4 (&c)[8][4], const bf16* const (&p)[8]) {
  asm volatile(
      "global_load_dwordx4 %0, %32, off\n\t"
      "global_load_dwordx4 %1, %32, off offset:64\n\t"
      "global_load_dwordx4 %2, %32, off offset:128\n\t"
      "global_load_dwordx4 %3, %32, off offset:192\n\t"
      "global_load_dwordx4 %4, %33, off\n\t"
      "global_load_dwordx4 %5, %33, off offset:64\n\t"
      "global_load_dwordx4 %6, %33, off offset:128\n\t"
      "global_load_dwordx4 %7, %33, off offset:192\n\t"
      "global_load_dwordx4 %8, %34, off\n\t"
      "global_load_dwordx4 %9, %34, off offset:64\n\t"
      "global_load_dwordx4 %10, %34, off offset:128\n\t"
      "global_load_dwordx4 %11, %34, off offset:192\n\t"
      "global_load_dwordx4 %12, %35, off\n\t"
      "global_load_dwordx4 %13, %35, off offset:64\n\t"
      "global_load_dwordx4 %14, %35, off offset:128\n\t"
      "global_load_dwordx4 %15, %35, off offset:192\n\t"
      "global_load_dwordx4 %16, %36, off\n\t"
      "global_load_dwordx4 %17, %36, off offset:64\n\t"
      "global_load_dwordx4 %18, %36, off offset:128\n\t"
      "global_load_dwordx4 %19, %36, off offset:192\n\t"
      "global_load_dwordx4 %20, %37, off\n\t"
      "global_load_dwordx4 %21, %37, off offset:64\n\t"
      "global_load_dwordx4 %22, %37, off offset:128\n\t"
      "global_load_dwordx4 %23, %37, off offset:192\n\t"
      "global_load_dwordx4 %24, %38, off\n\t"
      "global_load_dwordx4 %25, %38, off offset:64\n\t"
      "global_load_dwordx4 %26, %38, off offset:128\n\t"
      "global_load_dwordx4 %27, %38, off offset:192\n\t"
      "global_load_dwordx4 %28, %39, off\n\t"
      "global_load_dwordx4 %29, %39, off offset:64\n\t"
      "global_load_dwordx4 %30, %39, off offset:128\n\t"
      "global_load_dwordx4 %31, %39, off offset:192\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(c[0][0]), "=&v"(c[0][1]), "=&v"(c[0][2]), "=&v"(c[0][3]), "=&v"(c[1][0]), "=&v"(c[1][1]), "=&v"(c[1][2]), "=&v"(c[1][3]), "=&v"(c[2][0]), "=&v"(c[2][1]), "=&v"(c[2][2]), "=&v"(c[2][3]), "=&v"(c[3][0]), "=&v"(c[3][1]), "=&v"(c[3][2]), "=&v"(c[3][3]), "=&v"(c[4][0]), "=&v"(c[4][1]), "=&v"(c[4][2]), "=&v"(c[4][3]), "=&v"(c[5][0]), "=&v"(c[5][1]), "=&v"(c[5][2]), "=&v"(c[5][3]), "=&v"(c[6][0]), "=&v"(c[6][1]), "=&v"(c[6][2]), "=&v"(c[6][3]), "=&v"(c[7][0]), "=&v"(c[7][1]), "=&v"(c[7][2]), "=&v"(c[7][3])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}
// Epilogue of the persistent 256x256 kernels (gemm4p / gemm4q / gemm4r): bias / GELU / GELU' / aux
// product / beta C from the AGPR accumulators in the widened 16-B store layout, handed to sink(i, jp,
// o, o2) per lane chunk (o: column blocks 2 jp, 2 jp + 1 of the output C, o2: those of the second
// output aux of EPI_BIAS_GELU(_D)), to be paired by pack16 into one 16-B store.
// biasv: the lane's bias quads (HAS_BIAS); mrow = m0 + wm 128 + (lane & 15); nst: p_nst().
// Stores: the epilogue is store-ISSUE-bound (0.25 MB per CU per tile with GELU': ~240 of 490 us per
// launch went to 8-B stores, profiles/r3q_exp.log), so column blocks j = 2 jp, 2 jp + 1 are paired:
// one v_permlane16_swap per dword gives lanes g even 8 contiguous columns of block 2 jp and lanes g
// odd those of block 2 jp + 1 (cdna_hip_programming.md T21, 16-lane form) -> one 16-B store each.
// The swap is an involution: applied to an input tile read in that layout it restores the
// accumulator layout.
DEV int p_nst(int n0, int wn, int lane) { return n0 + wn * 128 + 16 * g_odd(lane) + 8 * (lane >> 5); }  // + 32 jp
DEV u32x4 pack16(bf16x4 a, bf16x4 b) {
  uint2 ua = __builtin_bit_cast(uint2, a), ub = __builtin_bit_cast(uint2, b);
  const auto rx = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
  const auto ry = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
  return u32x4{rx[0], ry[0], rx[1], ry[1]};
}
// plain 16-B stores: the nt policy ran the store-bound epilogues 3-4 % faster alone but the step 0.8 %
// slower (the consumers lose the outputs' MALL residency, profiles/r4b_store_nt_step_ab.log)
DEV void st_out(bf16* pp, u32x4 d) { *(u32x4*)pp = d; }
template <int EPI, bool ACC, class Sink>
DEV void p_epi_tile(const BigArgs& g, f32x4 (&acc)[8][8], const f32x4 (&biasv)[8], int mrow, int nst, Sink&& sink) {
  constexpr bool HAS_BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_D;
  constexpr bool IN_EPI = (EPI == EPI_NONE && ACC) || EPI == EPI_MUL_AUX;
  constexpr bool in_tile = IN_EPI;
  // the input tile (aux, or C for beta) whole, one wait before the first store: streaming it two rows
  // ahead of the stores measured the same (profiles/r4y2_epilogue_pipe_ab.log)
  uint4 cin[8][4];
  if (IN_EPI && in_tile) {
    const bf16* src = EPI == EPI_MUL_AUX ? g.aux : (const bf16*)g.C;
    const long ld = EPI == EPI_MUL_AUX ? g.ldaux : g.ldc;
    const bf16* rows[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) rows[i] = src + (long)(mrow + 16 * i) * ld + nst;
    load_tile16(cin, rows);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) {
      bf16x4 o[2], o2[2], ci[2];
      if (IN_EPI && in_tile) {     // input chunk back to the accumulator layout (blocks 2 jp, 2 jp + 1)
        const uint4 c4 = cin[i][jp];
        const auto rx = __builtin_amdgcn_permlane16_swap(c4.x, c4.z, false, false);
        const auto ry = __builtin_amdgcn_permlane16_swap(c4.y, c4.w, false, false);
        ci[0] = __builtin_bit_cast(bf16x4, make_uint2(rx[0], ry[0]));
        ci[1] = __builtin_bit_cast(bf16x4, make_uint2(rx[1], ry[1]));
      }
      float v[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = 2 * jp + h;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[h][r] = g.alpha * acc[i][j][r] + (HAS_BIAS ? biasv[j][r] : 0.f);
          if (IN_EPI && in_tile) {
            if (EPI == EPI_MUL_AUX) v[h][r] *= (float)ci[h][r];
            else v[h][r] += g.beta * (float)ci[h][r];
          }
        }
      }
      if (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_D) {
        // the chunk's 4 pairs through gelu2n together (independent chains interleaved)
        const f32x2 x[4] = {f32x2{v[0][0], v[0][1]}, f32x2{v[0][2], v[0][3]}, f32x2{v[1][0], v[1][1]},
                            f32x2{v[1][2], v[1][3]}};
        f32x2 gl[4], gd[4];
        gelu2n<4>(x, gl, EPI == EPI_BIAS_GELU_D ? &gd : nullptr);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (EPI == EPI_BIAS_GELU_D) {
            o2[h][0] = (bf16)gd[2 * h].x; o2[h][1] = (bf16)gd[2 * h].y;
            o2[h][2] = (bf16)gd[2 * h + 1].x; o2[h][3] = (bf16)gd[2 * h + 1].y;
          } else {     // pre-activation
            o2[h][0] = (bf16)v[h][0]; o2[h][1] = (bf16)v[h][1]; o2[h][2] = (bf16)v[h][2]; o2[h][3] = (bf16)v[h][3];
          }
          o[h][0] = (bf16)gl[2 * h].x; o[h][1] = (bf16)gl[2 * h].y;
          o[h][2] = (bf16)gl[2 * h + 1].x; o[h][3] = (bf16)gl[2 * h + 1].y;
        }
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          o[h][0] = (bf16)v[h][0]; o[h][1] = (bf16)v[h][1]; o[h][2] = (bf16)v[h][2]; o[h][3] = (bf16)v[h][3];
        }
      }
      sink(i, jp, o, o2);
    }
  }
}
// (no runtime store-policy branch around the tile's 64 stores: such block boundaries kept the scheduler
// from interleaving the GELU chains of neighbouring chunks -- an s_nop between most dependent packed FMAs)
template <int EPI, bool ACC>
DEV void p_store_tile(const BigArgs& g, f32x4 (&acc)[8][8], const f32x4 (&biasv)[8], int mrow, int n0, int wn,
                      int lane) {
  const int nst = p_nst(n0, wn, lane);
  bf16* Cb = (bf16*)g.C;
  p_epi_tile<EPI, ACC>(g, acc, biasv, mrow, nst, [&](int i, int jp, const bf16x4 (&o)[2], const bf16x4 (&o2)[2]) {
    const long m = mrow + 16 * i;
    if ((EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_D) && (EPI == EPI_BIAS_GELU_D || g.aux))
      st_out(g.aux + m * g.ldaux + nst + 32 * jp, pack16(o2[0], o2[1]));
    st_out(Cb + m * g.ldc + nst + 32 * jp, pack16(o[0], o[1]));
  });
}

#ifndef EEGF_P_NOP
#define EEGF_P_NOP 0
#endif
template <bool BKC, int EPI, bool ACC = false>     // ACC: EPI_NONE with C = alpha A B^T + beta C
__global__ void __launch_bounds__(NT4, 1) gemm4p_kernel(BigArgs g) {
  constexpr bool AKC = true;
  constexpr int LDS4 = NSLOT4 * SLOT4;
  constexpr bool HAS_BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_D;
  // an input tile: aux (EPI_MUL_AUX: activation' product) or beta * C (EPI_NONE, beta != 0: residual
  // accumulate), read by load_tile16 after the next tile's staging is issued
  constexpr bool IN_EPI = (EPI == EPI_NONE && ACC) || EPI == EPI_MUL_AUX;
  __shared__ __attribute__((aligned(16))) bf16 lds[LDS4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = g.N / TN, tiles_m = g.M / TM, ntiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int nk = g.K / BK4;
  int L = xcd_remap(blockIdx.x, G);
  if (L >= ntiles) return;

  // per-lane staging offsets (full tiles: no row / column clamp, so one set serves every tile)
  uint32_t voffA[4], voffB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wave * 4 + j) * 16 + (lane >> 2);
    voffA[j] = (uint32_t)(((long)r * g.lda + ((lane & 3) ^ sw4(r)) * 8) * 2);
    if (BKC) {
      voffB[j] = (uint32_t)(((long)r * g.ldb + ((lane & 3) ^ sw4(r)) * 8) * 2);
    } else {
      const int k = (wave * 4 + j) * 2 + (lane >> 5);
      voffB[j] = (uint32_t)(((long)k * g.ldb + ((lane & 31) ^ swz_k(k)) * 8) * 2);
    }
  }
  const long stepB = BKC ? BK4 : (long)BK4 * g.ldb;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(lds));
  // NOP: the K-loop's DMAs take SALU-computed bases (s_nop 0 after the M0 write, isa_lint-checked); the
  // prologue's come straight from tile_base's v_readfirstlane (s_nop 3)
  auto stage_part = [&](const bf16* bA, const bf16* bB, int slot, int j, auto Nc) __attribute__((always_inline)) {
    constexpr int NOP = decltype(Nc)::value;
    const bool kc = j < 4 ? AKC : BKC;
    const uint32_t dst = lds0 + 2u * (slot * SLOT4 + (j < 4 ? 0 : TM * BK4) +
                                      (wave * 4 + (j & 3)) * (kc ? 16 * BK4 : 2 * TN));
    if (j < 4) glds16_asm_sa<NOP>(bA, voffA[j & 3], dst);
    else glds16_asm_sa<NOP>(bB, voffB[j & 3], dst);
  };
  using NOP0 = std::integral_constant<int, EEGF_P_NOP>;
  using NOP3 = std::integral_constant<int, 3>;
  auto tile_base = [&](int l, const bf16*& bA, const bf16*& bB, int& m0, int& n0) {
    int tm, tn;
    tile_coords(g, l, tiles_m, tiles_n, tm, tn);
    m0 = __builtin_amdgcn_readfirstlane(tm * TM);
    n0 = __builtin_amdgcn_readfirstlane(tn * TN);
    bA = g.A + (long)m0 * g.lda;
    bB = BKC ? g.B + (long)n0 * g.ldb : g.B + n0;
  };
  auto stage_first = [&](const bf16* bA, const bf16* bB) {   // K-tiles 0 .. NSLOT4-1 -> slots 0 .. 4
    for (int kt = 0; kt < NSLOT4; ++kt)
      if (kt < nk)
        for (int j = 0; j < 8; ++j) stage_part(bA + kt * BK4, bB + kt * stepB, kt, j, NOP3{});
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int offA = (wm * 128 + fr) * BK4 + ((fq ^ sw4(fr)) << 3);
  const int offB = TM * BK4 + (wn * 128 + fr) * BK4 + ((fq ^ sw4(fr)) << 3);
  int tB0[8], tB1[8];
  if (!BKC) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = fr >> 2, p4 = fr & 3;
      const int col = wn * 128 + 16 * i + 4 * p4, ch = col >> 3, off = col & 7;
      const int ka = 8 * fq + q, kb = ka + 4;
      tB0[i] = TM * BK4 + ka * TN + (((ch ^ swz_k(ka)) << 3) | off);
      tB1[i] = TM * BK4 + kb * TN + (((ch ^ swz_k(kb)) << 3) | off);
    }
  }
  auto rdA = [&](const bf16* img, int i) { return *(const bf16x8*)(img + offA + i * 16 * BK4); };
  auto rdB = [&](const bf16* img, int i) {
    return BKC ? *(const bf16x8*)(img + offB + i * 16 * BK4) : rd_col_off(img, tB0[i], tB1[i]);
  };

  const bf16* baseA;
  const bf16* baseB;
  int m0, n0;
  tile_base(L, baseA, baseB, m0, n0);
  stage_first(baseA, baseB);
  f32x4 acc[8][8];
  // Cross-tile staging (nk >= 8): the K-loop tail of tile t stages tile t + 1's K-tiles 0 .. 4 into the
  // slots it frees (the ring runs on across tiles: slot0 = where the tile's K-tile 0 sits), those are
  // retired before the epilogue's first store, and tile t + 1 then skips its prologue wait and the
  // waits of K-tiles 0 .. 2 (their operands have landed).  The epilogue stores -- counted in vmcnt
  // with the LDS-DMA, so any wait behind them waits for them too -- drain under those K-tiles' MFMAs
  // instead of in front of them (the GELU' FFN1 epilogue is store-bound: profiles/r3q_epilogue_anatomy.log)
  const bool xs = nk >= 8;
  int slot0 = 0;
  bool landed = false;          // this tile's K-tiles 0 .. 4 retired (cross-staged and waited for)
  for (;;) {
    const int Ln = L + G;
    const bool more_tiles = Ln < ntiles;
    int m0n = 0, n0n = 0;
    const bf16* nA = nullptr;
    const bf16* nB = nullptr;
    if (more_tiles) tile_base(Ln, nA, nB, m0n, n0n);
    const bool cross = xs && more_tiles;
    // K-tiles 0 and 1 retired (older epilogue stores still counted only make this wait stricter)
    if (!landed) vm_wait_tiles(max(0, min(nk, NSLOT4) - 2));
    raw_barrier();
    bf16x8 fa[2][8], fb[2][8];
    const bf16* img0 = lds + slot0 * SLOT4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      fa[0][i] = rdA(img0, i);
      fb[0][i] = rdB(img0, i);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();

    auto ktile = [&](auto Hc, int k, int slot, int nslot, auto Ic, auto Tc) __attribute__((always_inline)) {
      constexpr int H = decltype(Hc)::value;
      constexpr bool INIT = decltype(Ic)::value, TAIL = decltype(Tc)::value;
      const bool more = !TAIL || k + 1 < nk;
      const bool own = !TAIL || k + NSLOT4 < nk;           // stage this tile's K-tile k + 5
      const bool st = own || cross;                        // ... or the next tile's K-tile k + 5 - nk
      const bf16* nimg = lds + nslot * SLOT4;
      const bf16* sA = own ? baseA + (k + NSLOT4) * BK4 : nA + (k + NSLOT4 - nk) * BK4;
      const bf16* sB = own ? baseB + (k + NSLOT4) * stepB : nB + (k + NSLOT4 - nk) * stepB;
      auto mma = [&](int s, int jj) {
        if (INIT) mma16_acc0(acc[s][jj], fb[H][jj], fa[H][s]);
        else mma16_acc(acc[s][jj], fb[H][jj], fa[H][s]);
      };
      // the next K-tile's fragments: one fa + one fb per 8-MFMA group (fb[7] read in group 7, ~6 MFMAs
      // before the wait); issuing them in groups 0..5 measured the same
      auto rd_next = [&](int s, int jj) __attribute__((always_inline)) {
        if (!more) return;
        if (jj == 0) fa[H ^ 1][s] = rdA(nimg, s);
        if (jj == 1) fb[H ^ 1][s] = rdB(nimg, s);
      };
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        mma(s, 0);
        rd_next(s, 0);
        __builtin_amdgcn_sched_barrier(0);
        mma(s, 1);
        rd_next(s, 1);
        __builtin_amdgcn_sched_barrier(0);
        mma(s, 2);
        if (st) stage_part(sA, sB, slot, s, NOP0{});
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int jj = 3; jj < 8; ++jj) {
          mma(s, jj);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // K-tile k + 2 retired (its fragments are read in the next K-tile): skipped when it landed before
      // the tile started (cross-staged, k + 2 <= 4) or when there is no such K-tile of this tile
      if (!(landed && k < NSLOT4 - 2) && k + 2 < nk) {
        if (!TAIL || cross) vm_wait_tiles(NSLOT4 - 2);
        else vm_wait_tiles(max(0, min(nk - 1, k + NSLOT4) - (k + 2)));
      } else if (!cross && k + 2 >= nk) {
        vm_wait_tiles(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      raw_barrier();
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using F = std::false_type;
    using T = std::true_type;
    auto nxt = [](int sl) { return sl == NSLOT4 - 1 ? 0 : sl + 1; };
    int slot = slot0;
    if (nk > NSLOT4) ktile(C0{}, 0, slot, nxt(slot), T{}, F{});
    else ktile(C0{}, 0, slot, nxt(slot), T{}, T{});
    slot = nxt(slot);
    int kt = 1;
    for (; kt + 1 + NSLOT4 < nk; kt += 2) {
      ktile(C1{}, kt, slot, nxt(slot), F{}, F{});
      slot = nxt(slot);
      ktile(C0{}, kt + 1, slot, nxt(slot), F{}, F{});
      slot = nxt(slot);
    }
    for (; kt < nk; kt += 2) {
      ktile(C1{}, kt, slot, nxt(slot), F{}, T{});
      slot = nxt(slot);
      if (kt + 1 < nk) {
        ktile(C0{}, kt + 1, slot, nxt(slot), F{}, T{});
        slot = nxt(slot);
      }
    }
    // every wave is past its last ring read (the final K-tile's barrier): the ring is free
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");

    // the bias (8 quads, L2-resident) before the prefetch, retired at once
    const int mrow = m0 + wm * 128 + (lane & 15);
    const int ncol = n0 + wn * 128 + 4 * (lane >> 4);
    f32x4 biasv[8];
    if (HAS_BIAS) load_bias8(biasv, g.bias + ncol);
    if (more_tiles && !cross) stage_first(nA, nB);
    // cross-staged: the next tile's K-tiles 0 .. 4 retired before the first store (load_bias8 /
    // load_tile16 wait for them too)
    if (cross) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    p_store_tile<EPI, ACC>(g, acc, biasv, mrow, n0, wn, lane);
    if (!more_tiles) break;
    L = Ln;
    m0 = m0n;
    n0 = n0n;
    baseA = nA;
    baseB = nB;
    // cross-staged: the ring runs on (next tile's K-tile 0 sits in the slot after this tile's last)
    landed = cross;
    if (cross) slot0 = (slot0 + nk) % NSLOT4;
  }
}

// ---------------------------------------------------------------------------------------------
// Whole-line staging of the persistent GEMMs (round 4, profiles/r4e_dma_line_pattern.log): gemm4p's
// LDS-DMA instruction covers 16 rows x 64 B of a K-contiguous operand (one 32-deep K-tile: half of every
// 128-B line it touches), which the CU's DMA path moves at 31 B/cycle from L2 against 46 B/cycle for
// 8 rows x 128 B, while a 256x256 K-tile needs 32 KB per 1,024 MFMA cycles.  gemm4r therefore stages
// K-tile PAIRS (64 deep) as operand images of 32 KB: [256 rows][64 k] per K-contiguous operand (16-B
// chunk c of row r stored at c ^ (r & 7): conflict-free ds_read_b128), [64 k][256 cols] per k-major one
// (gemm4p's swz_k image, two K-tiles stacked), 32 KB staged per K-tile, one 1-KB part per 8-MFMA group.
// (The first whole-line kernel, gemm4q, held a whole K-tile of A fragments in registers over a
// five-slot ring; gemm4r replaced it in round 5 with bitwise the same results, and it was retired in
// round 6 with the other superseded kernels: gemm_big_kernel, gemm8, gemm4h -- git history, 829c7a6.)
// Needs K % 64 == 0 and K >= 128 (launch_big routes other shapes to gemm4p).
constexpr int BKP = 64;                                // K per pair
constexpr int HSLOT = TM * BKP;                        // one operand image of a pair (32 KB)
#ifndef EEGF_Q_NOP
#define EEGF_Q_NOP 0
#endif
#ifndef EEGF_Q_SPOS
#define EEGF_Q_SPOS 4      // the group's LDS-DMA part goes after its MFMA EEGF_Q_SPOS (0..7)
#endif
// Persistent tile walk: round r of workgroup b takes logical tile r * G + xcd_remap(b), so each round an
// XCD runs the next contiguous block of 32 tiles of the whole grid (tile_coords' grouped raster keeps
// them on few A panels).  An XCD-blocked walk measured neutral (profiles/r5a_order_ab.log).
struct QWalk {
  int L, end, step;
};
DEV QWalk q_walk(int ntiles) { return {xcd_remap(blockIdx.x, gridDim.x), ntiles, (int)gridDim.x}; }

// ---------------------------------------------------------------------------------------------
// gemm4r: the whole-line K-tile pairs above with ROLLING A fragments.  Each A fragment is used by one
// 8-MFMA group, so it is read two groups ahead (across the K-tile boundary too) into four register sets
// instead of a whole K-tile ahead into sixteen (gemm4q): 48 fewer VGPRs in the K-loop.  The price is the
// ring: pair t's A image is read until the end of its odd K-tile, so it cannot take pair t + 2's B there.
// Instead A images rotate through three slots and B images through two (A of global pair u in slot
// 2 (u mod 3), B in 1 + 2 (u mod 2)): pair t + 2's A is staged during pair t's even K-tile into pair
// t - 1's A slot (free since the barrier that ends pair t - 1's odd K-tile -- a second barrier per
// pair), its B during the odd K-tile into pair t's B slot (read during pair t - 1's odd and pair t's
// even K-tile, free since the barrier that ends the even one): still 32 KB per K-tile.  The same MFMA K
// order and epilogue as gemm4q / gemm4p (bitwise the same results).  eegf_tune key 18.
template <bool BKC, int EPI, bool ACC = false>
__global__ void __launch_bounds__(NT4, 1) gemm4r_kernel(BigArgs g) {
  constexpr bool HAS_BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_D;
  __shared__ __attribute__((aligned(16))) bf16 lds[5 * HSLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = g.N / TN, tiles_m = g.M / TM, ntiles = tiles_m * tiles_n;
  const int np = g.K / BKP;
  const QWalk walk = q_walk(ntiles);
  int L = walk.L;
  if (L >= walk.end) return;

  const int kr = lane >> 3;
  const uint32_t voffA = (uint32_t)(((long)kr * g.lda + ((lane & 7) ^ kr) * 8) * 2);
  uint32_t voffB[4];
  if (BKC) {
    voffB[0] = (uint32_t)(((long)kr * g.ldb + ((lane & 7) ^ kr) * 8) * 2);
  } else {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int j = (v & 1) | ((v >> 1) << 2);
      const int k = (wave * 8 + j) * 2 + (lane >> 5);
      voffB[v] = (uint32_t)(((long)(lane >> 5) * g.ldb + ((lane & 31) ^ swz_k(k)) * 8) * 2);
    }
  }
  const long pstepB = BKC ? BKP : (long)BKP * g.ldb;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr_of(lds));
  using QNOP = std::integral_constant<int, EEGF_Q_NOP>;
  using PNOP = std::integral_constant<int, 3>;
  // part j < 8: an A part into slot ps; j >= 8: a B part (gemm4q's mapping)
  auto stage_part = [&](const bf16* bA, const bf16* bB, int ps, int j, auto NopC) __attribute__((always_inline)) {
    const int jj = j & 7, pr = wave * 8 + jj;
    constexpr int NOP = decltype(NopC)::value;
    if (j < 8) {
      glds16_asm_sa<NOP>(bA + (long)pr * 8 * g.lda, voffA, lds0 + 2u * (ps * HSLOT + pr * 8 * BKP));
    } else if (BKC) {
      glds16_asm_sa<NOP>(bB + (long)pr * 8 * g.ldb, voffB[0], lds0 + 2u * (ps * HSLOT + pr * 8 * BKP));
    } else {
      glds16_asm_sa<NOP>(bB + (long)pr * 2 * g.ldb, voffB[(jj & 1) | ((jj >> 2) << 1)], lds0 + 2u * (ps * HSLOT + pr * 2 * TN));
    }
  };
  auto tile_base = [&](int l, const bf16*& bA, const bf16*& bB, int& m0, int& n0) {
    int tm, tn;
    tile_coords(g, l, tiles_m, tiles_n, tm, tn);
    m0 = __builtin_amdgcn_readfirstlane(tm * TM);
    n0 = __builtin_amdgcn_readfirstlane(tn * TN);
    bA = g.A + (long)m0 * g.lda;
    bB = BKC ? g.B + (long)n0 * g.ldb : g.B + n0;
  };
  const int fr = lane & 15, fq = lane >> 4;
  const int offA0 = (wm * 128 + fr) * BKP + ((fq ^ (fr & 7)) << 3);
  const int offA1 = (wm * 128 + fr) * BKP + (((4 + fq) ^ (fr & 7)) << 3);
  const int offB0 = (wn * 128 + fr) * BKP + ((fq ^ (fr & 7)) << 3);
  const int offB1 = (wn * 128 + fr) * BKP + (((4 + fq) ^ (fr & 7)) << 3);
  int tB0[8], tB1[8];
  if (!BKC) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = fr >> 2, p4 = fr & 3;
      const int col = wn * 128 + 16 * i + 4 * p4, ch = col >> 3, off = col & 7;
      const int ka = 8 * fq + q, kb = ka + 4;
      tB0[i] = ka * TN + (((ch ^ swz_k(ka)) << 3) | off);
      tB1[i] = kb * TN + (((ch ^ swz_k(kb)) << 3) | off);
    }
  }
  auto rdA = [&](const bf16* img, auto Hc, int i) {
    return *(const bf16x8*)(img + (decltype(Hc)::value ? offA1 : offA0) + i * 16 * BKP);
  };
  auto rdB = [&](const bf16* img, auto Hc, int i) {
    constexpr int h = decltype(Hc)::value;
    return BKC ? *(const bf16x8*)(img + (h ? offB1 : offB0) + i * 16 * BKP)
               : rd_col_off(img + h * 32 * TN, tB0[i], tB1[i]);
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  auto anext = [](int a) { return a >= 4 ? a - 4 : a + 2; };      // A slot of the next pair: 0 -> 2 -> 4 -> 0

  const bf16* baseA;
  const bf16* baseB;
  int m0, n0;
  tile_base(L, baseA, baseB, m0, n0);
#pragma unroll 1
  for (int j = 0; j < 16; ++j) stage_part(baseA, baseB, j < 8 ? 0 : 1, j, PNOP{});                    // pair 0
#pragma unroll 1
  for (int j = 0; j < 16; ++j) stage_part(baseA + BKP, baseB + pstepB, j < 8 ? 2 : 3, j, PNOP{});    // pair 1
  f32x4 acc[8][8];
  int aS0 = 0, bS0 = 1;         // slots of the tile's pair-0 A and B
  bool landed = false;
  for (;;) {
    const int Ln = L + walk.step;
    const bool more_tiles = Ln < walk.end;
    int m0n = 0, n0n = 0;
    const bf16* nA = nullptr;
    const bf16* nB = nullptr;
    if (more_tiles) tile_base(Ln, nA, nB, m0n, n0n);
    if (!landed) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");      // pair 0 (pair 1 younger)
    raw_barrier();
    bf16x8 fa[4], fb[2][8];
    {
      const bf16* img0 = lds + aS0 * HSLOT;
      const bf16* imb0 = lds + bS0 * HSLOT;
      fa[0] = rdA(img0, C0{}, 0);
      fa[1] = rdA(img0, C0{}, 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) fb[0][i] = rdB(imb0, C0{}, i);
    }
    auto ktile = [&](auto Hc, int t, int aS, int bS, auto Ic, auto Tc) __attribute__((always_inline)) {
      constexpr int H = decltype(Hc)::value;
      constexpr bool INIT = decltype(Ic)::value, TAIL = decltype(Tc)::value;
      const bool more = !TAIL || H == 0 || t + 1 < np;
      const bf16* cimg = lds + aS * HSLOT;                                // this K-tile's A (half H)
      const bf16* nimg = H == 0 ? cimg : lds + anext(aS) * HSLOT;         // the next K-tile's A
      const bf16* nimb = lds + (H == 0 ? bS : (bS ^ 2)) * HSLOT;           // the next K-tile's B
      const bool own = !TAIL || t + 2 < np;
      const bool st = own || more_tiles;
      const int sslot = H == 0 ? anext(anext(aS)) : bS;                   // pair t + 2's A / B slot
      const bf16* sA = own ? baseA + (t + 2) * BKP : nA + (t + 2 - np) * BKP;
      const bf16* sB = own ? baseB + (t + 2) * pstepB : nB + (t + 2 - np) * pstepB;
      using HN = std::integral_constant<int, H ^ 1>;
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8) {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          if (INIT) mma16_acc0(acc[s8][jj], fb[H][jj], fa[s8 & 3]);
          else mma16_acc(acc[s8][jj], fb[H][jj], fa[s8 & 3]);
          if (jj == 0) {
            if (s8 + 2 < 8) fa[(s8 + 2) & 3] = rdA(cimg, Hc, s8 + 2);
            else if (more) fa[(s8 + 2) & 3] = rdA(nimg, HN{}, s8 - 6);
          }
          if (jj == 1 && more) fb[H ^ 1][s8] = rdB(nimb, HN{}, s8);
          if (jj == EEGF_Q_SPOS && st) stage_part(sA, sB, sslot, 8 * H + s8, QNOP{});
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (H == 0) {
        // pair t + 1 (staged during pair t - 1) must have landed before the next K-tile reads its B; the
        // barrier frees pair t's B slot for pair t + 2's B (this K-tile's 8 A parts are the younger ones)
        if (!TAIL || t + 1 < np) {
          if (st) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        raw_barrier();
      } else if (!TAIL || t + 1 < np) {
        // every wave is past its last read of pair t's A (consumed by this K-tile's MFMAs): pair t + 3's A
        // may land in its slot from the next even K-tile on
        raw_barrier();
      }
    };
    using F = std::false_type;
    using T = std::true_type;
    int aS = aS0, bS = bS0;
    if (np > 2) {
      ktile(C0{}, 0, aS, bS, T{}, F{});
      ktile(C1{}, 0, aS, bS, F{}, F{});
    } else {
      ktile(C0{}, 0, aS, bS, T{}, T{});
      ktile(C1{}, 0, aS, bS, F{}, T{});
    }
    aS = anext(aS);
    bS ^= 2;
#pragma unroll 1
    for (int t = 1; t + 2 < np; ++t) {
      ktile(C0{}, t, aS, bS, F{}, F{});
      ktile(C1{}, t, aS, bS, F{}, F{});
      aS = anext(aS);
      bS ^= 2;
    }
#pragma unroll 1
    for (int t = max(1, np - 2); t < np; ++t) {
      ktile(C0{}, t, aS, bS, F{}, T{});
      ktile(C1{}, t, aS, bS, F{}, T{});
      aS = anext(aS);
      bS ^= 2;
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    const int mrow = m0 + wm * 128 + (lane & 15);
    const int ncol = n0 + wn * 128 + 4 * (lane >> 4);
    f32x4 biasv[8];
    if (HAS_BIAS) load_bias8(biasv, g.bias + ncol);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    p_store_tile<EPI, ACC>(g, acc, biasv, mrow, n0, wn, lane);
    if (!more_tiles) break;
    L = Ln;
    m0 = m0n;
    n0 = n0n;
    baseA = nA;
    baseB = nB;
    landed = true;
    aS0 = aS;
    bS0 = bS;
  }
}

// eegf_tune key 11: the persistent kernels (gemm4r / gemm4p) for the bf16-output GEMMs they take: 1
// (default) every eligible shape (full 256 x 256 tiles, K-contiguous A: every BERT forward and input
// gradient of the bench step), 0 none (gemm4w, the non-persistent 4-wave kernel: the bit-identity
// reference of tests/test_gemm_gpu.py)
int g_persistent = 1;
// key 14: gemm4r (whole-line K-tile pairs, rolling A fragments) where K % 64 == 0 and K >= 128 (1,
// default), or gemm4p's 64-B half lines everywhere (0); bitwise the same results
int g_gemm4r = 1;
int cu_count() {
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  return cus;
}
int g_cu_reserve = 0;      // eegf_tune key 13
}  // namespace
// workgroups of a persistent grid: every CU but the reserved ones (room for RCCL kernels, key 13)
int persistent_cus() {
  const int n = cu_count() - g_cu_reserve;
  return n > 0 ? n : 1;
}
namespace {
// Routing of the 256-row GEMMs: bf16 outputs with a K-contiguous A on full tiles go to the persistent
// kernel (gemm4r where K splits into >= 2 K-tile pairs, else gemm4p); everything else -- ragged M / N,
// other epilogues, beta with an aux epilogue, and the fp32 split-K weight gradients -- to gemm4w.
template <bool AKC, bool BKC, int EPI, typename TO>
int launch_big(const BigArgs& a, int splits, hipStream_t s) {
  const int tiles = ((a.M + TM - 1) / TM) * ((a.N + TN - 1) / TN);
  if constexpr (AKC && sizeof(TO) == 2 && (EPI == EPI_NONE || EPI == EPI_BIAS || EPI == EPI_BIAS_GELU ||
                                           EPI == EPI_BIAS_GELU_D || (EPI == EPI_MUL_AUX && !BKC))) {
    // beta * C: the EPI_NONE input tile only (the aux epilogue ignores beta, as big_epilogue does)
    const bool beta_ok = a.beta == 0.f || EPI == EPI_NONE;
    const bool aux_ok = EPI != EPI_MUL_AUX || (a.aux && a.ldaux % 8 == 0 && (((uintptr_t)a.aux) & 15) == 0);
    if (g_persistent && beta_ok && aux_ok && splits == 1 && a.M % TM == 0 && a.N % TN == 0 && a.ldc % 8 == 0 &&
        (((uintptr_t)a.C) & 15) == 0 && a.K % BK4 == 0 && (((uintptr_t)a.bias) & 15) == 0) {
      const dim3 grid(tiles < persistent_cus() ? tiles : persistent_cus());
      bool acc = false;
      if constexpr (EPI == EPI_NONE) acc = a.beta != 0.f;
      // whole-line staging wherever K splits into >= 2 pairs of K-tiles: the forward layout 3-6 % faster
      // than gemm4p's half lines (profiles/r4u_gemm4q_ring5_ab.log), the input gradients 3-5 %
      // (profiles/r4ze_dgrad_gemm4q_ab.log), gemm4r's rolling A fragments another 2-14 % (r5t_4r_ab.log)
      const bool r = g_gemm4r && a.K % BKP == 0 && a.K >= 2 * BKP;
      if (acc) {
        if constexpr (EPI == EPI_NONE) {
          if (r) EEGF_LAUNCH((gemm4r_kernel<BKC, EPI, true>), grid, dim3(NT4), 0, s, a);
          else EEGF_LAUNCH((gemm4p_kernel<BKC, EPI, true>), grid, dim3(NT4), 0, s, a);
        }
      } else if (r) {
        EEGF_LAUNCH((gemm4r_kernel<BKC, EPI>), grid, dim3(NT4), 0, s, a);
      } else {
        EEGF_LAUNCH((gemm4p_kernel<BKC, EPI>), grid, dim3(NT4), 0, s, a);
      }
      return (int)hipGetLastError();
    }
  }
  EEGF_LAUNCH((gemm4w_kernel<AKC, BKC, EPI, TO>), dim3(tiles, splits), dim3(NT4), 0, s, a);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(256) big_splitk_reduce(const float* __restrict__ slabs, int splits, long MN, int N,
                                                         float* C, long ldc, float beta) {
  const long i4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= MN) return;
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < splits; ++s) o += *(const f32x4*)(slabs + (long)s * MN + i4);
  const long m = i4 / N, n = i4 % N;          // N % 4 == 0: a 4-group never crosses a row
  float* c = C + m * ldc + n;
  if (beta != 0.f) o += beta * *(const f32x4*)c;
  *(f32x4*)c = o;
}

// db[m] += sum over splits of part[s][m] (fixed order: bitwise reproducible)
DEV void rowsum_reduce_at(const float* __restrict__ part, int splits, int M, float* db, int m) {
  if (m >= M) return;
  float v = 0.f;
  for (int s = 0; s < splits; ++s) v += part[(long)s * M + m];
  db[m] += v;
}
__global__ void __launch_bounds__(256) rowsum_reduce(const float* __restrict__ part, int splits, int M, float* db) {
  rowsum_reduce_at(part, splits, M, db, blockIdx.x * 256 + threadIdx.x);
}
// the weight gradient's slab reduction and the bias gradient's row-sum reduction in one launch: blocks
// below nslab reduce the slabs (as big_splitk_reduce), the rest the row sums (as rowsum_reduce) -- two
// independent fixed-order sums, one launch instead of two per weight gradient (48 per step)
__global__ void __launch_bounds__(256) splitk_rowsum_reduce(const float* __restrict__ slabs, int splits, long MN, int N,
                                                            float* C, long ldc, float beta, int nslab,
                                                            const float* __restrict__ part, int M, float* db) {
  if ((int)blockIdx.x >= nslab) {
    rowsum_reduce_at(part, splits, M, db, ((int)blockIdx.x - nslab) * 256 + threadIdx.x);
    return;
  }
  const long i4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= MN) return;
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < splits; ++s) o += *(const f32x4*)(slabs + (long)s * MN + i4);
  const long m = i4 / N, n = i4 % N;
  float* c = C + m * ldc + n;
  if (beta != 0.f) o += beta * *(const f32x4*)c;
  *(f32x4*)c = o;
}

// split count of the weight-gradient GEMM (fp32 slabs over K = tokens): the count that fills whole
// waves of the CUs best with >= 2048-deep slices and slabs (+ extra fp32 elements per slab) within
// ws_bytes: e.g. 36 tiles x 7 = 252 workgroups, 27 x 9 = 243, 9 x 28 = 252
int wgrad_splits(int M, int N, int K, long ws_bytes, long extra) {
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  int splits = 1;
  double best = 0.0;
  for (int s = 1; s <= 64; ++s) {
    if (K / s < 2048 || (long)s * ((long)M * N + extra) * 4 > ws_bytes) break;
    const int wg = tiles * s, waves = (wg + 255) / 256;
    const double eff = (double)wg / (waves * 256.0) * (wg >= 192 ? 1.0 : wg / 192.0);
    if (eff > best + 1e-3) { best = eff; splits = s; }
  }
  return splits;
}

}  // namespace

// Weight gradient with the bias gradient fused (gemm.hip eegf_gemm_wgrad_bias): C[M][N] = A^T B + beta C
// over K tokens (A [K][M], B [K][N] bf16, both k-major), db[M] += A.sum(0), on the 4-wave kernel with
// fp32 split-K slabs followed by the fixed-order slab and row-sum reductions.  Returns 1 when the shape
// is not eligible (the caller then runs the plain GEMM and a column reduction).
int eegf_gemm_big_wgrad_bias(int M, int N, int K, const void* A, long lda, const void* B, long ldb, float* C, long ldc,
                             float beta, float* db, void* workspace, long ws_bytes, hipStream_t stream) {
  if (K % BK != 0 || M % 8 != 0 || N % 8 != 0 || M < 256 || N < 256 || K < 4096) return 1;
  if (lda % 8 || ldb % 8 || ldc % 4 || !workspace) return 1;
  if ((((uintptr_t)A | (uintptr_t)B) & 15) != 0) return 1;
  int splits = wgrad_splits(M, N, K, ws_bytes, M);
  if ((splits > 1 ? (long)splits * ((long)M * N + M) : (long)M) * 4 > ws_bytes) return 1;
  int ks = (K / splits + BK - 1) / BK * BK;
  splits = (K + ks - 1) / ks;
  float* slabs = (float*)workspace;
  float* part = slabs + (splits > 1 ? (long)splits * M * N : 0);
  BigArgs a{(const bf16*)A, (const bf16*)B, splits > 1 ? (void*)slabs : (void*)C, nullptr, nullptr, lda, ldb, ldc, 0,
            M, N, K, 1.0f, beta, 1.0f, splits > 1 ? ks : 0, part, g_ts_buf, group_for(N)};
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  EEGF_LAUNCH((gemm4w_kernel<false, false, EPI_NONE, float, true>), dim3(tiles, splits), dim3(NT4), 0,
                     stream, a);
  const int nrow = (M + 255) / 256;
  if (splits > 1) {
    const long MN = (long)M * N;
    const int nslab = (int)((MN / 4 + 255) / 256);
    EEGF_LAUNCH(splitk_rowsum_reduce, dim3((unsigned)(nslab + nrow)), dim3(256), 0, stream, (const float*)slabs,
                       splits, MN, N, C, ldc, beta, nslab, (const float*)part, M, db);
  } else {
    EEGF_LAUNCH(rowsum_reduce, dim3((unsigned)nrow), dim3(256), 0, stream, (const float*)part, splits, M, db);
  }
  return (int)hipGetLastError();
}

// Internal entry used by eegf_gemm (gemm.hip).  Returns 1 if the shape is not eligible.
//   bf16 out: token-sized forward / input-gradient GEMMs (A K-contiguous), any beta;
//   fp32 out: weight gradients (A, B k-major, EPI_NONE), split-K over the token axis with fp32 slabs
//             in `workspace` reduced in a fixed order (bitwise reproducible), beta applied once.
int eegf_gemm_big(int a_kc, int b_kc, int epi, int out_f32, int M, int N, int K, const void* A, long lda,
                  const void* B, long ldb, void* C, long ldc, const float* bias, void* aux, long ldaux, float alpha,
                  float beta, float epi_scale, void* workspace, long ws_bytes, hipStream_t stream) {
  if (K % BK != 0 || M % 8 != 0 || N % 8 != 0) return 1;
  if (lda % 8 || ldb % 8 || ldc % 8 || (aux && ldaux % 8)) return 1;
  if ((((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)aux) & 15) != 0) return 1;
  BigArgs a{(const bf16*)A, (const bf16*)B, C, bias, (bf16*)aux, lda, ldb, ldc, ldaux, M, N, K, alpha, beta,
            epi_scale, 0, nullptr, g_ts_buf, group_for(N)};
  if (out_f32) {
    if (a_kc || b_kc || epi != EPI_NONE || M < 256 || N < 256 || K < 4096 || ldc % 4) return 1;
    int splits = wgrad_splits(M, N, K, ws_bytes, 0);
    if (splits == 1) return launch_big<false, false, EPI_NONE, float>(a, 1, stream);
    int ks = (K / splits + BK - 1) / BK * BK;
    splits = (K + ks - 1) / ks;
    a.C = workspace;
    a.ksplit = ks;
    const int st = launch_big<false, false, EPI_NONE, float>(a, splits, stream);
    if (st) return st;
    const long MN = (long)M * N;
    EEGF_LAUNCH(big_splitk_reduce, dim3((unsigned)((MN / 4 + 255) / 256)), dim3(256), 0, stream,
                       (const float*)workspace, splits, MN, N, (float*)C, ldc, beta);
    return (int)hipGetLastError();
  }
  if (!a_kc || M < 2048 || N < 256) return 1;
  if (b_kc) {
    switch (epi) {
      case EPI_NONE: return launch_big<true, true, EPI_NONE, bf16>(a, 1, stream);
      case EPI_BIAS: return launch_big<true, true, EPI_BIAS, bf16>(a, 1, stream);
      case EPI_BIAS_GELU: return launch_big<true, true, EPI_BIAS_GELU, bf16>(a, 1, stream);
      case EPI_BIAS_RELU: return launch_big<true, true, EPI_BIAS_RELU, bf16>(a, 1, stream);
      case EPI_BIAS_TANH: return launch_big<true, true, EPI_BIAS_TANH, bf16>(a, 1, stream);
      case EPI_BIAS_GELU_D: return launch_big<true, true, EPI_BIAS_GELU_D, bf16>(a, 1, stream);
    }
  } else {
    switch (epi) {
      case EPI_NONE: return launch_big<true, false, EPI_NONE, bf16>(a, 1, stream);
      case EPI_DGELU: return launch_big<true, false, EPI_DGELU, bf16>(a, 1, stream);
      case EPI_DRELU: return launch_big<true, false, EPI_DRELU, bf16>(a, 1, stream);
      case EPI_DTANH: return launch_big<true, false, EPI_DTANH, bf16>(a, 1, stream);
      case EPI_MUL_AUX: return launch_big<true, false, EPI_MUL_AUX, bf16>(a, 1, stream);
    }
  }
  return 1;
}

extern int g_attn256_mode;     // attention.hip
extern int g_ln_fwd768;        // layernorm.hip

// Tuning / A-B hook (returns the old value; test and benchmark state, include/eegfusion.h lists the
// keys): 2 = L = 256 attention kernels (bit 0 forward, bit 1 backward); 6 / 7 = LayerNorm rows; 10 = the
// 768-wide LayerNorm forward; 11 = persistent GEMMs on / off; 13 = CUs left free by the persistent grids;
// 14 = gemm4r / gemm4p; 19 = the MFMA cross-attention kernels.
#if EEGF_DIAG
// Diagnostics builds only (-DEEGF_DIAG=1): every following gemm4w launch writes 4 phase timestamps + the
// CU id per workgroup into buf (int64 [grid.y][grid.x][8], s_memrealtime 100 MHz ticks) until called
// again with nullptr.  tools/gemm_phases.py.
extern "C" int eegf_gemm_big_timestamps(long long* buf) {
  g_ts_buf = buf;
  return 0;
}
#else
extern "C" int eegf_gemm_big_timestamps(long long* buf) { return buf ? EEGF_ERR_ARG : 0; }
#endif

extern int g_xbwd_mfma;   // decoder.hip
extern "C" int eegf_tune(int key, int value) {
  if (key == 19) { const int o = g_xbwd_mfma; if (value < 0 || value > 1) return EEGF_ERR_ARG; g_xbwd_mfma = value; return o; }
  if (key == 2) { const int o = g_attn256_mode; if (value < 0 || value > 3) return EEGF_ERR_ARG; g_attn256_mode = value; return o; }
  if (key == 7) { const int o = g_ln_bwd_rpb; if (value < 4 || value > 1024 || value % 4) return EEGF_ERR_ARG; g_ln_bwd_rpb = value; return o; }
  if (key == 10) { const int o = g_ln_fwd768; if (value < 0 || value > 1) return EEGF_ERR_ARG; g_ln_fwd768 = value; return o; }
  if (key == 11) { const int o = g_persistent; if (value < 0 || value > 1) return EEGF_ERR_ARG; g_persistent = value; return o; }
  if (key == 14) { const int o = g_gemm4r; if (value < 0 || value > 1) return EEGF_ERR_ARG; g_gemm4r = value; return o; }
  if (key == 13) { const int o = g_cu_reserve; if (value < 0 || value >= cu_count()) return EEGF_ERR_ARG; g_cu_reserve = value; return o; }
  if (key == 6) { const int o = g_ln_rpw; if (value < 1 || value > 64) return EEGF_ERR_ARG; g_ln_rpw = value; return o; }
  return EEGF_ERR_ARG;
}
