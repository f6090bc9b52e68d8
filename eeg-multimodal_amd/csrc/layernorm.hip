// layernorm.hip — residual-add + dropout + LayerNorm forward/backward, and strided row reductions.
//
// Replaces (per row of `width` features):
//   BertEmbeddings   LN(embeds + type[0] + pos[t]) then dropout          (modeling_bert.py:95-105)
//   BertSelfOutput / BertOutput   LN(dropout(dense) + residual)          (modeling_bert.py:282-351)
//   TransformerDecoderLayer norm1/2/3(x + dropout_k(block(x)))           (transformer.py:1158-1200)
// One wave per row, 4 features per lane-chunk (8-B bf16 / 16-B fp32 loads), fp32 statistics.
// The backward writes per-block partial sums of dgamma/dbeta (no atomics → bitwise reproducible);
// eegf_colsum reduces them (and bias / position-embedding gradients) in a second pass.
#include "common.h"
#include "eegfusion_internal.h"
#include <algorithm>

int g_ln_bwd_rpb = 64;  // rows per workgroup of eegf_ln_bwd for rows >= 65536 (eegf_tune key 7)
int g_ln_rpw = 16;  // max rows per wave of eegf_ln_fwd (eegf_tune key 6); see eegf_ln_fwd
// eegf_tune key 10: bf16 width-768 rows on ln_fwd768_kernel (1, default) or the generic kernel (0)
int g_ln_fwd768 = 1;

namespace {

template <typename T> struct V4;
template <> struct V4<float> {
  typedef f32x4 raw;
  static DEV f32x4 load(const float* p) { return *(const f32x4*)p; }
  static DEV f32x4 cvt(f32x4 v) { return v; }
  static DEV void store(float* p, f32x4 v) { *(f32x4*)p = v; }
};
template <> struct V4<bf16> {
  typedef bf16x4 raw;
  static DEV f32x4 load(const bf16* p) {
    bf16x4 v = *(const bf16x4*)p;
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
  static DEV f32x4 cvt(bf16x4 v) { return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]}; }
  static DEV void store(bf16* p, f32x4 v) {
    bf16x4 o;
    o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
    *(bf16x4*)p = o;
  }
};

// LayerNorm dropout stream (hidden dropout of BertEmbeddings / BertSelfOutput / BertOutput and the
// decoder's dropout1-3): the attention-probability stream of common.h (keep_bits8: Philox4x32-7,
// eight 16-bit draws per call): element e = row*W + col is kept iff halfword (e & 7) of call e >> 3
// clears thr16.  Lane l holds 4-element group g = l + 64c of chunk c, so lanes 2k, 2k+1 share one
// call per chunk: a chunk pair (c, c+1) costs one call per lane (even lanes draw chunk c's call,
// odd lanes chunk c+1's, swapped with one shuffle); an unpaired last chunk costs one call per lane.
// nib[c] bit j = keep bit of element col + j.  All 64 lanes of the wave must be active.
template <int NCH>
DEV void ln_keep(uint64_t seed, uint64_t offset, long row, int lane, float p, uint32_t (&nib)[NCH]) {
  const uint32_t thr = thr16_of(p);
  const int odd = lane & 1;
  const uint64_t rowcall = (uint64_t)row * (NCH * 32);
#pragma unroll
  for (int c = 0; c + 1 < NCH; c += 2) {
    const uint32_t mine = keep_bits8(seed, offset, rowcall + (uint64_t)(((lane & ~1) + 64 * (c + odd)) >> 1), thr);
    const uint32_t other = __shfl_xor(mine, 1, 64);
    nib[c] = ((odd ? other : mine) >> (4 * odd)) & 15u;
    nib[c + 1] = ((odd ? mine : other) >> (4 * odd)) & 15u;
  }
  if (NCH & 1) {
    const int c = NCH - 1;
    nib[c] = (keep_bits8(seed, offset, rowcall + (uint64_t)(((lane & ~1) + 64 * c) >> 1), thr) >> (4 * odd)) & 15u;
  }
}

struct LnFwdArgs {
  const void* x; const void* r; const float* table; const float* table2;
  const float* gamma; const float* beta;
  void* y; void* s; float* mean; float* rstd;
  long rows; int table_period; float eps; float p; int drop_mode; uint64_t seed, offset;
  int rpw;  // rows per wave (consecutive rows; eegf_tune key 6)
};

// One wave per row, rpw consecutive rows per wave (eegf_tune key 6); with rpw > 1 the next row's
// x / r are loaded before the current row is reduced (two rows of loads in flight per wave).
template <typename T, int NCH>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnFwdArgs a) {
  typedef typename V4<T>::raw R4;
  constexpr int W = NCH * 256;
  const int lane = threadIdx.x & 63;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * a.rpw;
  if (row0 >= a.rows) return;
  const long rend = row0 + a.rpw < a.rows ? row0 + a.rpw : a.rows;
  const bool drop = a.drop_mode != 0 && a.p > 0.f;
  const float dscale = drop ? 1.0f / (1.0f - a.p) : 1.0f;
  R4 px[NCH], pr[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    px[c] = *(const R4*)((const T*)a.x + row0 * W + col);
    if (a.r) pr[c] = *(const R4*)((const T*)a.r + row0 * W + col);
  }
  for (long row = row0; row < rend; ++row) {
    R4 cx[NCH], cr[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) { cx[c] = px[c]; cr[c] = pr[c]; }
    if (row + 1 < rend) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int col = (lane + 64 * c) * 4;
        px[c] = *(const R4*)((const T*)a.x + (row + 1) * W + col);
        if (a.r) pr[c] = *(const R4*)((const T*)a.r + (row + 1) * W + col);
      }
    }
    f32x4 v[NCH];
    float sum = 0.f;
    uint32_t nib[NCH];
    if (drop) ln_keep<NCH>(a.seed, a.offset, row, lane, a.p, nib);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      v[c] = V4<T>::cvt(cx[c]);
      if (drop && a.drop_mode == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[c][e] *= ((nib[c] >> e) & 1u) ? dscale : 0.f;
      }
      if (a.r) v[c] += V4<T>::cvt(cr[c]);
      if (a.table) v[c] += *(const f32x4*)(a.table + (row % a.table_period) * W + col);
      if (a.table2) v[c] += *(const f32x4*)(a.table2 + col);
      if (a.s) V4<T>::store((T*)a.s + row * W + col, v[c]);
      sum += v[c][0] + v[c][1] + v[c][2] + v[c][3];
    }
    const float mean = wave_sum(sum) * (1.0f / W);
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[c][e] - mean; sq += d * d; }
    const float rstd = rsqrtf(wave_sum(sq) * (1.0f / W) + a.eps);
    T* y = (T*)a.y + row * W;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      const f32x4 g = *(const f32x4*)(a.gamma + col), b = *(const f32x4*)(a.beta + col);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[c][e] - mean) * rstd * g[e] + b[e];
      if (drop && a.drop_mode == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] *= ((nib[c] >> e) & 1u) ? dscale : 0.f;
      }
      V4<T>::store(y + col, o);
    }
    if (lane == 0) {
      if (a.mean) a.mean[row] = mean;
      if (a.rstd) a.rstd[row] = rstd;
    }
  }
}

// bf16 rows of 768 (the BERT hidden LayerNorms): 16-B accesses for columns 0..511 (lane l owns 8l ..
// 8l + 7) and 8-B accesses for 512..767 (lane l owns 512 + 4l .. + 3), so 2 / 3 of the row moves in
// 1-KB wave-instructions (ln_fwd_kernel's 4-column lane chunks move 512 B per instruction).  The
// dropout stream is the same function of (row, column): columns 8l .. 8l + 7 are exactly call
// row * 96 + l (no cross-lane exchange), columns 512 + 4l .. are half of call row * 96 + 64 + l / 2.
DEV void ld8bf(const bf16* p, float (&v)[8]) {
  const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
}
DEV void st8bf(bf16* p, const float (&v)[8]) {
  bf16x8 x;
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = (bf16)v[e];
  *(bf16x8*)p = x;
}
__global__ void __launch_bounds__(256, 4) ln_fwd768_kernel(LnFwdArgs a) {   // 4 waves per SIMD: <= 128 VGPRs
  constexpr int W = 768;
  const int lane = threadIdx.x & 63;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * a.rpw;
  if (row0 >= a.rows) return;
  const long rend = row0 + a.rpw < a.rows ? row0 + a.rpw : a.rows;
  const bool drop = a.drop_mode != 0 && a.p > 0.f;
  const float dscale = drop ? 1.0f / (1.0f - a.p) : 1.0f;
  const uint32_t thr = thr16_of(a.p);
  const int ca = 8 * lane, cb = 512 + 4 * lane;      // the lane's column groups
  // gamma / beta of the lane's 12 columns, once per wave: inside the row loop hipcc re-loads them every
  // row (the y / s stores may alias them as far as it can tell); 6 % on the launch without the residual
  // store, step -0.3 ms (profiles/r4zj_ln_hoist_ab.log)
  float gm[12], bt[12];
  {
    const f32x4 g0 = *(const f32x4*)(a.gamma + ca), g1 = *(const f32x4*)(a.gamma + ca + 4), g2 = *(const f32x4*)(a.gamma + cb);
    const f32x4 b0 = *(const f32x4*)(a.beta + ca), b1 = *(const f32x4*)(a.beta + ca + 4), b2 = *(const f32x4*)(a.beta + cb);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gm[e] = g0[e]; gm[4 + e] = g1[e]; gm[8 + e] = g2[e];
      bt[e] = b0[e]; bt[4 + e] = b1[e]; bt[8 + e] = b2[e];
    }
  }
  const bf16* X = (const bf16*)a.x;
  const bf16* Rr = (const bf16*)a.r;
  bf16x8 pxa, pra = {};
  bf16x4 pxb, prb = {};
  pxa = *(const bf16x8*)(X + row0 * W + ca);
  pxb = *(const bf16x4*)(X + row0 * W + cb);
  if (Rr) { pra = *(const bf16x8*)(Rr + row0 * W + ca); prb = *(const bf16x4*)(Rr + row0 * W + cb); }
  for (long row = row0; row < rend; ++row) {
    const bf16x8 cxa = pxa, cra = pra;
    const bf16x4 cxb = pxb, crb = prb;
    if (row + 1 < rend) {
      pxa = *(const bf16x8*)(X + (row + 1) * W + ca);
      pxb = *(const bf16x4*)(X + (row + 1) * W + cb);
      if (Rr) { pra = *(const bf16x8*)(Rr + (row + 1) * W + ca); prb = *(const bf16x4*)(Rr + (row + 1) * W + cb); }
    }
    uint32_t ka = 0xFFu, kb = 0xFu;                   // keep bits: ka bit e <-> ca + e, kb bit e <-> cb + e
    if (drop) {
      ka = keep_bits8(a.seed, a.offset, (uint64_t)row * 96 + lane, thr);
      kb = (keep_bits8(a.seed, a.offset, (uint64_t)row * 96 + 64 + (lane >> 1), thr) >> (4 * (lane & 1))) & 0xFu;
    }
    float v[12];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)cxa[e];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[8 + e] = (float)cxb[e];
    if (drop && a.drop_mode == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= ((ka >> e) & 1u) ? dscale : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[8 + e] *= ((kb >> e) & 1u) ? dscale : 0.f;
    }
    if (Rr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += (float)cra[e];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[8 + e] += (float)crb[e];
    }
    if (a.table) {
      const float* tp = a.table + (row % a.table_period) * W;
      const f32x4 t0 = *(const f32x4*)(tp + ca), t1 = *(const f32x4*)(tp + ca + 4), t2 = *(const f32x4*)(tp + cb);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] += t0[e]; v[4 + e] += t1[e]; v[8 + e] += t2[e]; }
    }
    if (a.table2) {
      const f32x4 t0 = *(const f32x4*)(a.table2 + ca), t1 = *(const f32x4*)(a.table2 + ca + 4),
                  t2 = *(const f32x4*)(a.table2 + cb);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[e] += t0[e]; v[4 + e] += t1[e]; v[8 + e] += t2[e]; }
    }
    if (a.s) {
      bf16* sp = (bf16*)a.s + row * W;
      float va[8] = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
      st8bf(sp + ca, va);
      V4<bf16>::store(sp + cb, f32x4{v[8], v[9], v[10], v[11]});
    }
    float sum = 0.f;
#pragma unroll
    for (int e = 0; e < 12; ++e) sum += v[e];
    const float mean = wave_sum(sum) * (1.0f / W);
    float sq = 0.f;
#pragma unroll
    for (int e = 0; e < 12; ++e) { const float d = v[e] - mean; sq += d * d; }
    const float rstd = rsqrtf(wave_sum(sq) * (1.0f / W) + a.eps);
    float o[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) o[e] = (v[e] - mean) * rstd * gm[e] + bt[e];
    if (drop && a.drop_mode == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= ((ka >> e) & 1u) ? dscale : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[8 + e] *= ((kb >> e) & 1u) ? dscale : 0.f;
    }
    bf16* y = (bf16*)a.y + row * W;
    float oa[8] = {o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]};
    st8bf(y + ca, oa);
    V4<bf16>::store(y + cb, f32x4{o[8], o[9], o[10], o[11]});
    if (lane == 0) {
      if (a.mean) a.mean[row] = mean;
      if (a.rstd) a.rstd[row] = rstd;
    }
  }
}

struct LnBwdArgs {
  const void* dy; const void* s; const float* mean; const float* rstd; const float* gamma;
  void* dx; void* dr; float* dgamma_part; float* dbeta_part;
  long rows; int rows_per_block; float p; int drop_mode; uint64_t seed, offset;
};

template <typename T, int NCH>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnBwdArgs a) {
  constexpr int W = NCH * 256;
  __shared__ float red[2][4][W];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 dg[NCH], db[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) { dg[c] = f32x4{0, 0, 0, 0}; db[c] = f32x4{0, 0, 0, 0}; }
  f32x4 gam[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) gam[c] = *(const f32x4*)(a.gamma + (lane + 64 * c) * 4);

  const long r0 = (long)blockIdx.x * a.rows_per_block;
  for (int i = wave; i < a.rows_per_block; i += 4) {
    const long row = r0 + i;
    if (row >= a.rows) break;
    const float mean = a.mean[row], rstd = a.rstd[row];
    f32x4 dy[NCH], xh[NCH];
    float s1 = 0.f, s2 = 0.f;
    uint32_t nib[NCH];
    const bool drop = a.drop_mode != 0 && a.p > 0.f;
    const float dscale = drop ? 1.0f / (1.0f - a.p) : 1.0f;
    if (drop) ln_keep<NCH>(a.seed, a.offset, row, lane, a.p, nib);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      dy[c] = V4<T>::load((const T*)a.dy + row * W + col);
      if (drop && a.drop_mode == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) dy[c][e] *= ((nib[c] >> e) & 1u) ? dscale : 0.f;
      }
      const f32x4 sv = V4<T>::load((const T*)a.s + row * W + col);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[c][e] = (sv[e] - mean) * rstd;
        const float g = dy[c][e] * gam[c][e];
        s1 += g;
        s2 += g * xh[c][e];
        dg[c][e] += dy[c][e] * xh[c][e];
        db[c][e] += dy[c][e];
      }
    }
    s1 = wave_sum(s1) * (1.0f / W);
    s2 = wave_sum(s2) * (1.0f / W);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (lane + 64 * c) * 4;
      f32x4 ds;
#pragma unroll
      for (int e = 0; e < 4; ++e) ds[e] = rstd * (dy[c][e] * gam[c][e] - s1 - xh[c][e] * s2);
      if (a.dr) V4<T>::store((T*)a.dr + row * W + col, ds);
      if (drop && a.drop_mode == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ds[e] *= ((nib[c] >> e) & 1u) ? dscale : 0.f;
      }
      if (a.dx) V4<T>::store((T*)a.dx + row * W + col, ds);
    }
  }
  // per-block partial dgamma / dbeta (fixed order: bitwise reproducible)
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (lane + 64 * c) * 4;
    *(f32x4*)&red[0][wave][col] = dg[c];
    *(f32x4*)&red[1][wave][col] = db[c];
  }
  __syncthreads();
  for (int col = threadIdx.x; col < W; col += 256) {
    const float g = red[0][0][col] + red[0][1][col] + red[0][2][col] + red[0][3][col];
    const float b = red[1][0][col] + red[1][1][col] + red[1][2][col] + red[1][3][col];
    if (a.dgamma_part) a.dgamma_part[(long)blockIdx.x * W + col] = g;
    if (a.dbeta_part) a.dbeta_part[(long)blockIdx.x * W + col] = b;
  }
}

// ---- strided column sums: out[p, c] = sum_{r = p (mod period)} in[r*ld + c]  (+ beta*out) ----
// A period-P sum over contiguous rows is a plain column sum over rows/P rows of width P*width.
// Stage 1: each thread sums 8 adjacent columns (one 16-B bf16 / 2x16-B fp32 load per row) over a
// chunk of rows → fp32 partial [chunk][width].  Stage 2: 4 waves split the chunks of 64 columns,
// LDS combine, fixed order → bitwise reproducible.
template <typename T>
__global__ void __launch_bounds__(256) colsum_chunks(const T* __restrict__ in, long ld, long rows, int width,
                                                     long rows_per_chunk, float* __restrict__ ws) {
  const int c0 = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c0 >= width) return;
  const long r0 = (long)blockIdx.y * rows_per_chunk;
  const long r1 = min(rows, r0 + rows_per_chunk);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 + 8 <= width) {
    for (long r = r0; r < r1; ++r) {
      const T* p = in + r * ld + c0;
      if (sizeof(T) == 2) {
        const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
      } else {
        const f32x4 v0 = *(const f32x4*)p, v1 = *(const f32x4*)(p + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc[e] += v0[e]; acc[4 + e] += v1[e]; }
      }
    }
  } else {
    for (long r = r0; r < r1; ++r)
      for (int e = 0; e < 8 && c0 + e < width; ++e) acc[e] += to_f32(in[r * ld + c0 + e]);
  }
  float* o = ws + (long)blockIdx.y * width + c0;
  for (int e = 0; e < 8 && c0 + e < width; ++e) o[e] = acc[e];
}

template <typename T>
__global__ void __launch_bounds__(256) colsum_scalar(const T* __restrict__ in, long ld, long rows, int width,
                                                     long rows_per_chunk, float* __restrict__ ws) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= width) return;
  const long r0 = (long)blockIdx.y * rows_per_chunk, r1 = min(rows, r0 + rows_per_chunk);
  float acc = 0.f;
  for (long r = r0; r < r1; ++r) acc += to_f32(in[r * ld + c]);
  ws[(long)blockIdx.y * width + c] = acc;
}

// 16 waves per 64-column block, each summing chunks k = wave (mod 16) with 8 loads in flight (one
// load per memory round trip before: the 1,024-chunk combine of a 65,536-row bias gradient took 65 us
// for 3 MB on 12 workgroups); the 16 wave sums are added in a fixed order (deterministic)
constexpr int CW = 16;
__global__ void __launch_bounds__(64 * CW) colsum_combine(const float* __restrict__ ws, int chunks, int width,
                                                          float* __restrict__ out, float beta) {
  __shared__ float red[CW][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (c < width) {
    int k = wave;
    for (; k + 7 * CW < chunks; k += 8 * CW) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ws[(long)(k + u * CW) * width + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; k < chunks; k += CW) acc += ws[(long)k * width + c];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < width) {
    float v = red[0][lane];
#pragma unroll
    for (int w = 1; w < CW; ++w) v += red[w][lane];
    out[c] = beta != 0.f ? v + beta * out[c] : v;
  }
}

template <typename T>
int colsum_t(const void* in, long ld, long rows, int width, int period, float* ws, long ws_elems, float* out,
             float beta, hipStream_t st) {
  if (period > 1) {
    if (ld != width || rows % period != 0) return EEGF_ERR_ARG;
    rows /= period;
    width *= period;
    ld = width;
  }
  const bool vec = (width % 8 == 0) && (ld % 8 == 0) && (((uintptr_t)in & 15) == 0);
  const int xblocks = vec ? (width + 2047) / 2048 : (width + 255) / 256;
  long chunks = std::max(1L, std::min(rows / 32, (long)(1024 + xblocks - 1) / xblocks));
  while (chunks * width > ws_elems && chunks > 1) chunks = (chunks + 1) / 2;
  if (chunks * width > ws_elems) return EEGF_ERR_ARG;
  const long rpc = (rows + chunks - 1) / chunks;
  chunks = (rows + rpc - 1) / rpc;
  if (vec) EEGF_LAUNCH(colsum_chunks<T>, dim3(xblocks, (unsigned)chunks), dim3(256), 0, st, (const T*)in, ld, rows, width, rpc, ws);
  else EEGF_LAUNCH(colsum_scalar<T>, dim3(xblocks, (unsigned)chunks), dim3(256), 0, st, (const T*)in, ld, rows, width, rpc, ws);
  EEGF_LAUNCH(colsum_combine, dim3((width + 63) / 64), dim3(64 * CW), 0, st, ws, (int)chunks, width, out, beta);
  return (int)hipGetLastError();
}

template <typename T>
int ln_fwd_t(int nch, const LnFwdArgs& a, hipStream_t st) {
  const dim3 grid((unsigned)((a.rows + 4L * a.rpw - 1) / (4L * a.rpw)));
  switch (nch) {
    case 1: EEGF_LAUNCH((ln_fwd_kernel<T, 1>), grid, dim3(256), 0, st, a); break;
    case 2: EEGF_LAUNCH((ln_fwd_kernel<T, 2>), grid, dim3(256), 0, st, a); break;
    case 3: EEGF_LAUNCH((ln_fwd_kernel<T, 3>), grid, dim3(256), 0, st, a); break;
    case 4: EEGF_LAUNCH((ln_fwd_kernel<T, 4>), grid, dim3(256), 0, st, a); break;
    default: return EEGF_ERR_ARG;
  }
  return (int)hipGetLastError();
}

template <typename T>
int ln_bwd_t(int nch, const LnBwdArgs& a, hipStream_t st) {
  const dim3 grid((unsigned)((a.rows + a.rows_per_block - 1) / a.rows_per_block));
  switch (nch) {
    case 1: EEGF_LAUNCH((ln_bwd_kernel<T, 1>), grid, dim3(256), 0, st, a); break;
    case 2: EEGF_LAUNCH((ln_bwd_kernel<T, 2>), grid, dim3(256), 0, st, a); break;
    case 3: EEGF_LAUNCH((ln_bwd_kernel<T, 3>), grid, dim3(256), 0, st, a); break;
    case 4: EEGF_LAUNCH((ln_bwd_kernel<T, 4>), grid, dim3(256), 0, st, a); break;
    default: return EEGF_ERR_ARG;
  }
  return (int)hipGetLastError();
}

// ---- batched column sums: many small independent reductions in one launch ----
// Descriptor (6 x int64): src, dst, ld, rows, width | dtype << 32, float_bits(beta) | first_block << 32.
// Block b serves the descriptor whose block range holds b: 64 columns.  Thread t sums the 4 columns
// 4 (t & 15) .. of the rows r = t >> 4 (mod 16) with one 16-B (fp32) / 8-B (bf16) load per row, 4 rows in
// flight; the 16 row-group partials are combined in a fixed order (bitwise reproducible); dst[c] = sum +
// beta * dst[c].  Descriptors whose base, row stride or width are not 4-element aligned take the
// one-column-per-lane form.  (The 1-column form held ~2.3 TB/s on the 1,165-block batch of the bench
// step's LayerNorm / bias partials: 130 us, profiles/r5zh_kernel_stats.md.)
template <typename T>
DEV void colsum_rows4(const T* p, long ld, long rows, int rg, float (&acc)[4]) {
  long r = rg;
  for (; r + 48 < rows; r += 64) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = V4<T>::load(p + (r + 16 * u) * ld);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += v[u][e];
  }
  for (; r < rows; r += 16) {
    const f32x4 v = V4<T>::load(p + r * ld);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] += v[e];
  }
}
__global__ void __launch_bounds__(256) colsum_batch_kernel(const long long* __restrict__ desc, int n) {
  __shared__ float red[16][65];
  const int blk = blockIdx.x, tid = threadIdx.x;
  int d = 0;
  for (int i = 1; i < n; ++i) {
    if ((int)(desc[6 * i + 5] >> 32) <= blk) d = i;
    else break;
  }
  const long long* D = desc + 6 * d;
  const long ld = D[2], rows = D[3];
  const int width = (int)(D[4] & 0xffffffffLL), dtype = (int)(D[4] >> 32);
  const float beta = __int_as_float((int)(D[5] & 0xffffffffLL));
  const int c0 = (blk - (int)(D[5] >> 32)) * 64;
  const int esz = dtype == EEGF_BF16 ? 2 : 4;
  const bool vec = ((D[0] | (ld * esz)) & (4L * esz - 1)) == 0 && (width & 3) == 0;
  if (vec) {
    const int cq = tid & 15, rg = tid >> 4, c = c0 + 4 * cq;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < width) {
      if (dtype == EEGF_BF16) colsum_rows4((const bf16*)D[0] + c, ld, rows, rg, acc);
      else colsum_rows4((const float*)D[0] + c, ld, rows, rg, acc);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) red[rg][4 * cq + e] = acc[e];
  } else {
    const int lane = tid & 63, wave = tid >> 6, c = c0 + lane;
    const long r0 = rows * wave / 4, r1 = rows * (wave + 1) / 4;
    float acc = 0.f;
    if (c < width) {
      if (dtype == EEGF_BF16) {
        const bf16* p = (const bf16*)D[0] + c;
        for (long r = r0; r < r1; ++r) acc += (float)p[r * ld];
      } else {
        const float* p = (const float*)D[0] + c;
        for (long r = r0; r < r1; ++r) acc += p[r * ld];
      }
    }
    red[wave][lane] = acc;
  }
  __syncthreads();
  if (tid < 64 && c0 + tid < width) {
    const int c = c0 + tid, ng = vec ? 16 : 4;
    float v = 0.f;
    for (int i = 0; i < ng; ++i) v += red[i][tid];
    float* dst = (float*)D[1];
    dst[c] = beta != 0.f ? v + beta * dst[c] : v;
  }
}

}  // namespace

extern "C" int eegf_colsum_batch(int n, const long long* desc, int blocks, hipStream_t stream) {
  if (n <= 0 || !desc || blocks <= 0) return EEGF_ERR_ARG;
  EEGF_LAUNCH(colsum_batch_kernel, dim3(blocks), dim3(256), 0, stream, desc, n);
  return (int)hipGetLastError();
}

extern "C" int eegf_ln_fwd(int dtype, long rows, int width, const void* x, const void* r, const float* table,
                           int table_period, const float* table2, const float* gamma, const float* beta, float eps,
                           float drop_p, int drop_mode, unsigned long long seed, unsigned long long offset,
                           void* y, void* s_out, float* mean, float* rstd, hipStream_t stream) {
  if (rows <= 0 || width % 256 != 0 || width > 1024 || !x || !gamma || !beta || !y) return EEGF_ERR_ARG;
  if (table && table_period <= 0) return EEGF_ERR_ARG;
  if (drop_p < 0.f || drop_p >= 1.f || drop_mode < 0 || drop_mode > 2) return EEGF_ERR_ARG;
  LnFwdArgs a{x, r, table, table2, gamma, beta, y, s_out, mean, rstd, rows, table_period, eps, drop_p, drop_mode,
              seed, offset, 1};
  // rows per wave: up to g_ln_rpw while the grid keeps >= 1024 workgroups (4 per CU); measured at
  // 65536 x 768 bf16 (tools/ln_bench.py): 86 -> 67 us without, 97 -> 88 us with the residual store
  while (a.rpw * 2 <= g_ln_rpw && rows / (4L * a.rpw * 2) >= 1024) a.rpw *= 2;
  if (dtype == EEGF_F32) return ln_fwd_t<float>(width / 256, a, stream);
  if (dtype == EEGF_BF16 && width == 768 && g_ln_fwd768 &&
      ((((uintptr_t)x | (uintptr_t)r | (uintptr_t)y | (uintptr_t)s_out | (uintptr_t)table | (uintptr_t)table2 |
         (uintptr_t)gamma | (uintptr_t)beta) & 15) == 0)) {
    const dim3 grid((unsigned)((a.rows + 4L * a.rpw - 1) / (4L * a.rpw)));
    EEGF_LAUNCH(ln_fwd768_kernel, grid, dim3(256), 0, stream, a);
    return (int)hipGetLastError();
  }
  if (dtype == EEGF_BF16) return ln_fwd_t<bf16>(width / 256, a, stream);
  return EEGF_ERR_ARG;
}

extern "C" long eegf_ln_bwd_partial_rows(long rows) {
  // rows per block of eegf_ln_bwd: partial buffers hold ceil(rows / this) x width floats.  Below 65536
  // rows about 256 blocks (a multiple of 4 rows, 4 .. 64): the decoder's 256-row LayerNorms ran 4 blocks
  // of 64 rows, 16 waves on the whole chip (25.5 us each, 9 per step; profiles/r5zh_kernel_stats.md)
  if (rows >= 65536) return g_ln_bwd_rpb;
  const long r = (rows / 256 + 3) / 4 * 4;
  return r < 4 ? 4 : r > 64 ? 64 : r;
}

extern "C" int eegf_ln_bwd(int dtype, long rows, int width, const void* dy, const void* s, const float* mean,
                           const float* rstd, const float* gamma, float drop_p, int drop_mode,
                           unsigned long long seed, unsigned long long offset, void* dx, void* dr,
                           float* dgamma_part, float* dbeta_part, hipStream_t stream) {
  if (rows <= 0 || width % 256 != 0 || width > 1024 || !dy || !s || !mean || !rstd || !gamma) return EEGF_ERR_ARG;
  if (drop_p < 0.f || drop_p >= 1.f || drop_mode < 0 || drop_mode > 2) return EEGF_ERR_ARG;
  LnBwdArgs a{dy, s, mean, rstd, gamma, dx, dr, dgamma_part, dbeta_part, rows,
              (int)eegf_ln_bwd_partial_rows(rows), drop_p, drop_mode, seed, offset};
  if (dtype == EEGF_F32) return ln_bwd_t<float>(width / 256, a, stream);
  if (dtype == EEGF_BF16) return ln_bwd_t<bf16>(width / 256, a, stream);
  return EEGF_ERR_ARG;
}

extern "C" int eegf_colsum(int dtype, const void* in, long ld, long rows, int width, int period, float* ws,
                           long ws_elems, float* out, float beta, hipStream_t stream) {
  if (!in || !ws || !out || rows <= 0 || width <= 0 || period <= 0 || period > 65535) return EEGF_ERR_ARG;
  if (dtype == EEGF_F32) return colsum_t<float>(in, ld, rows, width, period, ws, ws_elems, out, beta, stream);
  if (dtype == EEGF_BF16) return colsum_t<bf16>(in, ld, rows, width, period, ws, ws_elems, out, beta, stream);
  return EEGF_ERR_ARG;
}
