// decoder.hip — single-query cross-attention of the 3-layer TransformerDecoder over the BERT memory.
//
// Reference: multihead_attn(x, memory, memory) inside TransformerDecoderLayer._mha_block
// (torch/nn/modules/transformer.py:1177-1196; F.multi_head_attention_forward), called from
// model.py:40-43 with tgt = the single action token.  The memory K/V projections are never
// materialised: for head h with projected query q_h,
//     score_j = q_h . (Wk_h M_j + bk_h) / 8 = q'_h . M_j + const,   q'_h = Wk_h^T q_h / 8
//     ctx_h   = sum_j p~_j (Wv_h M_j + bv_h) = Wv_h c_h + s_h bv_h,   c_h = sum_j p~_j M_j
// where p~ = dropout(p) (attention-probability dropout, F.multi_head_attention_forward dropout_p)
// and s_h = sum_j p~_j (1 without dropout).  The constant q_h.bk_h/8 cancels in the softmax.
//
// Kernels (HBM-bound on the memory M = [B, S, 768] in the encoder dtype):
//   xrow_dot   lane = one memory row j: out[b,h,j] = v[b,h,:] . M[b,j,:]   (v uniform → scalar loads)
//              forward: raw scores (v = q');  backward: dp~ (v = dc)
//   xctx       per (b, 256-column slab): softmax over j (recomputed per workgroup from the raw
//              scores), dropout, then c[h, cols] = sum_j p~[h][j] M[j][cols]; 4 waves split j
//   xbwd_cols  per (b, 256-column slab): softmax backward, then in one pass over M:
//              dq'[h, cols] = sum_j dsc[h][j] M[j][cols],  dM[j][cols] = sum_h p~ dc + dsc q'
//   xctx_mfma / xbwd_mfma  the same two for a bf16 memory on v_mfma_f32_16x16x4_f32 (the bench path)
// The q'/Wv/out-proj GEMMs are eegf_gemm; the s_h bv_h term is eegf_head_bias_fwd/bwd.
#include "common.h"
#include "eegfusion_internal.h"

// eegf_tune key 19: the bf16-memory context and backward on xctx_mfma_kernel / xbwd_mfma_kernel (1,
// default) or the VALU xctx_kernel / xbwd_cols_kernel (0)
int g_xbwd_mfma = 1;

namespace {

constexpr int E = 768, NH = 12, SLAB = 256;

template <typename T> DEV void load4(const T* p, float (&v)[4]);
template <> DEV void load4<float>(const float* p, float (&v)[4]) {
  const float4 x = *(const float4*)p;
  v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
}
template <> DEV void load4<bf16>(const bf16* p, float (&v)[4]) {
  const bf16x4 x = *(const bf16x4*)p;
  v[0] = (float)x[0]; v[1] = (float)x[1]; v[2] = (float)x[2]; v[3] = (float)x[3];
}
template <typename T> DEV void store4(T* p, const float (&v)[4]);
template <> DEV void store4<float>(float* p, const float (&v)[4]) { *(float4*)p = float4{v[0], v[1], v[2], v[3]}; }
template <> DEV void store4<bf16>(bf16* p, const float (&v)[4]) {
  bf16x4 o;
  o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
  *(bf16x4*)p = o;
}

// out[b,h,j] = vec[b,h,:] . M[b,j,:] (+ kbias[b,j]); grid (ceil(S/64), B), 256 threads:
// lane = row j, wave w = column quarter [192w, 192w+192) (8 columns per 16-B step, next step's
// row chunk prefetched), partial dot products reduced across the 4 waves through LDS.
template <typename T, typename TV>
__global__ void __launch_bounds__(256) xrow_dot_kernel(const T* __restrict__ mem, const TV* __restrict__ vec,
                                                       const float* __restrict__ kbias, int S, float* __restrict__ out) {
  constexpr int QW = E / 4;                       // 192 columns per wave
  __shared__ float red[4][NH][64];
  const int b = blockIdx.y, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int jr = j < S ? j : S - 1;
  const int c0 = wave * QW;
  const T* row = mem + ((long)b * S + jr) * E + c0;
  const TV* v = vec + (long)b * NH * E + c0;
  float acc[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) acc[h] = 0.f;
  float nx[8];
  load4<T>(row, *(float(*)[4])nx);
  load4<T>(row + 4, *(float(*)[4])(nx + 4));
#pragma unroll 1
  for (int c = 0; c < QW; c += 8) {
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = nx[e];
    if (c + 8 < QW) {
      load4<T>(row + c + 8, *(float(*)[4])nx);
      load4<T>(row + c + 12, *(float(*)[4])(nx + 4));
    }
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)                // 4 columns x 12 heads of v (scalar) per half-step
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[h] += m[4 * hf + e] * to_f32(v[h * E + c + 4 * hf + e]);
  }
#pragma unroll
  for (int h = 0; h < NH; ++h) red[wave][h][lane] = acc[h];
  __syncthreads();
  for (int i = threadIdx.x; i < NH * 64; i += 256) {
    const int h = i >> 6, l = i & 63, jj = blockIdx.x * 64 + l;
    if (jj < S) {
      const float kb = kbias ? kbias[(long)b * S + jj] : 0.f;
      out[((long)b * NH + h) * S + jj] = red[0][h][l] + red[1][h][l] + red[2][h][l] + red[3][h][l] + kb;
    }
  }
}

// Same product on the MFMA for a bf16 memory: grid (ceil(S/256), B), 4 waves x 16-row blocks.  The fp32
// vector is split as v = v_hi + v_lo (two bf16 operands, both multiplied against the exact bf16 memory
// and accumulated in fp32), so the scores keep ~2^-16 relative accuracy in v instead of bf16's 2^-8.
// A = memory rows straight from global (16 B per lane, 64 B row segments), B = v_hi / v_lo from LDS
// (heads padded 12 -> 16 with zeros).
constexpr int XR = 4;       // 64-row blocks per xrow_dot_mfma workgroup
constexpr int XW = 8;       // waves per xrow_dot_mfma workgroup (16-row blocks w, w + 8, ...): one
                            // workgroup per batch row at S = 256, so the CU's memory parallelism is
                            // its waves' loads in flight -- 4 waves held ~2.2 TB/s (profiles/r2am)
template <typename TV>
__global__ void __launch_bounds__(64 * XW) xrow_dot_mfma_kernel(const bf16* __restrict__ mem, const TV* __restrict__ vec,
                                                            const float* __restrict__ kbias, int S,
                                                            float* __restrict__ out) {
  // row stride E + 16 (98 bank quads = 2 mod 16): the 16-lane groups of the ds_read_b128 fragment reads
  // (rows li, chunk g) land on 16 distinct bank quads; E + 8 (1 mod 16) put rows 11 / 12 and 12 / 13 of
  // a group on one quad (2-way conflicts, 0.44 of the kernel's LDS cycles in r6x_pmc_table.md)
  constexpr int LDV = E + 16;
  __shared__ __attribute__((aligned(16))) bf16 vt[2][16 * LDV];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  // 4 consecutive elements per thread and every load of the loop issued before the first LDS store (one
  // load latency: the element-per-thread loop waited for each of its 24 loads in turn)
  constexpr int NV = 16 * E / 4 / (64 * XW);
  static_assert(NV * 4 * 64 * XW == 16 * E, "v staging covers 16 x 768");
  float4 xv[NV];
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = 4 * (tid + u * 64 * XW), h = i / E, c = i % E;
    if (h < NH) {
      float t[4];
      load4<TV>(vec + ((long)b * NH + h) * E + c, t);
      xv[u] = float4{t[0], t[1], t[2], t[3]};
    } else {
      xv[u] = float4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int i = 4 * (tid + u * 64 * XW), h = i / E, c = i % E;
    const float x[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
    bf16x4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      hi[e] = (bf16)x[e];
      lo[e] = (bf16)(x[e] - (float)hi[e]);
    }
    *(bf16x4*)(vt[0] + h * LDV + c) = hi;
    *(bf16x4*)(vt[1] + h * LDV + c) = lo;
  }
  __syncthreads();
  const bf16* vh = vt[0] + li * LDV + 8 * g;
  const bf16* vl = vt[1] + li * LDV + 8 * g;
  // the workgroup covers XR row blocks of 64 (amortises the v staging): wave w takes 16-row blocks
  // w, w + XW, ...; the whole 768-wide row segment's 24 loads are issued before the first MFMA
  for (int j0 = blockIdx.x * 64 * XR + wave * 16; j0 < min(S, (int)(blockIdx.x + 1) * 64 * XR); j0 += 16 * XW) {
    const bf16* row = mem + ((long)b * S + min(j0 + li, S - 1)) * E + 8 * g;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < E / 32; ++kc) {
      const bf16x8 a = *(const bf16x8*)(row + 32 * kc);
      acc = mma16(a, *(const bf16x8*)(vh + 32 * kc), acc);
      acc = mma16(a, *(const bf16x8*)(vl + 32 * kc), acc);
    }
    // acc[r] = out[row j0 + 4g + r][head li]
    if (li < NH) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = j0 + 4 * g + r;
        if (j < S) out[((long)b * NH + li) * S + j] = acc[r] + (kbias ? kbias[(long)b * S + j] : 0.f);
      }
    }
  }
}
template <typename T, typename TV>
void launch_xrow_dot(const T* mem, const TV* vec, const float* kbias, int B, int S, float* out, hipStream_t st) {
  if constexpr (sizeof(T) == 2)
    EEGF_LAUNCH((xrow_dot_mfma_kernel<TV>), dim3((S + 64 * XR - 1) / (64 * XR), B), dim3(64 * XW), 0, st, mem, vec,
                       kbias, S, out);
  else
    EEGF_LAUNCH((xrow_dot_kernel<T, TV>), dim3((S + 63) / 64, B), dim3(256), 0, st, mem, vec, kbias, S, out);
}

// Softmax (+dropout) of the 12 raw score rows of batch row b into LDS pt[S][12] (p~);
// workgroup slab 0 also stores the undropped p (for the backward) and s_h = sum_j p~.
DEV void softmax_rows(const float* __restrict__ raw, int S, int b, float p_drop, uint64_t seed, uint64_t offset,
                      bool write, float* __restrict__ probs, float* __restrict__ psum, float* pt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int h = wave; h < NH; h += nw) {
    const float* r = raw + ((long)b * NH + h) * S;
    // loops unrolled by 4: their independent loads issue together (the 1-by-1 loops waited for every
    // load in turn: ~24 dependent L2 round trips per workgroup before the first memory row)
    float mx = -3.0e38f;
#pragma unroll 4
    for (int j = lane; j < S; j += 64) mx = fmaxf(mx, r[j]);
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll 4
    for (int j = lane; j < S; j += 64) { const float e = __expf(r[j] - mx); pt[j * NH + h] = e; sum += e; }
    const float inv = 1.0f / wave_sum(sum);
    float ds = 0.f;
#pragma unroll 4
    for (int j = lane; j < S; j += 64) {
      const float p = pt[j * NH + h] * inv;
      if (write) probs[((long)b * NH + h) * S + j] = p;
      const float pd = p_drop > 0.f ? p * drop_mask1(seed, offset, ((uint64_t)b * NH + h) * S + j, p_drop) : p;
      pt[j * NH + h] = pd;
      ds += pd;
    }
    ds = wave_sum(ds);
    if (write && psum && lane == 0) psum[b * NH + h] = ds;
  }
}

DEV void lds_row12(const float* base, float (&v)[NH]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float4 x = *(const float4*)(base + 4 * k);
    v[4 * k] = x.x; v[4 * k + 1] = x.y; v[4 * k + 2] = x.z; v[4 * k + 3] = x.w;
  }
}

// Sum of the 8 waves' [12][4-column] partials in red[4][12][256]: waves 4-7 park theirs, waves 0-3
// add their own in place; the caller then sums the 4 slices (fixed order: deterministic).
DEV void reduce8_waves(const float (&acc)[NH][4], float* red, int wave, int lane) {
  if (wave >= 4) {
#pragma unroll
    for (int h = 0; h < NH; ++h)
      *(float4*)(red + ((wave - 4) * NH + h) * SLAB + lane * 4) = float4{acc[h][0], acc[h][1], acc[h][2], acc[h][3]};
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      float4* q = (float4*)(red + (wave * NH + h) * SLAB + lane * 4);
      const float4 o = *q;
      *q = float4{o.x + acc[h][0], o.y + acc[h][1], o.z + acc[h][2], o.w + acc[h][3]};
    }
  }
  __syncthreads();
}
DEV float red4(const float* red, int h, int c) {
  return red[(0 * NH + h) * SLAB + c] + red[(1 * NH + h) * SLAB + c] + red[(2 * NH + h) * SLAB + c] +
         red[(3 * NH + h) * SLAB + c];
}

// grid (E/256, B), 512 threads: lane owns 4 columns of the slab, wave w rows [w*S/8, (w+1)*S/8);
// the 8 per-wave partial contexts are summed in two rounds through a [4][12][256] LDS buffer.
template <typename T, typename TQ>
__global__ void __launch_bounds__(512) xctx_kernel(const T* __restrict__ mem, const float* __restrict__ raw, int S,
                                                   float p_drop, uint64_t seed, uint64_t offset,
                                                   float* __restrict__ probs, float* __restrict__ psum,
                                                   TQ* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* pt = sm;                       // [S][12]
  float* red = sm + S * NH;             // [4][12][256]
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  softmax_rows(raw, S, b, p_drop, seed, offset, blockIdx.x == 0, probs, psum, pt);
  __syncthreads();
  const int col = blockIdx.x * SLAB + lane * 4;
  float acc[NH][4];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[h][e] = 0.f;
  const int per = (S + 7) / 8, j0 = wave * per, j1 = min(S, j0 + per);
  const T* M = mem + (long)b * S * E + col;
#pragma unroll 4
  for (int j = j0; j < j1; ++j) {
    float m[4], p[NH];
    load4<T>(M + (long)j * E, m);
    lds_row12(pt + j * NH, p);
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[h][e] += p[h] * m[e];
  }
  reduce8_waves(acc, red, wave, lane);
  for (int i = tid; i < NH * SLAB; i += 512) {
    const int h = i / SLAB, c = i % SLAB;
    ctx[((long)b * NH + h) * E + blockIdx.x * SLAB + c] = from_f32<TQ>(red4(red, h, c));
  }
}

// The context on the fp32 MFMA for a bf16 memory: grid (E/256, B), 4 waves, the column layout of
// xbwd_mfma_kernel below (wave w: columns 256 slab + 64 w as four interleaved 16-column tiles):
// ctx^T[c][h] = sum_j M[j][c] p~[h][j] as v_mfma_f32_16x16x4_f32 (fp32 products and sums, as xctx_kernel).
// xctx_kernel at B = 256, S = 256: 37.9 us per launch, 2.6 TB/s (profiles/r5zm_kernel_stats.md).
template <typename TQ>
__global__ void __launch_bounds__(256) xctx_mfma_kernel(const bf16* __restrict__ mem, const float* __restrict__ raw, int S,
                                                        float p_drop, uint64_t seed, uint64_t offset,
                                                        float* __restrict__ probs, float* __restrict__ psum,
                                                        TQ* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float pt[];       // [Spad][12]
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int Spad = (S + 15) & ~15;
  softmax_rows(raw, S, b, p_drop, seed, offset, blockIdx.x == 0, probs, psum, pt);
  for (int i = S * NH + tid; i < Spad * NH; i += 256) pt[i] = 0.f;
  __syncthreads();
  const int cbase = blockIdx.x * SLAB + 64 * wave;
  const bf16* Mb = mem + (long)b * S * E + cbase + 4 * li;
  f32x4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x4 mc[4], mn[4];
  auto load_tile = [&](int jb, bf16x4 (&m)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) m[t] = *(const bf16x4*)(Mb + (long)min(jb + 4 * t + g, S - 1) * E);
  };
  load_tile(0, mc);
  for (int jb = 0; jb < Spad; jb += 16) {
    if (jb + 16 < Spad) load_tile(jb + 16, mn);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float pv = li < NH ? pt[(jb + 4 * t + g) * NH + li] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)mc[t][q], pv, acc[q], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) mc[t] = mn[t];
  }
  // acc[q][r] = ctx[h = li][cbase + 16 g + 4 r + q]
  if (li < NH) {
    TQ* dst = ctx + ((long)b * NH + li) * E + cbase + 16 * g;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = acc[q][r];
      store4<TQ>(dst + 4 * r, v);
    }
  }
}

// Backward, grid (E/256, B), 256 threads.  raw = dc . M_j (xrow_dot); dpsum[b,h] = dL/ds_h.
//   dp~ = raw + dpsum;  dp = dp~ * mask;  dsc = p (dp - sum_j p dp)
//   dq'[h,c] = sum_j dsc[h][j] M[j][c];   dM[j][c] (+)= sum_h p~[h][j] dc[h][c] + dsc[h][j] q'[h][c]
template <typename T, typename TQ>
__global__ void __launch_bounds__(512) xbwd_cols_kernel(const T* __restrict__ mem, const TQ* __restrict__ qp,
                                                        const float* __restrict__ probs, const float* __restrict__ raw,
                                                        const float* __restrict__ dpsum, const TQ* __restrict__ dc, int S,
                                                        float p_drop, uint64_t seed, uint64_t offset,
                                                        T* __restrict__ dmem, float beta, TQ* __restrict__ dqp) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* pt = sm;                 // [S][12] p~
  float* st = sm + S * NH;        // [S][12] dsc
  float* red = st + S * NH;       // [4][12][256]
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int h = wave; h < NH; h += 8) {
    const float* pr = probs + ((long)b * NH + h) * S;
    const float* dr = raw + ((long)b * NH + h) * S;
    const float dsh = dpsum ? dpsum[b * NH + h] : 0.f;
    float dot = 0.f;
    for (int j = lane; j < S; j += 64) {
      const float mk = p_drop > 0.f ? drop_mask1(seed, offset, ((uint64_t)b * NH + h) * S + j, p_drop) : 1.f;
      const float p = pr[j], dp = (dr[j] + dsh) * mk;
      pt[j * NH + h] = p * mk;
      st[j * NH + h] = dp;
      dot += p * dp;
    }
    dot = wave_sum(dot);
    for (int j = lane; j < S; j += 64) st[j * NH + h] = pr[j] * (st[j * NH + h] - dot);
  }
  __syncthreads();
  const int col = blockIdx.x * SLAB + lane * 4;
  float qr[NH][4], dcr[NH][4], acc[NH][4];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    load4<TQ>(qp + ((long)b * NH + h) * E + col, qr[h]);
    load4<TQ>(dc + ((long)b * NH + h) * E + col, dcr[h]);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[h][e] = 0.f;
  }
  const int per = (S + 7) / 8, j0 = wave * per, j1 = min(S, j0 + per);
  const T* M = mem + (long)b * S * E + col;
  T* dM = dmem + (long)b * S * E + col;
#pragma unroll 2
  for (int j = j0; j < j1; ++j) {
    float m[4], p[NH], d[NH], o[4] = {0.f, 0.f, 0.f, 0.f};
    load4<T>(M + (long)j * E, m);
    lds_row12(pt + j * NH, p);
    lds_row12(st + j * NH, d);
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[h][e] += d[h] * m[e];
        o[e] += p[h] * dcr[h][e] + d[h] * qr[h][e];
      }
    if (beta != 0.f) {
      float old[4];
      load4<T>(dM + (long)j * E, old);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] += beta * old[e];
    }
    store4<T>(dM + (long)j * E, o);
  }
  reduce8_waves(acc, red, wave, lane);
  for (int i = tid; i < NH * SLAB; i += 512) {
    const int h = i / SLAB, c = i % SLAB;
    dqp[((long)b * NH + h) * E + blockIdx.x * SLAB + c] = from_f32<TQ>(red4(red, h, c));
  }
}

// The same backward on the fp32 MFMA for a bf16 memory (v_mfma_f32_16x16x4_f32: fp32 products, fp32
// sums, as the VALU kernel above).  grid (E/256, B), 4 waves; wave w owns the 64 columns
// cbase = 256 slab + 64 w of every memory row, as four interleaved 16-column tiles q (MFMA row m <->
// column cbase + 4 m + q), so one 8-B load of M[j][cbase + 4 li ..] feeds all four tiles and the four
// tiles' accumulators hold 16 consecutive columns of one row:
//   dM^T[c][j] = sum_k B2[k][c] A2[j][k],  k < 24: A2 = [p~ | dsc] (LDS a2[j][k]), B2 = [dc ; q'] rows
//   dq'^T[c][h] = sum_j M[j][c] dsc[h][j]
// The softmax backward (the prologue) is the VALU kernel's.  Rows j >= S are zero in a2 (their M loads
// clamp to row S - 1 and contribute 0).  VALU kernel at B = 256, S = 256: 130 us per launch, 2.4 TB/s.
constexpr int A2LD = 25;     // a2 row stride (floats): 24 used
template <typename TQ>
__global__ void __launch_bounds__(256) xbwd_mfma_kernel(const bf16* __restrict__ mem, const TQ* __restrict__ qp,
                                                        const float* __restrict__ probs, const float* __restrict__ raw,
                                                        const float* __restrict__ dpsum, const TQ* __restrict__ dc, int S,
                                                        float p_drop, uint64_t seed, uint64_t offset,
                                                        bf16* __restrict__ dmem, float beta, TQ* __restrict__ dqp) {
  extern __shared__ __attribute__((aligned(16))) float a2[];        // [Spad][A2LD]
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int Spad = (S + 15) & ~15;
  for (int h = wave; h < NH; h += 4) {
    const float* pr = probs + ((long)b * NH + h) * S;
    const float* dr = raw + ((long)b * NH + h) * S;
    const float dsh = dpsum ? dpsum[b * NH + h] : 0.f;
    float dot = 0.f;
#pragma unroll 4
    for (int j = lane; j < S; j += 64) {
      const float mk = p_drop > 0.f ? drop_mask1(seed, offset, ((uint64_t)b * NH + h) * S + j, p_drop) : 1.f;
      const float p = pr[j], dp = (dr[j] + dsh) * mk;
      a2[j * A2LD + h] = p * mk;
      a2[j * A2LD + NH + h] = dp;
      dot += p * dp;
    }
    dot = wave_sum(dot);
#pragma unroll 4
    for (int j = lane; j < S; j += 64) a2[j * A2LD + NH + h] = pr[j] * (a2[j * A2LD + NH + h] - dot);
  }
  for (int i = S * A2LD + tid; i < Spad * A2LD; i += 256) a2[i] = 0.f;
  __syncthreads();
  const int cbase = blockIdx.x * SLAB + 64 * wave;
  // B2 rows k = g + 4 t (t < 6): columns cbase + 4 li + q -> bq[t][q]
  float bq[6][4];
#pragma unroll
  for (int t = 0; t < 6; ++t) {
    const int k = g + 4 * t;
    const TQ* src = k < NH ? dc + ((long)b * NH + k) * E : qp + ((long)b * NH + k - NH) * E;
    load4<TQ>(src + cbase + 4 * li, bq[t]);
  }
  const bf16* Mb = mem + (long)b * S * E + cbase + 4 * li;
  bf16* dMb = dmem + (long)b * S * E + cbase + 16 * g;
  f32x4 acc1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc1[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per 16-row tile: M rows jb + 4 t + g (t < 4) as 8-B loads; the old dM row jb + li as two 16-B loads
  auto load_tile = [&](int jb, bf16x4 (&m)[4], bf16x8 (&o)[2]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) m[t] = *(const bf16x4*)(Mb + (long)min(jb + 4 * t + g, S - 1) * E);
    if (beta != 0.f) {
      const bf16* src = dMb + (long)min(jb + li, S - 1) * E;
      o[0] = *(const bf16x8*)src;
      o[1] = *(const bf16x8*)(src + 8);
    }
  };
  bf16x4 mc[4], mn[4];
  bf16x8 oc[2], on[2];
  load_tile(0, mc, oc);
  for (int jb = 0; jb < Spad; jb += 16) {
    if (jb + 16 < Spad) load_tile(jb + 16, mn, on);
    // dq': k = rows jb + 4 t + g, n = head li
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float dv = li < NH ? a2[(jb + 4 * t + g) * A2LD + NH + li] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc1[q] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)mc[t][q], dv, acc1[q], 0, 0, 0);
    }
    // dM: k = g + 4 t, n = row jb + li
    f32x4 acc2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc2[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      const float av = a2[(jb + li) * A2LD + g + 4 * t];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc2[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(bq[t][q], av, acc2[q], 0, 0, 0);
    }
    // acc2[q][r] = dM[jb + li][cbase + 16 g + 4 r + q]
    if (jb + li < S) {
      bf16x8 v[2];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float x = acc2[q][r];
          if (beta != 0.f) x += beta * (float)oc[r >> 1][4 * (r & 1) + q];
          v[r >> 1][4 * (r & 1) + q] = (bf16)x;
        }
      bf16* dst = dMb + (long)(jb + li) * E;
      *(bf16x8*)dst = v[0];
      *(bf16x8*)(dst + 8) = v[1];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) mc[t] = mn[t];
    oc[0] = on[0];
    oc[1] = on[1];
  }
  // acc1[q][r] = dq'[h = li][cbase + 16 g + 4 r + q]
  if (li < NH) {
    TQ* dst = dqp + ((long)b * NH + li) * E + cbase + 16 * g;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = acc1[q][r];
      store4<TQ>(dst + 4 * r, v);
    }
  }
}

// x[b, c] += bias[c] * s[b, c / group]   (the s_h bv_h term of the dropped-out context)
__global__ void __launch_bounds__(256) head_bias_fwd_kernel(int B, int W, int group, float* __restrict__ x,
                                                            const float* __restrict__ bias, const float* __restrict__ s) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * W) return;
  const int b = (int)(i / W), c = (int)(i % W);
  x[i] += bias[c] * s[(long)b * (W / group) + c / group];
}
// ds[b, g] = sum_{c in g} dx[b,c] bias[c]: grid B, 256 threads (thread t: columns t, t+256, t+512;
// wave w reduces heads w, w+4, w+8).
__global__ void __launch_bounds__(256) head_bias_ds_kernel(int W, const float* __restrict__ dx,
                                                           const float* __restrict__ bias, float* __restrict__ ds) {
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int k = 0; k < W / 256; ++k) {
    const int c = t + 256 * k;
    const float v = wave_sum(dx[(long)b * W + c] * bias[c]);
    if (lane == 0) ds[(long)b * (W / 64) + 4 * k + wave] = v;
  }
}
// dbias[c] = beta*dbias[c] + sum_b dx[b,c] s[b, c/64]: grid W/64, 256 threads (wave w: rows w, w+4, ..).
__global__ void __launch_bounds__(256) head_bias_db_kernel(int B, int W, const float* __restrict__ dx,
                                                           const float* __restrict__ s, float* __restrict__ dbias,
                                                           float beta) {
  __shared__ float red[4][64];
  const int g = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = g * 64 + lane;
  float acc = 0.f;
#pragma unroll 8
  for (int b = wave; b < B; b += 4) acc += dx[(long)b * W + c] * s[(long)b * (W / 64) + g];
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    const float v = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    dbias[c] = v + (beta != 0.f ? beta * dbias[c] : 0.f);
  }
}

template <typename T, typename TQ>
int xfwd(int B, int S, const void* mem, const void* qp, const float* kb, float p, uint64_t seed, uint64_t off,
         float* ws, float* probs, float* psum, void* ctx, hipStream_t st) {
  launch_xrow_dot<T, TQ>((const T*)mem, (const TQ*)qp, kb, B, S, ws, st);
  if constexpr (sizeof(T) == 2) {
    if (g_xbwd_mfma) {
      const size_t lds = sizeof(float) * (size_t)((S + 15) & ~15) * NH;
      hipFuncSetAttribute((const void*)xctx_mfma_kernel<TQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      EEGF_LAUNCH((xctx_mfma_kernel<TQ>), dim3(E / SLAB, B), dim3(256), lds, st, (const bf16*)mem, ws, S, p,
                         seed, off, probs, psum, (TQ*)ctx);
      return (int)hipGetLastError();
    }
  }
  const size_t lds = sizeof(float) * ((size_t)S * NH + 4 * NH * SLAB);
  hipFuncSetAttribute((const void*)xctx_kernel<T, TQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  EEGF_LAUNCH((xctx_kernel<T, TQ>), dim3(E / SLAB, B), dim3(512), lds, st, (const T*)mem, ws, S, p, seed, off,
                     probs, psum, (TQ*)ctx);
  return (int)hipGetLastError();
}
template <typename T, typename TQ>
int xbwd(int B, int S, const void* mem, const void* qp, const float* probs, const float* dpsum, const void* dctx,
         float p, uint64_t seed, uint64_t off, float* ws, void* dmem, float beta, void* dqp, hipStream_t st) {
  launch_xrow_dot<T, TQ>((const T*)mem, (const TQ*)dctx, (const float*)nullptr, B, S, ws, st);
  if constexpr (sizeof(T) == 2) {
    if (g_xbwd_mfma) {
      const size_t lds = sizeof(float) * (size_t)((S + 15) & ~15) * A2LD;
      hipFuncSetAttribute((const void*)xbwd_mfma_kernel<TQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      EEGF_LAUNCH((xbwd_mfma_kernel<TQ>), dim3(E / SLAB, B), dim3(256), lds, st, (const bf16*)mem,
                         (const TQ*)qp, probs, ws, dpsum, (const TQ*)dctx, S, p, seed, off, (bf16*)dmem, beta, (TQ*)dqp);
      return (int)hipGetLastError();
    }
  }
  const size_t lds = sizeof(float) * ((size_t)2 * S * NH + 4 * NH * SLAB);
  hipFuncSetAttribute((const void*)xbwd_cols_kernel<T, TQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  EEGF_LAUNCH((xbwd_cols_kernel<T, TQ>), dim3(E / SLAB, B), dim3(512), lds, st, (const T*)mem, (const TQ*)qp,
                     probs, ws, dpsum, (const TQ*)dctx, S, p, seed, off, (T*)dmem, beta, (TQ*)dqp);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int eegf_xattn_fwd(int mem_dtype, int q_dtype, int B, int S, const void* mem, const void* qp,
                              const float* key_bias, float drop_p, unsigned long long seed, unsigned long long offset,
                              float* ws, float* probs, float* psum, void* ctx, hipStream_t stream) {
  if (B <= 0 || B > 65535 || S <= 0 || S > 1024 || !mem || !qp || !ws || !probs || !ctx) return EEGF_ERR_ARG;
  if (drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && !psum)) return EEGF_ERR_ARG;
  if (mem_dtype == EEGF_F32 && q_dtype == EEGF_F32)
    return xfwd<float, float>(B, S, mem, qp, key_bias, drop_p, seed, offset, ws, probs, psum, ctx, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_BF16)
    return xfwd<bf16, bf16>(B, S, mem, qp, key_bias, drop_p, seed, offset, ws, probs, psum, ctx, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_F32)
    return xfwd<bf16, float>(B, S, mem, qp, key_bias, drop_p, seed, offset, ws, probs, psum, ctx, stream);
  return EEGF_ERR_ARG;
}

extern "C" int eegf_xattn_bwd(int mem_dtype, int q_dtype, int B, int S, const void* mem, const void* qp,
                              const float* probs, const float* dpsum, const void* dctx, float drop_p,
                              unsigned long long seed, unsigned long long offset, float* ws, void* dmem, float beta,
                              void* dqp, hipStream_t stream) {
  if (B <= 0 || B > 65535 || S <= 0 || S > 1024 || !mem || !qp || !probs || !dctx || !ws || !dmem || !dqp)
    return EEGF_ERR_ARG;
  if (drop_p < 0.f || drop_p >= 1.f) return EEGF_ERR_ARG;
  if (mem_dtype == EEGF_F32 && q_dtype == EEGF_F32)
    return xbwd<float, float>(B, S, mem, qp, probs, dpsum, dctx, drop_p, seed, offset, ws, dmem, beta, dqp, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_BF16)
    return xbwd<bf16, bf16>(B, S, mem, qp, probs, dpsum, dctx, drop_p, seed, offset, ws, dmem, beta, dqp, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_F32)
    return xbwd<bf16, float>(B, S, mem, qp, probs, dpsum, dctx, drop_p, seed, offset, ws, dmem, beta, dqp, stream);
  return EEGF_ERR_ARG;
}

extern "C" int eegf_head_bias_fwd(int B, int W, int group, float* x, const float* bias, const float* s,
                                  hipStream_t stream) {
  if (B <= 0 || W <= 0 || group <= 0 || W % group != 0 || !x || !bias || !s) return EEGF_ERR_ARG;
  const long n = (long)B * W;
  EEGF_LAUNCH(head_bias_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, B, W, group, x,
                     bias, s);
  return (int)hipGetLastError();
}

extern "C" int eegf_head_bias_bwd(int B, int W, int group, const float* dx, const float* bias, const float* s,
                                  float* ds, float* dbias, float beta, hipStream_t stream) {
  if (B <= 0 || W <= 0 || group != 64 || W % 256 != 0 || !dx || !bias || !s || !ds) return EEGF_ERR_ARG;
  EEGF_LAUNCH(head_bias_ds_kernel, dim3(B), dim3(256), 0, stream, W, dx, bias, ds);
  if (dbias) EEGF_LAUNCH(head_bias_db_kernel, dim3(W / 64), dim3(256), 0, stream, B, W, dx, s, dbias, beta);
  return (int)hipGetLastError();
}
