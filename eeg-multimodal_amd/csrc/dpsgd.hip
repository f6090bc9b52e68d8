// dpsgd.hip — per-sample gradient clipping and Gaussian noise for DP-SGD (opacus
// make_private_with_epsilon as used by main_0430.py:143-162 and base_train.py:322-348), without
// materialising per-sample gradients.
//
// opacus computes grad_sample[b] for every trainable parameter (GradSampleModule hooks), the
// per-sample norm n_b = || (grad_sample_p[b])_p ||_2 over all trainable parameters, the clip factor
// c_b = min(1, C / (n_b + 1e-6)), the clipped sum sum_b c_b grad_sample[b] plus N(0, (sigma C)^2)
// noise, divided by the expected batch size (DPOptimizer pre_step).  Here:
//   * n_b^2 is accumulated site by site straight from the backward's operands:
//       - token-sequence Linear (BERT layer: T rows per sample): ||DY_b^T X_b||_F^2
//         = sum_{t,u} (x_t . x_u)(dy_t . dy_u) ("ghost norm": the two T x T Gram matrices of the
//         sample on the MFMA, 64 x 64 tile by tile, multiplied and reduced in registers) — eegf_ghost_norm;
//       - its bias: ||sum_t dy_t||^2; LayerNorm gamma / beta: ||sum_t dy_t * xhat_t||^2 + ||sum_t dy_t||^2
//         (xhat rebuilt from the saved pre-LN sum, mean, rstd) — eegf_seg_sqnorm;
//       - one-row-per-sample Linear (head, pooler, visual encoder): ||dy_b||^2 ||x_b||^2 (+ ||dy_b||^2
//         for the bias) — eegf_row_sqnorm;
//   * every per-sample gradient is linear in that sample's logit gradient, so the clipped sum is a
//     second backward with the logit-gradient rows scaled by c_b (eegf_dp_clip_rows);
//   * eegf_dp_noise adds the Gaussian noise (Philox4x32-10 + Box-Muller) and the 1/expected-batch
//     scale in one pass over a gradient range.
// All reductions run in a fixed order (deterministic).
#include "common.h"
#include "eegfusion_internal.h"

namespace {

// ---------------------------------------------------------------- ghost norm (MFMA Gram tiles)
// grid (S, ntiles): workgroup (s, t) takes upper-triangle tile t = (i, j), i <= j, of the sample's
// T/64 x T/64 block grid; 4 waves, wave w owns rows 16w..16w+15 of the 64 x 64 tile, 4 16-column
// blocks.  Fragments come straight from global memory (the sample's rows are L2-resident across the
// 10-36 tiles).  Writes part[s * ntiles + t] = weight * sum(Gx o Gy), weight 2 off the diagonal.
template <typename T>
__global__ void __launch_bounds__(256) ghost_norm_kernel(int Tn, int Dx, int Dy, const T* __restrict__ X, long ldx,
                                                         const T* __restrict__ DY, long ldy, float* __restrict__ part) {
  __shared__ float red[4];
  const int s = blockIdx.x, tile = blockIdx.y, ntiles = gridDim.y;
  const int nb = Tn / 64;
  int i = 0, j = 0, k = tile;                      // tile -> (i, j), row-major upper triangle
  while (k >= nb - i) { k -= nb - i; ++i; }
  j = i + k;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long r0 = (long)s * Tn + i * 64 + wave * 16 + (lane & 15);     // this lane's A row
  const long c0 = (long)s * Tn + j * 64 + (lane & 15);                 // B row of column block 0
  const int kk = 8 * (lane >> 4);
  float acc = 0.f;
  f32x4 gx[4], gy[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) gx[c] = gy[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < Dx; k0 += 32) {
    const auto a = ld_row8(X + r0 * ldx + k0 + kk);
#pragma unroll
    for (int c = 0; c < 4; ++c) gx[c] = mma16(a, ld_row8(X + (c0 + 16 * c) * ldx + k0 + kk), gx[c]);
  }
  for (int k0 = 0; k0 < Dy; k0 += 32) {
    const auto a = ld_row8(DY + r0 * ldy + k0 + kk);
#pragma unroll
    for (int c = 0; c < 4; ++c) gy[c] = mma16(a, ld_row8(DY + (c0 + 16 * c) * ldy + k0 + kk), gy[c]);
  }
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc += gx[c][r] * gy[c][r];
  acc = wave_sum(acc);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long)s * ntiles + tile] = (i == j ? 1.f : 2.f) * (((red[0] + red[1]) + red[2]) + red[3]);
}

// out[s] = beta * out[s] + sum_t part[s * n + t]   (fixed order)
__global__ void __launch_bounds__(256) rowsum_kernel(int S, int n, const float* __restrict__ part, float beta,
                                                     float* __restrict__ out) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= S) return;
  float v = 0.f;
  for (int t = 0; t < n; ++t) v += part[(long)s * n + t];
  out[s] = (beta != 0.f ? beta * out[s] : 0.f) + v;
}

// ------------------------------------------------------------- per-sample column-sum norms
// One workgroup per sample (rows s*T .. s*T+T-1): per column c, a_c = sum_t dy[t, c] (bias / LN beta);
// with LayerNorm stats (xs, mean, rstd non-null) also g_c = sum_t dy[t, c] * (xs[t, c] - mean[t]) rstd[t]
// (LN gamma).  out[s] = beta * out[s] + sum_c a_c^2 (+ g_c^2).
template <typename T>
__global__ void __launch_bounds__(256) seg_sqnorm_kernel(int Tn, int W, const T* __restrict__ dy, long ldd,
                                                         const T* __restrict__ xs, long ldx, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, int bias_term, float beta,
                                                         float* __restrict__ out) {
  __shared__ float red[4];
  const int s = blockIdx.x;
  const long row0 = (long)s * Tn;
  float v = 0.f;
  for (int c = threadIdx.x; c < W; c += 256) {
    float a = 0.f, g = 0.f;
    for (int t = 0; t < Tn; ++t) {
      const float d = to_f32(dy[(row0 + t) * ldd + c]);
      a += d;
      if (xs) g += d * (to_f32(xs[(row0 + t) * ldx + c]) - mean[row0 + t]) * rstd[row0 + t];
    }
    v += (bias_term ? a * a : 0.f) + g * g;
  }
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float tot = ((red[0] + red[1]) + red[2]) + red[3];
    out[s] = (beta != 0.f ? beta * out[s] : 0.f) + tot;
  }
}

// ------------------------------------------------------------------ one-row-per-sample Linear
// One wave per sample: out[s] += ||a_s||^2 * (b ? ||b_s||^2 : 1)
template <typename T>
__global__ void __launch_bounds__(256) row_sqnorm_kernel(int S, int Wa, const T* __restrict__ a, long lda, int Wb,
                                                         const T* __restrict__ b, long ldb, float* __restrict__ out) {
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (s >= S) return;
  float na = 0.f, nb = 0.f;
  for (int c = lane; c < Wa; c += 64) { const float x = to_f32(a[(long)s * lda + c]); na += x * x; }
  if (b)
    for (int c = lane; c < Wb; c += 64) { const float x = to_f32(b[(long)s * ldb + c]); nb += x * x; }
  na = wave_sum(na);
  nb = wave_sum(nb);
  if (lane == 0) out[s] += na * (b ? nb : 1.f);
}

// ------------------------------------------------------------------------------ clip factors
// c_s = min(1, C / (sqrt(psn_s) + 1e-6)) (opacus clip_and_accumulate); dl[s, :] *= c_s; clip[s] = c_s
__global__ void __launch_bounds__(256) clip_rows_kernel(int S, int ncls, const float* __restrict__ psn, float max_norm,
                                                        float* __restrict__ dl, float* __restrict__ clip) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= S) return;
  const float c = fminf(max_norm / (sqrtf(psn[s]) + 1e-6f), 1.0f);
  for (int k = 0; k < ncls; ++k) dl[(long)s * ncls + k] *= c;
  if (clip) clip[s] = c;
}

// ------------------------------------------------------------------------------ Gaussian noise
// g[i] = (g[i] + std * z_i) * scale; z_i standard normal from Philox4x32-10(counter i >> 2, offset;
// seed): words (x, y) -> Box-Muller pair for elements 4c, 4c+1; (z, w) -> 4c+2, 4c+3
__global__ void __launch_bounds__(256) dp_noise_kernel(long n, float* __restrict__ g, float std, float scale,
                                                       uint64_t seed, uint64_t offset) {
  const long c = (long)blockIdx.x * 256 + threadIdx.x;
  if (c * 4 >= n) return;
  const u32x4s r = philox4x32((uint32_t)c, (uint32_t)(c >> 32), (uint32_t)offset, (uint32_t)(offset >> 32),
                              (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  float z[4];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float u1 = u01_open0(w[2 * p]);                       // (0, 1]: log finite
    const float u2 = (float)(w[2 * p + 1] >> 8) * (1.0f / 16777216.0f);
    const float rad = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincosf(6.283185307179586f * u2, &sn, &cs);
    z[2 * p] = rad * cs;
    z[2 * p + 1] = rad * sn;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long i = c * 4 + k;
    if (i < n) g[i] = (g[i] + std * z[k]) * scale;
  }
}

}  // namespace

extern "C" long eegf_ghost_norm_workspace(int S, int T) {
  if (S <= 0 || T <= 0 || T % 64) return 0;
  const long nb = T / 64;
  return (long)S * (nb * (nb + 1) / 2);
}

extern "C" int eegf_ghost_norm(int dtype, int S, int T, int Dx, int Dy, const void* X, long ldx, const void* DY,
                               long ldy, float* ws, long ws_elems, float beta, float* out, hipStream_t stream) {
  if (S <= 0 || T <= 0 || T % 64 || Dx <= 0 || Dy <= 0 || Dx % 32 || Dy % 32 || !X || !DY || !ws || !out)
    return EEGF_ERR_ARG;
  if (ldx % 8 || ldy % 8 || ((uintptr_t)X | (uintptr_t)DY) & 15) return EEGF_ERR_ARG;
  const int nb = T / 64, ntiles = nb * (nb + 1) / 2;
  if (ws_elems < (long)S * ntiles) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)S, (unsigned)ntiles);
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(ghost_norm_kernel<float>, grid, dim3(256), 0, stream, T, Dx, Dy, (const float*)X, ldx,
                       (const float*)DY, ldy, ws);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(ghost_norm_kernel<bf16>, grid, dim3(256), 0, stream, T, Dx, Dy, (const bf16*)X, ldx,
                       (const bf16*)DY, ldy, ws);
  else return EEGF_ERR_ARG;
  EEGF_LAUNCH(rowsum_kernel, dim3((S + 255) / 256), dim3(256), 0, stream, S, ntiles, (const float*)ws, beta, out);
  return (int)hipGetLastError();
}

extern "C" int eegf_seg_sqnorm(int dtype, int S, int T, int W, const void* dy, long ldd, const void* xs, long ldx,
                               const float* mean, const float* rstd, int bias_term, float beta, float* out,
                               hipStream_t stream) {
  if (S <= 0 || T <= 0 || W <= 0 || !dy || !out) return EEGF_ERR_ARG;
  if (xs && (!mean || !rstd)) return EEGF_ERR_ARG;
  if (!xs && !bias_term) return EEGF_ERR_ARG;
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(seg_sqnorm_kernel<float>, dim3(S), dim3(256), 0, stream, T, W, (const float*)dy, ldd,
                       (const float*)xs, ldx, mean, rstd, bias_term, beta, out);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(seg_sqnorm_kernel<bf16>, dim3(S), dim3(256), 0, stream, T, W, (const bf16*)dy, ldd,
                       (const bf16*)xs, ldx, mean, rstd, bias_term, beta, out);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_row_sqnorm(int dtype, int S, int Wa, const void* a, long lda, int Wb, const void* b, long ldb,
                               float* out, hipStream_t stream) {
  if (S <= 0 || Wa <= 0 || !a || !out || (b && Wb <= 0)) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((S + 3) / 4));
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(row_sqnorm_kernel<float>, grid, dim3(256), 0, stream, S, Wa, (const float*)a, lda, Wb,
                       (const float*)b, ldb, out);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(row_sqnorm_kernel<bf16>, grid, dim3(256), 0, stream, S, Wa, (const bf16*)a, lda, Wb,
                       (const bf16*)b, ldb, out);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_dp_clip_rows(int S, int ncls, const float* psn, float max_norm, float* dlogits, float* clip,
                                 hipStream_t stream) {
  if (S <= 0 || ncls <= 0 || !psn || !dlogits || !(max_norm > 0.f)) return EEGF_ERR_ARG;
  EEGF_LAUNCH(clip_rows_kernel, dim3((S + 255) / 256), dim3(256), 0, stream, S, ncls, psn, max_norm, dlogits, clip);
  return (int)hipGetLastError();
}

extern "C" int eegf_dp_noise(long n, float* grad, float std, float scale, unsigned long long seed,
                             unsigned long long offset, hipStream_t stream) {
  if (n <= 0 || !grad || std < 0.f) return EEGF_ERR_ARG;
  const long calls = (n + 3) / 4;
  EEGF_LAUNCH(dp_noise_kernel, dim3((unsigned)((calls + 255) / 256)), dim3(256), 0, stream, n, grad, std, scale,
                     seed, offset);
  return (int)hipGetLastError();
}
