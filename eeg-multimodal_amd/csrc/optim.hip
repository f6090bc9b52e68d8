// optim.hip — fused Adam over a flat parameter arena, casts and small elementwise helpers.
//
// Replaces torch.optim.Adam(params, lr) (past_acc.py:159-160, train.py:77, base_train.py:170-171):
// one launch updates a contiguous range of the fp32 master arena (the two reference optimizers
// own disjoint ranges: model params and DP), and optionally refreshes the bf16 compute shadow
// of the same range in the same pass (no separate cast kernel on the hot path).  grad_scale folds the
// data-parallel 1/N average into the read of the all-reduced gradient sum (no separate scaling pass
// over the gradient arena; g * (1/N) in fp32 is the product torch's mul_ would store).
// Arithmetic follows torch's single-tensor Adam (torch/optim/adam.py _single_tensor_adam):
//   g = grad_scale*g + wd*p; m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g^2;
//   p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)     (m via lerp, as torch)
#include "common.h"
#include "eegfusion_internal.h"

namespace {

// ZERO (eegf_adam_consume): the gradient is written back as 0 once read, so the trainer's next backward
// accumulates into a clean arena without a separate fill pass over it (4 B more per parameter here
// instead of a 4-B-per-parameter memset launch: 148 M elements, 75 us per step)
template <bool ZERO>
__global__ void __launch_bounds__(256) adam_kernel(long n, float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16* __restrict__ shadow, float b1, float b2, float eps, float wd,
                                                   float gscale, float step_size, float sqrt_bc2) {
  const long i4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (i4 + 4 <= n) {
    f32x4 pv = *(const f32x4*)(p + i4), gv = *(const f32x4*)(g + i4);
    f32x4 mv = *(const f32x4*)(m + i4), vv = *(const f32x4*)(v + i4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float gr = gv[e] * gscale;
      if (wd != 0.f) gr += wd * pv[e];
      mv[e] = mv[e] + (1.f - b1) * (gr - mv[e]);              // exp_avg.lerp_(grad, 1-beta1)
      vv[e] = b2 * vv[e] + (1.f - b2) * gr * gr;
      const float denom = sqrtf(vv[e]) / sqrt_bc2 + eps;
      pv[e] = pv[e] - step_size * (mv[e] / denom);
    }
    *(f32x4*)(p + i4) = pv;
    *(f32x4*)(m + i4) = mv;
    *(f32x4*)(v + i4) = vv;
    if (ZERO) *(f32x4*)(g + i4) = f32x4{0.f, 0.f, 0.f, 0.f};
    if (shadow) {
      bf16x4 s;
      s[0] = (bf16)pv[0]; s[1] = (bf16)pv[1]; s[2] = (bf16)pv[2]; s[3] = (bf16)pv[3];
      *(bf16x4*)(shadow + i4) = s;
    }
  } else {
    for (long i = i4; i < n; ++i) {
      float gr = g[i] * gscale;
      if (wd != 0.f) gr += wd * p[i];
      m[i] = m[i] + (1.f - b1) * (gr - m[i]);
      v[i] = b2 * v[i] + (1.f - b2) * gr * gr;
      p[i] = p[i] - step_size * (m[i] / (sqrtf(v[i]) / sqrt_bc2 + eps));
      if (shadow) shadow[i] = (bf16)p[i];
      if (ZERO) g[i] = 0.f;
    }
  }
}

__global__ void __launch_bounds__(256) cast_kernel(long n, const float* __restrict__ src, bf16* __restrict__ dst) {
  const long i4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 + 4 <= n) {
    const f32x4 x = *(const f32x4*)(src + i4);
    bf16x4 s;
    s[0] = (bf16)x[0]; s[1] = (bf16)x[1]; s[2] = (bf16)x[2]; s[3] = (bf16)x[3];
    *(bf16x4*)(dst + i4) = s;
  } else {
    for (long i = i4; i < n; ++i) dst[i] = (bf16)src[i];
  }
}

__global__ void __launch_bounds__(256) key_bias_kernel(long n, const long long* __restrict__ mask, float* __restrict__ bias) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) bias[i] = mask[i] == 0 ? -1e30f : 0.f;
}

}  // namespace

namespace {
template <bool ZERO>
int adam_launch(long n, float* p, float* g, float* m, float* v, void* bf16_shadow, float lr, float beta1, float beta2,
                float eps, float weight_decay, float grad_scale, int step, hipStream_t stream) {
  if (n <= 0 || !p || !g || !m || !v || step <= 0) return EEGF_ERR_ARG;
  if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) != 0) return EEGF_ERR_ARG;
  if (bf16_shadow && ((uintptr_t)bf16_shadow & 7) != 0) return EEGF_ERR_ARG;
  const double bc1 = 1.0 - pow((double)beta1, step), bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)(lr / bc1), sqrt_bc2 = (float)sqrt(bc2);
  const long blocks = (n + 1023) / 1024;
  EEGF_LAUNCH(adam_kernel<ZERO>, dim3((unsigned)blocks), dim3(256), 0, stream, n, p, g, m, v, (bf16*)bf16_shadow,
              beta1, beta2, eps, weight_decay, grad_scale, step_size, sqrt_bc2);
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int eegf_adam(long n, float* p, const float* g, float* m, float* v, void* bf16_shadow, float lr, float beta1,
                         float beta2, float eps, float weight_decay, float grad_scale, int step, hipStream_t stream) {
  return adam_launch<false>(n, p, const_cast<float*>(g), m, v, bf16_shadow, lr, beta1, beta2, eps, weight_decay,
                            grad_scale, step, stream);
}

extern "C" int eegf_adam_consume(long n, float* p, float* g, float* m, float* v, void* bf16_shadow, float lr,
                                 float beta1, float beta2, float eps, float weight_decay, float grad_scale, int step,
                                 hipStream_t stream) {
  return adam_launch<true>(n, p, g, m, v, bf16_shadow, lr, beta1, beta2, eps, weight_decay, grad_scale, step, stream);
}

extern "C" int eegf_cast_f32_bf16(long n, const float* src, void* dst, hipStream_t stream) {
  if (n <= 0 || !src || !dst) return EEGF_ERR_ARG;
  if ((((uintptr_t)src) & 15) != 0 || (((uintptr_t)dst) & 7) != 0) return EEGF_ERR_ARG;
  EEGF_LAUNCH(cast_kernel, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, stream, n, src, (bf16*)dst);
  return (int)hipGetLastError();
}

extern "C" int eegf_key_bias(long n, const long long* mask, float* bias, hipStream_t stream) {
  if (n <= 0 || !mask || !bias) return EEGF_ERR_ARG;
  EEGF_LAUNCH(key_bias_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, n, mask, bias);
  return (int)hipGetLastError();
}
