// elementwise.hip — small bandwidth-bound helpers between the fused kernels.
//   eegf_axpby:    y = alpha*x + beta*y          (gradient sums where two paths meet)
//   eegf_tanh_bwd: dx = dy * (1 - y^2)           (BertPooler tanh, modeling_bert.py:457-462)
//   eegf_dropout:  x[i] *= mask(i / group)        (in place; group 1 = elementwise dropout, e.g. the
//                  decoder FFN's inner dropout transformer.py:1197-1199; group 64 = one draw per head, the
//                  decoder self-attention's dropout of its single attention weight transformer.py:1158-1176)
#include "common.h"
#include "eegfusion_internal.h"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) axpby_kernel(long n, float alpha, const T* __restrict__ x, float beta, T* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = from_f32<T>(alpha * to_f32(x[i]) + (beta != 0.f ? beta * to_f32(y[i]) : 0.f));
}

template <typename T>
__global__ void __launch_bounds__(256) tanh_bwd_kernel(long n, const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) { const float t = to_f32(y[i]); dx[i] = from_f32<T>(to_f32(dy[i]) * (1.f - t * t)); }
}

template <typename T>
__global__ void __launch_bounds__(256) dropout_kernel(long n, int group, float p, uint64_t seed, uint64_t offset,
                                                      T* __restrict__ x) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = from_f32<T>(to_f32(x[i]) * drop_mask1(seed, offset, (uint64_t)(i / group), p));
}

}  // namespace

extern "C" int eegf_axpby(int dtype, long n, float alpha, const void* x, float beta, void* y, hipStream_t stream) {
  if (n <= 0 || !x || !y) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == EEGF_F32) EEGF_LAUNCH(axpby_kernel<float>, grid, dim3(256), 0, stream, n, alpha, (const float*)x, beta, (float*)y);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(axpby_kernel<bf16>, grid, dim3(256), 0, stream, n, alpha, (const bf16*)x, beta, (bf16*)y);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_tanh_bwd(int dtype, long n, const void* dy, const void* y, void* dx, hipStream_t stream) {
  if (n <= 0 || !dy || !y || !dx) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == EEGF_F32) EEGF_LAUNCH(tanh_bwd_kernel<float>, grid, dim3(256), 0, stream, n, (const float*)dy, (const float*)y, (float*)dx);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(tanh_bwd_kernel<bf16>, grid, dim3(256), 0, stream, n, (const bf16*)dy, (const bf16*)y, (bf16*)dx);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_dropout(int dtype, long n, int group, float p, unsigned long long seed, unsigned long long offset,
                            void* x, hipStream_t stream) {
  if (n <= 0 || group <= 0 || p < 0.f || p >= 1.f || !x) return EEGF_ERR_ARG;
  if (p == 0.f) return 0;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == EEGF_F32) EEGF_LAUNCH(dropout_kernel<float>, grid, dim3(256), 0, stream, n, group, p, seed, offset, (float*)x);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(dropout_kernel<bf16>, grid, dim3(256), 0, stream, n, group, p, seed, offset, (bf16*)x);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

// Mean over the L rows of each sequence (TTCA's decoder output .mean(dim=1), TISC's
// eeg_txt_semantics_embedding.mean(dim=1) and its encoder's .mean(dim=0): custom_models/models.py:109,
// :253, :260): out[b] (fp32, row stride ld_out) = (1/L) sum_l x[b*L + l] (row stride ld_x);
// backward: dx[b*L + l] = beta dx[b*L + l] + dmean[b] / L.  One block per (b, 256-column slab),
// fixed summation order.
namespace {
template <typename T>
__global__ void __launch_bounds__(256) seq_mean_kernel(int L, int width, const T* __restrict__ x, long ldx,
                                                       float* __restrict__ out, long ldo) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= width) return;
  float s = 0.f;
  for (int l = 0; l < L; ++l) s += to_f32(x[((long)b * L + l) * ldx + c]);
  out[(long)b * ldo + c] = s / (float)L;
}
template <typename T>
__global__ void __launch_bounds__(256) seq_mean_bwd_kernel(int L, int width, const float* __restrict__ dmean, long ldm,
                                                           T* __restrict__ dx, long ldx, float beta) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= width) return;
  const float g = dmean[(long)b * ldm + c] / (float)L;
  for (int l = 0; l < L; ++l) {
    T* p = dx + ((long)b * L + l) * ldx + c;
    *p = from_f32<T>(beta != 0.f ? beta * to_f32(*p) + g : g);
  }
}
}  // namespace

extern "C" int eegf_seq_mean(int dtype, int B, int L, int width, const void* x, long ld_x, float* out, long ld_out,
                             hipStream_t stream) {
  if (B <= 0 || B > 65535 || L <= 0 || width <= 0 || !x || !out || ld_x < width || ld_out < width) return EEGF_ERR_ARG;
  const dim3 grid(B, (width + 255) / 256);
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(seq_mean_kernel<float>, grid, dim3(256), 0, stream, L, width, (const float*)x, ld_x, out, ld_out);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(seq_mean_kernel<bf16>, grid, dim3(256), 0, stream, L, width, (const bf16*)x, ld_x, out, ld_out);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_seq_mean_bwd(int dtype, int B, int L, int width, const float* dmean, long ld_dmean, void* dx,
                                 long ld_dx, float beta, hipStream_t stream) {
  if (B <= 0 || B > 65535 || L <= 0 || width <= 0 || !dmean || !dx || ld_dx < width || ld_dmean < width)
    return EEGF_ERR_ARG;
  const dim3 grid(B, (width + 255) / 256);
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(seq_mean_bwd_kernel<float>, grid, dim3(256), 0, stream, L, width, dmean, ld_dmean, (float*)dx,
                       ld_dx, beta);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(seq_mean_bwd_kernel<bf16>, grid, dim3(256), 0, stream, L, width, dmean, ld_dmean, (bf16*)dx,
                       ld_dx, beta);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

// Diagnostics (no reference counterpart): a stand-in for an RCCL all-reduce kernel's use of the CUs,
// for measuring on one GPU whether the gradient all-reduces issued during the backward (trainer.py
// GradReducer) can make progress while the backward's kernels hold the chip.  A fixed grid
// of `wgs` workgroups (RCCL runs one block per channel) walks x[0, n) with a grid-stride loop `passes`
// times, reading and rewriting every element unchanged (x * 1 + 0: the values stay bit-identical).
namespace {
__global__ void __launch_bounds__(256) ring_proxy_kernel(long n4, int passes, float* __restrict__ x) {
  const long stride = (long)gridDim.x * 256;
  for (int p = 0; p < passes; ++p) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
      f32x4 v = ((f32x4*)x)[i];
      // an opaque identity: the compiler may not drop the read-modify-write
      asm volatile("" : "+v"(v));
      ((f32x4*)x)[i] = v;
    }
    __syncthreads();
  }
}
}  // namespace

extern "C" int eegf_ring_proxy(long n, int passes, int wgs, float* x, hipStream_t stream) {
  if (n <= 0 || n % 4 || passes <= 0 || wgs <= 0 || wgs > 4096 || !x || (((uintptr_t)x) & 15)) return EEGF_ERR_ARG;
  EEGF_LAUNCH(ring_proxy_kernel, dim3(wgs), dim3(256), 0, stream, n / 4, passes, x);
  return (int)hipGetLastError();
}
