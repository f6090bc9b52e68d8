// elementwise.hip — small bandwidth-bound helpers between the fused kernels.
//   eegf_axpby:    y = alpha*x + beta*y          (gradient sums where two paths meet)
//   eegf_tanh_bwd: dx = dy * (1 - y^2)           (BertPooler tanh, modeling_bert.py:457-462)
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

}  // namespace

extern "C" int eegf_axpby(int dtype, long n, float alpha, const void* x, float beta, void* y, hipStream_t stream) {
  if (n <= 0 || !x || !y) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == EEGF_F32) hipLaunchKernelGGL(axpby_kernel<float>, grid, dim3(256), 0, stream, n, alpha, (const float*)x, beta, (float*)y);
  else if (dtype == EEGF_BF16) hipLaunchKernelGGL(axpby_kernel<bf16>, grid, dim3(256), 0, stream, n, alpha, (const bf16*)x, beta, (bf16*)y);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_tanh_bwd(int dtype, long n, const void* dy, const void* y, void* dx, hipStream_t stream) {
  if (n <= 0 || !dy || !y || !dx) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == EEGF_F32) hipLaunchKernelGGL(tanh_bwd_kernel<float>, grid, dim3(256), 0, stream, n, (const float*)dy, (const float*)y, (float*)dx);
  else if (dtype == EEGF_BF16) hipLaunchKernelGGL(tanh_bwd_kernel<bf16>, grid, dim3(256), 0, stream, n, (const bf16*)dy, (const bf16*)y, (bf16*)dx);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}
