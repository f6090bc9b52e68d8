// embed.hip — EEG input front-ends.
//
// Contract W (synthetic windows, BASELINE configs 2-5): the EEG window arrives channel x time
// [B, C, T] fp32; the per-time-step token encoder needs time-major rows [B*T, C].  One workgroup
// per (b, 64-step tile) reads the tile coalesced along time into LDS and writes it coalesced along
// channels (cast to the compute dtype) — the input of the eeg_encoder GEMM.
// Contract T (token ids, model.py / train.py): word-embedding gather feeding BertEmbeddings
// (modeling_bert.py:95-105) and its scatter-add backward.
#include "common.h"
#include "eegfusion_internal.h"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) window_tokens_kernel(const float* __restrict__ eeg, int C, int Tn,
                                                            T* __restrict__ tokens) {
  __shared__ float tile[128][65];
  const int b = blockIdx.y, t0 = blockIdx.x * 64, tid = threadIdx.x;
  const float* src = eeg + (long)b * C * Tn;
  for (int i = tid; i < C * 64; i += 256) {
    const int c = i / 64, t = i % 64;
    tile[c][t] = (t0 + t < Tn) ? src[(long)c * Tn + t0 + t] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < C * 64; i += 256) {
    const int t = i / C, c = i % C;
    if (t0 + t < Tn) tokens[((long)b * Tn + t0 + t) * C + c] = from_f32<T>(tile[c][t]);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gather_kernel(const long long* __restrict__ ids, const float* __restrict__ table,
                                                     int width, long rows, T* __restrict__ out) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* src = table + ids[row] * width;
  for (int c = threadIdx.x & 63; c < width; c += 64) out[row * width + c] = from_f32<T>(src[c]);
}

template <typename T>
__global__ void __launch_bounds__(256) scatter_add_kernel(const long long* __restrict__ ids, const T* __restrict__ d,
                                                          int width, long rows, float* __restrict__ table_grad) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  float* dst = table_grad + ids[row] * width;
  for (int c = threadIdx.x & 63; c < width; c += 64) atomicAdd(dst + c, to_f32(d[row * width + c]));
}

}  // namespace

extern "C" int eegf_window_tokens(int dtype, int B, int C, int T, const float* eeg, void* tokens, hipStream_t stream) {
  if (B <= 0 || C <= 0 || C > 128 || T <= 0 || !eeg || !tokens || B > 65535) return EEGF_ERR_ARG;
  const dim3 grid((T + 63) / 64, B);
  if (dtype == EEGF_F32) hipLaunchKernelGGL(window_tokens_kernel<float>, grid, dim3(256), 0, stream, eeg, C, T, (float*)tokens);
  else if (dtype == EEGF_BF16) hipLaunchKernelGGL(window_tokens_kernel<bf16>, grid, dim3(256), 0, stream, eeg, C, T, (bf16*)tokens);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_embed_gather(int dtype, long rows, int width, const long long* ids, const float* table, void* out,
                                 hipStream_t stream) {
  if (rows <= 0 || width <= 0 || !ids || !table || !out) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == EEGF_F32) hipLaunchKernelGGL(gather_kernel<float>, grid, dim3(256), 0, stream, ids, table, width, rows, (float*)out);
  else if (dtype == EEGF_BF16) hipLaunchKernelGGL(gather_kernel<bf16>, grid, dim3(256), 0, stream, ids, table, width, rows, (bf16*)out);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_embed_scatter_add(int dtype, long rows, int width, const long long* ids, const void* d,
                                      float* table_grad, hipStream_t stream) {
  if (rows <= 0 || width <= 0 || !ids || !d || !table_grad) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == EEGF_F32)
    hipLaunchKernelGGL(scatter_add_kernel<float>, grid, dim3(256), 0, stream, ids, (const float*)d, width, rows, table_grad);
  else if (dtype == EEGF_BF16)
    hipLaunchKernelGGL(scatter_add_kernel<bf16>, grid, dim3(256), 0, stream, ids, (const bf16*)d, width, rows, table_grad);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}
