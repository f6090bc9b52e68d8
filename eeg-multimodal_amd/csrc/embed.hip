// embed.hip — EEG input front-ends.
//
// Contract W (synthetic windows, BASELINE configs 2-5): the EEG window arrives channel x time
// [B, C, T] fp32; the per-time-step token encoder needs time-major rows [B*T, C].  One workgroup
// per (b, 64-step tile) reads the tile coalesced along time into LDS and writes it coalesced along
// channels (cast to the compute dtype) — the input of the eeg_encoder GEMM.
// Contract T (token ids, model.py / train.py): word-embedding gather feeding BertEmbeddings
// (modeling_bert.py:95-105) and its scatter-add backward; the varlen (pad-skipping) front-end: per-row
// lengths of the attention mask, the packed embedding gather (word + position rows of the real
// tokens only) and the padded <-> packed row moves around the BERT stack.
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

// lens[b] = number of nonzero mask entries of row b; *nonprefix |= 1 when a row is not of the form
// [1]*n + [0]*(L-n) (BertTokenizer right padding, get_embedding.py:115): the packed path needs it
__global__ void __launch_bounds__(64) seq_lengths_kernel(const long long* __restrict__ mask, int L, int* lens,
                                                        int* nonprefix) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const long long* m = mask + (long)b * L;
  int n = 0;
  for (int j = lane; j < L; j += 64) n += m[j] != 0;
  n = wave_sum_i(n);
  int bad = 0;
  for (int j = lane; j < L; j += 64) bad |= (m[j] != 0) != (j < n);
  bad = wave_sum_i(bad);
  if (lane == 0) {
    lens[b] = n;
    if (bad) atomicOr(nonprefix, 1);
  }
}

// packed row cu[b] + j (j < len_b) = word[ids[b, j]] + pos[j] (fp32 sum, one rounding to T);
// ids_packed[row] = ids[b, j].  4 rows (b, j) per block, 64 threads per row.
template <typename T>
__global__ void __launch_bounds__(256) varlen_embed_kernel(const int* __restrict__ cu, const long long* __restrict__ ids,
                                                           int L, int width, const float* __restrict__ word,
                                                           const float* __restrict__ pos, T* __restrict__ out,
                                                           long long* __restrict__ ids_packed) {
  const int b = blockIdx.y, j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int len = cu[b + 1] - cu[b];
  if (j >= len || j >= L) return;
  const long row = cu[b] + j;
  const long long id = ids[(long)b * L + j];
  const float* w = word + id * width;
  const float* p = pos + (long)j * width;
  for (int c = threadIdx.x & 63; c < width; c += 64) out[row * width + c] = from_f32<T>(w[c] + p[c]);
  if ((threadIdx.x & 63) == 0) ids_packed[row] = id;
}

// padded [B, S, width] <-> packed rows: to_padded: dst[b*S + j] = j < len_b ? src[cu[b] + j] : 0;
// else dst[cu[b] + j] = src[b*S + j] for j < len_b.  16-B chunks, 4 rows per block.
__global__ void __launch_bounds__(256) varlen_rows_kernel(const int* __restrict__ cu, int S, int chunks,
                                                          const char* __restrict__ src, long ld_src,
                                                          char* __restrict__ dst, long ld_dst, int to_padded) {
  const int b = blockIdx.y, j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= S) return;
  const int len = cu[b + 1] - cu[b];
  const long prow = (long)b * S + j, qrow = (long)cu[b] + j;
  if (to_padded) {
    char* d = dst + prow * ld_dst;
    for (int c = threadIdx.x & 63; c < chunks; c += 64)
      st16(d + 16 * c, j < len ? ld16(src + qrow * ld_src + 16 * c) : u32x4{0u, 0u, 0u, 0u});
  } else if (j < len) {
    char* d = dst + qrow * ld_dst;
    for (int c = threadIdx.x & 63; c < chunks; c += 64) st16(d + 16 * c, ld16(src + prow * ld_src + 16 * c));
  }
}

}  // namespace

extern "C" int eegf_seq_lengths(int B, int L, const long long* mask, int* lens, int* nonprefix, hipStream_t stream) {
  if (B <= 0 || L <= 0 || !mask || !lens || !nonprefix) return EEGF_ERR_ARG;
  hipMemsetAsync(nonprefix, 0, sizeof(int), stream);
  EEGF_LAUNCH(seq_lengths_kernel, dim3(B), dim3(64), 0, stream, mask, L, lens, nonprefix);
  return (int)hipGetLastError();
}

extern "C" int eegf_varlen_embed(int dtype, int B, int L, int width, const int* cu_seqlens, long packed_rows,
                                 long total_rows, const long long* ids, const float* word, const float* pos, void* out,
                                 long long* ids_packed, hipStream_t stream) {
  if (B <= 0 || B > 65535 || L <= 0 || width <= 0 || !cu_seqlens || !ids || !word || !pos || !out || !ids_packed ||
      packed_rows < 0 || total_rows < packed_rows)
    return EEGF_ERR_ARG;
  const size_t es = dtype == EEGF_BF16 ? 2 : dtype == EEGF_F32 ? 4 : 0;
  if (!es) return EEGF_ERR_ARG;
  if (total_rows > packed_rows) {      // pad rows: zero inputs, token id 0 (their gradients are zero)
    hipMemsetAsync((char*)out + packed_rows * width * es, 0, (total_rows - packed_rows) * width * es, stream);
    hipMemsetAsync(ids_packed + packed_rows, 0, (total_rows - packed_rows) * sizeof(long long), stream);
  }
  const dim3 grid((L + 3) / 4, B);
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(varlen_embed_kernel<float>, grid, dim3(256), 0, stream, cu_seqlens, ids, L, width, word, pos,
                       (float*)out, ids_packed);
  else
    EEGF_LAUNCH(varlen_embed_kernel<bf16>, grid, dim3(256), 0, stream, cu_seqlens, ids, L, width, word, pos,
                       (bf16*)out, ids_packed);
  return (int)hipGetLastError();
}

extern "C" int eegf_varlen_rows(int dtype, int B, int S, int width, const int* cu_seqlens, long packed_rows,
                                long total_rows, const void* src, long ld_src, void* dst, long ld_dst, int to_padded,
                                hipStream_t stream) {
  const size_t es = dtype == EEGF_BF16 ? 2 : dtype == EEGF_F32 ? 4 : 0;
  if (!es || B <= 0 || B > 65535 || S <= 0 || width <= 0 || (width * es) % 16 || !cu_seqlens || !src || !dst)
    return EEGF_ERR_ARG;
  if ((ld_src * es) % 16 || (ld_dst * es) % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16) return EEGF_ERR_ARG;
  if (!to_padded && total_rows > packed_rows)       // packed rows past the sequences: defined zeros
    hipMemset2DAsync((char*)dst + packed_rows * ld_dst * es, ld_dst * es, 0, width * es, total_rows - packed_rows,
                     stream);
  const dim3 grid((S + 3) / 4, B);
  EEGF_LAUNCH(varlen_rows_kernel, grid, dim3(256), 0, stream, cu_seqlens, S, (int)(width * es / 16),
                     (const char*)src, (long)(ld_src * es), (char*)dst, (long)(ld_dst * es), to_padded);
  return (int)hipGetLastError();
}

extern "C" int eegf_window_tokens(int dtype, int B, int C, int T, const float* eeg, void* tokens, hipStream_t stream) {
  if (B <= 0 || C <= 0 || C > 128 || T <= 0 || !eeg || !tokens || B > 65535) return EEGF_ERR_ARG;
  const dim3 grid((T + 63) / 64, B);
  if (dtype == EEGF_F32) EEGF_LAUNCH(window_tokens_kernel<float>, grid, dim3(256), 0, stream, eeg, C, T, (float*)tokens);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(window_tokens_kernel<bf16>, grid, dim3(256), 0, stream, eeg, C, T, (bf16*)tokens);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_embed_gather(int dtype, long rows, int width, const long long* ids, const float* table, void* out,
                                 hipStream_t stream) {
  if (rows <= 0 || width <= 0 || !ids || !table || !out) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == EEGF_F32) EEGF_LAUNCH(gather_kernel<float>, grid, dim3(256), 0, stream, ids, table, width, rows, (float*)out);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(gather_kernel<bf16>, grid, dim3(256), 0, stream, ids, table, width, rows, (bf16*)out);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_embed_scatter_add(int dtype, long rows, int width, const long long* ids, const void* d,
                                      float* table_grad, hipStream_t stream) {
  if (rows <= 0 || width <= 0 || !ids || !d || !table_grad) return EEGF_ERR_ARG;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(scatter_add_kernel<float>, grid, dim3(256), 0, stream, ids, (const float*)d, width, rows, table_grad);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(scatter_add_kernel<bf16>, grid, dim3(256), 0, stream, ids, (const bf16*)d, width, rows, table_grad);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}
