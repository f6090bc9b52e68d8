// decoder.hip — single-query cross-attention of the 3-layer TransformerDecoder over the BERT memory.
//
// Reference: multihead_attn(x, memory, memory) inside TransformerDecoderLayer._mha_block
// (torch/nn/modules/transformer.py:1177-1196; F.multi_head_attention_forward), called from
// model.py:40-43 with tgt = the single action token.  The memory K/V projections are never
// materialised: for head h with projected query q_h,
//     score_j = q_h . (Wk_h M_j + bk_h) / 8 = q'_h . M_j + const,   q'_h = Wk_h^T q_h / 8
//     ctx_h   = sum_j p_j (Wv_h M_j + bv_h) = Wv_h c_h + bv_h,        c_h = sum_j p_j M_j
// (the constant q_h.bk_h/8 cancels in the softmax).  These kernels compute p and c_h (forward) and
// dM, dq' (backward) by streaming M once or twice; the q', Wv c and projection GEMMs are eegf_gemm.
// One workgroup per batch row b; HBM-bound on M (S x 768 per row).
#include "common.h"
#include "eegfusion_internal.h"

namespace {

constexpr int E = 768, NH = 12, NCOL = 12;  // columns per lane: 768 / 64

template <typename T>
DEV void load_row12(const T* row, int lane, float (&v)[NCOL]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int col = (lane + 64 * i) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * i + e] = to_f32(row[col + e]);
  }
}
DEV int col_of(int lane, int k) { return (lane + 64 * (k >> 2)) * 4 + (k & 3); }

// ---- forward: scores, softmax (saved), context c[b,h,:] ----
template <typename T, typename TQ>
__global__ void __launch_bounds__(256) xattn_fwd_kernel(const T* __restrict__ mem, const TQ* __restrict__ qp,
                                                        const float* __restrict__ kbias, int S, float* __restrict__ probs,
                                                        TQ* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* qs = sm;               // [NH][E]
  float* ps = sm + NH * E;      // [NH][S]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* M = mem + (long)b * S * E;
  for (int i = tid; i < NH * E; i += 256) qs[i] = to_f32(qp[(long)b * NH * E + i]);
  __syncthreads();
  float qreg[NH][NCOL];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int k = 0; k < NCOL; ++k) qreg[h][k] = qs[h * E + col_of(lane, k)];
  // phase 1: raw scores
  for (int j = wave; j < S; j += 4) {
    float m[NCOL];
    load_row12(M + (long)j * E, lane, m);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < NCOL; ++k) acc += m[k] * qreg[h][k];
      acc = wave_sum(acc);
      if (lane == 0) ps[h * S + j] = acc + (kbias ? kbias[(long)b * S + j] : 0.f);
    }
  }
  __syncthreads();
  // phase 2: softmax over j per head (wave w: heads w, w+4, w+8)
  for (int h = wave; h < NH; h += 4) {
    float mx = -3.0e38f;
    for (int j = lane; j < S; j += 64) mx = fmaxf(mx, ps[h * S + j]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < S; j += 64) { const float e = __expf(ps[h * S + j] - mx); ps[h * S + j] = e; sum += e; }
    const float inv = 1.0f / wave_sum(sum);
    for (int j = lane; j < S; j += 64) {
      const float p = ps[h * S + j] * inv;
      ps[h * S + j] = p;
      probs[((long)b * NH + h) * S + j] = p;
    }
  }
  __syncthreads();
  // phase 3: c[h][col] = sum_j p[h][j] M[j][col]; wave w owns columns [192w, 192w+192), 3 per lane
  float acc[NH][3];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int k = 0; k < 3; ++k) acc[h][k] = 0.f;
  const int c0 = wave * 192 + lane;
  for (int j = 0; j < S; ++j) {
    const T* row = M + (long)j * E + c0;
    const float m0 = to_f32(row[0]), m1 = to_f32(row[64]), m2 = to_f32(row[128]);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const float p = ps[h * S + j];
      acc[h][0] += p * m0; acc[h][1] += p * m1; acc[h][2] += p * m2;
    }
  }
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int k = 0; k < 3; ++k) ctx[((long)b * NH + h) * E + c0 + 64 * k] = from_f32<TQ>(acc[h][k]);
}

// ---- backward ----
// dp[h][j] = dc[h].M[j];  dsc = p (dp - sum_j p dp);  dq'[h] = sum_j dsc[h][j] M[j];
// dM[j] (+)= sum_h p[h][j] dc[h] + dsc[h][j] q'[h]
template <typename T, typename TQ>
__global__ void __launch_bounds__(256) xattn_bwd_kernel(const T* __restrict__ mem, const TQ* __restrict__ qp,
                                                        const float* __restrict__ probs, const TQ* __restrict__ dc, int S,
                                                        T* __restrict__ dmem, float beta, TQ* __restrict__ dqp) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* qs = sm;                  // [NH][E] q'
  float* dcs = qs + NH * E;        // [NH][E] dc
  float* ps = dcs + NH * E;        // [NH][S] p
  float* dss = ps + NH * S;        // [NH][S] dp -> dsc
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* M = mem + (long)b * S * E;
  for (int i = tid; i < NH * E; i += 256) {
    qs[i] = to_f32(qp[(long)b * NH * E + i]);
    dcs[i] = to_f32(dc[(long)b * NH * E + i]);
  }
  for (int i = tid; i < NH * S; i += 256) ps[i] = probs[(long)b * NH * S + i];
  __syncthreads();
  {
    float dreg[NH][NCOL];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int k = 0; k < NCOL; ++k) dreg[h][k] = dcs[h * E + col_of(lane, k)];
    for (int j = wave; j < S; j += 4) {
      float m[NCOL];
      load_row12(M + (long)j * E, lane, m);
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < NCOL; ++k) acc += m[k] * dreg[h][k];
        acc = wave_sum(acc);
        if (lane == 0) dss[h * S + j] = acc;
      }
    }
  }
  __syncthreads();
  for (int h = wave; h < NH; h += 4) {
    float dot = 0.f;
    for (int j = lane; j < S; j += 64) dot += ps[h * S + j] * dss[h * S + j];
    dot = wave_sum(dot);
    for (int j = lane; j < S; j += 64) dss[h * S + j] = ps[h * S + j] * (dss[h * S + j] - dot);
  }
  __syncthreads();
  // dq'[h][col] = sum_j dsc[h][j] M[j][col]  (wave-owned column slices, as the forward context)
  {
    float acc[NH][3];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int k = 0; k < 3; ++k) acc[h][k] = 0.f;
    const int c0 = wave * 192 + lane;
    for (int j = 0; j < S; ++j) {
      const T* row = M + (long)j * E + c0;
      const float m0 = to_f32(row[0]), m1 = to_f32(row[64]), m2 = to_f32(row[128]);
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const float d = dss[h * S + j];
        acc[h][0] += d * m0; acc[h][1] += d * m1; acc[h][2] += d * m2;
      }
    }
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int k = 0; k < 3; ++k) dqp[((long)b * NH + h) * E + c0 + 64 * k] = from_f32<TQ>(acc[h][k]);
  }
  // dM[j][col] = sum_h p[h][j] dc[h][col] + dsc[h][j] q'[h][col]; each thread owns 3 columns
  {
    const int c0 = tid;  // columns tid, tid+256, tid+512
    float dcr[NH][3], qr[NH][3];
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int k = 0; k < 3; ++k) { dcr[h][k] = dcs[h * E + c0 + 256 * k]; qr[h][k] = qs[h * E + c0 + 256 * k]; }
    T* dM = dmem + (long)b * S * E;
    for (int j = 0; j < S; ++j) {
      float o[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        const float p = ps[h * S + j], d = dss[h * S + j];
#pragma unroll
        for (int k = 0; k < 3; ++k) o[k] += p * dcr[h][k] + d * qr[h][k];
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        T* dst = dM + (long)j * E + c0 + 256 * k;
        *dst = from_f32<T>(beta != 0.f ? o[k] + beta * to_f32(*dst) : o[k]);
      }
    }
  }
}

}  // namespace

template <typename T, typename TQ>
int xfwd(int B, int S, const void* mem, const void* qp, const float* kb, float* probs, void* ctx, hipStream_t st) {
  const size_t lds = sizeof(float) * (NH * E + NH * S);
  hipFuncSetAttribute((const void*)xattn_fwd_kernel<T, TQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((xattn_fwd_kernel<T, TQ>), dim3(B), dim3(256), lds, st, (const T*)mem, (const TQ*)qp, kb, S, probs,
                     (TQ*)ctx);
  return (int)hipGetLastError();
}
template <typename T, typename TQ>
int xbwd(int B, int S, const void* mem, const void* qp, const float* probs, const void* dctx, void* dmem, float beta,
         void* dqp, hipStream_t st) {
  const size_t lds = sizeof(float) * (2 * NH * E + 2 * NH * S);
  hipFuncSetAttribute((const void*)xattn_bwd_kernel<T, TQ>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((xattn_bwd_kernel<T, TQ>), dim3(B), dim3(256), lds, st, (const T*)mem, (const TQ*)qp, probs,
                     (const TQ*)dctx, S, (T*)dmem, beta, (TQ*)dqp);
  return (int)hipGetLastError();
}

extern "C" int eegf_xattn_fwd(int mem_dtype, int q_dtype, int B, int S, const void* mem, const void* qp,
                              const float* key_bias, float* probs, void* ctx, hipStream_t stream) {
  if (B <= 0 || S <= 0 || S > 2048 || !mem || !qp || !probs || !ctx) return EEGF_ERR_ARG;
  if (mem_dtype == EEGF_F32 && q_dtype == EEGF_F32) return xfwd<float, float>(B, S, mem, qp, key_bias, probs, ctx, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_BF16) return xfwd<bf16, bf16>(B, S, mem, qp, key_bias, probs, ctx, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_F32) return xfwd<bf16, float>(B, S, mem, qp, key_bias, probs, ctx, stream);
  return EEGF_ERR_ARG;
}

extern "C" int eegf_xattn_bwd(int mem_dtype, int q_dtype, int B, int S, const void* mem, const void* qp,
                              const float* probs, const void* dctx, void* dmem, float beta, void* dqp,
                              hipStream_t stream) {
  if (B <= 0 || S <= 0 || S > 2048 || !mem || !qp || !probs || !dctx || !dmem || !dqp) return EEGF_ERR_ARG;
  if (mem_dtype == EEGF_F32 && q_dtype == EEGF_F32)
    return xbwd<float, float>(B, S, mem, qp, probs, dctx, dmem, beta, dqp, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_BF16)
    return xbwd<bf16, bf16>(B, S, mem, qp, probs, dctx, dmem, beta, dqp, stream);
  if (mem_dtype == EEGF_BF16 && q_dtype == EEGF_F32)
    return xbwd<bf16, float>(B, S, mem, qp, probs, dctx, dmem, beta, dqp, stream);
  return EEGF_ERR_ARG;
}
