/* eegfusion.h — C-ABI of the MI355X-native EEG+action fusion training path.
 *
 * The reference (Rachfu/EEG-multimodal) has no native code: every device op below replaces an
 * implicit ATen / `transformers` op inside `ConcatModel.forward` (model.py:34-64,
 * past_acc.py:108-139, main_0430.py:108-123, python/src/custom_models/models.py:56-82) and its
 * autograd backward.  Each entry cites the reference call site it replaces.
 *
 * Contract for every entry point:
 *   - all pointers are caller-owned device pointers (row-major, contiguous unless a leading
 *     dimension / stride argument says otherwise); sizes are in elements;
 *   - no allocation, no host synchronisation, no global state: a caller may capture any sequence
 *     of calls into a hipGraph;
 *   - work is enqueued on `stream`;
 *   - returns 0 on success, EEGF_ERR_ARG (<0) on an argument error (nothing launched), or the
 *     hipError_t of the launch; never throws.
 */
#ifndef EEGFUSION_H
#define EEGFUSION_H

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

/* element types */
#define EEGF_F32 0
#define EEGF_BF16 1

#define EEGF_ERR_ARG (-1)

/* GEMM epilogues */
#define EPI_NONE 0       /* C = alpha*AB (+ beta*C)                                   */
#define EPI_BIAS 1       /* + bias[n]                           nn.Linear forward        */
#define EPI_BIAS_GELU 2  /* aux = AB+bias; C = gelu_erf(aux)    BertIntermediate         */
#define EPI_BIAS_RELU 3  /* C = relu(AB+bias)                   fc_layers[0..1]          */
#define EPI_BIAS_TANH 4  /* C = tanh(AB+bias)                   fc_layers[2..3], pooler  */
#define EPI_DGELU 5      /* C = AB * gelu'(aux)                 backward of EPI_BIAS_GELU */
#define EPI_DRELU 6      /* C = AB * (aux>0) * epi_scale        backward of relu(+dropout) */
#define EPI_DTANH 7      /* C = AB * (1-aux^2)                  backward of tanh         */

/* Every dense projection of the path: BERT Q/K/V/out/FFN (transformers modeling_bert.py:139-351),
 * pooler (modeling_bert.py:451-462), visual_encoder (model.py:18,36), decoder in_proj/out_proj/
 * linear1/linear2 (torch/nn/modules/transformer.py:1158-1200), fc_layers + classifier
 * (model.py:24-32,62-63), and their input-/weight-gradient GEMMs.
 *   C[z][m,n] = epi(alpha * sum_k A(m,k) B(k,n)) + beta*C[z][m,n]
 *   a_kcontig: A(m,k)=A[m*lda+k] else A[k*lda+m];  b_kcontig: B(k,n)=B[n*ldb+k] else B[k*ldb+n]
 * dtype: EEGF_F32 (out F32) or EEGF_BF16 (out BF16, or F32 for weight gradients). */
int eegf_gemm(int dtype, int out_dtype, int a_kcontig, int b_kcontig, int epi,
              int M, int N, int K, int batch,
              const void* A, long lda, long strideA,
              const void* B, long ldb, long strideB,
              void* C, long ldc, long strideC,
              const float* bias, void* aux, long ldaux, long strideAux,
              float alpha, float beta, float epi_scale, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* EEGFUSION_H */
