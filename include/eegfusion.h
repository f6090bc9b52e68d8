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
 *     of calls into a hipGraph.  The diagnostics are the exception, declared as such below and used
 *     by tests / benchmarks only: eegf_tune (process-global kernel-routing keys, A/B switches with
 *     production defaults; set them before launching, not concurrently with launches on other
 *     threads), the launch counters (eegf_launch_log_*, host-side) and eegf_gemm_big_timestamps
 *     (diagnostics builds only);
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
#define EPI_BIAS_GELU 2  /* aux = AB+bias (NULL: not stored); C = gelu_erf(AB+bias)  BertIntermediate */
#define EPI_BIAS_RELU 3  /* C = relu(AB+bias)                   fc_layers[0..1]          */
#define EPI_BIAS_TANH 4  /* C = tanh(AB+bias)                   fc_layers[2..3], pooler  */
#define EPI_DGELU 5      /* C = AB * gelu'(aux)                 backward of EPI_BIAS_GELU */
#define EPI_DRELU 6      /* C = AB * (aux>0) * epi_scale        backward of relu(+dropout) */
#define EPI_DTANH 7      /* C = AB * (1-aux^2)                  backward of tanh         */
#define EPI_BIAS_GELU_D 8 /* C = gelu_erf(AB+bias); aux = gelu_erf'(AB+bias)  (saves the derivative) */
#define EPI_MUL_AUX 9    /* C = AB * aux                        backward of EPI_BIAS_GELU_D */

/* Every dense projection of the path: BERT Q/K/V/out/FFN (transformers modeling_bert.py:139-351),
 * pooler (modeling_bert.py:451-462), visual_encoder (model.py:18,36), decoder in_proj/out_proj/
 * linear1/linear2 (torch/nn/modules/transformer.py:1158-1200), fc_layers + classifier
 * (model.py:24-32,62-63), and their input-/weight-gradient GEMMs.
 *   C[z][m,n] = epi(alpha * sum_k A(m,k) B(k,n)) + beta*C[z][m,n]
 *   a_kcontig: A(m,k)=A[m*lda+k] else A[k*lda+m];  b_kcontig: B(k,n)=B[n*ldb+k] else B[k*ldb+n]
 * dtype: EEGF_F32 (out F32) or EEGF_BF16 (out BF16, or F32: weight gradients, fp32 pooler output).
 * workspace (nullable, ws_bytes): fp32 split-K slabs; used when the tile grid under-fills the chip
 * and K is long (weight gradients over B*L tokens); the slabs are reduced in a fixed order. */
int eegf_gemm(int dtype, int out_dtype, int a_kcontig, int b_kcontig, int epi,
              int M, int N, int K, int batch,
              const void* A, long lda, long strideA,
              const void* B, long ldb, long strideB,
              void* C, long ldc, long strideC,
              const float* bias, long strideBias, void* aux, long ldaux, long strideAux,
              float alpha, float beta, float epi_scale, void* workspace, long ws_bytes,
              hipStream_t stream);
/* Tuning / A-B hook (tests and benchmarks; not part of the reference interface).  Returns the previous
 * value, or EEGF_ERR_ARG for an unknown key or an out-of-range value.  Every key selects between
 * kernels that compute the same results (bitwise, or up to summation order where stated); the defaults
 * are the production routes.
 *   key 2:  L = 256 attention kernels: bit 0 the persistent forward, bit 1 the persistent backward
 *           (default 3; 0 = the generic flash kernels, up to summation order);
 *   key 6:  maximum rows per wave of eegf_ln_fwd (1..64, default 16);
 *   key 7:  rows per workgroup of eegf_ln_bwd when rows >= 65536 (multiple of 4, default 64);
 *   key 10: bf16 768-wide rows of eegf_ln_fwd on the 16-B-access kernel (1, default) or the generic one (0);
 *   key 11: the persistent 256x256 GEMMs for the full-tile bf16-output GEMMs they take: 1 (default), 0 the
 *           non-persistent 4-wave kernel (bitwise the same results: tests/test_gemm_gpu.py);
 *   key 13: CUs left free by the persistent grids (0 = default): room for RCCL's kernels during the
 *           backward (tools/overlap_proxy.py prices it);
 *   key 14: the persistent GEMMs with K % 64 == 0 on gemm4r (whole-line K-tile pairs, rolling A
 *           fragments; 1, default) or gemm4p (64-B half lines; 0): bitwise the same results;
 *   key 19: eegf_xattn_fwd / _bwd with a bf16 memory: the context and backward on the fp32 MFMA (1, default)
 *           or the VALU kernels (0); fp32 products and sums either way, equal up to summation order.
 * Process-global (see the contract above): test / benchmark state, not for production callers. */
int eegf_tune(int key, int value);
/* Diagnostics (no reference counterpart), libraries built with -DEEGF_DIAG=1 only (elsewhere a non-null
 * buf returns EEGF_ERR_ARG): every following gemm4w launch writes 4 s_memrealtime stamps per workgroup
 * (start, prologue done, K-loop done, epilogue issued, slot 4 the CU id) into buf = int64
 * [grid.y][grid.x][8]; nullptr switches it off.  tools/gemm_phases.py. */
int eegf_gemm_big_timestamps(long long* buf);
/* Diagnostics (no reference counterpart): a stand-in for the CU use of an RCCL all-reduce kernel, for
 * the one-GPU overlap proxy of the gradient all-reduces (tools/overlap_proxy.py): `wgs`
 * workgroups read and rewrite x[0, n) unchanged `passes` times (n % 4 == 0, x 16-B aligned). */
int eegf_ring_proxy(long n, int passes, int wgs, float* x, hipStream_t stream);
/* Diagnostics (no reference counterpart): per-kernel launch counters.  Every kernel launch of the
 * library is counted on the host (one entry per kernel template instantiation) from load time or the
 * last reset.  eegf_launch_log_read writes "count<TAB>demangled kernel name\n" lines into buf (at most
 * cap bytes, NUL-terminated; buf may be NULL) and returns the bytes the whole text needs, NUL
 * included.  Process-global, like eegf_tune; the route-coverage test reads it
 * (tests/test_production_gpu.py). */
int eegf_launch_log_reset(void);
long eegf_launch_log_read(char* buf, long cap);
/* Weight gradient of an nn.Linear with its bias gradient fused (autograd of F.linear, the weight and
 * bias grads of every BERT projection, modeling_bert.py:139-351): dW [M][N] = dY^T X + beta dW over
 * K tokens, db [M] += dY.sum(0).  dY [K][M] (row stride ldd) and X [K][N] (ldx) bf16; dW, db fp32.
 * The row sums ride on the weight-gradient kernel: the workgroups of tile column 0 run one
 * v_mfma_f32_16x16x32_bf16 per 16-row block and K-tile against a ones operand (a column of the result
 * holds the K-tile's sum of one row), into a VGPR accumulator; deterministic, in the MFMA's summation
 * order (not bitwise the earlier VALU order), and reduced over the splits in a fixed order.  workspace: fp32 split-K slabs
 * (splits x (M*N + M) floats).  EEGF_ERR_ARG when the shape is not eligible (bf16, M, N >= 256,
 * K >= 4096, K % 64 == 0, 8-aligned dims, 16-B aligned dY / X, workspace too small): run eegf_gemm and
 * eegf_colsum instead. */
int eegf_gemm_wgrad_bias(int dtype, int M, int N, int K, const void* dY, long ldd, const void* X, long ldx,
                         float* dW, long ldw, float beta, float* db, void* workspace, long ws_bytes,
                         hipStream_t stream);
/* ---- contract T pad skipping (varlen BERT).  The reference runs BERT over the
 * padded 512 tokens (get_embedding.py:115) with the padded keys masked (model.py:37-43); the packed
 * rows of the real tokens give the same outputs.  cu_seqlens [B+1] int32 (device): sequence b owns
 * packed rows cu[b] .. cu[b+1]-1; packed_rows = cu[B]; total_rows >= packed_rows rounds the row count
 * up for the GEMM tiles (rows past packed_rows are written as zeros). */
/* lens[b] = nonzero entries of mask row b ([B, L] int64 attention_mask); *nonprefix = 1 when some row
 * is not [1]*n + [0]*(L-n) (then the packed path does not apply). */
int eegf_seq_lengths(int B, int L, const long long* mask, int* lens, int* nonprefix, hipStream_t stream);
/* BertEmbeddings word + position rows of the real tokens (modeling_bert.py:95-105, position_ids =
 * arange): out[cu[b]+j] = word[ids[b,j]] + pos[j] (fp32 sum, one rounding), ids_packed[cu[b]+j] =
 * ids[b,j]; the token-type row is added by eegf_ln_fwd (table2). */
int eegf_varlen_embed(int dtype, int B, int L, int width, const int* cu_seqlens, long packed_rows,
                      long total_rows, const long long* ids, const float* word, const float* pos, void* out,
                      long long* ids_packed, hipStream_t stream);
/* padded [B, S, width] (row stride ld) <-> packed rows: to_padded = 1 writes every padded row (zeros
 * past each sequence: the decoder memory / pooler input); 0 writes the packed rows (and zeros rows
 * packed_rows .. total_rows-1).  16-B aligned rows. */
int eegf_varlen_rows(int dtype, int B, int S, int width, const int* cu_seqlens, long packed_rows, long total_rows,
                     const void* src, long ld_src, void* dst, long ld_dst, int to_padded, hipStream_t stream);
/* Packed self-attention (BertSelfAttention over each sequence's real tokens, no key bias): as
 * eegf_attn_fwd with the rows of sequence b at cu[b] ..; max_len = the padded length L of the batch
 * (>= every sequence length): LSE is [B, 12, max_len] and the dropout element numbering is the padded
 * ((b*12 + h)*L + q)*L + key, so a packed batch draws exactly its padded form's masks.  key_bias
 * [B, max_len] (nullable) is added to the scores as in eegf_attn_fwd: with uniform cu_seqlens
 * (cu[b] = b*L) these kernels also run the padded layout at any L (the dense ones need L % 256). */
int eegf_attn_varlen_fwd(int dtype, int B, int H, int max_len, const int* cu_seqlens, long packed_rows,
                         long total_rows, const void* qkv, long ld_qkv, const float* key_bias, float scale,
                         float drop_p,
                         unsigned long long seed, unsigned long long offset, void* out, long ld_out, float* lse,
                         hipStream_t stream);
long eegf_attn_varlen_bwd_workspace(long total_rows, int max_len);
int eegf_attn_varlen_bwd(int dtype, int B, int H, int max_len, const int* cu_seqlens, long packed_rows,
                         long total_rows, const void* qkv, long ld_qkv, const float* key_bias, float scale,
                         float drop_p,
                         unsigned long long seed, unsigned long long offset, const void* out, const void* dout,
                         long ld_out, const float* lse, void* dqkv, float* dq_workspace, hipStream_t stream);

/* ---- modality variants (custom_models/models.py:84-272) */
/* Self-attention over S <= 8 tokens per sample (TISC's TransformerEncoder over [mean(EEG seq), action],
 * models.py:227-228, F.multi_head_attention_forward): rows n*S .. n*S+S-1 of qkv [N*S, >= 2304]; one wave
 * per (sample, head); probs [N, 12, S, S] fp32 = the undropped softmax (saved for the backward);
 * attention-weight dropout by Philox element ((n*12 + h)*S + i)*S + j. */
int eegf_attn_small_fwd(int dtype, int N, int S, const void* qkv, long ld_qkv, float scale, float drop_p,
                        unsigned long long seed, unsigned long long offset, void* out, long ld_out, float* probs,
                        hipStream_t stream);
int eegf_attn_small_bwd(int dtype, int N, int S, const void* qkv, long ld_qkv, const float* probs, const void* dout,
                        long ld_out, float scale, float drop_p, unsigned long long seed, unsigned long long offset,
                        void* dqkv, long ld_dqkv, hipStream_t stream);
/* out[b] (fp32) = mean of rows b*L .. b*L+L-1 of x (TTCA decoder output / TISC sequence and token
 * means, models.py:109, :253, :260); backward dx rows = beta dx + dmean[b] / L. */
int eegf_seq_mean(int dtype, int B, int L, int width, const void* x, long ld_x, float* out, long ld_out,
                  hipStream_t stream);
int eegf_seq_mean_bwd(int dtype, int B, int L, int width, const float* dmean, long ld_dmean, void* dx, long ld_dx,
                      float beta, hipStream_t stream);

/* fusion variants (eegf_fusion_fwd/bwd) */
#define FUSE_CONCAT 0        /* model.py ConcatModel.feature: minmax(cat)            model.py:46-50      */
#define FUSE_PRICONCAT 1     /* main_0430 ConcatModel: DP_guarantee(dp_mode=None)=id main_0430.py:118    */
#define FUSE_PRICONCAT_LAP 2 /* DP_guarantee('feature_all_lap'): minmax + row Laplace main_0430.py:76-85 */
#define FUSE_PRIGUMBEL 3     /* past_acc / TICA_LapDropout gate                      past_acc.py:120-136 */

/* Residual + dropout + LayerNorm, one row of `width` (multiple of 256, <= 1024) per wave:
 *   v = drop(x) [drop_mode 1] + r + table[row % table_period] + table2;  y = LN(v) [drop on y: mode 2]
 * Replaces BertEmbeddings LN+dropout (modeling_bert.py:95-105), BertSelfOutput/BertOutput
 * (:282-293, :340-351) and the decoder's norm1/2/3 (transformer.py:1158-1200).  Stores the
 * pre-LN sum `s_out` and per-row mean/rstd for the backward. */
int eegf_ln_fwd(int dtype, long rows, int width, const void* x, const void* r, const float* table,
                int table_period, const float* table2, const float* gamma, const float* beta, float eps,
                float drop_p, int drop_mode, unsigned long long seed, unsigned long long offset,
                void* y, void* s_out, float* mean, float* rstd, hipStream_t stream);
/* rows handled per workgroup by eegf_ln_bwd: partial dgamma/dbeta buffers are ceil(rows/this) x width */
long eegf_ln_bwd_partial_rows(long rows);
/* LayerNorm backward: dx = grad wrt x (dropout mask applied for mode 1), dr = grad wrt the
 * residual / table inputs (nullable); per-block partial dgamma/dbeta (reduce with eegf_colsum). */
int eegf_ln_bwd(int dtype, long rows, int width, const void* dy, const void* s, const float* mean,
                const float* rstd, const float* gamma, float drop_p, int drop_mode,
                unsigned long long seed, unsigned long long offset, void* dx, void* dr,
                float* dgamma_part, float* dbeta_part, hipStream_t stream);
/* out[p, c] = sum_{r = p mod period} in[r*ld + c] (+ beta*out); fp32 accumulation, two passes,
 * deterministic.  Bias gradients (period 1), position-embedding gradients (period L), LayerNorm
 * partial reduction.  ws: scratch of ws_elems floats. */
int eegf_colsum(int dtype, const void* in, long ld, long rows, int width, int period, float* ws,
                long ws_elems, float* out, float beta, hipStream_t stream);
/* Batched column sums (bias / LayerNorm gradients of a whole backward pass in one launch): desc is a
 * device array of n descriptors of 6 int64 each: src, dst (fp32), ld, rows, width | dtype << 32,
 * float_bits(beta) | first_block << 32, where descriptor i owns blocks [first_block_i,
 * first_block_{i+1}) (ceil(width / 64) blocks each, first_block ascending); blocks = total.
 * dst[c] = sum_r src[r*ld + c] + beta * dst[c], fixed order (deterministic). */
int eegf_colsum_batch(int n, const long long* desc, int blocks, hipStream_t stream);

/* Multi-head self-attention (12 x 64) over the fused QKV projection [B, L, ld_qkv>=2304]
 * (BertSelfAttention, modeling_bert.py:139-199).  key_bias [B, L]: 0 or -1e30 (nullable).
 * drop_p: dropout of the attention probabilities (modeling_bert.py:131,198; 0 = off), Philox
 * (seed, offset), element ((b*12+h)*L+q)*L+key.  out [B, L, ld_out>=768]; lse [B, 12, L] saved
 * for the backward.  drop_bits (nullable, used when drop_p > 0): receives the keep mask, one bit per
 * probability, [B*12][L][L/32] u32, bit t of word j <-> key 32j+t, for eegf_attn_bwd.  L % 128 == 0. */
int eegf_attn_fwd(int dtype, int B, int H, int L, const void* qkv, long ld_qkv, const float* key_bias,
                  float scale, float drop_p, unsigned long long seed, unsigned long long offset,
                  void* out, long ld_out, float* lse, unsigned int* drop_bits, hipStream_t stream);
/* fp32 workspace (elements) eegf_attn_bwd needs for dQ accumulation (0 when L <= 256). */
long eegf_attn_bwd_workspace(int B, int L);
/* Attention backward: writes dQ|dK|dV into dqkv [B, L, ld_qkv] (same layout as qkv).  drop_p,
 * seed, offset as in the forward; drop_bits: the forward's keep mask (nullable: the mask is
 * regenerated from the Philox stream).  L % 256 == 0. */
int eegf_attn_bwd(int dtype, int B, int H, int L, const void* qkv, long ld_qkv, const float* key_bias,
                  float scale, float drop_p, unsigned long long seed, unsigned long long offset,
                  const void* out, const void* dout, long ld_out, const float* lse,
                  const unsigned int* drop_bits, void* dqkv, float* dq_workspace, hipStream_t stream);

/* Decoder cross-attention over the BERT memory with a single query token
 * (TransformerDecoderLayer._mha_block, transformer.py:1177-1196; model.py:40-43), in the
 * reduced form: qp [B,12,768] = Wk_h^T q_h / 8 (by eegf_gemm); probs [B,12,S] (undropped p)
 * saved; ctx [B,12,768] = sum_j p~_j M_j with p~ = dropout(p) (drop_p, Philox element
 * (b*12+h)*S+j); psum [B,12] = sum_j p~_j (required when drop_p > 0; the caller adds
 * psum_h * bv_h with eegf_head_bias_fwd).  key_bias [B,S] nullable.  ws: B*12*S floats.
 * mem_dtype: the encoder's dtype; q_dtype: the decoder's (bf16 mode runs the decoder in fp32:
 * F32 with a BF16 memory).  S <= 1024. */
int eegf_xattn_fwd(int mem_dtype, int q_dtype, int B, int S, const void* mem, const void* qp,
                   const float* key_bias, float drop_p, unsigned long long seed, unsigned long long offset,
                   float* ws, float* probs, float* psum, void* ctx, hipStream_t stream);
/* Backward: dctx = dL/dctx [B,12,768]; dpsum [B,12] = dL/dpsum (nullable);
 * dmem [B,S,768] (= result + beta*dmem), dqp [B,12,768].  ws: B*12*S floats. */
int eegf_xattn_bwd(int mem_dtype, int q_dtype, int B, int S, const void* mem, const void* qp,
                   const float* probs, const float* dpsum, const void* dctx, float drop_p,
                   unsigned long long seed, unsigned long long offset, float* ws, void* dmem,
                   float beta, void* dqp, hipStream_t stream);
/* x[b,c] += bias[c] * s[b, c/group]  (fp32; the psum_h * bv_h term of the cross-attention). */
int eegf_head_bias_fwd(int B, int W, int group, float* x, const float* bias, const float* s,
                       hipStream_t stream);
/* ds[b,g] = sum_{c in g} dx[b,c] bias[c];  dbias[c] = sum_b dx[b,c] s[b,c/group] + beta*dbias[c]
 * (dbias nullable).  group == 64. */
int eegf_head_bias_bwd(int B, int W, int group, const float* dx, const float* bias, const float* s,
                       float* ds, float* dbias, float beta, hipStream_t stream);

/* Fused concat [pooled|img|cross] -> min-max -> privacy stage (variant FUSE_*), one row per
 * workgroup (model.py:46-61, past_acc.py:120-136, main_0430.py:76-85).  noise/gumbels (fp32
 * [B,2304] / [2,B,2304]) and row_noise [B] are injected draws (parity) or NULL: Philox(seed,
 * offset).  eps_mode 0 = newfrac 1/ln(.), 1 = new ln(.); eps_a = exp(eps); lap_scale = 1/eps.
 * Saves xn (normalised feature), argmin/argmax/range per row for the backward. */
int eegf_fusion_fwd(int dtype, int B, int variant, const void* pooled, long ld_pooled, const void* img,
                    long ld_img, const void* cross, long ld_cross, const float* DP, const float* noise,
                    const float* gumbels, const float* row_noise, int hard, int eps_mode, float eps_a,
                    float lap_scale, unsigned long long seed, unsigned long long offset, void* out,
                    float* xn, int* amin, int* amax, float* range, hipStream_t stream);
/* Backward to the three encoder outputs; ddp_rows [B,2304] (nullable) receives per-row dL/dDP
 * (reduce with eegf_colsum). */
int eegf_fusion_bwd(int dtype, int B, int variant, const void* dout, const float* xn, const int* amin,
                    const int* amax, const float* range, const float* DP, const float* noise,
                    const float* gumbels, int hard, int eps_mode, float eps_a, unsigned long long seed,
                    unsigned long long offset, void* d_pooled, long ld_pooled, void* d_img, long ld_img,
                    void* d_cross, long ld_cross, float* ddp_rows, hipStream_t stream);
/* F.cross_entropy (reduction 0 = mean: past_acc.py:73; 1 = sum: train.py:69,111) + argmax
 * correct count; dlogits = dL/dlogits * dscale (nullable). */
int eegf_cross_entropy(int dtype, int B, int C, const void* logits, const long long* labels,
                       int reduction, float dscale, float* loss, int* correct, void* dlogits,
                       hipStream_t stream);

/* PriGumbel-v1 gate (train_val.py:95-123, the model of :125-158): x [B,768] fp32 (fc2 output, row
 * stride ldx), w [768] (raw, no sigmoid); m_j = F.gumbel_softmax((w_j, 1-w_j), tau, hard)[1] with one
 * Gumbel pair per feature for the whole batch (gumbels [768,2] = -log Exp(1) injected, or Philox);
 * res = x m / (1 - w); out = row min-max(res) + row Laplace(0, lap_scale) (row_noise [B] injected or
 * Philox).  Saves xn, argmin/argmax/range for the backward. */
int eegf_v1_gate_fwd(int B, const float* x, long ldx, const float* w, const float* gumbels, const float* row_noise,
                     float tau, int hard, float lap_scale, unsigned long long seed, unsigned long long offset,
                     float* out, float* xn, int* amin, int* amax, float* range, hipStream_t stream);
/* Backward: dx [B,768] (row stride ldx); dw_rows [B,768] per-row dL/dw (nullable; reduce with
 * eegf_colsum), the straight-through estimator for hard masks. */
int eegf_v1_gate_bwd(int B, const float* dout, const float* x, long ldx, const float* w, const float* gumbels,
                     const float* xn, const int* amin, const int* amax, const float* range, float tau, int hard,
                     unsigned long long seed, unsigned long long offset, float* dx, float* dw_rows,
                     hipStream_t stream);
/* loss_function's privacy term (train_val.py:88-90): loss = max_j((1-w_j) eps_a + w_j) (nullable);
 * dw[argmax] += dscale (1 - eps_a) (nullable; first index on ties). */
int eegf_v1_wloss(int D, const float* w, float eps_a, float dscale, float* loss, float* dw, hipStream_t stream);

/* feawei DP initialisation (past_acc.py:98-103 with k = 1, zscore = 1; past_acc_feawei.py:153-163
 * with k = 5, zscore = 0): colsum [D] = column sums over `count` rows of the normalised features
 * (eegf_colsum with beta = 1 across batches); z = (m - mean m) / std m (population std) or z = m;
 * dp[c] = base[c] + (1 - sigmoid(k z_c)) - 0.5, base = cat(0.4, 0.5, 0.3 per 768) in the reference. */
int eegf_feawei_init(int D, const float* colsum, long count, float k, int zscore, const float* base, float* dp,
                     hipStream_t stream);

/* y = alpha*x + beta*y ; dx = dy*(1-y^2) */
int eegf_axpby(int dtype, long n, float alpha, const void* x, float beta, void* y, hipStream_t stream);
int eegf_tanh_bwd(int dtype, long n, const void* dy, const void* y, void* dx, hipStream_t stream);
/* In-place dropout x[i] *= mask(i / group) (Philox element i/group of (seed, offset); kept
 * elements scale by 1/(1-p)).  group 1: elementwise (decoder FFN inner dropout,
 * transformer.py:1197-1199); group 64: one draw per head (decoder self-attention weight dropout,
 * transformer.py:1158-1176).  Applying it to the gradient gives the backward. */
int eegf_dropout(int dtype, long n, int group, float p, unsigned long long seed, unsigned long long offset,
                 void* x, hipStream_t stream);

/* torch.optim.Adam step over a contiguous fp32 range (+ optional bf16 shadow refresh); the gradient
 * read is g * grad_scale (1 for a plain step, 1/N to average an all-reduced sum over N ranks). */
int eegf_adam(long n, float* p, const float* g, float* m, float* v, void* bf16_shadow, float lr,
              float beta1, float beta2, float eps, float weight_decay, float grad_scale, int step, hipStream_t stream);
/* eegf_adam that also writes g[i] = 0 once read: the optimizer step and the next iteration's
 * optimizer.zero_grad() (past_acc.py:197,204) in one pass over the gradient range. */
int eegf_adam_consume(long n, float* p, float* g, float* m, float* v, void* bf16_shadow, float lr,
                      float beta1, float beta2, float eps, float weight_decay, float grad_scale, int step,
                      hipStream_t stream);
int eegf_cast_f32_bf16(long n, const float* src, void* dst, hipStream_t stream);
/* attention_mask (int64, 1 = keep) -> additive key bias (0 / -1e30) */
int eegf_key_bias(long n, const long long* mask, float* bias, hipStream_t stream);

/* EEG window [B,C,T] fp32 (channel x time) -> time-major tokens [B*T, C] (contract W). */
int eegf_window_tokens(int dtype, int B, int C, int T, const float* eeg, void* tokens, hipStream_t stream);
/* word-embedding gather / scatter-add (contract T; modeling_bert.py:101-102) */
int eegf_embed_gather(int dtype, long rows, int width, const long long* ids, const float* table, void* out,
                      hipStream_t stream);
int eegf_embed_scatter_add(int dtype, long rows, int width, const long long* ids, const void* d,
                           float* table_grad, hipStream_t stream);

/* ---- DP-SGD: per-sample clipping + Gaussian noise (opacus make_private_with_epsilon as used by
 * main_0430.py:143-162 and python/src/custom_models/base_train.py:322-348; opacus's GradSampleModule
 * + DPOptimizer.pre_step), without materialising per-sample gradients.  out[s] accumulates the
 * squared per-sample gradient norm of sample s; beta scales the previous value (0 or 1). */
/* fp32 partial-sum elements eegf_ghost_norm needs: S * (T/64)(T/64 + 1)/2 */
long eegf_ghost_norm_workspace(int S, int T);
/* Token-sequence Linear (T rows per sample, T % 64 == 0): out[s] = beta*out[s] + ||DY_s^T X_s||_F^2
 * = sum_{t,u} (x_t.x_u)(dy_t.dy_u) (the two Gram matrices on the MFMA, tile by tile).  X [S*T, Dx],
 * DY [S*T, Dy] row-major with leading dimensions; Dx, Dy % 32 == 0. */
int eegf_ghost_norm(int dtype, int S, int T, int Dx, int Dy, const void* X, long ldx, const void* DY, long ldy,
                    float* ws, long ws_elems, float beta, float* out, hipStream_t stream);
/* Per-sample column sums over T rows: out[s] = beta*out[s] + [bias_term] sum_c (sum_t dy[t,c])^2 (a bias
 * or LN beta) and, with LayerNorm statistics (xs = pre-LN sum, mean, rstd; nullable),
 * + sum_c (sum_t dy[t,c] xhat[t,c])^2 (LN gamma).  Each term only for a trainable parameter; xs == NULL
 * with bias_term == 0 is an argument error.  T = 1 gives per-row norms. */
int eegf_seg_sqnorm(int dtype, int S, int T, int W, const void* dy, long ldd, const void* xs, long ldx,
                    const float* mean, const float* rstd, int bias_term, float beta, float* out, hipStream_t stream);
/* One row per sample (head / pooler / visual Linear): out[s] += ||a_s||^2 * (b ? ||b_s||^2 : 1). */
int eegf_row_sqnorm(int dtype, int S, int Wa, const void* a, long lda, int Wb, const void* b, long ldb, float* out,
                    hipStream_t stream);
/* c_s = min(1, max_norm / (sqrt(psn_s) + 1e-6)); dlogits[s, :] *= c_s; clip[s] = c_s (nullable). */
int eegf_dp_clip_rows(int S, int ncls, const float* psn, float max_norm, float* dlogits, float* clip,
                      hipStream_t stream);
/* grad[i] = (grad[i] + std * N(0,1)) * scale (Philox4x32-10 (seed, offset) + Box-Muller). */
int eegf_dp_noise(long n, float* grad, float std, float scale, unsigned long long seed, unsigned long long offset,
                  hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* EEGFUSION_H */
