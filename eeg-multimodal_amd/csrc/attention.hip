// attention.hip — fused multi-head self-attention forward/backward (BERT, 12 heads x 64).
//
// Replaces BertSelfAttention's  softmax(Q K^T / 8 + key_mask) V   (modeling_bert.py:139-199,
// sdpa/eager :111-136) and its autograd backward.  Q/K/V are read straight out of the fused
// QKV projection output [B, L, 3*768]; the context is written as [B, L, 768].
//
// Forward: grid (L/128, H, B), 8 waves x 16 queries.  S^T = K Q^T is computed "swapped" so the
// accumulator of S^T is directly the B operand of O^T = V^T P^T (k order permuted consistently,
// V^T read with ds_read_b64_tr_b16).  K/V tiles of 64 keys staged through LDS; online softmax.
// Stores LSE (natural log, scaled-score units) for the backward.  Attention-probability dropout
// (eager_attention_forward dropout(attn_weights), modeling_bert.py:131,198) is applied to P before PV with
// a Philox mask regenerated in the backward.
// Backward: grid (L/256, H, B), 8 waves x 32 keys; per 32-query chunk: S, P (from LSE), dP,
// dS = P (dP - rowsum(dO o O)); dV += P^T dO and dK += dS^T Q accumulate in registers; dS goes
// through LDS once for dQ = dS K.  With L <= 256 every dQ element is produced by exactly one
// workgroup (plain stores); for longer sequences dQ is accumulated with fp32 atomics.
#include "common.h"
#include "eegfusion_internal.h"

namespace {

constexpr int DH = 64;          // head dim
constexpr float NEG = -1e30f;   // masked-key score (finfo.min semantics: never NaN)

template <typename T> constexpr int pad16() { return 16 / (int)sizeof(T); }

struct AttnArgs {
  const void* qkv; void* out; float* lse; const float* kbias;
  const void* o; const void* dout; void* dqkv; float* dq_acc;
  int B, H, L; long ld_qkv, ld_out; float scale;
  float p; uint64_t seed, offset;   // attention-probability dropout (p = 0: off)
  uint32_t* bits;                   // dropout keep bits: written by the forward, read by the backward
  const int* cu;                    // varlen (packed rows): sequence b = rows cu[b] .. cu[b+1]-1, L = max length
};

// Dropout numbering of the attention probabilities (every attention kernel, so forward and backward
// agree): element (b, h, q, key) with key = 32 c + 16 j + 4 u + r is kept iff halfword 4 j + r of the
// Philox-7 call attn_call(b, h, q, c, u) is >= thr16 (keep_bits8 / philox4x32_r<7>, common.h).  The
// eight draws of a call are exactly the keys one MFMA lane (g = u) holds for query q in the forward's
// S^T layout (rows 4g + r of the 16-key blocks 2c and 2c + 1, i.e. one pack_acc fragment), so the
// forward applies them to its own probabilities with no cross-lane exchange.
DEV uint64_t attn_call(const AttnArgs& a, int b, int h, long q, long c, int u) {
  return (((uint64_t)b * a.H + h) * a.L + q) * (uint64_t)(4 * ((a.L + 31) >> 5)) + 4 * c + u;
}
// Forward layout: lane (g, li) of query q needs keys k0 + 16 f + 4 g + r (f = 0..3, k0 % 64 == 0):
// nib[f] bit r.  Calls (q, k0 / 32 + cc, g), cc = 0, 1, hold f = 2 cc (halfwords 0-3) and 2 cc + 1 (4-7).
DEV void attn_mask_fwd(const AttnArgs& a, int b, int h, long q, long k0, int g, uint32_t thr, uint32_t (&nib)[4]) {
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    const uint32_t bits = keep_bits8(a.seed, a.offset, attn_call(a, b, h, q, (k0 >> 5) + cc, g), thr);
    nib[2 * cc] = bits & 0xFu;
    nib[2 * cc + 1] = bits >> 4;
  }
}
// Backward layout: lane (g, li) needs mask[q0 + 16 qf + 4 g + r][kw + 16 f + li] as bit t = 4 qf + r of
// m8[f] (kw % 32 == 0).  The eight queries' calls of key group u = li >> 2 serve the whole lane quad
// (li & ~3 .. +3): lane al = li & 3 draws those of queries t = 2 al, 2 al + 1 and the quad exchanges
// the bytes; lane al keeps bit 4 f + al of every byte (key kw + 16 f + 4 u + al).
DEV void attn_mask_bwd(const AttnArgs& a, int b, int h, long q0, long kw, int lane, uint32_t thr, uint32_t (&m8)[2]) {
  const int g = lane >> 4, li = lane & 15, u = li >> 2, al = li & 3;
  uint32_t pair = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int t = 2 * al + k;
    pair |= keep_bits8(a.seed, a.offset, attn_call(a, b, h, q0 + 16 * (t >> 2) + 4 * g + (t & 3), kw >> 5, u), thr)
            << (8 * k);
  }
  m8[0] = m8[1] = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint32_t v = (uint32_t)__shfl((int)pair, (lane & ~3) | s, 64);    // bytes of queries 2 s, 2 s + 1
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int f = 0; f < 2; ++f) m8[f] |= ((v >> (8 * k + 4 * f + al)) & 1u) << (2 * s + k);
  }
}

// Keep bits of the attention-probability dropout, row-major per (b, h): word (q, j) of L/32 words per
// query row, bit t <-> key 32 j + t.  The forward stores them (a.bits non-null) so the backward reads
// them instead of regenerating the Philox stream.  Forward lane (g, li) of query q holds nib[f]
// (bit r <-> key k0 + 16 f + 4 g + r, f = 0..3, k0 % 64 == 0): the group's two words are OR-reduced
// over the 4 lanes g (all lanes must call this) and stored by lanes g = 0.
DEV void store_bits_fwd(const AttnArgs& a, int b, int h, long q, long k0, int g, const uint32_t (&nib)[4]) {
  uint32_t w0 = (nib[0] << (4 * g)) | (nib[1] << (16 + 4 * g));
  uint32_t w1 = (nib[2] << (4 * g)) | (nib[3] << (16 + 4 * g));
  w0 |= (uint32_t)__shfl_xor((int)w0, 16, 64);
  w1 |= (uint32_t)__shfl_xor((int)w1, 16, 64);
  w0 |= (uint32_t)__shfl_xor((int)w0, 32, 64);
  w1 |= (uint32_t)__shfl_xor((int)w1, 32, 64);
  if (g == 0) *(uint2*)(a.bits + (((long)b * a.H + h) * a.L + q) * (a.L / 32) + k0 / 32) = make_uint2(w0, w1);
}
// Backward layout of the same bits (as attn_mask_bwd): bit t8 <-> row 16 (t8 >> 2) + 4 g + (t8 & 3) of the
// rows starting at rowbits (wpr words per row), key kb + li.
DEV uint32_t load_bits_bwd(const uint32_t* rowbits, int wpr, long kb, int g, int li) {
  const int j = (int)((kb + li) >> 5), t = (int)((kb + li) & 31);
  uint32_t m = 0;
#pragma unroll
  for (int t8 = 0; t8 < 8; ++t8) m |= ((rowbits[(16 * (t8 >> 2) + 4 * g + (t8 & 3)) * wpr + j] >> t) & 1u) << t8;
  return m;
}

// Cooperative copy of `rows` x 64 elements (row stride `ld` in global) into LDS [rows][64+pad].
template <typename T, int NTHR>
DEV void stage_rows(T* lds, int ldl, const T* g, long ld, int rows, int tid) {
  constexpr int VE = 16 / (int)sizeof(T);
  constexpr int CPR = DH / VE;                 // 16-B chunks per row
  for (int c = tid; c < rows * CPR; c += NTHR) {
    const int r = c / CPR, cc = (c % CPR) * VE;
    st16(lds + r * ldl + cc, ld16(g + (long)r * ld + cc));
  }
}

// stage_rows for a ragged tail: rows >= valid are zero-filled (valid may be <= 0: all zero)
template <typename T, int NTHR>
DEV void stage_rows_vl(T* lds, int ldl, const T* g, long ld, int rows, int valid, int tid) {
  constexpr int VE = 16 / (int)sizeof(T);
  constexpr int CPR = DH / VE;
  for (int c = tid; c < rows * CPR; c += NTHR) {
    const int r = c / CPR, cc = (c % CPR) * VE;
    st16(lds + r * ldl + cc, r < valid ? ld16(g + (long)r * ld + cc) : u32x4{0u, 0u, 0u, 0u});
  }
}

// Sequence b of the launch: first row and length.  Dense: rows b*L .., length L.  Varlen (a.cu): the
// packed rows cu[b] .. cu[b+1]-1 (flash-attn cu_seqlens); the dropout element index keeps the padded
// (b, h, q, key) numbering with L = the padded length, so a packed batch draws the masks of its
// padded form.
template <bool VL>
DEV void attn_seq(const AttnArgs& a, int b, long& row0, int& len) {
  if (VL) { row0 = a.cu[b]; len = a.cu[b + 1] - a.cu[b]; }
  else { row0 = (long)b * a.L; len = a.L; }
}

template <typename T, bool VL = false>
__global__ void __launch_bounds__(512) attn_fwd_kernel(AttnArgs a) {
  using F = typename Frag8<T>::type;
  constexpr int KT = 64, LDK = DH + pad16<T>();
  __shared__ __attribute__((aligned(16))) T lds[2 * KT * LDK];
  T* Ks = lds;
  T* Vs = lds + KT * LDK;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y;
  long row0;
  int len;
  attn_seq<VL>(a, b, row0, len);
  if (VL && (int)blockIdx.x * 128 >= len) return;                   // uniform: past this sequence
  const int q = blockIdx.x * 128 + wave * 16 + li;                  // this lane's query (B/C column)
  const T* base = (const T*)a.qkv + row0 * a.ld_qkv;
  const T* Qg = base + h * DH;
  const T* Kg = base + 768 + h * DH;
  const T* Vg = base + 1536 + h * DH;
  const int qr = VL ? min(q, len - 1) : q;                          // ragged tail: clamped, never stored

  F qf[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) qf[c] = ld_row8(Qg + (long)qr * a.ld_qkv + 32 * c + 8 * g);

  f32x4 o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = f32x4{0, 0, 0, 0};
  float m = NEG, l = 0.f;
  const float* kb = a.kbias ? a.kbias + (long)b * a.L : nullptr;
  const uint32_t thr = thr16_of(a.p);
  const float dscale = 1.0f / (1.0f - a.p);

  for (int k0 = 0; k0 < len; k0 += KT) {
    __syncthreads();
    if (VL && k0 + KT > len) {
      stage_rows_vl<T, 512>(Ks, LDK, Kg + (long)k0 * a.ld_qkv, a.ld_qkv, KT, len - k0, tid);
      stage_rows_vl<T, 512>(Vs, LDK, Vg + (long)k0 * a.ld_qkv, a.ld_qkv, KT, len - k0, tid);
    } else {
      stage_rows<T, 512>(Ks, LDK, Kg + (long)k0 * a.ld_qkv, a.ld_qkv, KT, tid);
      stage_rows<T, 512>(Vs, LDK, Vg + (long)k0 * a.ld_qkv, a.ld_qkv, KT, tid);
    }
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      s[f] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int c = 0; c < 2; ++c) s[f] = mma16(ld_row8(Ks + (16 * f + li) * LDK + 32 * c + 8 * g), qf[c], s[f]);
    }
    // s[f][r]: key = k0 + 16f + 4g + r, query = q
    float tmax = NEG;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = s[f][r] * a.scale;
        const int key = k0 + 16 * f + 4 * g + r;
        // the key-bias row holds a.L entries: keys past the sequence are never read (a ragged or
        // uniform length below the 64-key block would read the next row / past the buffer)
        if (kb && (!VL || key < len)) v += kb[key];
        if (VL && key >= len) v = NEG;                                   // keys past the sequence
        s[f][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float alpha = __expf(m - mn);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s[f][r] = __expf(s[f][r] - mn); ps += s[f][r]; }
    l = l * alpha + ps;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] *= alpha;
    if (a.p > 0.f) {   // O accumulates dropout(P) V; the normaliser l stays the undropped sum
      uint32_t nib[4];
      attn_mask_fwd(a, b, h, q, k0, g, thr, nib);
      if (a.bits) store_bits_fwd(a, b, h, q, k0, g, nib);
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[f][r] = (nib[f] >> r) & 1u ? s[f][r] * dscale : 0.f;
    }
    // O^T[d, q] += sum_key V[key, d] P[q, key]   (k order: {4g..4g+3 of frag 2c, of frag 2c+1})
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const F pb = pack_acc<T>(s[2 * c], s[2 * c + 1]);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = mma16(ld_col4x2(Vs, LDK, 32 * c + 4 * g, 32 * c + 16 + 4 * g, 16 * e, lane), pb, o[e]);
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.0f / l;
  if (VL && q >= len) return;
  T* out = (T*)a.out + (row0 + q) * a.ld_out + h * DH;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    // o[e][r]: d = 16e + 4g + r
#pragma unroll
    for (int r = 0; r < 4; ++r) out[16 * e + 4 * g + r] = from_f32<T>(o[e][r] * inv);
  }
  if (g == 0) a.lse[((long)b * a.H + h) * a.L + q] = m + __logf(l);
}

template <typename T, bool VL = false>
__global__ void __launch_bounds__(512) attn_bwd_kernel(AttnArgs a) {
  using F = typename Frag8<T>::type;
  constexpr int KB = 256, QC = 32, LDK = DH + pad16<T>(), LDS_ = KB + pad16<T>();
  constexpr int SZ_K = KB * LDK, SZ_Q = QC * LDK, SZ_S = QC * LDS_;
  __shared__ __attribute__((aligned(16))) T lds[SZ_K + 3 * SZ_Q + SZ_S];
  __shared__ float lse_s[QC], dd_s[QC];
  T* Ks = lds;
  T* Qs = Ks + SZ_K;
  T* dOs = Qs + SZ_Q;
  T* Os = dOs + SZ_Q;
  T* dSs = Os + SZ_Q;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, li = lane & 15;
  const int b = blockIdx.z, h = blockIdx.y, kb0 = blockIdx.x * KB;
  long row0;
  int len;
  attn_seq<VL>(a, b, row0, len);
  if (VL && kb0 >= len) return;                                     // uniform: past this sequence
  const int kw0 = kb0 + wave * 32;                                    // this wave's 32 keys
  const T* base = (const T*)a.qkv + row0 * a.ld_qkv;
  const T* Qg = base + h * DH;
  const T* Kg = base + 768 + h * DH;
  const T* Vg = base + 1536 + h * DH;
  const T* Og = (const T*)a.o + row0 * a.ld_out + h * DH;
  const T* dOg = (const T*)a.dout + row0 * a.ld_out + h * DH;
  const float* lse = a.lse + ((long)b * a.H + h) * a.L;
  const float* kbias = a.kbias ? a.kbias + (long)b * a.L : nullptr;
  // dQ: one key block per sequence -> plain stores; varlen always sums through dq_acc when any
  // sequence may span two blocks (L > 256), so every row of the launch takes one path
  const int nkb = VL ? (a.L > KB ? 2 : 1) : a.L / KB;
  const uint32_t thr = thr16_of(a.p);
  const float dscale = 1.0f / (1.0f - a.p);

  // this wave's K and V as B operands (key = column): lane holds [key kw0+16f+li][d 32c+8g..]
  F kf[2][2], vf[2][2];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int kr = VL ? min(kw0 + 16 * f + li, len - 1) : kw0 + 16 * f + li;
      kf[f][c] = ld_row8(Kg + (long)kr * a.ld_qkv + 32 * c + 8 * g);
      vf[f][c] = ld_row8(Vg + (long)kr * a.ld_qkv + 32 * c + 8 * g);
    }
  float kbv[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    // keys past the sequence: p = 0, and their bias is never read (the 256-key block of a uniform
    // launch with L < 256 would read the next row's bias / past the end of the buffer)
    const int key = kw0 + 16 * f + li;
    kbv[f] = (VL && key >= len) ? NEG : (kbias ? kbias[key] : 0.f);
  }

  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e) { dk[f][e] = f32x4{0, 0, 0, 0}; dv[f][e] = f32x4{0, 0, 0, 0}; }

  if (VL) stage_rows_vl<T, 512>(Ks, LDK, Kg + (long)kb0 * a.ld_qkv, a.ld_qkv, KB, len - kb0, tid);
  else stage_rows<T, 512>(Ks, LDK, Kg + (long)kb0 * a.ld_qkv, a.ld_qkv, KB, tid);

  for (int q0 = 0; q0 < len; q0 += QC) {
    __syncthreads();
    if (VL) {      // rows past the sequence zero-filled: they add nothing to dK / dV
      stage_rows_vl<T, 512>(Qs, LDK, Qg + (long)q0 * a.ld_qkv, a.ld_qkv, QC, len - q0, tid);
      stage_rows_vl<T, 512>(dOs, LDK, dOg + (long)q0 * a.ld_out, a.ld_out, QC, len - q0, tid);
      stage_rows_vl<T, 512>(Os, LDK, Og + (long)q0 * a.ld_out, a.ld_out, QC, len - q0, tid);
    } else {
      stage_rows<T, 512>(Qs, LDK, Qg + (long)q0 * a.ld_qkv, a.ld_qkv, QC, tid);
      stage_rows<T, 512>(dOs, LDK, dOg + (long)q0 * a.ld_out, a.ld_out, QC, tid);
      stage_rows<T, 512>(Os, LDK, Og + (long)q0 * a.ld_out, a.ld_out, QC, tid);
    }
    if (tid < QC) lse_s[tid] = (!VL || q0 + tid < len) ? lse[q0 + tid] : 0.f;
    __syncthreads();
    {  // D[q] = sum_d dO[q,d] O[q,d]: 16 lanes per query
      const int qq = tid >> 4, part = tid & 15;
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < 4; ++d) acc += to_f32(dOs[qq * LDK + part * 4 + d]) * to_f32(Os[qq * LDK + part * 4 + d]);
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 16);
      if (part == 0) dd_s[qq] = acc;
    }
    __syncthreads();
    // S = Q K^T and dP = dO V^T : rows = queries (4g+r within q-frag), cols = keys (li)
    f32x4 p[2][2], ds[2][2];
    uint32_t m8[2] = {0xFFu, 0xFFu};
    if (a.p > 0.f) {
      if (a.bits) {
#pragma unroll
        for (int f = 0; f < 2; ++f)
          m8[f] = load_bits_bwd(a.bits + (((long)b * a.H + h) * a.L + q0) * (a.L / 32), a.L / 32, kw0 + 16 * f, g, li);
      } else {
        attn_mask_bwd(a, b, h, q0, kw0, lane, thr, m8);
      }
    }
#pragma unroll
    for (int qf = 0; qf < 2; ++qf) {
      F qa[2], da[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        qa[c] = ld_row8(Qs + (16 * qf + li) * LDK + 32 * c + 8 * g);
        da[c] = ld_row8(dOs + (16 * qf + li) * LDK + 32 * c + 8 * g);
      }
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        f32x4 s = f32x4{0, 0, 0, 0}, dp = f32x4{0, 0, 0, 0};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          s = mma16(qa[c], kf[f][c], s);
          dp = mma16(da[c], vf[f][c], dp);
        }
        // with dropout Z: O = (P o Z) V, so dV uses P o Z and dP = Z o (dO V^T); D = rowsum(dO o O)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qi = 16 * qf + 4 * g + r;
          float pv = __expf(s[r] * a.scale + kbv[f] - lse_s[qi]);
          if (VL && q0 + qi >= len) pv = 0.f;                          // query rows past the sequence
          const float mk = (m8[f] >> (4 * qf + r)) & 1u ? dscale : 0.f;
          s[r] = pv * mk;
          dp[r] = pv * (dp[r] * mk - dd_s[qi]);
        }
        p[qf][f] = s;
        ds[qf][f] = dp;
      }
    }
    // dV[key, d] += sum_q P[q,key] dO[q,d];  dK[key, d] += sum_q dS[q,key] Q[q,d]
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const F pa = pack_acc<T>(p[0][f], p[1][f]);
      const F sa = pack_acc<T>(ds[0][f], ds[1][f]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dv[f][e] = mma16(pa, ld_col4x2(dOs, LDK, 4 * g, 16 + 4 * g, 16 * e, lane), dv[f][e]);
        dk[f][e] = mma16(sa, ld_col4x2(Qs, LDK, 4 * g, 16 + 4 * g, 16 * e, lane), dk[f][e]);
      }
    }
    // dS -> LDS [q][key - kb0]
#pragma unroll
    for (int qf = 0; qf < 2; ++qf)
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          dSs[(16 * qf + 4 * g + r) * LDS_ + wave * 32 + 16 * f + li] = from_f32<T>(ds[qf][f][r]);
    __syncthreads();
    {  // dQ[q, d] = scale * sum_key dS[q,key] K[key,d]; wave -> (q-frag w>>2, d-frag w&3)
      const int qf = wave >> 2, e = wave & 3;
      f32x4 acc = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int kc = 0; kc < KB / 32; ++kc)
        acc = mma16(ld_row8(dSs + (16 * qf + li) * LDS_ + 32 * kc + 8 * g),
                    ld_col8(Ks, LDK, 32 * kc + 8 * g, 16 * e, lane), acc);
      // acc[r]: q = q0 + 16qf + 4g + r, d = 16e + li
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (VL && q0 + 16 * qf + 4 * g + r >= len) continue;
        const long qrow = row0 + q0 + 16 * qf + 4 * g + r;
        const int d = 16 * e + li;
        if (nkb == 1) ((T*)a.dqkv)[qrow * a.ld_qkv + h * DH + d] = from_f32<T>(acc[r] * a.scale);
        else atomicAdd(a.dq_acc + qrow * 768 + h * DH + d, acc[r] * a.scale);
      }
    }
  }
  // write dK, dV: dk[f][e][r] / dv[f][e][r] hold key kw0 + 16f + 4g + r, d = 16e + li
  T* dqkv = (T*)a.dqkv + row0 * a.ld_qkv;
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long key = kw0 + 16 * f + 4 * g + r;
        if (VL && key >= len) continue;
        const int d = 16 * e + li;
        dqkv[key * a.ld_qkv + 768 + h * DH + d] = from_f32<T>(dk[f][e][r] * a.scale);
        dqkv[key * a.ld_qkv + 1536 + h * DH + d] = from_f32<T>(dv[f][e][r]);
      }
}

__global__ void dq_convert_kernel(const float* dq_acc, void* dqkv, int is_bf16, long rows, long ld) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * 768) return;
  const long r = i / 768, c = i % 768;
  if (is_bf16) ((bf16*)dqkv)[r * ld + c] = (bf16)dq_acc[i];
  else ((float*)dqkv)[r * ld + c] = dq_acc[i];
}

#include "attention256.inc"

}  // namespace

int persistent_cus();    // gemm_big.hip: CU count minus the eegf_tune key 13 reserve

namespace {
// persistent L = 256 kernels: one workgroup per CU (capped by the item count)
int l256_grid(int items) {
  const int cus = persistent_cus();
  return items < cus ? items : cus;
}
}  // namespace

// Which directions take the L = 256 kernels: bit 0 forward, bit 1 backward (eegf_tune key 2,
// initial value from EEGF_ATTN256 = 0 / fwd / bwd / all).  Default both: B=256, p=0.1 the persistent
// backward takes 399 us against 473 for attn_bwd_kernel (profiles/r2g_attn_ab.log).
int g_attn256_mode = [] {
  const char* e = getenv("EEGF_ATTN256");
  if (!e) return 3;
  if (e[0] == '0') return 0;
  if (e[0] == 'b') return 2;
  if (e[0] == 'a') return 3;
  return 1;
}();

namespace {
// the L = 256 kernels draw with 32-bit call numbers (keep01x8_c32 / keep_bits8_c32): every call of the
// launch, < B H L 4 ceil(L / 32), must fit (B <= 43690 at H = 12); larger B runs the generic kernels
// and they index in 32 bits (attention256.inc): every element offset (rows x the larger stride, the
// keep-bit bytes) must stay below 2^31
bool l256_path(int dtype, int B, int H, int L, const float* key_bias, bool bwd, long ld_qkv, long ld_out) {
  const bool c32 = (uint64_t)B * H * L * 4 * ((L + 31) / 32) <= (1ull << 32);
  const bool i32 = (uint64_t)B * L * (uint64_t)(ld_qkv > ld_out ? ld_qkv : ld_out) < (1ull << 31) &&
                   (uint64_t)B * H * L * (L / 8) < (1ull << 31);
  return (g_attn256_mode & (bwd ? 2 : 1)) && dtype == EEGF_BF16 && L == LF && H == 12 && !key_bias && c32 && i32;
}

}  // namespace

extern "C" int eegf_attn_fwd(int dtype, int B, int H, int L, const void* qkv, long ld_qkv, const float* key_bias,
                             float scale, float drop_p, unsigned long long seed, unsigned long long offset,
                             void* out, long ld_out, float* lse, unsigned int* drop_bits, hipStream_t stream) {
  if (B <= 0 || H != 12 || L <= 0 || L % 128 != 0 || !qkv || !out || !lse || ld_qkv < 2304 || ld_out < 768)
    return EEGF_ERR_ARG;
  if (B > 65535 || drop_p < 0.f || drop_p >= 1.f) return EEGF_ERR_ARG;
  AttnArgs a{qkv, out, lse, key_bias, nullptr, nullptr, nullptr, nullptr, B, H, L, ld_qkv, ld_out, scale,
             drop_p, seed, offset, drop_p > 0.f ? drop_bits : nullptr};
  if (l256_path(dtype, B, H, L, key_bias, false, ld_qkv, ld_out)) {
    const dim3 g1(l256_grid(B * H));
    if (a.bits) EEGF_LAUNCH((attn_fwd256_kernel<true, true>), g1, dim3(512), 0, stream, a);
    else if (drop_p > 0.f) EEGF_LAUNCH(attn_fwd256_kernel<true>, g1, dim3(512), 0, stream, a);
    else EEGF_LAUNCH(attn_fwd256_kernel<false>, g1, dim3(512), 0, stream, a);
    return (int)hipGetLastError();
  }
  const dim3 grid(L / 128, H, B);
  if (dtype == EEGF_F32) EEGF_LAUNCH(attn_fwd_kernel<float>, grid, dim3(512), 0, stream, a);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(attn_fwd_kernel<bf16>, grid, dim3(512), 0, stream, a);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" long eegf_attn_bwd_workspace(int B, int L) { return L > 256 ? (long)B * L * 768 : 0; }

extern "C" int eegf_attn_bwd(int dtype, int B, int H, int L, const void* qkv, long ld_qkv, const float* key_bias,
                             float scale, float drop_p, unsigned long long seed, unsigned long long offset,
                             const void* out, const void* dout, long ld_out, const float* lse,
                             const unsigned int* drop_bits, void* dqkv, float* dq_workspace, hipStream_t stream) {
  if (B <= 0 || H != 12 || L <= 0 || L % 256 != 0 || !qkv || !out || !dout || !lse || !dqkv) return EEGF_ERR_ARG;
  if (ld_qkv < 2304 || ld_out < 768 || B > 65535 || drop_p < 0.f || drop_p >= 1.f) return EEGF_ERR_ARG;
  if (L > 256 && !dq_workspace) return EEGF_ERR_ARG;
  if (L > 256) hipMemsetAsync(dq_workspace, 0, sizeof(float) * (size_t)B * L * 768, stream);
  AttnArgs a{qkv, nullptr, const_cast<float*>(lse), key_bias, out, dout, dqkv, dq_workspace, B, H, L, ld_qkv, ld_out,
             scale, drop_p, seed, offset, drop_p > 0.f ? const_cast<uint32_t*>(drop_bits) : nullptr};
  if (l256_path(dtype, B, H, L, key_bias, true, ld_qkv, ld_out)) {
    const dim3 g1(l256_grid(B * H));
    if (drop_p > 0.f) EEGF_LAUNCH(attn_bwd256_kernel<true>, g1, dim3(512), 0, stream, a);
    else EEGF_LAUNCH(attn_bwd256_kernel<false>, g1, dim3(512), 0, stream, a);
    return (int)hipGetLastError();
  }
  const dim3 grid(L / 256, H, B);
  if (dtype == EEGF_F32) EEGF_LAUNCH(attn_bwd_kernel<float>, grid, dim3(512), 0, stream, a);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(attn_bwd_kernel<bf16>, grid, dim3(512), 0, stream, a);
  else return EEGF_ERR_ARG;
  if (L > 256) {
    const long n = (long)B * L * 768;
    EEGF_LAUNCH(dq_convert_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, dq_workspace, dqkv,
                       dtype == EEGF_BF16, (long)B * L, ld_qkv);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Varlen (packed) self-attention for contract T pad skipping: the padded keys of
// BertSelfAttention are masked (model.py:43, modeling_bert.py extended mask), so the packed rows of
// each sequence give the real rows' outputs of the padded computation exactly.
extern "C" int eegf_attn_varlen_fwd(int dtype, int B, int H, int max_len, const int* cu_seqlens, long packed_rows,
                                    long total_rows, const void* qkv, long ld_qkv, const float* key_bias,
                                    float scale, float drop_p,
                                    unsigned long long seed, unsigned long long offset, void* out, long ld_out,
                                    float* lse, hipStream_t stream) {
  if (B <= 0 || B > 65535 || H != 12 || max_len <= 0 || !cu_seqlens || !qkv || !out || !lse) return EEGF_ERR_ARG;
  if (ld_qkv < 2304 || ld_out < 768 || drop_p < 0.f || drop_p >= 1.f || packed_rows < 0 || total_rows < packed_rows)
    return EEGF_ERR_ARG;
  const size_t es = dtype == EEGF_BF16 ? 2 : dtype == EEGF_F32 ? 4 : 0;
  if (!es) return EEGF_ERR_ARG;
  if (total_rows > packed_rows)        // rows past the packed sequences: defined zeros
    hipMemsetAsync((char*)out + packed_rows * ld_out * es, 0, (total_rows - packed_rows) * ld_out * es, stream);
  AttnArgs a{qkv, out, lse, key_bias, nullptr, nullptr, nullptr, nullptr, B, H, max_len, ld_qkv, ld_out, scale,
             drop_p, seed, offset, nullptr, cu_seqlens};
  const dim3 grid((max_len + 127) / 128, H, B);
  if (dtype == EEGF_F32) EEGF_LAUNCH((attn_fwd_kernel<float, true>), grid, dim3(512), 0, stream, a);
  else EEGF_LAUNCH((attn_fwd_kernel<bf16, true>), grid, dim3(512), 0, stream, a);
  return (int)hipGetLastError();
}

extern "C" long eegf_attn_varlen_bwd_workspace(long total_rows, int max_len) {
  return max_len > 256 ? total_rows * 768 : 0;
}

extern "C" int eegf_attn_varlen_bwd(int dtype, int B, int H, int max_len, const int* cu_seqlens, long packed_rows,
                                    long total_rows, const void* qkv, long ld_qkv, const float* key_bias,
                                    float scale, float drop_p,
                                    unsigned long long seed, unsigned long long offset, const void* out,
                                    const void* dout, long ld_out, const float* lse, void* dqkv, float* dq_workspace,
                                    hipStream_t stream) {
  if (B <= 0 || B > 65535 || H != 12 || max_len <= 0 || !cu_seqlens || !qkv || !out || !dout || !lse || !dqkv)
    return EEGF_ERR_ARG;
  if (ld_qkv < 2304 || ld_out < 768 || drop_p < 0.f || drop_p >= 1.f || packed_rows < 0 || total_rows < packed_rows)
    return EEGF_ERR_ARG;
  if (max_len > 256 && !dq_workspace) return EEGF_ERR_ARG;
  const size_t es = dtype == EEGF_BF16 ? 2 : dtype == EEGF_F32 ? 4 : 0;
  if (!es) return EEGF_ERR_ARG;
  if (total_rows > packed_rows)
    hipMemsetAsync((char*)dqkv + packed_rows * ld_qkv * es, 0, (total_rows - packed_rows) * ld_qkv * es, stream);
  if (max_len > 256) hipMemsetAsync(dq_workspace, 0, sizeof(float) * (size_t)total_rows * 768, stream);
  AttnArgs a{qkv, nullptr, const_cast<float*>(lse), key_bias, out, dout, dqkv, dq_workspace, B, H, max_len, ld_qkv,
             ld_out, scale, drop_p, seed, offset, nullptr, cu_seqlens};
  const dim3 grid((max_len + 255) / 256, H, B);
  if (dtype == EEGF_F32) EEGF_LAUNCH((attn_bwd_kernel<float, true>), grid, dim3(512), 0, stream, a);
  else EEGF_LAUNCH((attn_bwd_kernel<bf16, true>), grid, dim3(512), 0, stream, a);
  if (max_len > 256) {
    const long n = total_rows * 768;
    EEGF_LAUNCH(dq_convert_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, dq_workspace, dqkv,
                       dtype == EEGF_BF16, total_rows, ld_qkv);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Self-attention over a handful of tokens (S <= 8): the TransformerEncoder of TISC_LapDropout runs
// its 12-head attention over the 2 tokens [mean(EEG sequence), action] of each sample
// (custom_models/models.py:227-228, :258-260; F.multi_head_attention_forward).  One wave per
// (sample n, head h), lane = head dimension d: q_i . k_j by wave reductions, softmax over j, the
// attention-weight dropout (Philox element ((n*12 + h)*S + i)*S + j, drop_mask1), ctx_i = sum_j p~_ij v_j.
// Rows of sample n are n*S .. n*S + S-1 of qkv [N*S, 3*768] / out [N*S, 768].  probs (undropped
// softmax, [N, 12, S, S] fp32) is saved for the backward.
namespace {
constexpr int SMAX = 8;

template <typename T>
__global__ void __launch_bounds__(64) attn_small_fwd_kernel(int S, const T* __restrict__ qkv, long ld, float scale,
                                                            float p, uint64_t seed, uint64_t offset, T* __restrict__ out,
                                                            long ldo, float* __restrict__ probs) {
  const int n = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  float q[SMAX], k[SMAX], v[SMAX];
  for (int i = 0; i < S; ++i) {
    const T* r = qkv + ((long)n * S + i) * ld + h * DH + d;
    q[i] = to_f32(r[0]) * scale;
    k[i] = to_f32(r[768]);
    v[i] = to_f32(r[1536]);
  }
  const float dscale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  for (int i = 0; i < S; ++i) {
    float sc[SMAX], mx = -INFINITY;
    for (int j = 0; j < S; ++j) {
      sc[j] = wave_sum(q[i] * k[j]);
      mx = fmaxf(mx, sc[j]);
    }
    float den = 0.f;
    for (int j = 0; j < S; ++j) { sc[j] = expf(sc[j] - mx); den += sc[j]; }
    float o = 0.f;
    for (int j = 0; j < S; ++j) {
      const float pij = sc[j] / den;
      const long e = (((long)n * 12 + h) * S + i) * S + j;
      if (d == 0) probs[e] = pij;
      const float m = p > 0.f ? drop_mask1(seed, offset, (uint64_t)e, p) : dscale;
      o += pij * m * v[j];
    }
    out[((long)n * S + i) * ldo + h * DH + d] = from_f32<T>(o);
  }
}

// dV_j = sum_i p~_ij dctx_i; dp~_ij = dctx_i . v_j; dp_ij = m_ij dp~_ij; ds_ij = p_ij (dp_ij - sum_k p_ik dp_ik);
// dq_i = scale sum_j ds_ij k_j; dk_j = scale sum_i ds_ij q_i
template <typename T>
__global__ void __launch_bounds__(64) attn_small_bwd_kernel(int S, const T* __restrict__ qkv, long ld,
                                                            const float* __restrict__ probs, const T* __restrict__ dout,
                                                            long ldo, float scale, float p, uint64_t seed,
                                                            uint64_t offset, T* __restrict__ dqkv, long ldd) {
  const int n = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  float q[SMAX], k[SMAX], v[SMAX], g[SMAX], dq[SMAX], dk[SMAX], dv[SMAX];
  for (int i = 0; i < S; ++i) {
    const T* r = qkv + ((long)n * S + i) * ld + h * DH + d;
    q[i] = to_f32(r[0]);
    k[i] = to_f32(r[768]);
    v[i] = to_f32(r[1536]);
    g[i] = to_f32(dout[((long)n * S + i) * ldo + h * DH + d]);
    dq[i] = dk[i] = dv[i] = 0.f;
  }
  const float dscale = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  for (int i = 0; i < S; ++i) {
    float pr[SMAX], dp[SMAX], sdot = 0.f;
    for (int j = 0; j < S; ++j) {
      const long e = (((long)n * 12 + h) * S + i) * S + j;
      pr[j] = probs[e];
      const float m = p > 0.f ? drop_mask1(seed, offset, (uint64_t)e, p) : dscale;
      dv[j] += pr[j] * m * g[i];
      dp[j] = m * wave_sum(g[i] * v[j]);
      sdot += pr[j] * dp[j];
    }
    for (int j = 0; j < S; ++j) {
      const float ds = pr[j] * (dp[j] - sdot) * scale;
      dq[i] += ds * k[j];
      dk[j] += ds * q[i];
    }
  }
  for (int i = 0; i < S; ++i) {
    T* r = dqkv + ((long)n * S + i) * ldd + h * DH + d;
    r[0] = from_f32<T>(dq[i]);
    r[768] = from_f32<T>(dk[i]);
    r[1536] = from_f32<T>(dv[i]);
  }
}
}  // namespace

extern "C" int eegf_attn_small_fwd(int dtype, int N, int S, const void* qkv, long ld_qkv, float scale, float drop_p,
                                   unsigned long long seed, unsigned long long offset, void* out, long ld_out,
                                   float* probs, hipStream_t stream) {
  if (N <= 0 || N > 65535 || S <= 0 || S > SMAX || !qkv || !out || !probs || ld_qkv < 2304 || ld_out < 768 ||
      drop_p < 0.f || drop_p >= 1.f)
    return EEGF_ERR_ARG;
  const dim3 grid(N, 12);
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(attn_small_fwd_kernel<float>, grid, dim3(64), 0, stream, S, (const float*)qkv, ld_qkv, scale,
                       drop_p, seed, offset, (float*)out, ld_out, probs);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(attn_small_fwd_kernel<bf16>, grid, dim3(64), 0, stream, S, (const bf16*)qkv, ld_qkv, scale,
                       drop_p, seed, offset, (bf16*)out, ld_out, probs);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_attn_small_bwd(int dtype, int N, int S, const void* qkv, long ld_qkv, const float* probs,
                                   const void* dout, long ld_out, float scale, float drop_p, unsigned long long seed,
                                   unsigned long long offset, void* dqkv, long ld_dqkv, hipStream_t stream) {
  if (N <= 0 || N > 65535 || S <= 0 || S > SMAX || !qkv || !probs || !dout || !dqkv || ld_qkv < 2304 ||
      ld_out < 768 || ld_dqkv < 2304 || drop_p < 0.f || drop_p >= 1.f)
    return EEGF_ERR_ARG;
  const dim3 grid(N, 12);
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(attn_small_bwd_kernel<float>, grid, dim3(64), 0, stream, S, (const float*)qkv, ld_qkv, probs,
                       (const float*)dout, ld_out, scale, drop_p, seed, offset, (float*)dqkv, ld_dqkv);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(attn_small_bwd_kernel<bf16>, grid, dim3(64), 0, stream, S, (const bf16*)qkv, ld_qkv, probs,
                       (const bf16*)dout, ld_out, scale, drop_p, seed, offset, (bf16*)dqkv, ld_dqkv);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}
