// common.h — shared device helpers for the EEG+action fusion path (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this directory:
//   * element type T is either `float` (fp32 parity mode) or `bf16` (performance mode);
//     accumulation is always fp32.
//   * an MFMA "k32 fragment" is 8 consecutive contraction-axis elements held by one lane:
//       lane l, group g = l >> 4, owns k = 8g .. 8g+7 of a 32-deep chunk,
//       row/col index = l & 15 of a 16-wide tile.
//     bf16 consumes it in one v_mfma_f32_16x16x32_bf16; fp32 consumes it as eight
//     v_mfma_f32_16x16x4_f32 (lane group g feeds k = 8g+t to instruction t).  Both sum the
//     same 32 products, so every kernel is written once for both precisions.
//   * C/D layout of a 16x16 accumulator: col = l & 15, row = 4*(l >> 4) + reg.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) float f32x8;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

template <typename T> struct Frag8;
template <> struct Frag8<bf16> { typedef bf16x8 type; };
template <> struct Frag8<float> { typedef f32x8 type; };

#define DEV __device__ __forceinline__

// LDS-DMA (global_load_lds_dwordx4: 16 B per lane, written lane-linearly from the wave-uniform
// LDS address lds_base) issued as inline asm.  With the builtin, hipcc's waitcnt pass puts an
// s_waitcnt vmcnt(0) in front of every ds_read_b64_tr_b16 that follows an LDS-DMA (it cannot tell
// which LDS the transpose read touches), which drains the staging pipeline of every kernel that
// reads a k-major operand.  Hidden in asm, the DMA is invisible to the pass: its completion is
// tracked by the kernels' own counted s_waitcnt vmcnt + barriers (the pass's waits for ordinary
// loads only get more conservative, never wrong: vmcnt retires in order).  M0 is set in the same
// asm statement; nothing else in these kernels uses M0.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
DEV void glds16_asm(const void* g, const void* lds_base) {
  typedef __attribute__((address_space(3))) void lv;
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lv*)lds_base);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(l) : "memory", "m0");
}
// saddr form: wave-uniform 64-bit base + per-lane 32-bit byte offset (no 64-bit address VGPRs).
// Wait states: the base SGPRs are often written by a VALU just before the statement
// (v_readfirstlane_b32 below, or v_readlane_b32 restoring a spilled SGPR), and a VMEM instruction
// reading an SGPR a VALU wrote needs 5 wait states, which hipcc does not insert inside asm.  The
// s_mov to M0 (1) + s_nop 3 (4) give 5; they also cover the 1 state the LDS-DMA needs after the M0
// write.  tools/isa_lint.py checks every LDS-DMA of the built library for both hazards.
DEV void glds16_asm_s(const void* base, uint32_t voff, const void* lds_base) {
  typedef __attribute__((address_space(3))) void lv;
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lv*)lds_base);
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const uint64_t bu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 3\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(bu), "s"(l)
               : "memory", "m0");
}
// saddr form with a 32-bit LDS byte address (no generic->LDS pointer cast per call) and a base the
// caller knows to be wave-uniform
// EEGF_DMA_POL: cache-policy bits of the saddr LDS-DMA (diagnostic A/B builds; default none)
#ifndef EEGF_DMA_POL
#define EEGF_DMA_POL ""
#endif
// NOP: wait states after the M0 write (s_nop NOP).  3 (default) covers a base a VALU wrote just before
// the statement; callers whose bases are SALU-computed may pass 0 (the 1 state the DMA needs after the M0
// write) -- tools/isa_lint.py / tests/test_isa_lint_cpu.py check every site of the built library.
template <int NOP = 3>
DEV void glds16_asm_sa(const void* base, uint32_t voff, uint32_t lds_addr) {
  // readfirstlane: a no-op on a base the compiler already keeps in SGPRs, and it keeps the "s"
  // constraint satisfiable when control flow elsewhere in the kernel makes it place the base in VGPRs
  const uint64_t b = (uint64_t)(uintptr_t)base;
  const uint64_t bu = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop %3\n\tglobal_load_lds_dwordx4 %0, %1" EEGF_DMA_POL ::"v"(voff), "s"(bu),
               "s"(lds_addr), "i"(NOP) : "memory", "m0");
}
DEV uint32_t lds_addr_of(const void* p) {
  typedef __attribute__((address_space(3))) void lv;
  return (uint32_t)(uintptr_t)(lv*)p;
}
#pragma clang diagnostic pop

DEV float to_f32(float x) { return x; }
DEV float to_f32(bf16 x) { return (float)x; }
template <typename T> DEV T from_f32(float x);
template <> DEV float from_f32<float>(float x) { return x; }
template <> DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }

DEV f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
DEV f32x4 mma16(f32x8 a, f32x8 b, f32x4 c) {
#pragma unroll
  for (int t = 0; t < 8; ++t) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[t], c, 0, 0, 0);
  return c;
}

// 8 contiguous elements (16-B aligned) from LDS or global.
DEV bf16x8 ld_row8(const bf16* p) { return *(const bf16x8*)p; }
DEV f32x8 ld_row8(const float* p) {
  f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  f32x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// 8 elements down a column of an LDS tile stored [k][col] with leading dimension ld:
// returns tile[(k0 + j) * ld + c0 + (lane & 15)], j = 0..7.
// bf16 uses two ds_read_b64_tr_b16 (lane 4q+p of a 16-group addresses row q, cols 4p..4p+3;
// lane i receives column i of the 4 rows).  k0 may differ per 16-lane group.
DEV bf16x8 ld_col8(const bf16* tile, int ld, int k0, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const bf16* a0 = tile + (k0 + q) * ld + c0 + 4 * p;
  const bf16* a1 = a0 + 4 * ld;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
DEV f32x8 ld_col8(const float* tile, int ld, int k0, int c0, int lane) {
  f32x8 r;
  const float* p = tile + k0 * ld + c0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = p[j * ld];
  return r;
}

// Same as ld_col8 but for a "split" k pattern: rows k0+0..3 and k1+0..3
// (used when an accumulator tile is re-used as an operand; see attention kernels).
DEV bf16x8 ld_col4x2(const bf16* tile, int ld, int k0, int k1, int c0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const bf16* a0 = tile + (k0 + q) * ld + c0 + 4 * p;
  const bf16* a1 = tile + (k1 + q) * ld + c0 + 4 * p;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
DEV f32x8 ld_col4x2(const float* tile, int ld, int k0, int k1, int c0, int lane) {
  f32x8 r;
  const float* p0 = tile + k0 * ld + c0 + (lane & 15);
  const float* p1 = tile + k1 * ld + c0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) { r[j] = p0[j * ld]; r[4 + j] = p1[j * ld]; }
  return r;
}

// Pack two accumulator tiles (rows 4g+r of tile a and of tile b) into one k32 operand
// fragment whose k order is {4g+0..3 of a, 4g+0..3 of b}.  The partner operand must use
// the same permuted k order (ld_col4x2 with k0 = 4g, k1 = 16 + 4g).
template <typename T> DEV typename Frag8<T>::type pack_acc(f32x4 a, f32x4 b);
template <> DEV bf16x8 pack_acc<bf16>(f32x4 a, f32x4 b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}
template <> DEV f32x8 pack_acc<float>(f32x4 a, f32x4 b) {
  f32x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// 16-byte vector load/store of raw bytes
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
DEV u32x4 ld16(const void* p) { return *(const u32x4*)p; }
DEV void st16(void* p, u32x4 v) { *(u32x4*)p = v; }

// wave reductions (64 lanes)
DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
DEV float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
// torch.relu: NaN propagates (fmaxf(NaN, 0) would return 0 and hide a NaN row from the forward
// while the backward's 0 * NaN still poisons the gradients)
DEV float relu_nan(float v) { return v < 0.f ? 0.f : v; }

// XCD-aware bijective remap of a 1-D block id (blocks b and b+8 share an XCD under the
// observed round-robin dispatch; this makes consecutive logical tiles share one XCD's L2).
DEV int xcd_remap(int orig, int nwg) {
  if (nwg < 16) return orig;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// erf(x/sqrt 2) by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7), sharing exp(-x^2/2) with the
// GELU derivative: one v_exp + one v_rcp instead of the library erff's branchy polynomial.
DEV float erf_half(float x, float e) {            // e = exp(-x*x/2)
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __frcp_rn(1.0f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return copysignf(1.0f - poly * e, x);
}
DEV float gelu_f(float x) {
  const float e = __expf(-0.5f * x * x);
  return 0.5f * x * (1.0f + erf_half(x, e));
}
DEV float gelu_grad(float x) {
  const float e = __expf(-0.5f * x * x);
  return 0.5f * (1.0f + erf_half(x, e)) + x * 0.39894228040143268f * e;
}
// Packed-fp32 GELU on pairs: the upper normal tail q = 1 - Phi(|x|) = phi(x) t P(t), t = 1 / (1 + p |x|)
// (A&S 26.2.17, the same approximation as erf_half's 7.1.26 with its constants folded: |error| of Phi
// <= 7.5e-8), phi(x) = exp2(-x^2 log2(e) / 2 - log2(sqrt(2 pi))) the normal density, so
// Phi(x) = 0.5 + copysign(0.5 - q, x), gelu = x Phi and gelu' = Phi + x phi.  19 VALU per pair (gelu'), 18
// (gelu): the epilogue that runs it is VALU-issue-bound (profiles/r5d_sink_ab.log, r5j_*).
typedef float f32x2 __attribute__((ext_vector_type(2)));
DEV void gelu2(f32x2 x, f32x2& gl, f32x2* gd) {
  const f32x2 x2 = x * x;
  const f32x2 ea = x2 * (-0.72134752044448170f) + (-1.3257480647361593f);     // log2 phi(x)
  f32x2 e;                                                                     // phi(x)
  e.x = __builtin_amdgcn_exp2f(ea.x);
  e.y = __builtin_amdgcn_exp2f(ea.y);
  f32x2 t;                               // scalar FMAs take |x| as a free source modifier
  t.x = __builtin_amdgcn_rcpf(fmaf(fabsf(x.x), 0.23164188826636040f, 1.0f));
  t.y = __builtin_amdgcn_rcpf(fmaf(fabsf(x.y), 0.23164188826636040f, 1.0f));
  f32x2 poly = t * 1.3302744295891231f + (-1.8212559791077754f);
  poly = poly * t + 1.7814779365698128f;
  poly = poly * t + (-0.35656378124891560f);
  poly = poly * t + 0.31938153025994087f;
  poly = poly * t;
  const f32x2 qm = poly * e + (-0.5f);                                         // q - 0.5 <= 0
  f32x2 us;                                                                    // sign(x) (0.5 - q)
  us.x = copysignf(qm.x, x.x);
  us.y = copysignf(qm.y, x.y);
  const f32x2 h = us + 0.5f;                                                   // Phi(x)
  gl = x * h;
  if (gd) *gd = x * e + h;                                                     // Phi(x) + x phi(x)
}

// gelu2 on N independent pairs, every step issued for all N before the next: the same operations
// (bitwise the same results), but each dependent packed FMA finds N - 1 others between it and its
// source, so the hazard recognizer needs no s_nop (one per dependent v_pk_* pair otherwise)
template <int N>
DEV void gelu2n(const f32x2 (&x)[N], f32x2 (&gl)[N], f32x2 (*gd)[N]) {
  f32x2 e[N], t[N], poly[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const f32x2 x2 = x[n] * x[n];
    const f32x2 ea = x2 * (-0.72134752044448170f) + (-1.3257480647361593f);
    e[n].x = __builtin_amdgcn_exp2f(ea.x);
    e[n].y = __builtin_amdgcn_exp2f(ea.y);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    t[n].x = __builtin_amdgcn_rcpf(fmaf(fabsf(x[n].x), 0.23164188826636040f, 1.0f));
    t[n].y = __builtin_amdgcn_rcpf(fmaf(fabsf(x[n].y), 0.23164188826636040f, 1.0f));
  }
#pragma unroll
  for (int n = 0; n < N; ++n) poly[n] = t[n] * 1.3302744295891231f + (-1.8212559791077754f);
#pragma unroll
  for (int n = 0; n < N; ++n) poly[n] = poly[n] * t[n] + 1.7814779365698128f;
#pragma unroll
  for (int n = 0; n < N; ++n) poly[n] = poly[n] * t[n] + (-0.35656378124891560f);
#pragma unroll
  for (int n = 0; n < N; ++n) poly[n] = poly[n] * t[n] + 0.31938153025994087f;
#pragma unroll
  for (int n = 0; n < N; ++n) poly[n] = poly[n] * t[n];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const f32x2 qm = poly[n] * e[n] + (-0.5f);
    f32x2 us;
    us.x = copysignf(qm.x, x[n].x);
    us.y = copysignf(qm.y, x[n].y);
    poly[n] = us + 0.5f;                                                       // Phi(x)
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    gl[n] = x[n] * poly[n];
    if (gd) (*gd)[n] = x[n] * e[n] + poly[n];
  }
}

// gelu(x) and gelu'(x) together (one exp, one erf): the forward stores gelu' for the backward
DEV void gelu_fg(float x, float& gl, float& gd) {
  const float e = __expf(-0.5f * x * x);
  const float h = 0.5f * (1.0f + erf_half(x, e));
  gl = x * h;
  gd = h + x * 0.39894228040143268f * e;
}

// ---------------------------------------------------------------------------------------
// Counter-based RNG: Philox4x32-10 (Salmon et al., SC'11).  Every random draw in the path
// (dropout masks, Laplace noise, Gumbel noise) is a pure function of (seed, stream, counter),
// so forward and backward regenerate identical masks and the CPU oracle can replay them.
// ---------------------------------------------------------------------------------------
struct u32x4s { uint32_t x, y, z, w; };
DEV uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t* hi) {
  uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}
template <int ROUNDS>
DEV u32x4s philox4x32_r(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    uint32_t hi0, hi1;
    uint32_t lo0 = mulhilo(0xD2511F53u, c0, &hi0);
    uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, &hi1);
    // three-input XORs as one v_bitop3_b32 each (truth table 0x96; hipcc emits two v_xor_b32 for
    // a ^ b ^ c): 2 instead of 4 bitwise VALU ops per round beside the two v_mad_u64_u32
    uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96), n1 = lo1;
    uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96), n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
DEV u32x4s philox4x32(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  return philox4x32_r<10>(c0, c1, c2, c3, k0, k1);
}
// uniform in (0, 1]: (x + 1) * 2^-32 with x in [0, 2^32)  → never exactly 0
DEV float u01_open0(uint32_t x) { return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f); }

// Dropout keep-mask, shared by every dropout site: element e of a site keyed (seed, offset) is kept
// iff word (e & 3) of philox(e >> 2, offset; seed) >= p * 2^32; kept elements scale by 1/(1-p).
// drop_mask4 returns the 4 consecutive elements 4*e4 .. 4*e4+3.
DEV void drop_mask4(uint64_t seed, uint64_t offset, uint64_t e4, float p, float (&m)[4]) {
  const u32x4s r = philox4x32((uint32_t)e4, (uint32_t)(e4 >> 32), (uint32_t)offset, (uint32_t)(offset >> 32),
                              (uint32_t)seed, (uint32_t)(seed >> 32));
  const float scale = 1.0f / (1.0f - p);
  const uint32_t thr = (uint32_t)fminf(p * 4294967296.0f, 4294967295.0f);
  m[0] = r.x >= thr ? scale : 0.f;
  m[1] = r.y >= thr ? scale : 0.f;
  m[2] = r.z >= thr ? scale : 0.f;
  m[3] = r.w >= thr ? scale : 0.f;
}
// Attention-probability stream (L^2 draws per head, the only site where the draw cost shows):
// Philox4x32-7 (Random123: BigCrush-clean at 7 rounds), eight 16-bit draws per call.  Element e
// is kept iff halfword (e & 7) of philox7(e >> 3, offset; seed) >= thr16 = (uint32)(p * 65536)
// (halfword k = bits 16*(k&1).. of word k>>1).  Returns the 8 keep bits (bit k = element 8c+k).
// Both halfwords of a word against thr16 at once: saturating packed subtract of (thr16 - 1), then
// min with 1 -> 0 / 1 in bits 0 and 16.  (Written as asm: hipcc turns the elementwise builtins back
// into 8 v_cmp + v_cndmask pairs with SGPR-mask hazards -- 14 VALU per call here vs ~21 + s_nops.)
DEV uint32_t pk_keep01(uint32_t w, uint32_t thrm1x2, uint32_t ones) {
  uint32_t d, m;
  asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(d) : "v"(w), "v"(thrm1x2));
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(d), "v"(ones));
  return m;
}
DEV uint32_t keep_bits8(uint64_t seed, uint64_t offset, uint64_t call, uint32_t thr16) {
  const u32x4s r = philox4x32_r<7>((uint32_t)call, (uint32_t)(call >> 32), (uint32_t)offset,
                                   (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t tm = (thr16 - 1u) & 0xFFFFu, tm2 = tm | (tm << 16), ones = 0x00010001u;
  // word j's halfword keep flags land at bits 2j (low half) and 16 + 2j (high half)
  const uint32_t b = pk_keep01(r.x, tm2, ones) | (pk_keep01(r.y, tm2, ones) << 2) |
                     (pk_keep01(r.z, tm2, ones) << 4) | (pk_keep01(r.w, tm2, ones) << 6);
  const uint32_t bits = (b & 0x55u) | (b >> 15);     // bit k = halfword k
  return thr16 ? bits : 0xFFu;                       // thr16 = 0 (p < 2^-16): every element kept
}
// keep_bits8 for a call number known to fit 32 bits (counter word 1 = 0): the same draws; with the
// high word a constant, the first round's output word 0 and the second round's first product are
// wave-uniform (scalar), one v_mad_u64_u32 fewer per call
DEV uint32_t keep_bits8_c32(uint64_t seed, uint64_t offset, uint32_t call, uint32_t thr16) {
  const u32x4s r = philox4x32_r<7>(call, 0u, (uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)seed,
                                   (uint32_t)(seed >> 32));
  const uint32_t tm = (thr16 - 1u) & 0xFFFFu, tm2 = tm | (tm << 16), ones = 0x00010001u;
  const uint32_t b = pk_keep01(r.x, tm2, ones) | (pk_keep01(r.y, tm2, ones) << 2) |
                     (pk_keep01(r.z, tm2, ones) << 4) | (pk_keep01(r.w, tm2, ones) << 6);
  const uint32_t bits = (b & 0x55u) | (b >> 15);
  return thr16 ? bits : 0xFFu;
}
DEV uint32_t thr16_of(float p) { return (uint32_t)fminf(p * 65536.0f, 65535.0f); }
// The same eight keep decisions as 0 / 1 halfword multipliers (word j -> halfwords 2j, 2j + 1), for
// applying a call's draws to eight packed bf16 values at once with v_pk_mul_lo_u16 (thr16 > 0)
DEV u32x4 keep01x8(uint64_t seed, uint64_t offset, uint64_t call, uint32_t thr16) {
  const u32x4s r = philox4x32_r<7>((uint32_t)call, (uint32_t)(call >> 32), (uint32_t)offset,
                                   (uint32_t)(offset >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t tm = (thr16 - 1u) & 0xFFFFu, tm2 = tm | (tm << 16), ones = 0x00010001u;
  return u32x4{pk_keep01(r.x, tm2, ones), pk_keep01(r.y, tm2, ones), pk_keep01(r.z, tm2, ones),
               pk_keep01(r.w, tm2, ones)};
}
// keep01x8 for a call number known to fit 32 bits (see keep_bits8_c32)
DEV u32x4 keep01x8_c32(uint64_t seed, uint64_t offset, uint32_t call, uint32_t thr16) {
  const u32x4s r = philox4x32_r<7>(call, 0u, (uint32_t)offset, (uint32_t)(offset >> 32), (uint32_t)seed,
                                   (uint32_t)(seed >> 32));
  const uint32_t tm = (thr16 - 1u) & 0xFFFFu, tm2 = tm | (tm << 16), ones = 0x00010001u;
  return u32x4{pk_keep01(r.x, tm2, ones), pk_keep01(r.y, tm2, ones), pk_keep01(r.z, tm2, ones),
               pk_keep01(r.w, tm2, ones)};
}
// bf16 pair x (0 or 1 per halfword): the value itself or +0, bit-exact (asm: one VALU)
DEV uint32_t pk_mul_u16(uint32_t a, uint32_t b) {
  uint32_t d;
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}

DEV float drop_mask1(uint64_t seed, uint64_t offset, uint64_t e, float p) {
  float m[4];
  drop_mask4(seed, offset, e >> 2, p, m);
  const int k = (int)(e & 3);
  return k == 0 ? m[0] : k == 1 ? m[1] : k == 2 ? m[2] : m[3];
}
