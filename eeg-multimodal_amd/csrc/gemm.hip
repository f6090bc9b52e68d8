// gemm.hip — MFMA GEMM with fused epilogues for every dense projection on the path.
//
//   C[m, n] = epi( alpha * sum_k A(m, k) * B(k, n) ) + beta * C[m, n]      (batched over z)
//
// Operand layouts (row-major storage, leading dimensions in elements):
//   A_KC: A(m,k) = A[m*lda + k]   (contraction axis contiguous)   else A[k*lda + m]
//   B_KC: B(k,n) = B[n*ldb + k]   (nn.Linear weight [out,in])      else B[k*ldb + n]
// Forward Linear = (A_KC, B_KC); input-gradient = (A_KC, !B_KC); weight-gradient = (!A_KC, !B_KC).
//
// Tile 128x128, one k-step = 128 bytes of contraction per row (bf16: 64, f32: 32), 256 threads
// = 4 waves in a 2x2 grid, each wave 64x64 = 4x4 accumulators of 16x16.  Strided (k-major) LDS
// tiles are read with ds_read_b64_tr_b16 (bf16).  Global loads are 16 B per lane, staged
// through registers one k-step ahead of the MFMAs (issue early, write LDS after the barrier).
#include "common.h"
#include "eegfusion_internal.h"
#include <cstdlib>

namespace {

constexpr int BM = 128, BN = 128, NT = 256;

struct GemmArgs {
  const void* A; const void* B; void* C; const float* bias; void* aux;
  long lda, ldb, ldc, ldaux;
  long sA, sB, sC, sAux, sBias;
  int M, N, K;
  float alpha, beta, epi_scale;
  int ksplit;          // >0: split-K slice length (grid.z = slices, C = fp32 slabs [z][M][N])
  int lds_epi;         // LDS-staged coalesced epilogue (bf16 out, beta == 0)
  int bt;              // output tile: 128 or 64
};

DEV void load4(const float* p, float (&v)[4]) { const f32x4 x = *(const f32x4*)p; v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3]; }
DEV void load4(const bf16* p, float (&v)[4]) { const bf16x4 x = *(const bf16x4*)p; v[0] = (float)x[0]; v[1] = (float)x[1]; v[2] = (float)x[2]; v[3] = (float)x[3]; }
DEV void store4(float* p, const float (&v)[4]) { *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]}; }
DEV void store4(bf16* p, const float (&v)[4]) {
  bf16x4 x; x[0] = (bf16)v[0]; x[1] = (bf16)v[1]; x[2] = (bf16)v[2]; x[3] = (bf16)v[3];
  *(bf16x4*)p = x;
}

// Coalesced copy of a 128x128 bf16 tile between LDS [128][ldl] and global (rows m0.., cols n0..),
// 16 B per lane (16 lanes per 256-B row), edge-guarded.  LOAD: global -> LDS, else LDS -> global.
template <bool LOAD>
DEV void tile_io(bf16* lds, int ldl, bf16* gp, long ld, int m0, int n0, int M, int N, int tid) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = tid + 256 * k;
    const int r = c >> 4, cc = (c & 15) * 8;
    const int m = m0 + r, n = n0 + cc;
    if (m >= M || n >= N) continue;
    bf16* g = gp + (long)m * ld + n;
    bf16* l = lds + r * ldl + cc;
    if (n + 8 <= N && ((uintptr_t)g & 15) == 0) {
      if (LOAD) st16(l, ld16(g)); else st16(g, ld16(l));
    } else {
      for (int e = 0; e < 8 && n + e < N; ++e) { if (LOAD) l[e] = g[e]; else g[e] = l[e]; }
    }
  }
}

template <typename T, int BT = 128>
struct TileCfg {
  static constexpr int KT = 128 / (int)sizeof(T);        // contraction elements per k-step
  static constexpr int VE = 16 / (int)sizeof(T);         // elements per 16-B chunk
  // K-contiguous LDS tile: [BT rows][KT], rows of exactly 128 B with 16-B chunk c of row r stored at
  // c ^ kc_swz(r) (below).  The round-5 layout padded each row by 16 B (36 words): ds_read_b128 serves
  // a wave in four 16-lane groups of mixed rows and chunks (MI355X_MICROARCH.md, LDS table), and rows
  // 10 / 12 and 11 / 13 of such a group met on one bank quad -- 2-way conflicts, 0.17-0.33 of the fp32
  // decoder GEMMs' LDS cycles in profiles/r6x_pmc_table.md
  static constexpr int RS_KC = KT;
  // k-major LDS tile: [KT rows][BT] + 32 B pad per row
  static constexpr int RS_KM = BT + 2 * VE;
  // fp32 k-major tiles: rows 8 apart (the four 16-lane groups of an fp32 ld_col8) would sit a multiple
  // of 64 banks apart (8 x 72 / 8 x 136 words: 4-way conflicts, 0.33-0.44 of LDS cycles in the round-5
  // counters), so every block of 8 rows is shifted by 16 more words: the four groups land on disjoint
  // 16-bank quarters.  The shift keeps every 16-B row chunk aligned.  bf16 tiles read through
  // ds_read_b64_tr_b16 and keep the plain layout.
  static constexpr int SKEW = sizeof(T) == 4 ? 16 : 0;
  static DEV int skew(int krow) { return SKEW * ((krow >> 3) & 3); }
  static constexpr int SZ_KC = BT * RS_KC;
  // chunk swizzle of the K-contiguous tiles: a function of bits 1-2 of the row, so every fragment read
  // (rows r0 + (lane & 15), r0 % 16 == 0) and every staging store (rows (tid >> 3) + 32 i) keeps one
  // per-lane value.  Chosen by exhaustive search over the linear XOR maps of the row's low bits: every
  // 16-lane group of the bf16 (chunk 4 kc + lane / 16) and fp32 (chunks 2 (lane / 16) + {0, 1}) fragment
  // reads covers the 16 bank quads once; the 8-lane ds_write_b128 groups write one whole 128-B row
  static DEV int kc_swz(int r) { return (((r >> 1) & 1) << 2) ^ (((r >> 2) & 1) * 3); }
  static constexpr int SZ_KM = KT * RS_KM + 3 * SKEW;
  static constexpr int CHUNKS = BT * 8 / NT;             // 16-B chunks per thread per operand tile
};

// Load one operand tile (BT x 128 B) into CHUNKS x 16-B registers per thread (guarded at the edges).
// KC: the K-contiguous layout (tile rows = m or n index).
template <typename T, bool KC, int BT>
DEV void load_tile(u32x4* reg, const T* __restrict__ base, long ld, int mn0, int k0, int MN,
                   int K, int tid) {
  using C = TileCfg<T, BT>;
#pragma unroll
  for (int i = 0; i < C::CHUNKS; ++i) {
    const int c = tid + NT * i;
    int r, col;            // r = tile row, col = element offset within row
    if (KC) { r = c >> 3; col = (c & 7) * C::VE; }
    else    { constexpr int CPR = BT / C::VE; r = c / CPR; col = (c % CPR) * C::VE; }
    const int row_idx = KC ? mn0 + r : k0 + r;       // index along the strided axis
    const int col_idx = KC ? k0 + col : mn0 + col;   // index along the contiguous axis
    const int row_lim = KC ? MN : K;
    const int col_lim = KC ? K : MN;
    const T* p = base + (long)row_idx * ld + col_idx;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row_idx < row_lim) {
      if (col_idx + C::VE <= col_lim && ((uintptr_t)p & 15) == 0) {
        v = ld16(p);
      } else {
        T tmp[C::VE];
#pragma unroll
        for (int e = 0; e < C::VE; ++e) tmp[e] = (col_idx + e < col_lim) ? p[e] : from_f32<T>(0.f);
        v = *(u32x4*)tmp;
      }
    }
    reg[i] = v;
  }
}

// 8 contiguous K elements at K offset kk (a multiple of 8) of a swizzled K-contiguous tile row
DEV bf16x8 ld_kc8(const bf16* row, int kk, int s) { return *(const bf16x8*)(row + (((kk >> 3) ^ s) << 3)); }
DEV f32x8 ld_kc8(const float* row, int kk, int s) {
  const f32x4 a = *(const f32x4*)(row + (((kk >> 2) ^ s) << 2));
  const f32x4 b = *(const f32x4*)(row + ((((kk >> 2) + 1) ^ s) << 2));
  f32x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

template <typename T, bool KC, int BT>
DEV void store_tile(T* lds, const u32x4* reg, int tid) {
  using C = TileCfg<T, BT>;
#pragma unroll
  for (int i = 0; i < C::CHUNKS; ++i) {
    const int c = tid + NT * i;
    int r, col;
    if (KC) { r = c >> 3; col = (c & 7) * C::VE; }
    else    { constexpr int CPR = BT / C::VE; r = c / CPR; col = (c % CPR) * C::VE; }
    st16(lds + (KC ? r * C::RS_KC + (((c & 7) ^ C::kc_swz(r)) * C::VE) : r * C::RS_KM + C::skew(r) + col), reg[i]);
  }
}

// BT: output tile BT x BT (128, or 64 for the batch-row GEMMs whose 128-tile grids would leave most
// CUs idle); 4 waves in 2 x 2, each a (BT/2) x (BT/2) block of NI x NI 16x16 accumulators.
template <typename T, bool AKC, bool BKC, typename TO, int EPI, int BT = 128>
__global__ void __launch_bounds__(NT) gemm_kernel(GemmArgs g) {
  using C = TileCfg<T, BT>;
  constexpr int WT = BT / 2, NI = WT / 16;
  using F = typename Frag8<T>::type;
  constexpr int SZA = AKC ? C::SZ_KC : C::SZ_KM;
  constexpr int SZB = BKC ? C::SZ_KC : C::SZ_KM;
  // the bf16 LDS-staged epilogue reuses the array as a [128][BN + 8] output tile (34.8 KB, more than the
  // two unpadded 16-KB operand tiles)
  constexpr int SZE = (sizeof(T) == 2 && BT == 128) ? BM * (BN + 8) : 0;
  __shared__ __attribute__((aligned(16))) T lds[SZA + SZB > SZE ? SZA + SZB : SZE];
  T* As = lds;
  T* Bs = lds + SZA;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (g.N + BT - 1) / BT, tiles_m = (g.M + BT - 1) / BT;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int m0 = tm * BT, n0 = tn * BT;
  const int z = blockIdx.y;
  int kbeg = 0, kend = g.K;
  if (g.ksplit > 0) { kbeg = blockIdx.z * g.ksplit; kend = min(g.K, kbeg + g.ksplit); }

  const T* A = (const T*)g.A + (long)z * g.sA;
  const T* B = (const T*)g.B + (long)z * g.sB;

  // acc[i][j] holds the TRANSPOSED 16x16 tile (operands swapped in the MFMA): lane l owns
  // C[m = m0 + wm*WT + 16i + (l&15)][n = n0 + wn*WT + 16j + 4*(l>>4) + r], r = 0..3, i.e. four
  // consecutive columns of one row -> 8/16-byte epilogue loads and stores.
  f32x4 acc[NI][NI];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[C::CHUNKS], rb[C::CHUNKS];
  const int kcs = C::kc_swz(lane & 15);     // the K-contiguous fragment rows' chunk swizzle
  const int nk = (kend - kbeg + C::KT - 1) / C::KT;
  load_tile<T, AKC, BT>(ra, A, g.lda, m0, kbeg, g.M, kend, tid);
  load_tile<T, BKC, BT>(rb, B, g.ldb, n0, kbeg, g.N, kend, tid);

  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();                     // previous k-step's LDS reads are done
    store_tile<T, AKC, BT>(As, ra, tid);
    store_tile<T, BKC, BT>(Bs, rb, tid);
    __syncthreads();
    if (kt + 1 < nk) {                   // issue next k-step's global loads under the MFMAs
      load_tile<T, AKC, BT>(ra, A, g.lda, m0, kbeg + (kt + 1) * C::KT, g.M, kend, tid);
      load_tile<T, BKC, BT>(rb, B, g.ldb, n0, kbeg + (kt + 1) * C::KT, g.N, kend, tid);
    }
#pragma unroll
    for (int kc = 0; kc < C::KT / 32; ++kc) {
      F a[NI], b[NI];
      const int kk = kc * 32 + 8 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int r = wm * WT + i * 16;
        if (AKC) a[i] = ld_kc8(As + (r + (lane & 15)) * C::RS_KC, kk, kcs);
        else     a[i] = ld_col8(As + C::skew(kk), C::RS_KM, kk, r, lane);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int c = wn * WT + j * 16;
        if (BKC) b[j] = ld_kc8(Bs + (c + (lane & 15)) * C::RS_KC, kk, kcs);
        else     b[j] = ld_col8(Bs + C::skew(kk), C::RS_KM, kk, c, lane);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = mma16(b[j], a[i], acc[i][j]);
    }
  }

  // ---- epilogue ----
  if (g.ksplit > 0) {                    // split-K: raw fp32 partial slab, reduced by gemm_splitk_reduce
    // slabs [split][batch][M][N] (batched split-K: plain GEMMs only, gemm_splitk_reduce_batched)
    float* slab = (float*)g.C + ((long)blockIdx.z * gridDim.y + z) * g.M * g.N;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int m = m0 + wm * WT + i * 16 + (lane & 15);
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int n = n0 + wn * WT + j * 16 + 4 * (lane >> 4);
        float* cp = slab + (long)m * g.N + n;
        const f32x4 v = acc[i][j] * g.alpha;
        if (n + 3 < g.N && ((uintptr_t)cp & 15) == 0) *(f32x4*)cp = v;
        else
          for (int r = 0; r < 4; ++r) if (n + r < g.N) cp[r] = v[r];
      }
    }
    return;
  }
  TO* Cp = (TO*)g.C + (long)z * g.sC;
  TO* aux = (TO*)g.aux + (long)z * g.sAux;
  const float* biasp = g.bias ? g.bias + (long)z * g.sBias : nullptr;
  constexpr bool HAS_BIAS = EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_TANH ||
                            EPI == EPI_BIAS_GELU_D;
  constexpr bool HAS_AUX = EPI == EPI_BIAS_GELU || EPI == EPI_DGELU || EPI == EPI_DRELU || EPI == EPI_DTANH ||
                           EPI == EPI_BIAS_GELU_D || EPI == EPI_MUL_AUX;
  constexpr bool AUX_IN = EPI == EPI_DGELU || EPI == EPI_DRELU || EPI == EPI_DTANH || EPI == EPI_MUL_AUX;
  constexpr bool TWO_OUT = EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_D;   // C and aux both written
  if constexpr (sizeof(TO) == 2 && sizeof(T) == 2 && BT == 128) {
    if (g.beta == 0.f && g.lds_epi) {
      // LDS-staged epilogue: the 128x128 bf16 tile goes through LDS so every global access is a
      // full 16-B-per-lane row segment (a wave writes 4 x 256-B rows per instruction).
      constexpr int LDC = BN + 8;
      bf16* ct = (bf16*)lds;
      __syncthreads();
      if (AUX_IN) {
        tile_io<true>(ct, LDC, (bf16*)aux, g.ldaux, m0, n0, g.M, g.N, tid);
        __syncthreads();
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int nl = wn * 64 + j * 16 + 4 * (lane >> 4);
        const int n = n0 + nl;
        float bias[4] = {0.f, 0.f, 0.f, 0.f};
        if (HAS_BIAS)
          for (int r = 0; r < 4; ++r) bias[r] = (n + r < g.N) ? biasp[n + r] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ml = wm * 64 + i * 16 + (lane & 15);
          bf16* lp = ct + ml * LDC + nl;
          float av[4] = {0.f, 0.f, 0.f, 0.f};
          if (AUX_IN) load4(lp, av);
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = g.alpha * acc[i][j][r];
            if (EPI == EPI_BIAS) v += bias[r];
            else if (EPI == EPI_BIAS_GELU) v = g.aux ? v + bias[r] : gelu_f(v + bias[r]);
            else if (EPI == EPI_BIAS_RELU) v = relu_nan(v + bias[r]);
            else if (EPI == EPI_BIAS_TANH) v = tanhf(v + bias[r]);
            else if (EPI == EPI_DGELU) v *= gelu_grad(av[r]);
            else if (EPI == EPI_DRELU) v = av[r] > 0.f ? v * g.epi_scale : 0.f;
            else if (EPI == EPI_DTANH) v *= (1.f - av[r] * av[r]);
            else if (EPI == EPI_MUL_AUX) v *= av[r];
            if (EPI == EPI_BIAS_GELU_D) {     // aux round first: gelu'; acc keeps gelu for the C round
              float gl, gd;
              gelu_fg(v + bias[r], gl, gd);
              acc[i][j][r] = gl;
              o[r] = gd;
            } else {
              acc[i][j][r] = v;               // BIAS_GELU keeps the pre-activation
              o[r] = v;
            }
          }
          store4(lp, o);
        }
      }
      __syncthreads();
      if ((EPI == EPI_BIAS_GELU && g.aux) || EPI == EPI_BIAS_GELU_D) {
        tile_io<false>(ct, LDC, (bf16*)aux, g.ldaux, m0, n0, g.M, g.N, tid);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = EPI == EPI_BIAS_GELU_D ? acc[i][j][r] : gelu_f(acc[i][j][r]);
            store4(ct + (wm * 64 + i * 16 + (lane & 15)) * LDC + wn * 64 + j * 16 + 4 * (lane >> 4), o);
          }
        __syncthreads();
      }
      tile_io<false>(ct, LDC, (bf16*)Cp, g.ldc, m0, n0, g.M, g.N, tid);
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int n = n0 + wn * WT + j * 16 + 4 * (lane >> 4);
    if (n >= g.N) continue;
    const bool nfull = n + 3 < g.N;
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (HAS_BIAS) {
      if (nfull && ((uintptr_t)(biasp + n) & 15) == 0) {
        const f32x4 bv = *(const f32x4*)(biasp + n);
        bias[0] = bv[0]; bias[1] = bv[1]; bias[2] = bv[2]; bias[3] = bv[3];
      } else {
        for (int r = 0; r < 4; ++r) if (n + r < g.N) bias[r] = biasp[n + r];
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int m = m0 + wm * WT + i * 16 + (lane & 15);
      if (m >= g.M) continue;
      TO* cp = Cp + (long)m * g.ldc + n;
      TO* ap = HAS_AUX && g.aux ? aux + (long)m * g.ldaux + n : nullptr;
      const bool vec = nfull && ((uintptr_t)cp & (4 * sizeof(TO) - 1)) == 0 &&
                       (!ap || ((uintptr_t)ap & (4 * sizeof(TO) - 1)) == 0);
      float av[4] = {0.f, 0.f, 0.f, 0.f}, cv[4] = {0.f, 0.f, 0.f, 0.f};
      if (vec) {
        if (AUX_IN) load4(ap, av);
        if (g.beta != 0.f) load4(cp, cv);
      } else {
        for (int r = 0; r < 4; ++r)
          if (n + r < g.N) {
            if (AUX_IN) av[r] = to_f32(ap[r]);
            if (g.beta != 0.f) cv[r] = to_f32(cp[r]);
          }
      }
      float o[4], pre[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = g.alpha * acc[i][j][r];
        if (EPI == EPI_BIAS) v += bias[r];
        else if (EPI == EPI_BIAS_GELU) { v += bias[r]; pre[r] = v; v = gelu_f(v); }
        else if (EPI == EPI_BIAS_GELU_D) { float gl; gelu_fg(v + bias[r], gl, pre[r]); v = gl; }
        else if (EPI == EPI_MUL_AUX) v *= av[r];
        else if (EPI == EPI_BIAS_RELU) v = relu_nan(v + bias[r]);
        else if (EPI == EPI_BIAS_TANH) v = tanhf(v + bias[r]);
        else if (EPI == EPI_DGELU) v *= gelu_grad(av[r]);
        else if (EPI == EPI_DRELU) v = av[r] > 0.f ? v * g.epi_scale : 0.f;
        else if (EPI == EPI_DTANH) v *= (1.f - av[r] * av[r]);
        if (g.beta != 0.f) v += g.beta * cv[r];
        o[r] = v;
      }
      if (vec) {
        store4(cp, o);
        if (TWO_OUT && ap) store4(ap, pre);
      } else {
        for (int r = 0; r < 4; ++r)
          if (n + r < g.N) {
            cp[r] = from_f32<TO>(o[r]);
            if (TWO_OUT && ap) ap[r] = from_f32<TO>(pre[r]);
          }
      }
    }
  }
}

// out = epi(sum_s slab[s] + bias) (+ beta*out): the split-K combine, elementwise with the epilogue
// (slabs already hold alpha*AB).  Fixed summation order -> bitwise reproducible.
template <typename TO, int EPI>
__global__ void __launch_bounds__(256) gemm_splitk_reduce(const float* __restrict__ slabs, int splits, int M, int N,
                                                          TO* C, long ldc, float beta, const float* bias, TO* aux,
                                                          long ldaux, float epi_scale) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)M * N;
  if (e >= total) return;
  float v = 0.f;
  for (int s = 0; s < splits; ++s) v += slabs[(long)s * total + e];
  const long m = e / N, n = e % N;
  TO* c = C + m * ldc + n;
  if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_TANH ||
      EPI == EPI_BIAS_GELU_D)
    v += bias[n];
  if (EPI == EPI_BIAS_GELU) { if (aux) aux[m * ldaux + n] = from_f32<TO>(v); v = gelu_f(v); }
  else if (EPI == EPI_BIAS_GELU_D) { float gl, gd; gelu_fg(v, gl, gd); aux[m * ldaux + n] = from_f32<TO>(gd); v = gl; }
  else if (EPI == EPI_MUL_AUX) v *= to_f32(aux[m * ldaux + n]);
  else if (EPI == EPI_BIAS_RELU) v = relu_nan(v);
  else if (EPI == EPI_BIAS_TANH) v = tanhf(v);
  else if (EPI == EPI_DGELU) v *= gelu_grad(to_f32(aux[m * ldaux + n]));
  else if (EPI == EPI_DRELU) v = to_f32(aux[m * ldaux + n]) > 0.f ? v * epi_scale : 0.f;
  else if (EPI == EPI_DTANH) { const float y = to_f32(aux[m * ldaux + n]); v *= 1.f - y * y; }
  if (beta != 0.f) v += beta * to_f32(*c);
  *c = from_f32<TO>(v);
}

// the batched plain form: C[b] = sum_s slab[s][b] + beta C[b] (C[b] at C + b strideC, row stride ldc),
// the same fixed summation order
template <typename TO>
__global__ void __launch_bounds__(256) gemm_splitk_reduce_batched(const float* __restrict__ slabs, int splits, int batch,
                                                                  int M, int N, TO* C, long ldc, long strideC,
                                                                  float beta) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long mn = (long)M * N, total = mn * batch;
  if (e >= total) return;
  float v = 0.f;
  for (int s = 0; s < splits; ++s) v += slabs[(long)s * total + e];
  const long b = e / mn, r = e % mn, m = r / N, n = r % N;
  TO* c = C + b * strideC + m * ldc + n;
  if (beta != 0.f) v += beta * to_f32(*c);
  *c = from_f32<TO>(v);
}

template <typename TO>
int splitk_reduce_t(int epi, const float* ws, int splits, int M, int N, void* C, long ldc, float beta,
                    const float* bias, void* aux, long ldaux, float scale, hipStream_t st) {
  const dim3 grid((unsigned)(((long)M * N + 255) / 256));
#define RED(E) EEGF_LAUNCH((gemm_splitk_reduce<TO, E>), grid, dim3(256), 0, st, ws, splits, M, N, (TO*)C, ldc, \
                                  beta, bias, (TO*)aux, ldaux, scale)
  switch (epi) {
    case EPI_NONE: RED(EPI_NONE); break;
    case EPI_BIAS: RED(EPI_BIAS); break;
    case EPI_BIAS_GELU: RED(EPI_BIAS_GELU); break;
    case EPI_BIAS_RELU: RED(EPI_BIAS_RELU); break;
    case EPI_BIAS_TANH: RED(EPI_BIAS_TANH); break;
    case EPI_DGELU: RED(EPI_DGELU); break;
    case EPI_DRELU: RED(EPI_DRELU); break;
    case EPI_DTANH: RED(EPI_DTANH); break;
    case EPI_BIAS_GELU_D: RED(EPI_BIAS_GELU_D); break;
    case EPI_MUL_AUX: RED(EPI_MUL_AUX); break;
    default: return EEGF_ERR_ARG;
  }
#undef RED
  return (int)hipGetLastError();
}

int splitk_reduce_dispatch(int epi, int out_bf16, const float* ws, int splits, int M, int N, void* C, long ldc,
                           float beta, float alpha, const float* bias, void* aux, long ldaux, float scale,
                           hipStream_t st) {
  (void)alpha;
  return out_bf16 ? splitk_reduce_t<bf16>(epi, ws, splits, M, N, C, ldc, beta, bias, aux, ldaux, scale, st)
                  : splitk_reduce_t<float>(epi, ws, splits, M, N, C, ldc, beta, bias, aux, ldaux, scale, st);
}

template <typename T, bool AKC, bool BKC, typename TO, int EPI>
int launch(const GemmArgs& a, int batch, hipStream_t s, int splits = 1) {
  if (a.bt == 64) {
    const int tiles = ((a.M + 63) / 64) * ((a.N + 63) / 64);
    EEGF_LAUNCH((gemm_kernel<T, AKC, BKC, TO, EPI, 64>), dim3(tiles, batch, splits), dim3(NT), 0, s, a);
  } else {
    const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    EEGF_LAUNCH((gemm_kernel<T, AKC, BKC, TO, EPI>), dim3(tiles, batch, splits), dim3(NT), 0, s, a);
  }
  return (int)hipGetLastError();
}

template <typename T, typename TO>
int dispatch_layout_split(int akc, int bkc, const GemmArgs& a, hipStream_t s, int splits) {
  if (akc && bkc) return launch<T, true, true, TO, EPI_NONE>(a, 1, s, splits);
  if (akc && !bkc) return launch<T, true, false, TO, EPI_NONE>(a, 1, s, splits);
  if (!akc && !bkc) return launch<T, false, false, TO, EPI_NONE>(a, 1, s, splits);
  return launch<T, false, true, TO, EPI_NONE>(a, 1, s, splits);
}

template <typename T, typename TO, int EPI>
int dispatch_layout(int akc, int bkc, const GemmArgs& a, int batch, hipStream_t s) {
  if (akc && bkc) return launch<T, true, true, TO, EPI>(a, batch, s);
  if (akc && !bkc) return launch<T, true, false, TO, EPI>(a, batch, s);
  if (!akc && !bkc) return launch<T, false, false, TO, EPI>(a, batch, s);
  return launch<T, false, true, TO, EPI>(a, batch, s);
}

template <typename T, typename TO>
int dispatch_epi(int epi, int akc, int bkc, const GemmArgs& a, int batch, hipStream_t s) {
  switch (epi) {
    case EPI_NONE: return dispatch_layout<T, TO, EPI_NONE>(akc, bkc, a, batch, s);
    case EPI_BIAS: return launch<T, true, true, TO, EPI_BIAS>(a, batch, s);
    case EPI_BIAS_GELU: return launch<T, true, true, TO, EPI_BIAS_GELU>(a, batch, s);
    case EPI_BIAS_RELU: return launch<T, true, true, TO, EPI_BIAS_RELU>(a, batch, s);
    case EPI_BIAS_TANH: return launch<T, true, true, TO, EPI_BIAS_TANH>(a, batch, s);
    case EPI_DGELU: return launch<T, true, false, TO, EPI_DGELU>(a, batch, s);
    case EPI_DRELU: return launch<T, true, false, TO, EPI_DRELU>(a, batch, s);
    case EPI_DTANH: return launch<T, true, false, TO, EPI_DTANH>(a, batch, s);
    case EPI_BIAS_GELU_D: return launch<T, true, true, TO, EPI_BIAS_GELU_D>(a, batch, s);
    case EPI_MUL_AUX: return launch<T, true, false, TO, EPI_MUL_AUX>(a, batch, s);
  }
  return EEGF_ERR_ARG;
}

}  // namespace

int eegf_gemm_big(int a_kc, int b_kc, int epi, int out_f32, int M, int N, int K, const void* A, long lda,
                  const void* B, long ldb, void* C, long ldc, const float* bias, void* aux, long ldaux, float alpha,
                  float beta, float epi_scale, void* workspace, long ws_bytes, hipStream_t stream);
int eegf_gemm_big_wgrad_bias(int M, int N, int K, const void* A, long lda, const void* B, long ldb, float* C, long ldc,
                             float beta, float* db, void* workspace, long ws_bytes, hipStream_t stream);

static int gemm_impl(int dtype, int out_dtype, int a_kcontig, int b_kcontig, int epi, int M, int N, int K, int batch,
                     const void* A, long lda, long strideA, const void* B, long ldb, long strideB, void* C, long ldc,
                     long strideC, const float* bias, long strideBias, void* aux, long ldaux, long strideAux,
                     float alpha, float beta, float epi_scale, void* workspace, long ws_bytes, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || !A || !B || !C) return EEGF_ERR_ARG;
  if (batch > 65535) return EEGF_ERR_ARG;
  if (epi < EPI_NONE || epi > EPI_MUL_AUX) return EEGF_ERR_ARG;
  const bool has_bias = epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_RELU || epi == EPI_BIAS_TANH ||
                        epi == EPI_BIAS_GELU_D;
  const bool aux_in = epi == EPI_DGELU || epi == EPI_DRELU || epi == EPI_DTANH || epi == EPI_MUL_AUX;
  if (has_bias && !bias) return EEGF_ERR_ARG;
  if ((aux_in || epi == EPI_BIAS_GELU_D) && !aux) return EEGF_ERR_ARG;    // BIAS_GELU: aux optional
  if (aux_in && beta != 0.f) return EEGF_ERR_ARG;                           // aux replaces C
  if (epi != EPI_NONE) {
    const bool fwd = epi <= EPI_BIAS_TANH || epi == EPI_BIAS_GELU_D;
    if (fwd && !(a_kcontig && b_kcontig)) return EEGF_ERR_ARG;
    if (!fwd && !(a_kcontig && !b_kcontig)) return EEGF_ERR_ARG;
  }
  GemmArgs a{A, B, C, bias, aux, lda, ldb, ldc, ldaux, strideA, strideB, strideC, strideAux, strideBias, M, N, K, alpha, beta, epi_scale, 0,
             1, 128};
  if (dtype == EEGF_BF16 && batch == 1) {
    const int st = eegf_gemm_big(a_kcontig, b_kcontig, epi, out_dtype == EEGF_F32, M, N, K, A, lda, B, ldb, C, ldc,
                                 bias, aux, ldaux, alpha, beta, epi_scale, workspace, ws_bytes, stream);
    if (st != 1) return st;
  }
  // under-filled grids (the batch-row decoder / head GEMMs, M = B): 64 x 64 tiles quadruple the
  // workgroups; then split-K for long contractions (weight gradients, K = tokens) and for the
  // batch-row GEMMs; the fixed-order slab reduction applies the epilogue.
  if (((M + BM - 1) / BM) * ((N + BN - 1) / BN) * batch < 192) a.bt = 64;
  // (32 x 32 tiles over the whole K instead of split-K measured slower: a 256 x 768 x 768 fp32 product
  // took 19.3 us on 192 workgroups against 11.7 us + a 5 us reduce on 48 tiles x 4 splits,
  // profiles/r6e_prof_ab.log)
  const int tiles = ((M + a.bt - 1) / a.bt) * ((N + a.bt - 1) / a.bt);
  if (batch > 1 && epi == EPI_NONE && workspace && tiles * batch <= 256 && K >= 512) {
    // batched plain GEMMs on an under-filled grid (the decoder's per-head dq = dqp Wk_h, 48 workgroups
    // over K = 768 took 28 us): split K as for the batch-row GEMMs, slabs [split][batch][M][N]
    const int kt = dtype == EEGF_F32 ? 32 : 64;
    const int min_slice = dtype == EEGF_F32 ? 128 : 256;
    int splits = 1;
    while (splits * tiles * batch < 512 && K / (splits * 2) >= min_slice) splits *= 2;
    while (splits > 1 && (long)splits * batch * M * N * 4 > ws_bytes) splits /= 2;
    if (splits > 1) {
      int ks = (K + splits - 1) / splits;
      ks = (ks + kt - 1) / kt * kt;
      splits = (K + ks - 1) / ks;
      GemmArgs b = a;
      b.C = workspace; b.ksplit = ks; b.alpha = alpha;
      int st;
      if (dtype == EEGF_F32) {
        if (out_dtype != EEGF_F32) return EEGF_ERR_ARG;
        st = a_kcontig && b_kcontig ? launch<float, true, true, float, EPI_NONE>(b, batch, stream, splits)
           : a_kcontig ? launch<float, true, false, float, EPI_NONE>(b, batch, stream, splits)
           : b_kcontig ? launch<float, false, true, float, EPI_NONE>(b, batch, stream, splits)
                       : launch<float, false, false, float, EPI_NONE>(b, batch, stream, splits);
        if (st) return st;
        const dim3 grid((unsigned)(((long)batch * M * N + 255) / 256));
        EEGF_LAUNCH(gemm_splitk_reduce_batched<float>, grid, dim3(256), 0, stream, (const float*)workspace,
                           splits, batch, M, N, (float*)C, ldc, strideC, beta);
        return (int)hipGetLastError();
      }
    }
  }
  if (batch == 1 && workspace && tiles < 512 && (K >= 4096 || (tiles <= 256 && K >= 512))) {
    const int kt = dtype == EEGF_F32 ? 32 : 64;
    int splits = 1;
    // fp32 batch-row GEMMs (decoder / head, 48-96 tiles): slices down to 128 so ~200 workgroups fill
    // the CUs (one 64x64 fp32 tile over K = 768 is ~5 us of MFMA on one CU)
    const int min_slice = K >= 4096 ? 1024 : (dtype == EEGF_F32 ? 128 : 256);
    while (splits * tiles < 512 && K / (splits * 2) >= min_slice) splits *= 2;
    while (splits > 1 && (long)splits * M * N * 4 > ws_bytes) splits /= 2;
    if (splits > 1) {
      int ks = (K + splits - 1) / splits;
      ks = (ks + kt - 1) / kt * kt;
      splits = (K + ks - 1) / ks;
      GemmArgs b = a;
      b.C = workspace; b.ksplit = ks; b.alpha = alpha;
      int st;
      if (dtype == EEGF_F32) st = dispatch_layout_split<float, float>(a_kcontig, b_kcontig, b, stream, splits);
      else st = dispatch_layout_split<bf16, float>(a_kcontig, b_kcontig, b, stream, splits);
      if (st) return st;
      return splitk_reduce_dispatch(epi, out_dtype == EEGF_BF16, (const float*)workspace, splits, M, N, C, ldc, beta,
                                    alpha, bias, aux, ldaux, epi_scale, stream);
    }
  }
  if (dtype == EEGF_F32) {
    if (out_dtype != EEGF_F32) return EEGF_ERR_ARG;
    return dispatch_epi<float, float>(epi, a_kcontig, b_kcontig, a, batch, stream);
  }
  if (dtype == EEGF_BF16) {
    if (out_dtype == EEGF_BF16) return dispatch_epi<bf16, bf16>(epi, a_kcontig, b_kcontig, a, batch, stream);
    if (out_dtype == EEGF_F32) return dispatch_epi<bf16, float>(epi, a_kcontig, b_kcontig, a, batch, stream);
  }
  return EEGF_ERR_ARG;
}

extern "C" int eegf_gemm(int dtype, int out_dtype, int a_kcontig, int b_kcontig, int epi,
                         int M, int N, int K, int batch,
                         const void* A, long lda, long strideA,
                         const void* B, long ldb, long strideB,
                         void* C, long ldc, long strideC,
                         const float* bias, long strideBias, void* aux, long ldaux, long strideAux,
                         float alpha, float beta, float epi_scale, void* workspace, long ws_bytes,
                         hipStream_t stream) {
  return gemm_impl(dtype, out_dtype, a_kcontig, b_kcontig, epi, M, N, K, batch, A, lda, strideA, B, ldb, strideB, C,
                   ldc, strideC, bias, strideBias, aux, ldaux, strideAux, alpha, beta, epi_scale, workspace, ws_bytes,
                   stream);
}

extern "C" int eegf_gemm_wgrad_bias(int dtype, int M, int N, int K, const void* dY, long ldd, const void* X, long ldx,
                                    float* dW, long ldw, float beta, float* db, void* workspace, long ws_bytes,
                                    hipStream_t stream) {
  if (dtype != EEGF_BF16 || !dY || !X || !dW || !db || M <= 0 || N <= 0 || K <= 0) return EEGF_ERR_ARG;
  const int st = eegf_gemm_big_wgrad_bias(M, N, K, dY, ldd, X, ldx, dW, ldw, beta, db, workspace, ws_bytes, stream);
  return st == 1 ? EEGF_ERR_ARG : st;
}
