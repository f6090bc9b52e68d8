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

namespace {

constexpr int BM = 128, BN = 128, NT = 256;

struct GemmArgs {
  const void* A; const void* B; void* C; const float* bias; void* aux;
  long lda, ldb, ldc, ldaux;
  long sA, sB, sC, sAux, sBias;
  int M, N, K;
  float alpha, beta, epi_scale;
};

DEV float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
DEV float gelu_grad(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

template <typename T>
struct TileCfg {
  static constexpr int KT = 128 / (int)sizeof(T);        // contraction elements per k-step
  static constexpr int VE = 16 / (int)sizeof(T);         // elements per 16-B chunk
  // K-contiguous LDS tile: [128 rows][KT] + 16 B pad per row
  static constexpr int RS_KC = KT + VE;
  // k-major LDS tile: [KT rows][128] + 32 B pad per row
  static constexpr int RS_KM = 128 + 2 * VE;
  static constexpr int SZ_KC = 128 * RS_KC;
  static constexpr int SZ_KM = KT * RS_KM;
};

// Load one 16-KB operand tile into 4 x 16-B registers per thread (guarded at the edges).
// rows_is_mn: true for the K-contiguous layout (tile rows = m or n index).
template <typename T, bool KC>
DEV void load_tile(u32x4 (&reg)[4], const T* __restrict__ base, long ld, int mn0, int k0, int MN, int K, int tid) {
  using C = TileCfg<T>;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + NT * i;
    int r, col;            // r = tile row, col = element offset within row
    if (KC) { r = c >> 3; col = (c & 7) * C::VE; }
    else    { constexpr int CPR = 128 / C::VE; r = c / CPR; col = (c % CPR) * C::VE; }
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

template <typename T, bool KC>
DEV void store_tile(T* lds, const u32x4 (&reg)[4], int tid) {
  using C = TileCfg<T>;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + NT * i;
    int r, col;
    if (KC) { r = c >> 3; col = (c & 7) * C::VE; }
    else    { constexpr int CPR = 128 / C::VE; r = c / CPR; col = (c % CPR) * C::VE; }
    st16(lds + r * (KC ? C::RS_KC : C::RS_KM) + col, reg[i]);
  }
}

template <typename T, bool AKC, bool BKC, typename TO, int EPI>
__global__ void __launch_bounds__(NT) gemm_kernel(GemmArgs g) {
  using C = TileCfg<T>;
  using F = typename Frag8<T>::type;
  constexpr int SZA = AKC ? C::SZ_KC : C::SZ_KM;
  constexpr int SZB = BKC ? C::SZ_KC : C::SZ_KM;
  __shared__ __attribute__((aligned(16))) T lds[SZA + SZB];
  T* As = lds;
  T* Bs = lds + SZA;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (g.N + BN - 1) / BN, tiles_m = (g.M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.y;

  const T* A = (const T*)g.A + (long)z * g.sA;
  const T* B = (const T*)g.B + (long)z * g.sB;
  TO* Cp = (TO*)g.C + (long)z * g.sC;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  const int nk = (g.K + C::KT - 1) / C::KT;
  load_tile<T, AKC>(ra, A, g.lda, m0, 0, g.M, g.K, tid);
  load_tile<T, BKC>(rb, B, g.ldb, n0, 0, g.N, g.K, tid);

  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();                     // previous k-step's LDS reads are done
    store_tile<T, AKC>(As, ra, tid);
    store_tile<T, BKC>(Bs, rb, tid);
    __syncthreads();
    if (kt + 1 < nk) {                   // issue next k-step's global loads under the MFMAs
      load_tile<T, AKC>(ra, A, g.lda, m0, (kt + 1) * C::KT, g.M, g.K, tid);
      load_tile<T, BKC>(rb, B, g.ldb, n0, (kt + 1) * C::KT, g.N, g.K, tid);
    }
#pragma unroll
    for (int kc = 0; kc < C::KT / 32; ++kc) {
      F a[4], b[4];
      const int kk = kc * 32 + 8 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16;
        if (AKC) a[i] = ld_row8(As + (r + (lane & 15)) * C::RS_KC + kk);
        else     a[i] = ld_col8(As, C::RS_KM, kk, r, lane);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = wn * 64 + j * 16;
        if (BKC) b[j] = ld_row8(Bs + (c + (lane & 15)) * C::RS_KC + kk);
        else     b[j] = ld_col8(Bs, C::RS_KM, kk, c, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mma16(a[i], b[j], acc[i][j]);
    }
  }

  // ---- epilogue ----
  TO* aux = (TO*)g.aux + (long)z * g.sAux;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + (lane & 15);
    if (n >= g.N) continue;
    float bias = 0.f;
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_TANH) bias = g.bias[(long)z * g.sBias + n];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= g.M) continue;
        float v = g.alpha * acc[i][j][r];
        if (EPI == EPI_BIAS) v += bias;
        else if (EPI == EPI_BIAS_GELU) {
          v += bias;
          aux[(long)m * g.ldaux + n] = from_f32<TO>(v);
          v = gelu_f(v);
        } else if (EPI == EPI_BIAS_RELU) v = fmaxf(v + bias, 0.f);
        else if (EPI == EPI_BIAS_TANH) v = tanhf(v + bias);
        else if (EPI == EPI_DGELU) v *= gelu_grad(to_f32(aux[(long)m * g.ldaux + n]));
        else if (EPI == EPI_DRELU) v = to_f32(aux[(long)m * g.ldaux + n]) > 0.f ? v * g.epi_scale : 0.f;
        else if (EPI == EPI_DTANH) { const float y = to_f32(aux[(long)m * g.ldaux + n]); v *= (1.f - y * y); }
        TO* cp = Cp + (long)m * g.ldc + n;
        if (g.beta != 0.f) v += g.beta * to_f32(*cp);
        *cp = from_f32<TO>(v);
      }
    }
  }
}

template <typename T, bool AKC, bool BKC, typename TO, int EPI>
int launch(const GemmArgs& a, int batch, hipStream_t s) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_kernel<T, AKC, BKC, TO, EPI>), dim3(tiles, batch), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
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
  }
  return EEGF_ERR_ARG;
}

}  // namespace

extern "C" int eegf_gemm(int dtype, int out_dtype, int a_kcontig, int b_kcontig, int epi,
                         int M, int N, int K, int batch,
                         const void* A, long lda, long strideA,
                         const void* B, long ldb, long strideB,
                         void* C, long ldc, long strideC,
                         const float* bias, long strideBias, void* aux, long ldaux, long strideAux,
                         float alpha, float beta, float epi_scale, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || !A || !B || !C) return EEGF_ERR_ARG;
  if (batch > 65535) return EEGF_ERR_ARG;
  const bool has_bias = epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_RELU || epi == EPI_BIAS_TANH;
  if (has_bias && !bias) return EEGF_ERR_ARG;
  if ((epi == EPI_BIAS_GELU || epi == EPI_DGELU || epi == EPI_DRELU || epi == EPI_DTANH) && !aux) return EEGF_ERR_ARG;
  if (epi != EPI_NONE) {
    const bool fwd = epi <= EPI_BIAS_TANH;
    if (fwd && !(a_kcontig && b_kcontig)) return EEGF_ERR_ARG;
    if (!fwd && !(a_kcontig && !b_kcontig)) return EEGF_ERR_ARG;
  }
  GemmArgs a{A, B, C, bias, aux, lda, ldb, ldc, ldaux, strideA, strideB, strideC, strideAux, strideBias, M, N, K, alpha, beta, epi_scale};
  if (dtype == EEGF_F32) {
    if (out_dtype != EEGF_F32) return EEGF_ERR_ARG;
    return dispatch_epi<float, float>(epi, a_kcontig, b_kcontig, a, batch, stream);
  }
  if (dtype == EEGF_BF16) {
    if (out_dtype == EEGF_BF16) return dispatch_epi<bf16, bf16>(epi, a_kcontig, b_kcontig, a, batch, stream);
    if (out_dtype == EEGF_F32) {
      if (epi != EPI_NONE) return EEGF_ERR_ARG;
      return dispatch_layout<bf16, float, EPI_NONE>(a_kcontig, b_kcontig, a, batch, stream);
    }
  }
  return EEGF_ERR_ARG;
}
