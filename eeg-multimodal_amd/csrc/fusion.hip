// fusion.hip — fused feature concat + row min-max + privacy stage (PriGumbel / PriConcat), and
// the cross-entropy loss, forward and backward.
//
//   concat:    f = [pooled | img | cross]  (B x 2304, EEG || action || cross)    model.py:46
//   min-max:   xn = (f - min f) / (max f - min f), no epsilon                      model.py:47-50
//   PriGumbel: w = sigmoid(DP); y = xn + n * eps_hat(w), n ~ Laplace(0,1);
//              eps_hat = 1/ln((e^eps - w)/(1-w)) ("newfrac", past_acc.py:132) or ln(...) ("new",
//              model.py:57); m = gumbel_softmax(stack(w, 1-w), tau=1, hard, dim=0);
//              out = y*m0 + y*m1                                                   past_acc.py:130-136
//   PriConcat: DP_guarantee(f, eps, dp_mode) — identity as ConcatModel.forward calls it
//              (main_0430.py:118), or 'feature_all_lap': minmax + one Laplace(0,1/eps) per row.
// One 768-thread workgroup (12 waves) per sample row, thread t owning features t, 768 + t and 1536 + t
// (one element of each encoder's row: three coalesced row reads, no branch); the Laplace/Gumbel draws
// come from Philox(seed, offset, element) unless injected (parity mode), and are regenerated in the
// backward.  Round 5 ran 256 threads x 9 elements: one wave per SIMD with nine serial Philox + log
// chains per lane, 19-20 us per launch at B = 256 (latency-bound, ~0.35 TB/s).
#include "common.h"
#include "eegfusion_internal.h"

namespace {

constexpr int D3 = 2304, D1 = 768;
constexpr int FT = 768, FW = FT / 64, PER = D3 / FT;  // fusion kernels: 768 threads, 12 waves, 3 features each

struct FusionArgs {
  const void* pooled; const void* img; const void* cross; long ld_pooled, ld_img, ld_cross;
  const float* DP; const float* noise; const float* gumbels; const float* row_noise;
  int B, variant, hard, eps_mode; float eps_a, lap_scale, tau;
  uint64_t seed, offset;
  void* out; float* xn; int* amin; int* amax; float* range;
  // backward
  const void* dout; void* d_pooled; void* d_img; void* d_cross; float* ddp_rows;
};

template <typename T>
DEV float feat(const FusionArgs& a, int b, int j) {
  if (j < D1) return to_f32(((const T*)a.pooled)[(long)b * a.ld_pooled + j]);
  if (j < 2 * D1) return to_f32(((const T*)a.img)[(long)b * a.ld_img + j - D1]);
  return to_f32(((const T*)a.cross)[(long)b * a.ld_cross + j - 2 * D1]);
}

DEV float gumbel_of(uint32_t word) {
  const float u = ((float)(word >> 9) + 0.5f) * 0x1p-23f;
  return -logf(-logf(u));
}

// laplace(0,1), gumbel_0, gumbel_1 for element (b, j)
DEV void draws(const FusionArgs& a, int b, int j, float& n, float& g0, float& g1) {
  const long e = (long)b * D3 + j;
  if (a.noise && a.gumbels) {
    n = a.noise[e];
    g0 = a.gumbels[e];
    g1 = a.gumbels[(long)a.B * D3 + e];
    return;
  }
  const u32x4s r = philox4x32((uint32_t)e, (uint32_t)(e >> 32), (uint32_t)a.offset, (uint32_t)(a.offset >> 32),
                              (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
  // torch Laplace.rsample: u ~ U[finfo.eps - 1, 1), n = -sign(u) log1p(-|u|)   (laplace.py:83-86)
  const float u = (float)(r.x >> 8) * (1.0f / 16777216.0f) * (2.0f - 1.1920929e-7f) + (1.1920929e-7f - 1.0f);
  n = a.noise ? a.noise[e] : -copysignf(1.f, u) * log1pf(-fabsf(u)) * (u == 0.f ? 0.f : 1.f);
  // gumbel = -log(E), E ~ Exp(1) = -log(U).  U = (k + 1/2) 2^-23, k in [0, 2^23), lies strictly
  // inside (0, 1): its largest value 1 - 2^-24 is an fp32 number (a 24-bit k + 1/2 would round to
  // 2^24, U = 1, E = 0, g = inf and a NaN softmax).  Accurate logf: the fast log of 1 - 2^-24 is 0.
  g0 = a.gumbels ? a.gumbels[e] : gumbel_of(r.y);
  g1 = a.gumbels ? a.gumbels[(long)a.B * D3 + e] : gumbel_of(r.z);
}

DEV float row_laplace(const FusionArgs& a, int b) {
  if (a.row_noise) return a.row_noise[b];
  const u32x4s r = philox4x32((uint32_t)b, 0x5eedu, (uint32_t)a.offset, (uint32_t)(a.offset >> 32),
                              (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
  const float u = (float)(r.x >> 8) * (1.0f / 16777216.0f) * (2.0f - 1.1920929e-7f) + (1.1920929e-7f - 1.0f);
  return -a.lap_scale * copysignf(1.f, u) * log1pf(-fabsf(u)) * (u == 0.f ? 0.f : 1.f);
}

struct GateVals { float w, eh, ys0, ys1, r0, r1, n; };

DEV GateVals gate(const FusionArgs& a, int b, int j) {
  GateVals v;
  const float dp = a.DP[j];
  v.w = 1.0f / (1.0f + __expf(-dp));
  const float lr = __logf((a.eps_a - v.w) / (1.0f - v.w));
  v.eh = a.eps_mode == 0 ? 1.0f / lr : lr;
  float g0, g1;
  draws(a, b, j, v.n, g0, g1);
  const float z0 = (v.w + g0) / a.tau, z1 = ((1.0f - v.w) + g1) / a.tau;
  const float mz = fmaxf(z0, z1);
  const float e0 = __expf(z0 - mz), e1 = __expf(z1 - mz), s = e0 + e1;
  v.ys0 = e0 / s;
  v.ys1 = e1 / s;
  if (a.hard) {
    const float h0 = v.ys0 >= v.ys1 ? 1.f : 0.f;   // argmax, first index on ties
    v.r0 = (h0 - v.ys0) + v.ys0;
    v.r1 = ((1.f - h0) - v.ys1) + v.ys1;
  } else {
    v.r0 = v.ys0;
    v.r1 = v.ys1;
  }
  return v;
}

// block argmin/argmax (first index on ties: the (value, index) order is total, so the result does
// not depend on the reduction order); NW waves
template <int NW = 4>
DEV void block_minmax(float& vmin, int& imin, float& vmax, int& imax) {
  __shared__ float smin[NW], smax[NW];
  __shared__ int simin[NW], simax[NW];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(vmin, o, 64), oM = __shfl_xor(vmax, o, 64);
    const int oi = __shfl_xor(imin, o, 64), oI = __shfl_xor(imax, o, 64);
    if (om < vmin || (om == vmin && oi < imin)) { vmin = om; imin = oi; }
    if (oM > vmax || (oM == vmax && oI < imax)) { vmax = oM; imax = oI; }
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smin[wave] = vmin; simin[wave] = imin; smax[wave] = vmax; simax[wave] = imax; }
  __syncthreads();
  vmin = smin[0]; imin = simin[0]; vmax = smax[0]; imax = simax[0];
  for (int w = 1; w < NW; ++w) {
    if (smin[w] < vmin || (smin[w] == vmin && simin[w] < imin)) { vmin = smin[w]; imin = simin[w]; }
    if (smax[w] > vmax || (smax[w] == vmax && simax[w] < imax)) { vmax = smax[w]; imax = simax[w]; }
  }
}

template <int NW = 4>
DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) s += red[w];
  return s;
}

template <typename T>
__global__ void __launch_bounds__(FT) fusion_fwd_kernel(FusionArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  float x[PER];
  float vmin = 3.4e38f, vmax = -3.4e38f;
  int imin = 0x7fffffff, imax = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = tid + FT * k;
    x[k] = feat<T>(a, b, j);
    if (x[k] < vmin) { vmin = x[k]; imin = j; }
    if (x[k] > vmax) { vmax = x[k]; imax = j; }
  }
  T* out = (T*)a.out + (long)b * D3;
  if (a.variant == FUSE_PRICONCAT) {                      // DP_guarantee(dp_mode=None): identity
#pragma unroll
    for (int k = 0; k < PER; ++k) out[tid + FT * k] = from_f32<T>(x[k]);
    return;
  }
  // the gate (DP load, Philox, Laplace / Gumbel logs, softmax) does not depend on the row's min / max:
  // computed before the block reduction, so its latency overlaps the feature loads and the barriers
  GateVals gv[PER];
  if (a.variant == FUSE_PRIGUMBEL) {
#pragma unroll
    for (int k = 0; k < PER; ++k) gv[k] = gate(a, b, tid + FT * k);
  }
  const float rn = a.variant == FUSE_PRICONCAT_LAP ? row_laplace(a, b) : 0.f;
  block_minmax<FW>(vmin, imin, vmax, imax);
  const float R = vmax - vmin;
  if (tid == 0 && a.amin) { a.amin[b] = imin; a.amax[b] = imax; a.range[b] = R; }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = tid + FT * k;
    const float xn = (x[k] - vmin) / R;
    if (a.xn) a.xn[(long)b * D3 + j] = xn;
    float o;
    if (a.variant == FUSE_PRIGUMBEL) {
      const GateVals& g = gv[k];
      const float y = xn + g.n * g.eh;
      o = y * g.r0 + y * g.r1;
    } else if (a.variant == FUSE_PRICONCAT_LAP) {
      o = xn + rn;
    } else {
      o = xn;
    }
    out[j] = from_f32<T>(o);
  }
}

template <typename T>
__global__ void __launch_bounds__(FT) fusion_bwd_kernel(FusionArgs a) {
  __shared__ float red[FW];
  const int b = blockIdx.x, tid = threadIdx.x;
  const T* dout = (const T*)a.dout + (long)b * D3;
  float dxn[PER], xn[PER];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = tid + FT * k;
    const float d = to_f32(dout[j]);
    if (a.variant == FUSE_PRIGUMBEL) {
      const GateVals g = gate(a, b, j);
      xn[k] = a.xn[(long)b * D3 + j];
      const float dy = d * g.r0 + d * g.r1;
      dxn[k] = dy;
      if (a.ddp_rows) {
        const float y = xn[k] + g.n * g.eh;
        const float deh = dy * g.n;
        const float am1 = a.eps_a - 1.0f;
        const float dehdw = (a.eps_mode == 0 ? -g.eh * g.eh : 1.0f) * am1 / ((a.eps_a - g.w) * (1.0f - g.w));
        const float G = d * y;                                       // dL/dm_k (both k)
        const float sg = G * g.ys0 + G * g.ys1;
        const float dz0 = g.ys0 * (G - sg) / a.tau, dz1 = g.ys1 * (G - sg) / a.tau;
        const float dw = deh * dehdw + dz0 - dz1;
        a.ddp_rows[(long)b * D3 + j] = dw * g.w * (1.0f - g.w);
      }
    } else if (a.variant == FUSE_PRICONCAT) {
      dxn[k] = d;
      xn[k] = 0.f;
    } else {
      xn[k] = a.xn[(long)b * D3 + j];
      dxn[k] = d;
    }
    s1 += dxn[k] * (xn[k] - 1.0f);
    s2 += dxn[k] * xn[k];
  }
  float R = 1.f;
  int imin = -1, imax = -1;
  if (a.variant != FUSE_PRICONCAT) {
    s1 = block_sum<FW>(s1, red);
    s2 = block_sum<FW>(s2, red);
    R = a.range[b];
    imin = a.amin[b];
    imax = a.amax[b];
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int j = tid + FT * k;
    float dx = dxn[k] / R;
    if (j == imin) dx += s1 / R;
    if (j == imax) dx -= s2 / R;
    if (j < D1) ((T*)a.d_pooled)[(long)b * a.ld_pooled + j] = from_f32<T>(dx);
    else if (j < 2 * D1) ((T*)a.d_img)[(long)b * a.ld_img + j - D1] = from_f32<T>(dx);
    else ((T*)a.d_cross)[(long)b * a.ld_cross + j - 2 * D1] = from_f32<T>(dx);
  }
}

// cross-entropy over C classes (F.cross_entropy, mean or sum) + argmax correct count
template <typename T>
__global__ void __launch_bounds__(256) ce_kernel(const T* logits, const long long* labels, int B, int C, int reduction,
                                                 float dscale, float* loss, int* correct, T* dlogits) {
  __shared__ float red[4];
  __shared__ int redc[4];
  float l = 0.f;
  int c = 0;
  const float norm = reduction == 0 ? 1.0f / B : 1.0f;
  for (int b = threadIdx.x; b < B; b += 256) {
    const T* z = logits + (long)b * C;
    float mx = -3.4e38f;
    int am = 0;
    for (int k = 0; k < C; ++k) { const float v = to_f32(z[k]); if (v > mx) { mx = v; am = k; } }
    float s = 0.f;
    for (int k = 0; k < C; ++k) s += __expf(to_f32(z[k]) - mx);
    const float lse = mx + __logf(s);
    const int y = (int)labels[b];
    l += lse - to_f32(z[y]);
    c += (am == y);
    if (dlogits)
      for (int k = 0; k < C; ++k)
        dlogits[(long)b * C + k] = from_f32<T>((__expf(to_f32(z[k]) - lse) - (k == y ? 1.f : 0.f)) * norm * dscale);
  }
  l = wave_sum(l);
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = l; redc[threadIdx.x >> 6] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (loss) *loss = (red[0] + red[1] + red[2] + red[3]) * norm;
    if (correct) *correct = redc[0] + redc[1] + redc[2] + redc[3];
  }
}

// feawei DP initialisation (past_acc.py:98-103; past_acc_feawei.py:153-163): m = colsum / count is the
// column mean of the normalised features of a forward pass over the train set; z = (m - mean m) /
// std m (np.std, ddof 0) when zscore, else z = m; w = 1 - sigmoid(k z) in fp32;
// DP = (base + w) - 0.5.  One 256-thread workgroup; mean and variance accumulate in fp64 (the
// reference's feature matrix is a float64 numpy array), two passes.
DEV double block_sum_f64(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void feawei_kernel(int D, const float* colsum, double inv_count, float k,
                                                     int zscore, const float* base, float* dp) {
  __shared__ double red[4];
  double mu = 0.0, sd = 1.0;
  if (zscore) {
    double s = 0.0;
    for (int c = threadIdx.x; c < D; c += 256) s += (double)colsum[c] * inv_count;
    mu = block_sum_f64(s, red) / D;
    double q = 0.0;
    for (int c = threadIdx.x; c < D; c += 256) {
      const double d = (double)colsum[c] * inv_count - mu;
      q += d * d;
    }
    sd = sqrt(block_sum_f64(q, red) / D);
  }
  for (int c = threadIdx.x; c < D; c += 256) {
    const double m = (double)colsum[c] * inv_count;
    const float x = (float)((double)k * (zscore ? (m - mu) / sd : m));
    const float w = 1.0f - 1.0f / (1.0f + expf(-x));
    dp[c] = (base[c] + w) - 0.5f;
  }
}

// ---------------------------------------------------------------------------------------------
// PriGumbel-v1 (train_val.py:95-158): after fc1 + ReLU + fc2 the 768-wide feature x goes through
//   gumbel_dropout: logits_j = (w_j, 1 - w_j) (raw w, no sigmoid), m_j = gumbel_softmax(logits_j,
//     tau, hard)[1] with ONE Gumbel pair per feature shared by the whole batch (the [768, 2] call,
//     dim -1); hard = straight-through one-hot of the argmax (first index on ties);
//     res = x * m / (1 - w)                                                     :95-101
//   Lap_noise: row min-max of res, + one Laplace(0, 1/eps) draw per row          :114-123
// and the loss adds max_j((1 - w_j) e^eps + w_j) (loss_function :80-93).  Draws: Philox(seed, offset,
// counter j) words y, z for the feature's pair, the row draw as row_laplace; or injected.
constexpr int V1D = 768, V1PER = V1D / 256;

struct V1Vals { float m, dmdw; };

DEV V1Vals v1_mask(const FusionArgs& a, int j) {
  float g0, g1;
  if (a.gumbels) {
    g0 = a.gumbels[2 * j];
    g1 = a.gumbels[2 * j + 1];
  } else {
    const u32x4s r = philox4x32((uint32_t)j, 0x76316731u, (uint32_t)a.offset, (uint32_t)(a.offset >> 32),
                                (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
    g0 = gumbel_of(r.y);
    g1 = gumbel_of(r.z);
  }
  const float w = a.DP[j];
  const float z0 = (w + g0) / a.tau, z1 = ((1.0f - w) + g1) / a.tau;
  const float mz = fmaxf(z0, z1);
  const float e0 = __expf(z0 - mz), e1 = __expf(z1 - mz), sm = e0 + e1;
  const float s0 = e0 / sm, s1 = e1 / sm;
  V1Vals v;
  v.m = a.hard ? (((s0 >= s1 ? 0.f : 1.f) - s1) + s1) : s1;
  v.dmdw = -2.0f * s0 * s1 / a.tau;          // d s1 / d w (the straight-through estimator keeps it)
  return v;
}

// one workgroup per row; a.pooled = x [B, 768] fp32 (row stride ld_pooled), a.DP = w [768]
__global__ void __launch_bounds__(256) v1_fwd_kernel(FusionArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* x = (const float*)a.pooled + (long)b * a.ld_pooled;
  float r[V1PER];
  float vmin = 3.4e38f, vmax = -3.4e38f;
  int imin = 0x7fffffff, imax = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < V1PER; ++k) {
    const int j = tid + 256 * k;
    const V1Vals v = v1_mask(a, j);
    r[k] = x[j] * v.m / (1.0f - a.DP[j]);
    if (r[k] < vmin) { vmin = r[k]; imin = j; }
    if (r[k] > vmax) { vmax = r[k]; imax = j; }
  }
  block_minmax(vmin, imin, vmax, imax);
  const float R = vmax - vmin;
  if (tid == 0) { a.amin[b] = imin; a.amax[b] = imax; a.range[b] = R; }
  const float rn = row_laplace(a, b);
  float* out = (float*)a.out + (long)b * V1D;
#pragma unroll
  for (int k = 0; k < V1PER; ++k) {
    const int j = tid + 256 * k;
    const float xn = (r[k] - vmin) / R;
    a.xn[(long)b * V1D + j] = xn;
    out[j] = xn + rn;
  }
}

__global__ void __launch_bounds__(256) v1_bwd_kernel(FusionArgs a) {
  __shared__ float red[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* dout = (const float*)a.dout + (long)b * V1D;
  const float* x = (const float*)a.pooled + (long)b * a.ld_pooled;
  float d[V1PER], xn[V1PER];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < V1PER; ++k) {
    const int j = tid + 256 * k;
    d[k] = dout[j];
    xn[k] = a.xn[(long)b * V1D + j];
    s1 += d[k] * (xn[k] - 1.0f);
    s2 += d[k] * xn[k];
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  const float R = a.range[b];
  const int imin = a.amin[b], imax = a.amax[b];
  float* dx = (float*)a.d_pooled + (long)b * a.ld_pooled;
#pragma unroll
  for (int k = 0; k < V1PER; ++k) {
    const int j = tid + 256 * k;
    float dr = d[k] / R;
    if (j == imin) dr += s1 / R;
    if (j == imax) dr -= s2 / R;
    const V1Vals v = v1_mask(a, j);
    const float iw = 1.0f / (1.0f - a.DP[j]);
    dx[j] = dr * v.m * iw;
    if (a.ddp_rows) a.ddp_rows[(long)b * V1D + j] = dr * x[j] * (v.dmdw * iw + v.m * iw * iw);
  }
}

// loss_w = max_j((1 - w_j) a + w_j), a = e^eps (first index on ties, torch.max); dw[j*] += dscale (1 - a)
__global__ void __launch_bounds__(256) v1_wloss_kernel(int D, const float* __restrict__ w, float eps_a, float dscale,
                                                       float* __restrict__ loss, float* __restrict__ dw) {
  float vmax = -3.4e38f, vmin = 3.4e38f;
  int imax = 0x7fffffff, imin = 0x7fffffff;
  for (int j = threadIdx.x; j < D; j += 256) {
    const float v = (1.0f - w[j]) * eps_a + w[j];
    if (v > vmax) { vmax = v; imax = j; }
  }
  block_minmax(vmin, imin, vmax, imax);
  if (threadIdx.x == 0) {
    if (loss) *loss = vmax;
    if (dw) dw[imax] += dscale * (1.0f - eps_a);
  }
}

}  // namespace

extern "C" int eegf_fusion_fwd(int dtype, int B, int variant, const void* pooled, long ld_pooled, const void* img,
                               long ld_img, const void* cross, long ld_cross, const float* DP, const float* noise,
                               const float* gumbels, const float* row_noise, int hard, int eps_mode, float eps_a,
                               float lap_scale, unsigned long long seed, unsigned long long offset, void* out,
                               float* xn, int* amin, int* amax, float* range, hipStream_t stream) {
  if (B <= 0 || B > 0x7fffffff / D3 || !pooled || !img || !cross || !out) return EEGF_ERR_ARG;
  if (variant < FUSE_CONCAT || variant > FUSE_PRIGUMBEL) return EEGF_ERR_ARG;
  if (variant == FUSE_PRIGUMBEL && (!DP || eps_a <= 1.0f)) return EEGF_ERR_ARG;
  if ((noise == nullptr) != (gumbels == nullptr) && variant == FUSE_PRIGUMBEL) return EEGF_ERR_ARG;
  FusionArgs a{};
  a.pooled = pooled; a.img = img; a.cross = cross; a.ld_pooled = ld_pooled; a.ld_img = ld_img; a.ld_cross = ld_cross;
  a.DP = DP; a.noise = noise; a.gumbels = gumbels; a.row_noise = row_noise; a.B = B; a.variant = variant;
  a.hard = hard; a.eps_mode = eps_mode; a.eps_a = eps_a; a.lap_scale = lap_scale; a.tau = 1.0f;
  a.seed = seed; a.offset = offset; a.out = out; a.xn = xn; a.amin = amin; a.amax = amax; a.range = range;
  if (variant != FUSE_PRICONCAT && (!amin || !amax || !range)) return EEGF_ERR_ARG;
  if (dtype == EEGF_F32) EEGF_LAUNCH(fusion_fwd_kernel<float>, dim3(B), dim3(FT), 0, stream, a);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(fusion_fwd_kernel<bf16>, dim3(B), dim3(FT), 0, stream, a);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_fusion_bwd(int dtype, int B, int variant, const void* dout, const float* xn, const int* amin,
                               const int* amax, const float* range, const float* DP, const float* noise,
                               const float* gumbels, int hard, int eps_mode, float eps_a, unsigned long long seed,
                               unsigned long long offset, void* d_pooled, long ld_pooled, void* d_img, long ld_img,
                               void* d_cross, long ld_cross, float* ddp_rows, hipStream_t stream) {
  if (B <= 0 || !dout || !d_pooled || !d_img || !d_cross) return EEGF_ERR_ARG;
  if (variant < FUSE_CONCAT || variant > FUSE_PRIGUMBEL) return EEGF_ERR_ARG;
  if (variant != FUSE_PRICONCAT && (!xn || !amin || !amax || !range)) return EEGF_ERR_ARG;
  if (variant == FUSE_PRIGUMBEL && (!DP || eps_a <= 1.0f)) return EEGF_ERR_ARG;
  FusionArgs a{};
  a.dout = dout; a.xn = const_cast<float*>(xn); a.amin = const_cast<int*>(amin); a.amax = const_cast<int*>(amax);
  a.range = const_cast<float*>(range); a.DP = DP; a.noise = noise; a.gumbels = gumbels; a.B = B;
  a.variant = variant; a.hard = hard; a.eps_mode = eps_mode; a.eps_a = eps_a; a.tau = 1.0f; a.seed = seed;
  a.offset = offset; a.d_pooled = d_pooled; a.ld_pooled = ld_pooled; a.d_img = d_img; a.ld_img = ld_img;
  a.d_cross = d_cross; a.ld_cross = ld_cross; a.ddp_rows = ddp_rows;
  if (dtype == EEGF_F32) EEGF_LAUNCH(fusion_bwd_kernel<float>, dim3(B), dim3(FT), 0, stream, a);
  else if (dtype == EEGF_BF16) EEGF_LAUNCH(fusion_bwd_kernel<bf16>, dim3(B), dim3(FT), 0, stream, a);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_cross_entropy(int dtype, int B, int C, const void* logits, const long long* labels,
                                  int reduction, float dscale, float* loss, int* correct, void* dlogits,
                                  hipStream_t stream) {
  if (B <= 0 || C <= 0 || C > 64 || !logits || !labels) return EEGF_ERR_ARG;
  if (dtype == EEGF_F32)
    EEGF_LAUNCH(ce_kernel<float>, dim3(1), dim3(256), 0, stream, (const float*)logits, labels, B, C, reduction,
                       dscale, loss, correct, (float*)dlogits);
  else if (dtype == EEGF_BF16)
    EEGF_LAUNCH(ce_kernel<bf16>, dim3(1), dim3(256), 0, stream, (const bf16*)logits, labels, B, C, reduction,
                       dscale, loss, correct, (bf16*)dlogits);
  else return EEGF_ERR_ARG;
  return (int)hipGetLastError();
}

extern "C" int eegf_v1_gate_fwd(int B, const float* x, long ldx, const float* w, const float* gumbels,
                                const float* row_noise, float tau, int hard, float lap_scale, unsigned long long seed,
                                unsigned long long offset, float* out, float* xn, int* amin, int* amax, float* range,
                                hipStream_t stream) {
  if (B <= 0 || !x || !w || !out || !xn || !amin || !amax || !range || !(tau > 0.f) || ldx < V1D) return EEGF_ERR_ARG;
  FusionArgs a{};
  a.pooled = x; a.ld_pooled = ldx; a.DP = w; a.gumbels = gumbels; a.row_noise = row_noise; a.B = B; a.hard = hard;
  a.tau = tau; a.lap_scale = lap_scale; a.seed = seed; a.offset = offset; a.out = out; a.xn = xn; a.amin = amin;
  a.amax = amax; a.range = range;
  EEGF_LAUNCH(v1_fwd_kernel, dim3(B), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

extern "C" int eegf_v1_gate_bwd(int B, const float* dout, const float* x, long ldx, const float* w,
                                const float* gumbels, const float* xn, const int* amin, const int* amax,
                                const float* range, float tau, int hard, unsigned long long seed,
                                unsigned long long offset, float* dx, float* dw_rows, hipStream_t stream) {
  if (B <= 0 || !dout || !x || !w || !xn || !amin || !amax || !range || !dx || !(tau > 0.f) || ldx < V1D)
    return EEGF_ERR_ARG;
  FusionArgs a{};
  a.dout = dout; a.pooled = x; a.ld_pooled = ldx; a.DP = w; a.gumbels = gumbels; a.xn = const_cast<float*>(xn);
  a.amin = const_cast<int*>(amin); a.amax = const_cast<int*>(amax); a.range = const_cast<float*>(range); a.B = B;
  a.hard = hard; a.tau = tau; a.seed = seed; a.offset = offset; a.d_pooled = dx; a.ddp_rows = dw_rows;
  EEGF_LAUNCH(v1_bwd_kernel, dim3(B), dim3(256), 0, stream, a);
  return (int)hipGetLastError();
}

extern "C" int eegf_v1_wloss(int D, const float* w, float eps_a, float dscale, float* loss, float* dw,
                             hipStream_t stream) {
  if (D <= 0 || !w) return EEGF_ERR_ARG;
  EEGF_LAUNCH(v1_wloss_kernel, dim3(1), dim3(256), 0, stream, D, w, eps_a, dscale, loss, dw);
  return (int)hipGetLastError();
}

extern "C" int eegf_feawei_init(int D, const float* colsum, long count, float k, int zscore, const float* base,
                                float* dp, hipStream_t stream) {
  if (D <= 0 || count <= 0 || !colsum || !base || !dp) return EEGF_ERR_ARG;
  EEGF_LAUNCH(feawei_kernel, dim3(1), dim3(256), 0, stream, D, colsum, 1.0 / (double)count, k, zscore,
                     base, dp);
  return (int)hipGetLastError();
}
