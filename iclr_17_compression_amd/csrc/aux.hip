// Parameter packing, the factorised rate model as stand-alone kernels, and deterministic
// partial-sum reductions (gfx950). All memory-bound / parameter-sized work.
#include <string.h>

#include "common.h"

namespace iclr17 {

void deconv_phase_taps(int K, int s, int p, int ry, int rx, int* kh_out, int* kw_out, int* count);

namespace {

hipStream_t S(void* s) { return (hipStream_t)s; }

struct TapList {
  int kh[25];
  int kw[25];
};

// Element i of each packed layout (a pure index map of the reference tensor, so a batch of
// packs can run in one launch: pack_batch_kernel below).
// conv1 [N][3][9][9] → [64 quads][N][4], k = c·81 + kh·9 + kw, k ≥ 243 zero.
__device__ __forceinline__ float pk_conv1(const float* __restrict__ w, int N, long i) {
  const int e = i & 3, n = (int)((i >> 2) % N), q = (int)((i >> 2) / N);
  const int k = 4 * q + e;
  return k < 243 ? w[(long)n * 243 + k] : 0.f;
}

// conv1 [N][3][9][9] → [64 quads][N][4] in the x6 kernel's k order (engine_fp32.hip,
// conv1_x6_kernel): k' = 8g + e; g < 27: (c, kh) = (g / 9, g % 9), kw = e; g = 27: zero;
// g ≥ 28: pair (g − 28)·8 + e (< 27, else zero), kw = 8.
__device__ __forceinline__ float pk_conv1_x6(const float* __restrict__ w, int N, long i) {
  const int e4 = i & 3, n = (int)((i >> 2) % N), q = (int)((i >> 2) / N);
  const int k = 4 * q + e4, g = k >> 3, e = k & 7;
  int src = -1;
  if (g < 27) {
    src = g * 9 + e;
  } else if (g >= 28) {
    const int p = (g - 28) * 8 + e;
    if (p < 27) src = p * 9 + 8;
  }
  return src >= 0 ? w[(long)n * 243 + src] : 0.f;
}

// conv k5 [co][ci][5][5] → [25 taps][ci/4][co][4], tap = kh·5 + kw.
__device__ __forceinline__ float pk_conv5(const float* __restrict__ w, int N, long i) {
  const int e = i & 3;
  const int co = (int)((i >> 2) % N);
  const long r = (i >> 2) / N;
  const int q = (int)(r % (N / 4)), tap = (int)(r / (N / 4));
  const int ci = 4 * q + e;
  return w[((long)co * N + ci) * 25 + tap];
}

// deconv k5 [ci][co][5][5] → phase-major taps [25][ci/4][co][4].
__device__ __forceinline__ float pk_deconv5(const float* __restrict__ w, int N, const TapList& tl,
                                            long i) {
  const int e = i & 3;
  const int co = (int)((i >> 2) % N);
  const long r = (i >> 2) / N;
  const int q = (int)(r % (N / 4)), tap = (int)(r / (N / 4));
  const int ci = 4 * q + e;
  return w[((long)ci * N + co) * 25 + tl.kh[tap] * 5 + tl.kw[tap]];
}

// deconv3 [ci][3][9][9] → all-phase [9 neighbours][ci/4][48][4]; column n = co·16 + ry·4 + rx,
// neighbour (dy, dx) ∈ {-1,0,1}², kernel tap k = r + 4 − 4d (zero outside 0..8).
__device__ __forceinline__ float pk_deconv9(const float* __restrict__ w, int N, long i) {
  const int e = i & 3;
  const int n = (int)((i >> 2) % 48);
  const long r = (i >> 2) / 48;
  const int q = (int)(r % (N / 4)), nb = (int)(r / (N / 4));
  const int ci = 4 * q + e;
  const int co = n >> 4, ry = (n >> 2) & 3, rx = n & 3;
  const int dy = nb / 3 - 1, dx = nb % 3 - 1;
  const int kh = ry + 4 - 4 * dy, kw = rx + 4 - 4 * dx;
  float v = 0.f;
  if (kh >= 0 && kh < 9 && kw >= 0 && kw < 9) v = w[(((long)ci * 3 + co) * 9 + kh) * 9 + kw];
  return v;
}

// models/GDN.py:73-79 reparametrisation; gamma packed [C/4][C][4] (packed[q][i][e] = γ[i][4q+e]).
__device__ __forceinline__ void pk_gdn(const float* __restrict__ beta, const float* __restrict__ gamma,
                                       float* __restrict__ beta_eff, float* __restrict__ gp,
                                       float* __restrict__ gpt, int C, float bbound, float gbound,
                                       float ped, int i) {
  if (i < C) {
    const float m = fmaxf(beta[i], bbound);
    beta_eff[i] = m * m - ped;
  }
  if (i < C * C) {
    const int e = i & 3, row = (i >> 2) % C, q = (i >> 2) / C;
    const float m = fmaxf(gamma[(long)row * C + 4 * q + e], gbound);
    gp[i] = m * m - ped;
    if (gpt != nullptr) {
      const float mt = fmaxf(gamma[(long)(4 * q + e) * C + row], gbound);
      gpt[i] = mt * mt - ped;
    }
  }
}

__global__ void pack_conv1_kernel(const float* __restrict__ w, float* __restrict__ out, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 256 * N) out[i] = pk_conv1(w, N, i);
}

__global__ void pack_conv1_x6_kernel(const float* __restrict__ w, float* __restrict__ out, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 256 * N) out[i] = pk_conv1_x6(w, N, i);
}

__global__ void pack_conv5_kernel(const float* __restrict__ w, float* __restrict__ out, int N) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 25L * N * N) out[i] = pk_conv5(w, N, i);
}

__global__ void pack_deconv5_kernel(const float* __restrict__ w, float* __restrict__ out, int N,
                                    TapList tl) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 25L * N * N) out[i] = pk_deconv5(w, N, tl, i);
}

__global__ void pack_deconv9_kernel(const float* __restrict__ w, float* __restrict__ out, int N) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 9L * N * 48) out[i] = pk_deconv9(w, N, i);
}

__global__ void pack_gdn_kernel(const float* __restrict__ beta, const float* __restrict__ gamma,
                                float* __restrict__ beta_eff, float* __restrict__ gp,
                                float* __restrict__ gpt, int C, float bbound, float gbound,
                                float ped) {
  pk_gdn(beta, gamma, beta_eff, gp, gpt, C, bbound, gbound, ped, blockIdx.x * blockDim.x + threadIdx.x);
}

struct RatePtrs {
  const float* p[11];  // h1 b1 a1 h2 b2 a2 h3 b3 a3 h4 b4
};

__device__ __forceinline__ float softplus_ref(float x) {
  // torch.nn.functional.softplus(beta=1, threshold=20)
  return x > 20.f ? x : log1pf(expf(x));
}

__device__ __forceinline__ void pk_rate(const RatePtrs& rp, float* __restrict__ out, int C, int c) {
  for (int k = 0; k < 3; ++k) {
    out[(3 * k + 0) * C + c] = softplus_ref(rp.p[3 * k + 0][c]);
    out[(3 * k + 1) * C + c] = rp.p[3 * k + 1][c];
    out[(3 * k + 2) * C + c] = tanhf(rp.p[3 * k + 2][c]);
  }
  out[9 * C + c] = softplus_ref(rp.p[9][c]);
  out[10 * C + c] = rp.p[10][c];
}

__global__ void pack_rate_kernel(RatePtrs rp, float* __restrict__ out, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) pk_rate(rp, out, C, c);
}

// A batch of packing jobs in one launch (iclr17_pack_batch): job j owns the global thread range
// [begin[j], begin[j+1]) (block-aligned, so a workgroup serves one job); thread i of a job
// computes element i of its layout — or, for a split job, one 8-element group of
// iclr17_split_packed.
constexpr int PACK_MAXJ = 20;
struct PackJob {
  int kind, N, taps, K;
  const float* src0;
  const float* src1;
  void* dst0;
  void* dst1;
  void* dst2;
  float f0, f1, f2;
  long count;
};
struct PackBatch {
  int n;
  long begin[PACK_MAXJ + 1];
  PackJob job[PACK_MAXJ];
  TapList tl;
  RatePtrs rp;
};

__global__ void __launch_bounds__(256) pack_batch_kernel(const PackBatch b) {
  const long gi = (long)blockIdx.x * 256 + threadIdx.x;
  int j = 0;
  while (j + 1 < b.n && gi >= b.begin[j + 1]) ++j;
  const PackJob& J = b.job[j];
  const long i = gi - b.begin[j];
  if (i >= J.count) return;
  float* out = (float*)J.dst0;
  switch (J.kind) {
    case ICLR17_W_CONV1: out[i] = pk_conv1(J.src0, J.N, i); break;
    case ICLR17_W_CONV1_X6: out[i] = pk_conv1_x6(J.src0, J.N, i); break;
    case ICLR17_W_CONV5: out[i] = pk_conv5(J.src0, J.N, i); break;
    case ICLR17_W_DECONV5: out[i] = pk_deconv5(J.src0, J.N, b.tl, i); break;
    case ICLR17_W_DECONV9: out[i] = pk_deconv9(J.src0, J.N, i); break;
    case ICLR17_PACK_GDN:
      pk_gdn(J.src0, J.src1, out, (float*)J.dst1, (float*)J.dst2, J.N, J.f0, J.f1, J.f2, (int)i);
      break;
    case ICLR17_PACK_RATE: pk_rate(b.rp, out, J.N, (int)i); break;
    case ICLR17_PACK_SPLIT:
      split_packed_group(J.src0, J.K, J.N, J.count * 8, (unsigned short*)J.dst0, i);
      break;
  }
}

__global__ void bit_estimator_kernel(const float* __restrict__ x, int64_t n, int C, int64_t inner,
                                     const float* __restrict__ rp, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)((i / inner) % C);
    out[i] = bitparm_cdf(x[i], rp, C, c);
  }
}

// One Bitparm layer (bitEstimator.py:20-25): ta == nullptr selects the final (sigmoid) form.
__global__ void bitparm_kernel(const float* __restrict__ x, int64_t n, int C, int64_t inner,
                               const float* __restrict__ sp, const float* __restrict__ bb,
                               const float* __restrict__ ta, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)((i / inner) % C);
    const float t = x[i] * sp[c] + bb[c];
    out[i] = ta == nullptr ? 1.0f / (1.0f + expf(-t)) : t + tanhf(t) * ta[c];
  }
}

// Autograd of the stand-alone BitEstimator / Bitparm forward (bitEstimator.py:20-42) for an
// upstream gradient g = ∂L/∂out, op for op as rate_bwd_element (engine_fp32.hip) does for the
// rate term. rp is the packed [11][C] table (softplus(h_k), b_k, tanh(a_k) for k = 1..3 at
// slots 3k-3.., softplus(h4), b4 at 9, 10). MODE 0: the 4-layer BitEstimator; 1: one non-final
// Bitparm (slots 0-2); 2: the final Bitparm (slots 9, 10). One workgroup per (channel, chunk of
// that channel's elements): ∂x per element, and the 11 per-channel parameter partials summed in
// a fixed order into partial[chunk][11][C] (iclr17_rate_param_grad turns them into ∂h, ∂b, ∂a).
template <int MODE>
__global__ void __launch_bounds__(256) bitest_bwd_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ g, int64_t E,
                                                         int C, int64_t inner,
                                                         const float* __restrict__ rp,
                                                         float* __restrict__ dx, int64_t per,
                                                         float* __restrict__ partial) {
  __shared__ float red[4][11];
  const int c = blockIdx.x, chunk = blockIdx.y;
  const int64_t e0 = (int64_t)chunk * per;
  const int64_t e1 = e0 + per < E ? e0 + per : E;
  constexpr int K0 = MODE == 1 ? 0 : (MODE == 2 ? 3 : 0);   // first non-final layer
  constexpr int K1 = MODE == 1 ? 1 : (MODE == 2 ? 0 : 3);   // non-final layers
  constexpr bool FINAL = MODE != 1;
  float pg[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) pg[k] = 0.f;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const int64_t i = (e / inner) * C * inner + (int64_t)c * inner + e % inner;
    float v = x[i];
    float xs[4], Ts[3];
#pragma unroll
    for (int k = 0; k < K1; ++k) {
      xs[k] = v;
      const float t = v * rp[(3 * (K0 + k)) * C + c] + rp[(3 * (K0 + k) + 1) * C + c];
      const float T = tanhf(t);
      v = t + T * rp[(3 * (K0 + k) + 2) * C + c];
      Ts[k] = T;
    }
    float gx = g[i];
    if (FINAL) {
      xs[3] = v;
      const float F = 1.0f / (1.0f + expf(-(v * rp[9 * C + c] + rp[10 * C + c])));
      const float gt4 = (gx * (1.0f - F)) * F;              // sigmoid backward
      pg[10] += gt4;                                        // b4
      pg[9] += gt4 * xs[3];                                 // softplus(h4)
      gx = gt4 * rp[9 * C + c];
    }
#pragma unroll
    for (int k = K1 - 1; k >= 0; --k) {
      const int s3 = 3 * (K0 + k);
      const float T = Ts[k];
      const float gT = gx * rp[(s3 + 2) * C + c];
      pg[s3 + 2] += gx * T;                                 // tanh(a_k)
      const float gt = gx + gT * (1.0f - T * T);            // tanh backward
      pg[s3 + 1] += gt;                                     // b_k
      pg[s3] += gt * xs[k];                                 // softplus(h_k)
      gx = gt * rp[s3 * C + c];
    }
    dx[i] = gx;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 11; ++k) {
    const float v = wave_sum(pg[k]);
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 11) {
    const int k = threadIdx.x;
    partial[((int64_t)chunk * 11 + k) * C + c] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
  }
}

// One Bitparm's parameters into the packed [11][C] slots its MODE reads (zeros elsewhere).
__global__ void pack_bitparm_kernel(const float* __restrict__ h, const float* __restrict__ b,
                                    const float* __restrict__ a, float* __restrict__ rp, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  for (int k = 0; k < 11; ++k) rp[k * C + c] = 0.f;
  const int s = a != nullptr ? 0 : 9;
  rp[s * C + c] = softplus_ref(h[c]);
  rp[(s + 1) * C + c] = b[c];
  if (a != nullptr) rp[2 * C + c] = tanhf(a[c]);
}

__global__ void softplus_tanh_kernel(const float* __restrict__ h, const float* __restrict__ a,
                                     float* __restrict__ sp, float* __restrict__ ta, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  sp[c] = softplus_ref(h[c]);
  if (a != nullptr) ta[c] = tanhf(a[c]);
}

constexpr int kRateChunk = 4096;  // latents per partial (fixed → deterministic sums)

// Σ bits over a fixed 4096-element chunk of one image's latent; partial[b][chunk].
__global__ void rate_bits_kernel(const float* __restrict__ z, int C, int HW, int layout,
                                 const float* __restrict__ rp, double* __restrict__ partial,
                                 int chunks) {
  __shared__ float red[4];
  const int b = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const long per_image = (long)C * HW;
  const long lo = (long)ch * kRateChunk;
  const long hi = lo + kRateChunk < per_image ? lo + kRateChunk : per_image;
  float s = 0.f;
  for (long j = lo + threadIdx.x; j < hi; j += 256) {
    const int c = layout == ICLR17_LAYOUT_NCHW ? (int)(j / HW) : (int)(j % C);
    s += element_bits(z[(long)b * per_image + j], rp, C, c);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 4; ++w) t += (double)red[w];
    partial[(long)b * chunks + ch] = t;
  }
}

// Per-image sums of T partials, then their total. One workgroup of 16 waves: wave w reduces
// images w, w + 16, … (lane-strided sums, then a fixed butterfly), thread 0 adds the images in
// order. Fixed order throughout: bitwise reproducible for a given (B, T).
__global__ void __launch_bounds__(1024) reduce_partials_kernel(const double* __restrict__ partial,
                                                               int B, int T, double* per_image,
                                                               float* total, double scale) {
  __shared__ double img[1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double acc = 0.0;
  for (int b0 = 0; b0 < B; b0 += 1024) {
    const int nb = B - b0 < 1024 ? B - b0 : 1024;
    for (int b = wave; b < nb; b += 16) {
      const double* p = partial + (long)(b0 + b) * T;
      double s = 0.0;
      for (int t = lane; t < T; t += 64) s += p[t];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane == 0) {
        img[b] = s;
        if (per_image) per_image[b0 + b] = s;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int b = 0; b < nb; ++b) acc += img[b];
    __syncthreads();
  }
  if (threadIdx.x == 0 && total) *total = (float)(acc * scale);
}

// ∂L/∂recon of train.py's intended loss (mse of the unclipped recon, model.py:61) plus an optional
// gradient arriving at the clipped output (clamp(0,1) backward mask), as autograd evaluates them:
//   mean backward g/numel, pow backward ·(2·d), clamp backward · [0 ≤ r ≤ 1].
__global__ void grad_recon_kernel(const float* __restrict__ recon, const float* __restrict__ x,
                                  const float* __restrict__ g_mse, const float* __restrict__ g_clip,
                                  long n, float numel, float* __restrict__ out) {
  const float gm = g_mse != nullptr ? g_mse[0] / numel : 0.0f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float r = recon[i];
    float g = 0.0f;
    if (g_mse != nullptr) g = gm * (2.0f * (r - x[i]));
    if (g_clip != nullptr && r >= 0.0f && r <= 1.0f) g = g + g_clip[i];
    out[i] = g;
  }
}

// GDN.py:73-79 backward: β_eff = lb(β)² − ped, LowerBound passes g where x ≥ bound or g < 0.
__global__ void gdn_param_chain_kernel(const float* __restrict__ beta, const float* __restrict__ gamma,
                                       const float* __restrict__ dbeta_eff,
                                       const float* __restrict__ dgamma_eff, int C, float bbound,
                                       float gbound, float* __restrict__ dbeta,
                                       float* __restrict__ dgamma) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < C) {
    const float x = beta[i], lb = fmaxf(x, bbound);
    const float g = dbeta_eff[i] * (2.0f * lb);
    dbeta[i] = (x >= bbound || g < 0.0f) ? g : 0.0f;
  }
  if (i < C * C) {
    const float x = gamma[i], lb = fmaxf(x, gbound);
    const float g = dgamma_eff[i] * (2.0f * lb);
    dgamma[i] = (x >= gbound || g < 0.0f) ? g : 0.0f;
  }
}

// Rate-model parameter gradients from per-tile partials [T][11][C] (fixed-order sum) through
// softplus (h) and tanh (a): outputs in the order h1 b1 a1 h2 b2 a2 h3 b3 a3 h4 b4.
struct RateGradPtrs {
  float* p[11];
};

// One workgroup per (parameter k, 64 channels): T rows split over 4 lane groups, combined in
// fixed order, then the softplus / tanh chain rule (torch softplus_backward, tanh_backward).
__global__ void rate_param_chain_kernel(const float* __restrict__ part, int T, int C, RatePtrs rp,
                                        RateGradPtrs out) {
  __shared__ double red[4][64];
  const int k = blockIdx.y;
  const int cl = threadIdx.x & 63, gq = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0;
  if (c < C)
    for (int t = gq; t < T; t += 4) s += (double)part[((long)t * 11 + k) * C + c];
  red[gq][cl] = s;
  __syncthreads();
  if (gq != 0 || c >= C) return;
  const float g = (float)(((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl]);
  const int role = k % 3;
  float v;
  if (role == 0) {        // d softplus(h) → dh (beta 1, threshold 20)
    const float h = rp.p[k][c];
    const float z = expf(h);
    v = h > 20.0f ? g : g * z / (z + 1.0f);
  } else if (role == 1) {
    v = g;
  } else {                // d tanh(a) → da
    const float ta = tanhf(rp.p[k][c]);
    v = g * (1.0f - ta * ta);
  }
  out.p[k][c] = v;
}

}  // namespace
}  // namespace iclr17

using namespace iclr17;

extern "C" {

size_t iclr17_packed_weight_size(int which, int N) {
  switch (which) {
    case ICLR17_W_CONV1:
    case ICLR17_W_CONV1_X6: return (size_t)256 * N;
    case ICLR17_W_CONV5:
    case ICLR17_W_DECONV5: return (size_t)25 * N * N;
    case ICLR17_W_DECONV9: return (size_t)9 * N * 48;
    default: return 0;
  }
}

static int deconv5_taps(TapList* tl) {
  int n = 0;
  for (int ry = 0; ry < 2; ++ry)
    for (int rx = 0; rx < 2; ++rx) {
      int c = 0;
      deconv_phase_taps(5, 2, 2, ry, rx, tl->kh + n, tl->kw + n, &c);
      n += c;
    }
  return n;
}

int iclr17_pack_weight(int which, const float* w, float* packed, int N, void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "pack_weight: N=%d unsupported", N);
  ICLR17_REQUIRE(w && packed, ICLR17_EINVAL, "pack_weight: null pointer");
  const size_t total = iclr17_packed_weight_size(which, N);
  ICLR17_REQUIRE(total > 0, ICLR17_EINVAL, "pack_weight: unknown weight kind %d", which);
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = S(stream);
  switch (which) {
    case ICLR17_W_CONV1: hipLaunchKernelGGL(pack_conv1_kernel, grid, dim3(256), 0, st, w, packed, N); break;
    case ICLR17_W_CONV1_X6: hipLaunchKernelGGL(pack_conv1_x6_kernel, grid, dim3(256), 0, st, w, packed, N); break;
    case ICLR17_W_CONV5: hipLaunchKernelGGL(pack_conv5_kernel, grid, dim3(256), 0, st, w, packed, N); break;
    case ICLR17_W_DECONV5: {
      TapList tl;
      const int n = deconv5_taps(&tl);
      ICLR17_REQUIRE(n == 25, ICLR17_EINVAL, "pack_weight: deconv tap count %d", n);
      hipLaunchKernelGGL(pack_deconv5_kernel, grid, dim3(256), 0, st, w, packed, N, tl);
      break;
    }
    case ICLR17_W_DECONV9: hipLaunchKernelGGL(pack_deconv9_kernel, grid, dim3(256), 0, st, w, packed, N); break;
  }
  return check_launch("pack_weight");
}

// The packs of a parameter update in two launches: every non-split job, then the splits (which
// may read packs made by the first). Jobs are checked like the single-pack entry points.
int iclr17_pack_batch(const iclr17_pack_job* jobs, int n, const float* const* rate_params,
                      void* stream) {
  ICLR17_REQUIRE(jobs && n >= 0, ICLR17_EINVAL, "pack_batch: bad arguments");
  hipStream_t st = S(stream);
  PackBatch b;
  memset(&b, 0, sizeof(b));
  ICLR17_REQUIRE(deconv5_taps(&b.tl) == 25, ICLR17_EINVAL, "pack_batch: deconv tap count");
  if (rate_params)
    for (int k = 0; k < 11; ++k) {
      ICLR17_REQUIRE(rate_params[k], ICLR17_EINVAL, "pack_batch: null rate parameter %d", k);
      b.rp.p[k] = rate_params[k];
    }
  int rate_jobs = 0;
  for (int phase = 0; phase < 2; ++phase) {
    b.n = 0;
    long total = 0;
    auto flush = [&]() -> int {
      if (b.n == 0) return 0;
      b.begin[b.n] = total;
      hipLaunchKernelGGL(pack_batch_kernel, dim3((unsigned)(total / 256)), dim3(256), 0, st, b);
      b.n = 0;
      total = 0;
      return check_launch("pack_batch");
    };
    for (int j = 0; j < n; ++j) {
      const iclr17_pack_job& q = jobs[j];
      if ((q.kind == ICLR17_PACK_SPLIT) != (phase == 1)) continue;
      PackJob J;
      memset(&J, 0, sizeof(J));
      J.kind = q.kind;
      J.N = q.N;
      J.taps = q.taps;
      J.K = q.K;
      J.src0 = q.src0;
      J.src1 = q.src1;
      J.dst0 = q.dst0;
      J.dst1 = q.dst1;
      J.dst2 = q.dst2;
      J.f0 = q.f0;
      J.f1 = q.f1;
      J.f2 = q.f2;
      switch (q.kind) {
        case ICLR17_W_CONV1: case ICLR17_W_CONV1_X6: case ICLR17_W_CONV5: case ICLR17_W_DECONV5:
        case ICLR17_W_DECONV9:
          ICLR17_REQUIRE(q.N == 128 || q.N == 192, ICLR17_EUNSUPPORTED, "pack_batch: N=%d", q.N);
          ICLR17_REQUIRE(q.src0 && q.dst0, ICLR17_EINVAL, "pack_batch: null weight pointer (job %d)", j);
          J.count = (long)iclr17_packed_weight_size(q.kind, q.N);
          break;
        case ICLR17_PACK_GDN:
          ICLR17_REQUIRE(q.N > 0 && q.N % 4 == 0, ICLR17_EINVAL, "pack_batch: GDN C=%d", q.N);
          ICLR17_REQUIRE(q.src0 && q.src1 && q.dst0 && q.dst1, ICLR17_EINVAL,
                         "pack_batch: null GDN pointer (job %d)", j);
          J.count = (long)q.N * q.N;
          break;
        case ICLR17_PACK_RATE:
          ICLR17_REQUIRE(rate_params && q.dst0 && q.N > 0 && ++rate_jobs == 1, ICLR17_EINVAL,
                         "pack_batch: one rate job, with rate_params");
          J.count = q.N;
          break;
        case ICLR17_PACK_SPLIT:
          ICLR17_REQUIRE(q.src0 && q.dst0 && q.taps > 0 && q.K > 0 && q.K % 8 == 0 && q.N > 0,
                         ICLR17_EINVAL, "pack_batch: bad split job %d", j);
          J.count = (long)q.taps * (q.K / 8) * q.N;
          break;
        default:
          ICLR17_REQUIRE(false, ICLR17_EINVAL, "pack_batch: unknown job kind %d", q.kind);
      }
      if (b.n == PACK_MAXJ) {
        const int rc = flush();
        if (rc) return rc;
      }
      b.job[b.n] = J;
      b.begin[b.n] = total;
      total += (J.count + 255) / 256 * 256;
      ++b.n;
    }
    const int rc = flush();
    if (rc) return rc;
  }
  return 0;
}

int iclr17_pack_gdn(const float* beta, const float* gamma, float* beta_eff, float* gamma_packed,
                    float* gamma_packed_t, int C, float beta_bound, float gamma_bound,
                    float pedestal, void* stream) {
  ICLR17_REQUIRE(C > 0 && C % 4 == 0, ICLR17_EINVAL, "pack_gdn: C=%d must be a multiple of 4", C);
  ICLR17_REQUIRE(beta && gamma && beta_eff && gamma_packed, ICLR17_EINVAL, "pack_gdn: null pointer");
  const int total = C * C;
  hipLaunchKernelGGL(pack_gdn_kernel, dim3((total + 255) / 256), dim3(256), 0, S(stream), beta,
                     gamma, beta_eff, gamma_packed, gamma_packed_t, C, beta_bound, gamma_bound, pedestal);
  return check_launch("pack_gdn");
}

int iclr17_pack_rate(const float* h1, const float* b1, const float* a1, const float* h2,
                     const float* b2, const float* a2, const float* h3, const float* b3,
                     const float* a3, const float* h4, const float* b4, float* packed, int C,
                     void* stream) {
  RatePtrs rp = {{h1, b1, a1, h2, b2, a2, h3, b3, a3, h4, b4}};
  for (int i = 0; i < 11; ++i) ICLR17_REQUIRE(rp.p[i], ICLR17_EINVAL, "pack_rate: null parameter %d", i);
  ICLR17_REQUIRE(packed && C > 0, ICLR17_EINVAL, "pack_rate: bad output");
  hipLaunchKernelGGL(pack_rate_kernel, dim3((C + 255) / 256), dim3(256), 0, S(stream), rp, packed, C);
  return check_launch("pack_rate");
}

int iclr17_bit_estimator(const float* x, int64_t n, int C, int64_t inner,
                         const float* rate_packed, float* out, void* stream) {
  ICLR17_REQUIRE(n >= 0 && C > 0 && inner > 0, ICLR17_EINVAL, "bit_estimator: bad shape");
  if (n == 0) return ICLR17_OK;
  ICLR17_REQUIRE(x && rate_packed && out, ICLR17_EINVAL, "bit_estimator: null pointer");
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(bit_estimator_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), x, n,
                     C, inner, rate_packed, out);
  return check_launch("bit_estimator");
}

int iclr17_bitparm(const float* x, int64_t n, int C, int64_t inner, const float* h,
                   const float* b, const float* a, float* work, float* out, void* stream) {
  ICLR17_REQUIRE(n >= 0 && C > 0 && inner > 0, ICLR17_EINVAL, "bitparm: bad shape");
  if (n == 0) return ICLR17_OK;
  ICLR17_REQUIRE(x && h && b && work && out, ICLR17_EINVAL, "bitparm: null pointer");
  hipStream_t st = S(stream);
  float* sp = work;
  float* ta = a != nullptr ? work + C : nullptr;
  hipLaunchKernelGGL(softplus_tanh_kernel, dim3((C + 255) / 256), dim3(256), 0, st, h, a, sp, ta, C);
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(bitparm_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, C, inner, sp,
                     b, ta, out);
  return check_launch("bitparm");
}

int iclr17_bitest_bwd_chunks(int64_t n, int C) {
  const int64_t E = C > 0 ? n / C : 0;   // elements per channel
  const int64_t per = 16384;
  int64_t t = (E + per - 1) / per;
  return (int)(t < 1 ? 1 : t);
}

static int bitest_bwd_launch(int mode, const float* x, const float* g, int64_t n, int C,
                             int64_t inner, const float* rp, float* dx, float* partial,
                             hipStream_t st) {
  const int T = iclr17_bitest_bwd_chunks(n, C);
  const int64_t E = n / C;
  const int64_t per = (E + T - 1) / T;
  const dim3 grid(C, T);
  if (mode == 0)
    hipLaunchKernelGGL(bitest_bwd_kernel<0>, grid, dim3(256), 0, st, x, g, E, C, inner, rp, dx, per, partial);
  else if (mode == 1)
    hipLaunchKernelGGL(bitest_bwd_kernel<1>, grid, dim3(256), 0, st, x, g, E, C, inner, rp, dx, per, partial);
  else
    hipLaunchKernelGGL(bitest_bwd_kernel<2>, grid, dim3(256), 0, st, x, g, E, C, inner, rp, dx, per, partial);
  return check_launch("bit_estimator_bwd");
}

int iclr17_bit_estimator_bwd(const float* x, const float* g, int64_t n, int C, int64_t inner,
                             const float* rate_packed, float* dx, float* partial, void* stream) {
  ICLR17_REQUIRE(n > 0 && C > 0 && inner > 0 && n % C == 0, ICLR17_EINVAL,
                 "bit_estimator_bwd: bad shape");
  ICLR17_REQUIRE(x && g && rate_packed && dx && partial, ICLR17_EINVAL,
                 "bit_estimator_bwd: null pointer");
  return bitest_bwd_launch(0, x, g, n, C, inner, rate_packed, dx, partial, S(stream));
}

int iclr17_bitparm_bwd(const float* x, const float* g, int64_t n, int C, int64_t inner,
                       const float* h, const float* b, const float* a, float* work, float* dx,
                       float* partial, void* stream) {
  ICLR17_REQUIRE(n > 0 && C > 0 && inner > 0 && n % C == 0, ICLR17_EINVAL, "bitparm_bwd: bad shape");
  ICLR17_REQUIRE(x && g && h && b && work && dx && partial, ICLR17_EINVAL,
                 "bitparm_bwd: null pointer");
  hipStream_t st = S(stream);
  hipLaunchKernelGGL(pack_bitparm_kernel, dim3((C + 255) / 256), dim3(256), 0, st, h, b, a, work, C);
  int rc = check_launch("bitparm_bwd_pack");
  if (rc) return rc;
  return bitest_bwd_launch(a != nullptr ? 1 : 2, x, g, n, C, inner, work, dx, partial, st);
}

int iclr17_rate_bits_partials(int C, int h, int w) {
  const long n = (long)C * h * w;
  return (int)((n + kRateChunk - 1) / kRateChunk);
}

int iclr17_rate_bits(const float* z, int B, int C, int h, int w, int layout,
                     const float* rate_packed, double* bits_partial, void* stream) {
  ICLR17_REQUIRE(B > 0 && C > 0 && h > 0 && w > 0, ICLR17_EINVAL, "rate_bits: bad shape");
  ICLR17_REQUIRE(layout == ICLR17_LAYOUT_NCHW || layout == ICLR17_LAYOUT_NHWC, ICLR17_EINVAL,
                 "rate_bits: bad layout");
  ICLR17_REQUIRE(z && rate_packed && bits_partial, ICLR17_EINVAL, "rate_bits: null pointer");
  const int chunks = iclr17_rate_bits_partials(C, h, w);
  hipLaunchKernelGGL(rate_bits_kernel, dim3(B * chunks), dim3(256), 0, S(stream), z, C, h * w,
                     layout, rate_packed, bits_partial, chunks);
  return check_launch("rate_bits");
}

int iclr17_reduce_partials(const double* partial, int B, int T, double* per_image, float* total,
                           double scale, void* stream) {
  ICLR17_REQUIRE(partial && B > 0 && T > 0, ICLR17_EINVAL, "reduce_partials: bad arguments");
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(1024), 0, S(stream), partial, B, T,
                     per_image, total, scale);
  return check_launch("reduce_partials");
}

int iclr17_grad_recon(const float* recon, const float* x, const float* g_mse, const float* g_clip,
                      int64_t n, float* g_recon, void* stream) {
  ICLR17_REQUIRE(recon && x && g_recon && n > 0, ICLR17_EINVAL, "grad_recon: bad arguments");
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(grad_recon_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), recon, x,
                     g_mse, g_clip, (long)n, (float)n, g_recon);
  return check_launch("grad_recon");
}

int iclr17_gdn_param_chain(const float* beta, const float* gamma, const float* dbeta_eff,
                           const float* dgamma_eff, int C, float beta_bound, float gamma_bound,
                           float* dbeta, float* dgamma, void* stream) {
  ICLR17_REQUIRE(beta && gamma && dbeta_eff && dgamma_eff && dbeta && dgamma && C > 0,
                 ICLR17_EINVAL, "gdn_param_chain: bad arguments");
  hipLaunchKernelGGL(gdn_param_chain_kernel, dim3((C * C + 255) / 256), dim3(256), 0, S(stream),
                     beta, gamma, dbeta_eff, dgamma_eff, C, beta_bound, gamma_bound, dbeta, dgamma);
  return check_launch("gdn_param_chain");
}

int iclr17_rate_param_grad(const float* partial, int T, int C, const float* h1, const float* a1,
                           const float* h2, const float* a2, const float* h3, const float* a3,
                           const float* h4, float* dh1, float* db1, float* da1, float* dh2,
                           float* db2, float* da2, float* dh3, float* db3, float* da3, float* dh4,
                           float* db4, void* stream) {
  RatePtrs rp = {{h1, nullptr, a1, h2, nullptr, a2, h3, nullptr, a3, h4, nullptr}};
  RateGradPtrs o = {{dh1, db1, da1, dh2, db2, da2, dh3, db3, da3, dh4, db4}};
  for (int i = 0; i < 11; ++i) ICLR17_REQUIRE(o.p[i], ICLR17_EINVAL, "rate_param_grad: null output %d", i);
  ICLR17_REQUIRE(partial && T > 0 && C > 0 && h1 && a1 && h2 && a2 && h3 && a3 && h4, ICLR17_EINVAL,
                 "rate_param_grad: bad arguments");
  hipLaunchKernelGGL(rate_param_chain_kernel, dim3((C + 63) / 64, 11), dim3(256), 0, S(stream),
                     partial, T, C, rp, o);
  return check_launch("rate_param_grad");
}

}  // extern "C"
