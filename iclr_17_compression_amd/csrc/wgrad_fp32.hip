// Weight / parameter gradients of the codec layers (gfx950, exact-f32 MFMA), split-K over
// pixels with fixed-order partial sums (bitwise reproducible).
//
//   wgrad_k5  dW[m][c][kh][kw] = Σ_{b,o} G[b,o,m] · X[b, 2o−2+k, c]      (NHWC G and X)
//             conv2/conv3 (G = ∂u, X = layer input) and deconv1/deconv2 (G = deconv input,
//             X = ∂(deconv output)) — both land in PyTorch's [m][c][kh][kw] weight layout.
//             With 1 tap, stride 1 and X squared on load it is the GDN parameter gradient
//             dγ_eff[i][j] = Σ_p dn[p][i] · u[p][j]² (the conv2d weight grad of GDN.py:83).
//   wgrad_k9  dW[m][c][kh][kw] = Σ_{b,o} G[b,o,m] · X[b, c, 4o−4+k]       (NCHW 3-channel X)
//             conv1 (G = ∂u1, X = image) and deconv3 (G = s2, X = ∂recon).
//
// GEMM mapping: M = m (all of it per workgroup, 4 waves × 48/32 rows), N = 64 columns of
// (tap, c), K = pixels. Both operands are staged through LDS ([pixel][channel] rows, coalesced
// 16-byte loads); a lane's 4 k-values are 4 consecutive pixels (scalar LDS reads).
#include "common.h"

namespace iclr17 {
namespace {

hipStream_t S(void* s) { return (hipStream_t)s; }

constexpr int KP = 32;  // pixels per k-step

template <int M, bool SQUARE>
__global__ void __launch_bounds__(256) wgrad_k5_kernel(const float* __restrict__ G,
                                                       const float* __restrict__ X, int B, int Ho,
                                                       int Wo, int Hi, int Wi, int C, int ksize,
                                                       int stride, int pad, int nsplit,
                                                       float* __restrict__ part) {
  constexpr int MT = M / 4 / 16;   // m-tiles per wave (3 for 192, 2 for 128)
  constexpr int NT = 4;            // 64 columns
  constexpr int GS = M + 4, XS = 64 + 4;
  __shared__ __attribute__((aligned(16))) float smem[2 * KP * GS + 2 * KP * XS];
  float* sG = smem;
  float* sX = smem + 2 * KP * GS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntap = ksize * ksize;
  const int tap = blockIdx.x % ntap, ct = blockIdx.x / ntap;
  const int kh = tap / ksize, kw = tap % ksize;
  const int split = blockIdx.y;
  const long P = (long)B * Ho * Wo;
  const long per = ((P + nsplit - 1) / nsplit + KP - 1) / KP * KP;
  const long p0 = split * per;
  const long p1 = p0 + per < P ? p0 + per : P;
  const int nsteps = p1 > p0 ? (int)((p1 - p0 + KP - 1) / KP) : 0;

  constexpr int GL = KP * M / 4 / 256;   // float4 loads of G per thread per step
  f4 rg[GL], rx[2];
  auto load = [&](int s) {
    const long pb = p0 + (long)s * KP;
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      const int idx = tid + 256 * i;
      const int pr = idx / (M / 4), c4 = idx % (M / 4);
      const long p = pb + pr;
      rg[i] = p < p1 ? *(const f4*)(G + p * M + c4 * 4) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i;
      const int pr = idx >> 4, c4 = idx & 15;
      const long p = pb + pr;
      f4 v = f4{0.f, 0.f, 0.f, 0.f};
      if (p < p1) {
        const int ow = (int)(p % Wo);
        const long q = p / Wo;
        const int oh = (int)(q % Ho);
        const int b = (int)(q / Ho);
        const int iy = oh * stride - pad + kh, ix = ow * stride - pad + kw;
        if (iy >= 0 && iy < Hi && ix >= 0 && ix < Wi) {
          v = *(const f4*)(X + (((long)b * Hi + iy) * Wi + ix) * C + ct * 64 + c4 * 4);
          if (SQUARE) v = v * v;
        }
      }
      rx[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < GL; ++i) {
      const int idx = tid + 256 * i;
      *(f4*)(sG + buf * KP * GS + (idx / (M / 4)) * GS + (idx % (M / 4)) * 4) = rg[i];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i;
      *(f4*)(sX + buf * KP * XS + (idx >> 4) * XS + (idx & 15) * 4) = rx[i];
    }
  };

  f4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};

  if (nsteps > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  const int m0 = wave * MT * 16;
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    if (s + 1 < nsteps) load(s + 1);
    const float* g = sG + cur * KP * GS;
    const float* x = sX + cur * KP * XS;
#pragma unroll
    for (int kb = 0; kb < KP / 16; ++kb) {
      const int pr = kb * 16 + 4 * (lane >> 4);
      f4 af[MT], bf[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int e = 0; e < 4; ++e) af[mt][e] = g[(pr + e) * GS + m0 + mt * 16 + (lane & 15)];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) bf[nt][e] = x[(pr + e) * XS + nt * 16 + (lane & 15)];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16(af[mt][e], bf[nt][e], acc[mt][nt]);
    }
    if (s + 1 < nsteps) store(cur ^ 1);
    __syncthreads();
  }
  // part[split][m][c][tap]  (the PyTorch [m][c][kh][kw] layout)
  float* out = part + (long)split * M * C * ntap;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + mt * 16 + 4 * (lane >> 4) + r;
        const int c = ct * 64 + nt * 16 + (lane & 15);
        out[((long)m * C + c) * ntap + tap] = acc[mt][nt][r];
      }
}

// conv1 / deconv3 weight gradient: K = 243 = (c, kh, kw) of a 9×9 stride-4 pad-4 window on a
// 3-channel NCHW image X; pixels iterate over 8×8 output tiles whose 37×37×3 input patch is
// staged in LDS (as in the conv1 forward kernel).
constexpr int P9 = 37, P9PLANE = P9 * P9, P9ZERO = 3 * P9PLANE;

template <int M>
__global__ void __launch_bounds__(256) wgrad_k9_kernel(const float* __restrict__ G,
                                                       const float* __restrict__ X, int B, int Ho,
                                                       int Wo, int nsplit, float* __restrict__ part) {
  constexpr int MT = M / 4 / 16;
  constexpr int NT = 4;
  constexpr int GS = M + 4;
  constexpr int OFF_G = (P9ZERO + 4 + 64 + 64 + 3) / 4 * 4;
  __shared__ __attribute__((aligned(16))) float smem[OFF_G + 64 * GS];
  int* ktab = (int*)(smem + P9ZERO + 4);
  int* mtab = ktab + 64;
  float* sG = smem + OFF_G;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ktile = blockIdx.x;  // 4 tiles of 64 k values (243 used)
  const int split = blockIdx.y;
  const int H = Ho * 4, W = Wo * 4;
  const int tiles_x = (Wo + 7) / 8, tiles_y = (Ho + 7) / 8;
  const int ntiles = B * tiles_x * tiles_y;
  const int per = (ntiles + nsplit - 1) / nsplit;
  const int t0 = split * per, t1 = t0 + per < ntiles ? t0 + per : ntiles;
  if (tid < 64) {
    const int k = ktile * 64 + tid;
    int off = P9ZERO;
    if (k < 243) off = (k / 81) * P9PLANE + ((k % 81) / 9) * P9 + k % 9;
    ktab[tid] = off;
    mtab[tid] = (tid >> 3) * 4 * P9 + (tid & 7) * 4;
  }
  if (tid == 0) smem[P9ZERO] = 0.f;

  f4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
  const int m0 = wave * MT * 16;
  for (int tl = t0; tl < t1; ++tl) {
    const int tx = tl % tiles_x, ty = (tl / tiles_x) % tiles_y, b = tl / (tiles_x * tiles_y);
    __syncthreads();  // previous tile's reads done
    const int iy0 = ty * 32 - 4, ix0 = tx * 32 - 4;
    for (int idx = tid; idx < 3 * P9PLANE; idx += 256) {
      const int c = idx / P9PLANE, rem = idx - c * P9PLANE;
      const int r = rem / P9, col = rem - r * P9;
      const int iy = iy0 + r, ix = ix0 + col;
      float v = 0.f;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = X[(((long)b * 3 + c) * H + iy) * W + ix];
      smem[idx] = v;
    }
    for (int idx = tid; idx < 64 * (M / 4); idx += 256) {
      const int pr = idx / (M / 4), c4 = idx % (M / 4);
      const int oy = ty * 8 + (pr >> 3), ox = tx * 8 + (pr & 7);
      f4 v = f4{0.f, 0.f, 0.f, 0.f};
      if (oy < Ho && ox < Wo) v = *(const f4*)(G + (((long)b * Ho + oy) * Wo + ox) * M + c4 * 4);
      *(f4*)(sG + pr * GS + c4 * 4) = v;
    }
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int pr = kb * 16 + 4 * (lane >> 4);
      f4 af[MT], bf[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int e = 0; e < 4; ++e) af[mt][e] = sG[(pr + e) * GS + m0 + mt * 16 + (lane & 15)];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int ko = ktab[nt * 16 + (lane & 15)];
#pragma unroll
        for (int e = 0; e < 4; ++e) bf[nt][e] = ko == P9ZERO ? 0.f : smem[ko + mtab[pr + e]];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16(af[mt][e], bf[nt][e], acc[mt][nt]);
    }
  }
  float* out = part + (long)split * M * 243;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + mt * 16 + 4 * (lane >> 4) + r;
        const int k = ktile * 64 + nt * 16 + (lane & 15);
        if (k < 243) out[(long)m * 243 + k] = acc[mt][nt][r];
      }
}

// out[i] = Σ_s part[s][i], fixed order.
__global__ void sum_splits_kernel(const float* __restrict__ part, int nsplit, long n,
                                  float* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nsplit; ++k) s += part[(long)k * n + i];
    out[i] = s;
  }
}

// out[c] = Σ_t part[t][c]: 64 columns per workgroup, T split over 4 lane groups (strided), the 4
// partial sums combined in order through LDS — fixed order, bitwise reproducible.
__global__ void sum_rows_kernel(const float* __restrict__ part, int T, int C, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < C)
    for (int t = g; t < T; t += 4) s += part[(long)t * C + c];
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < C) out[c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

// Column sums of a [P][C] row-major matrix (NHWC activations): part[chunk][c].
__global__ void colsum_kernel(const float* __restrict__ A, long P, int C, int chunk,
                              float* __restrict__ part) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long p0 = (long)blockIdx.y * chunk;
  const long p1 = p0 + chunk < P ? p0 + chunk : P;
  float s = 0.f;
  for (long p = p0; p < p1; ++p) s += A[p * C + c];
  part[(long)blockIdx.y * C + c] = s;
}

// Per-channel sums of an NCHW tensor [B][C][HW]: part[b][c] (one workgroup per (b, c)).
__global__ void plane_sum_kernel(const float* __restrict__ A, int C, long HW, float* __restrict__ part) {
  __shared__ float red[4];
  const long base = (long)blockIdx.x * HW;
  float s = 0.f;
  for (long i = threadIdx.x; i < HW; i += 256) s += A[base + i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

int wgrad9_splits(int ntiles) { return ntiles < 128 ? ntiles : 128; }

int wgrad_splits(long P, int tiles) {
  // enough workgroups to fill 256 CUs twice, at least ~256 pixels per split
  int s = (512 + tiles - 1) / tiles;
  const long maxs = P / 256 > 1 ? P / 256 : 1;
  if (s > maxs) s = (int)maxs;
  if (s < 1) s = 1;
  return s;
}

}  // namespace
}  // namespace iclr17

using namespace iclr17;

extern "C" {

int iclr17_sum_rows(const float* part, int T, int C, float* out, void* stream);

size_t iclr17_wgrad_workspace_size(int kind, int B, int Ho, int Wo, int M, int C) {
  const long P = (long)B * Ho * Wo;
  if (kind == 9) return (size_t)wgrad9_splits(B * ((Wo + 7) / 8) * ((Ho + 7) / 8)) * M * 243;
  const int ntap = kind == 1 ? 1 : 25;
  const int tiles = ntap * (C / 64);
  return (size_t)wgrad_splits(P, tiles) * M * C * ntap;
}

int iclr17_wgrad_k5(const float* G, const float* X, int B, int Ho, int Wo, int M, int C,
                    float* workspace, float* dW, void* stream) {
  ICLR17_REQUIRE(B > 0 && Ho > 0 && Wo > 0, ICLR17_EINVAL, "wgrad_k5: bad shape");
  ICLR17_REQUIRE((M == 128 || M == 192) && C % 64 == 0 && C > 0, ICLR17_EUNSUPPORTED,
                 "wgrad_k5: M=%d C=%d unsupported", M, C);
  ICLR17_REQUIRE(G && X && workspace && dW, ICLR17_EINVAL, "wgrad_k5: null pointer");
  const long P = (long)B * Ho * Wo;
  const int tiles = 25 * (C / 64);
  const int ns = wgrad_splits(P, tiles);
  hipStream_t st = S(stream);
  dim3 grid(tiles, ns);
  if (M == 192)
    hipLaunchKernelGGL((wgrad_k5_kernel<192, false>), grid, dim3(256), 0, st, G, X, B, Ho, Wo, 2 * Ho, 2 * Wo, C, 5, 2, 2, ns, workspace);
  else
    hipLaunchKernelGGL((wgrad_k5_kernel<128, false>), grid, dim3(256), 0, st, G, X, B, Ho, Wo, 2 * Ho, 2 * Wo, C, 5, 2, 2, ns, workspace);
  int rc = check_launch("wgrad_k5");
  if (rc) return rc;
  const long n = (long)M * C * 25;
  hipLaunchKernelGGL(sum_splits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, workspace, ns, n, dW);
  return check_launch("wgrad_k5_sum");
}

int iclr17_wgrad_k9(const float* G, const float* X, int B, int Ho, int Wo, int M,
                    float* workspace, float* dW, void* stream) {
  ICLR17_REQUIRE(B > 0 && Ho > 0 && Wo > 0, ICLR17_EINVAL, "wgrad_k9: bad shape");
  ICLR17_REQUIRE(M == 128 || M == 192, ICLR17_EUNSUPPORTED, "wgrad_k9: M=%d unsupported", M);
  ICLR17_REQUIRE(G && X && workspace && dW, ICLR17_EINVAL, "wgrad_k9: null pointer");
  const int ns = wgrad9_splits(B * ((Wo + 7) / 8) * ((Ho + 7) / 8));
  hipStream_t st = S(stream);
  dim3 grid(4, ns);
  if (M == 192)
    hipLaunchKernelGGL((wgrad_k9_kernel<192>), grid, dim3(256), 0, st, G, X, B, Ho, Wo, ns, workspace);
  else
    hipLaunchKernelGGL((wgrad_k9_kernel<128>), grid, dim3(256), 0, st, G, X, B, Ho, Wo, ns, workspace);
  int rc = check_launch("wgrad_k9");
  if (rc) return rc;
  const long n = (long)M * 243;
  hipLaunchKernelGGL(sum_splits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, workspace, ns, n, dW);
  return check_launch("wgrad_k9_sum");
}

size_t iclr17_gdn_wgrad_workspace_size(long P, int C) {
  return (size_t)wgrad_splits(P, C / 64) * C * C;
}

// GDN.py:83 parameter gradients from dn (∂L/∂n, NHWC [P][C]) and the saved input u:
//   dgamma_eff[i][j] = Σ_p dn[p][i] · u[p][j]²,  dbeta_eff[i] = Σ_p dn[p][i].
int iclr17_gdn_wgrad(const float* dn, const float* u, long P, int C, float* workspace,
                     float* dgamma_eff, void* stream) {
  ICLR17_REQUIRE(P > 0 && (C == 128 || C == 192), ICLR17_EUNSUPPORTED, "gdn_wgrad: C=%d", C);
  ICLR17_REQUIRE(dn && u && workspace && dgamma_eff, ICLR17_EINVAL, "gdn_wgrad: null pointer");
  const int ns = wgrad_splits(P, C / 64);
  hipStream_t st = S(stream);
  dim3 grid(C / 64, ns);
  // a 1×1 "conv" over a P×1 grid: Ho = P, Wo = 1
  if (C == 192)
    hipLaunchKernelGGL((wgrad_k5_kernel<192, true>), grid, dim3(256), 0, st, dn, u, 1, (int)P, 1, (int)P, 1, C, 1, 1, 0, ns, workspace);
  else
    hipLaunchKernelGGL((wgrad_k5_kernel<128, true>), grid, dim3(256), 0, st, dn, u, 1, (int)P, 1, (int)P, 1, C, 1, 1, 0, ns, workspace);
  int rc = check_launch("gdn_wgrad");
  if (rc) return rc;
  const long n = (long)C * C;
  hipLaunchKernelGGL(sum_splits_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, workspace, ns, n, dgamma_eff);
  return check_launch("gdn_wgrad_sum");
}

// out[c] = Σ_t part[t][c] (fixed order; T rows split over 4 thread groups, combined in order).
int iclr17_sum_rows(const float* part, int T, int C, float* out, void* stream) {
  ICLR17_REQUIRE(part && out && T > 0 && C > 0, ICLR17_EINVAL, "sum_rows: bad arguments");
  hipLaunchKernelGGL(sum_rows_kernel, dim3((C + 63) / 64), dim3(256), 0, S(stream), part, T, C, out);
  return check_launch("sum_rows");
}

// Bias gradient of a layer whose output gradient is NHWC [P][C]: db[c] = Σ_p G[p][c].
// workspace: 1024*C floats (1024 fixed row chunks, then iclr17_sum_rows).
int iclr17_bias_grad_nhwc(const float* G, long P, int C, float* workspace, float* db, void* stream) {
  ICLR17_REQUIRE(P > 0 && C > 0 && G && workspace && db, ICLR17_EINVAL, "bias_grad_nhwc: bad arguments");
  hipStream_t st = S(stream);
  const int chunk = (int)((P + 1023) / 1024);
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 255) / 256, 1024), dim3(256), 0, st, G, P, C, chunk, workspace);
  int rc = check_launch("bias_grad_nhwc");
  if (rc) return rc;
  return iclr17_sum_rows(workspace, 1024, C, db, stream);
}

// Bias gradient from an NCHW gradient [B][C][HW] (deconv3 output): workspace B*C floats.
int iclr17_bias_grad_nchw(const float* G, int B, int C, long HW, float* workspace, float* db,
                          void* stream) {
  ICLR17_REQUIRE(B > 0 && C > 0 && HW > 0 && G && workspace && db, ICLR17_EINVAL, "bias_grad_nchw: bad arguments");
  hipStream_t st = S(stream);
  hipLaunchKernelGGL(plane_sum_kernel, dim3(B * C), dim3(256), 0, st, G, C, HW, workspace);
  int rc = check_launch("bias_grad_nchw");
  if (rc) return rc;
  // part is [B][C] → sum over b for each c
  return iclr17_sum_rows(workspace, B, C, db, stream);
}

}  // extern "C"
