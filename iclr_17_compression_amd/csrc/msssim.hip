// MS-SSIM on the GPU — models/ms_ssim_torch.py:5-196 as train.py:178 calls it
// (ms_ssim(clipped, x, data_range=1.0): 11-tap σ=1.5 Gaussian, 5 levels, weights
// 0.0448 0.2856 0.3001 0.2363 0.1333), per image.
//
// Per level one kernel does the whole SSIM: a 16×64 output tile of one image plane stages its
// 26×74 input window of X and Y in LDS, runs the separable 'valid' filter (along W, then along
// H — the reference's order) on X, Y, X², Y² and XY, forms the cs and ssim maps and leaves one
// partial sum per tile (fixed-order reductions: results are bitwise reproducible). A second
// kernel does the 2×2 average pooling (one zero row/column of padding on odd sizes, counted in
// the average: avg_pool2d's defaults), and a last one forms
//   ms_ssim = Π_{l<4} (cs_l^w_l · ssim_4^w_4)
// exactly as ms_ssim_torch.py:189-190 does (the last level's ssim enters every factor; its cs is
// unused).
#include <string.h>

#include "common.h"

namespace iclr17 {
namespace {

constexpr int WIN = 11, TOH = 16, TOW = 64;
constexpr int IH = TOH + WIN - 1, IW = TOW + WIN - 1;   // 26 × 74 input window
constexpr int LEVELS = 5;
__constant__ float c_msssim_w[LEVELS] = {0.0448f, 0.2856f, 0.3001f, 0.2363f, 0.1333f};
// The reference's fp32 window (ms_ssim_torch.py:5-18: exp(−c²/(2·1.5²)) normalised by its sum,
// evaluated by torch-CPU fp32), bit for bit (tests/test_library.py recomputes it from the oracle).
__constant__ float c_gauss[WIN] = {
    0x1.0d957p-10f, 0x1.f1fe02p-8f, 0x1.26eb18p-5f, 0x1.bff0fep-4f, 0x1.b43c3ep-3f, 0x1.10656p-2f,
    0x1.b43c3ep-3f, 0x1.bff0fep-4f, 0x1.26eb18p-5f, 0x1.f1fe02p-8f, 0x1.0d957p-10f};

struct Level {
  int H, W;         // input size of the level
  long off;         // offset of the level's planes in the pyramid buffer (floats; level 0: -1)
  int tiles;        // output tiles per plane
};

__global__ void __launch_bounds__(256) ssim_level_kernel(const float* __restrict__ X,
                                                         const float* __restrict__ Y, int H,
                                                         int W, float c1, float c2,
                                                         double* __restrict__ partial) {
  __shared__ float sx[IH][IW + 1], sy[IH][IW + 1];
  __shared__ float h[5][IH][TOW + 1];
  __shared__ double red[2][256];
  const int Ho = H - (WIN - 1), Wo = W - (WIN - 1);
  const int plane = blockIdx.z;
  const int r0 = blockIdx.y * TOH, c0 = blockIdx.x * TOW;
  const float* xp = X + (long)plane * H * W;
  const float* yp = Y + (long)plane * H * W;
  float g[WIN];
#pragma unroll
  for (int k = 0; k < WIN; ++k) g[k] = c_gauss[k];

  for (int i = threadIdx.x; i < IH * IW; i += 256) {
    const int r = i / IW, c = i % IW;
    const int gr = r0 + r, gc = c0 + c;
    const bool ok = gr < H && gc < W;
    sx[r][c] = ok ? xp[(long)gr * W + gc] : 0.f;
    sy[r][c] = ok ? yp[(long)gr * W + gc] : 0.f;
  }
  __syncthreads();
  // along W: 26 rows × 64 columns, five filtered quantities
  for (int i = threadIdx.x; i < IH * TOW; i += 256) {
    const int r = i / TOW, c = i % TOW;
    float ax = 0.f, ay = 0.f, axx = 0.f, ayy = 0.f, axy = 0.f;
#pragma unroll
    for (int k = 0; k < WIN; ++k) {
      const float xv = sx[r][c + k], yv = sy[r][c + k];
      ax += g[k] * xv;
      ay += g[k] * yv;
      axx += g[k] * (xv * xv);
      ayy += g[k] * (yv * yv);
      axy += g[k] * (xv * yv);
    }
    h[0][r][c] = ax;
    h[1][r][c] = ay;
    h[2][r][c] = axx;
    h[3][r][c] = ayy;
    h[4][r][c] = axy;
  }
  __syncthreads();
  // along H, then the maps (ms_ssim_torch.py:59-73)
  double s_ssim = 0.0, s_cs = 0.0;
  for (int i = threadIdx.x; i < TOH * TOW; i += 256) {
    const int r = i / TOW, c = i % TOW;
    if (r0 + r >= Ho || c0 + c >= Wo) continue;
    float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < WIN; ++k)
#pragma unroll
      for (int q = 0; q < 5; ++q) m[q] += g[k] * h[q][r + k][c];
    const float mx = m[0], my = m[1];
    const float mxx = mx * mx, myy = my * my, mxy = mx * my;
    const float vx = 1.0f * (m[2] - mxx), vy = 1.0f * (m[3] - myy), cxy = 1.0f * (m[4] - mxy);
    const float cs = (2.0f * cxy + c2) / (vx + vy + c2);
    const float ssim = ((2.0f * mxy + c1) / (mxx + myy + c1)) * cs;
    s_ssim += (double)ssim;
    s_cs += (double)cs;
  }
  red[0][threadIdx.x] = s_ssim;
  red[1][threadIdx.x] = s_cs;
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int t = 0; t < 256; ++t) {
      a += red[0][t];
      b += red[1][t];
    }
    const long tile = ((long)plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    partial[2 * tile] = a;
    partial[2 * tile + 1] = b;
  }
}

// F.avg_pool2d(kernel 2, stride 2, padding (H % 2, W % 2)), count_include_pad: /4 always
__global__ void __launch_bounds__(256) avgpool2_kernel(const float* __restrict__ in, int P, int H,
                                                       int W, float* __restrict__ out) {
  const int ph = H % 2, pw = W % 2;
  const int Ho = (H + 2 * ph - 2) / 2 + 1, Wo = (W + 2 * pw - 2) / 2 + 1;
  const long n = (long)P * Ho * Wo;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int ox = (int)(i % Wo);
    const long t = i / Wo;
    const int oy = (int)(t % Ho);
    const long p = t / Ho;
    const float* src = in + p * H * W;
    float s = 0.f;
    for (int dy = 0; dy < 2; ++dy)
      for (int dx = 0; dx < 2; ++dx) {
        const int iy = 2 * oy - ph + dy, ix = 2 * ox - pw + dx;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) s += src[(long)iy * W + ix];
      }
    out[i] = s / 4.0f;
  }
}

// per-image means of a level: Σ over the 3 planes × tiles in a fixed order / (3·Ho·Wo)
__global__ void level_means_kernel(const double* __restrict__ partial, int B, int tiles, long count,
                                   double* __restrict__ means /* [B][2] */) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double a = 0.0, c = 0.0;
  for (long t = 0; t < 3L * tiles; ++t) {
    a += partial[2 * ((long)b * 3 * tiles + t)];
    c += partial[2 * ((long)b * 3 * tiles + t) + 1];
  }
  means[2 * b] = a / (double)count;
  means[2 * b + 1] = c / (double)count;
}

__global__ void msssim_combine_kernel(const double* __restrict__ means /* [L][B][2] */, int B,
                                      float* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float ssim_last = (float)means[((LEVELS - 1) * B + b) * 2];
  float prod = 1.0f;
  for (int l = 0; l < LEVELS - 1; ++l) {
    const float cs = (float)means[(l * B + b) * 2 + 1];
    prod = prod * (powf(cs, c_msssim_w[l]) * powf(ssim_last, c_msssim_w[LEVELS - 1]));
  }
  out[b] = prod;
}

int level_plan(int H, int W, Level* lv, int B, long* pyr_floats, long* partial_doubles) {
  long off = 0, part = 0;
  for (int l = 0; l < LEVELS; ++l) {
    if (H < WIN || W < WIN) return -1;
    lv[l].H = H;
    lv[l].W = W;
    lv[l].off = l == 0 ? -1 : off;
    if (l > 0) off += 2L * B * 3 * H * W;   // X and Y planes of this level
    lv[l].tiles = ((W - WIN + 1 + TOW - 1) / TOW) * ((H - WIN + 1 + TOH - 1) / TOH);
    part += 2L * B * 3 * lv[l].tiles;
    H = (H + 2 * (H % 2) - 2) / 2 + 1;
    W = (W + 2 * (W % 2) - 2) / 2 + 1;
  }
  *pyr_floats = off;
  *partial_doubles = part;
  return 0;
}

}  // namespace
}  // namespace iclr17

using namespace iclr17;

extern "C" {

size_t iclr17_ms_ssim_workspace_size(int B, int H, int W) {
  Level lv[LEVELS];
  long pyr = 0, part = 0;
  if (B <= 0 || level_plan(H, W, lv, B, &pyr, &part) != 0) return 0;
  // pyramid floats | partial doubles | per-level means [L][B][2] doubles (+ alignment slack)
  return (size_t)pyr * 4 + (size_t)part * 8 + (size_t)LEVELS * B * 2 * 8 + 256;
}

int iclr17_ms_ssim(const float* x, const float* y, int B, int H, int W, float data_range,
                   void* workspace, size_t workspace_bytes, float* out, void* stream) {
  ICLR17_REQUIRE(x && y && workspace && out && B > 0, ICLR17_EINVAL, "ms_ssim: null pointer");
  Level lv[LEVELS];
  long pyr = 0, part = 0;
  ICLR17_REQUIRE(level_plan(H, W, lv, B, &pyr, &part) == 0, ICLR17_EINVAL,
                 "ms_ssim: %dx%d is too small for 5 levels of an 11-tap window", H, W);
  ICLR17_REQUIRE(workspace_bytes >= iclr17_ms_ssim_workspace_size(B, H, W), ICLR17_EINVAL,
                 "ms_ssim: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  float* pyrbuf = (float*)ws;
  double* partial = (double*)(ws + pyr * 4);
  double* means = partial + part;
  const float c1 = (0.01f * data_range) * (0.01f * data_range);
  const float c2 = (0.03f * data_range) * (0.03f * data_range);
  const float* X = x;
  const float* Y = y;
  double* pl = partial;
  for (int l = 0; l < LEVELS; ++l) {
    const int Hl = lv[l].H, Wl = lv[l].W;
    if (l > 0) {
      float* Xn = pyrbuf + lv[l].off;
      float* Yn = Xn + (long)B * 3 * Hl * Wl;
      const int Hp = lv[l - 1].H, Wp = lv[l - 1].W;
      const long n = (long)B * 3 * Hl * Wl;
      const int blocks = (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192);
      hipLaunchKernelGGL(avgpool2_kernel, dim3(blocks), dim3(256), 0, st, X, B * 3, Hp, Wp, Xn);
      hipLaunchKernelGGL(avgpool2_kernel, dim3(blocks), dim3(256), 0, st, Y, B * 3, Hp, Wp, Yn);
      X = Xn;
      Y = Yn;
    }
    const int Ho = Hl - WIN + 1, Wo = Wl - WIN + 1;
    dim3 grid((Wo + TOW - 1) / TOW, (Ho + TOH - 1) / TOH, B * 3);
    hipLaunchKernelGGL(ssim_level_kernel, grid, dim3(256), 0, st, X, Y, Hl, Wl, c1, c2, pl);
    hipLaunchKernelGGL(level_means_kernel, dim3((B + 63) / 64), dim3(64), 0, st, pl, B,
                       lv[l].tiles, 3L * Ho * Wo, means + (long)l * B * 2);
    pl += 2L * B * 3 * lv[l].tiles;
  }
  hipLaunchKernelGGL(msssim_combine_kernel, dim3((B + 63) / 64), dim3(64), 0, st, means, B, out);
  return check_launch("ms_ssim");
}

}  // extern "C"
