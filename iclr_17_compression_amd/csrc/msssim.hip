// MS-SSIM on the GPU — models/ms_ssim_torch.py:5-196 as train.py:178 calls it
// (ms_ssim(clipped, x, data_range=1.0): 11-tap σ=1.5 Gaussian, 5 levels, weights
// 0.0448 0.2856 0.3001 0.2363 0.1333), per image.
//
// Per level one kernel does the whole SSIM: a 16×64 output tile of one image plane stages its
// 26×74 input window of X and Y in LDS (49 KB: 3 workgroups per CU; 32×64 tiles were 1.5 %
// slower at 2), runs the separable 'valid' filter (along W, then along
// H — the reference's order) on X, Y, X², Y² and XY, forms the cs and ssim maps and leaves one
// partial sum per tile. Both passes slide the window in registers (a W-pass thread filters 4
// consecutive columns of a row from 14 loaded values, an H-pass thread 4 consecutive rows of a
// column from 14), so each filtered value costs ~2 LDS reads instead of 11; every output keeps
// the reference's tap order. A second kernel does the 2×2 average pooling (one zero row/column
// of padding on odd sizes, counted in the average: avg_pool2d's defaults), and a last one, one
// workgroup per image, reduces the per-tile partials of all levels (fixed-order trees: results
// are bitwise reproducible) and forms
//   ms_ssim = Π_{l<4} (cs_l^w_l · ssim_4^w_4)
// exactly as ms_ssim_torch.py:189-190 does (the last level's ssim enters every factor; its cs is
// unused).
#include <string.h>

#include "common.h"

namespace iclr17 {
namespace {

constexpr int WIN = 11, TOH = 16, TOW = 64;
constexpr int IH = TOH + WIN - 1, IW = TOW + WIN - 1;   // 26 × 74 input window at TOH = 16
constexpr int IWP = 76;                                 // LDS row stride: 16-byte rows
constexpr int RS = TOH / 4;                             // H-pass rows per thread (wave = strip)
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

struct FinishPlan {
  long poff[LEVELS];     // first partial (doubles) of each level
  int tiles[LEVELS];     // tiles per plane
  double count[LEVELS];  // 3 · Ho · Wo
};

// g·v + acc: one fused multiply-add (the filter's rounding differs from the reference's
// torch-CPU convolution either way; MS-SSIM parity is a 1e-5 relative tolerance)
__device__ __forceinline__ float fmac(float g, float v, float acc) {
  return __builtin_fmaf(g, v, acc);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(256, 2) ssim_level_kernel(const float* __restrict__ X,
                                                            const float* __restrict__ Y, int H,
                                                            int W, float c1, float c2,
                                                            double* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) float sx[IH * IWP], sy[IH * IWP];
  __shared__ __attribute__((aligned(16))) float h[5][IH][TOW];
  __shared__ double red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int Ho = H - (WIN - 1), Wo = W - (WIN - 1);
  const int plane = blockIdx.z;
  const int r0 = blockIdx.y * TOH, c0 = blockIdx.x * TOW;
  const float* xp = X + (long)plane * H * W;
  const float* yp = Y + (long)plane * H * W;
  float g[WIN];
#pragma unroll
  for (int k = 0; k < WIN; ++k) g[k] = c_gauss[k];

  for (int i = tid; i < IH * IW; i += 256) {
    const int r = i / IW, c = i - r * IW;
    const int gr = r0 + r, gc = c0 + c;
    const bool ok = gr < H && gc < W;
    sx[r * IWP + c] = ok ? xp[(long)gr * W + gc] : 0.f;
    sy[r * IWP + c] = ok ? yp[(long)gr * W + gc] : 0.f;
  }
  __syncthreads();
  // along W: 42 rows × 16 column quads; a thread filters columns cq .. cq+3 of row r
  for (int task = tid; task < IH * (TOW / 4); task += 256) {
    const int r = task >> 4, cq = (task & 15) * 4;
    float xv[16], yv[16];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const f4 a = *(const f4*)(sx + r * IWP + cq + 4 * v);
      const f4 b = *(const f4*)(sy + r * IWP + cq + 4 * v);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xv[4 * v + e] = a[e];
        yv[4 * v + e] = b[e];
      }
    }
    f4 o[5];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float ax = 0.f, ay = 0.f, axx = 0.f, ayy = 0.f, axy = 0.f;
#pragma unroll
      for (int k = 0; k < WIN; ++k) {
        const float xk = xv[j + k], yk = yv[j + k];
        ax = fmac(g[k], xk, ax);
        ay = fmac(g[k], yk, ay);
        axx = fmac(g[k], xk * xk, axx);
        ayy = fmac(g[k], yk * yk, ayy);
        axy = fmac(g[k], xk * yk, axy);
      }
      o[0][j] = ax;
      o[1][j] = ay;
      o[2][j] = axx;
      o[3][j] = ayy;
      o[4][j] = axy;
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) *(f4*)(&h[q][r][cq]) = o[q];
  }
  __syncthreads();
  // along H: wave w filters rows RS·w .. RS·w + RS − 1 of column lane, then the maps
  // (ms_ssim_torch.py:59-73)
  const int rs = wave * RS;
  float m[5][RS];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    float v[RS + WIN - 1];
#pragma unroll
    for (int i = 0; i < RS + WIN - 1; ++i) v[i] = h[q][rs + i][lane];
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < WIN; ++k) acc = fmac(g[k], v[j + k], acc);
      m[q][j] = acc;
    }
  }
  double s_ssim = 0.0, s_cs = 0.0;
  if (c0 + lane < Wo) {
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      if (r0 + rs + j >= Ho) break;
      const float mx = m[0][j], my = m[1][j];
      const float mxx = mx * mx, myy = my * my, mxy = mx * my;
      const float vx = 1.0f * (m[2][j] - mxx), vy = 1.0f * (m[3][j] - myy),
                  cxy = 1.0f * (m[4][j] - mxy);
      const float cs = (2.0f * cxy + c2) / (vx + vy + c2);
      const float ssim = ((2.0f * mxy + c1) / (mxx + myy + c1)) * cs;
      s_ssim += (double)ssim;
      s_cs += (double)cs;
    }
  }
  s_ssim = wave_sum_d(s_ssim);
  s_cs = wave_sum_d(s_cs);
  if (lane == 0) {
    red[0][wave] = s_ssim;
    red[1][wave] = s_cs;
  }
  __syncthreads();
  if (tid == 0) {
    const long tile = ((long)plane * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    partial[2 * tile] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    partial[2 * tile + 1] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
  }
}

// F.avg_pool2d(kernel 2, stride 2, padding (H % 2, W % 2)), count_include_pad: /4 always.
// grid (⌈Wo/256⌉, Ho, 2P): output row oy of plane z % P of X (z < P) or Y.
__global__ void __launch_bounds__(256) avgpool2_kernel(const float* __restrict__ inx,
                                                       const float* __restrict__ iny, int P, int H,
                                                       int W, float* __restrict__ outx,
                                                       float* __restrict__ outy) {
  const int ph = H % 2, pw = W % 2;
  const int Ho = (H + 2 * ph - 2) / 2 + 1, Wo = (W + 2 * pw - 2) / 2 + 1;
  const int ox = blockIdx.x * 256 + threadIdx.x, oy = blockIdx.y;
  if (ox >= Wo) return;
  const int z = blockIdx.z;
  const int p = z < P ? z : z - P;
  const float* src = (z < P ? inx : iny) + (long)p * H * W;
  float s = 0.f;
  for (int dy = 0; dy < 2; ++dy)
    for (int dx = 0; dx < 2; ++dx) {
      const int iy = 2 * oy - ph + dy, ix = 2 * ox - pw + dx;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) s += src[(long)iy * W + ix];
    }
  (z < P ? outx : outy)[((long)p * Ho + oy) * Wo + ox] = s / 4.0f;
}

// One workgroup per image: the per-level means (Σ over the 3 planes × tiles, a fixed-order
// strided sum + tree, / (3·Ho·Wo)) and the MS-SSIM product.
__global__ void __launch_bounds__(256) msssim_finish_kernel(const double* __restrict__ partial,
                                                            const FinishPlan pl, int B,
                                                            double* __restrict__ means /* [L][B][2] */,
                                                            float* __restrict__ out) {
  __shared__ double red[2][256];
  const int b = blockIdx.x, tid = threadIdx.x;
  for (int l = 0; l < LEVELS; ++l) {
    const long n = 3L * pl.tiles[l];
    const double* p = partial + pl.poff[l] + 2 * (long)b * n;
    double a = 0.0, c = 0.0;
    for (long t = tid; t < n; t += 256) {
      a += p[2 * t];
      c += p[2 * t + 1];
    }
    red[0][tid] = a;
    red[1][tid] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) {
        red[0][tid] += red[0][tid + s];
        red[1][tid] += red[1][tid + s];
      }
      __syncthreads();
    }
    if (tid == 0) {
      means[((long)l * B + b) * 2] = red[0][0] / pl.count[l];
      means[((long)l * B + b) * 2 + 1] = red[1][0] / pl.count[l];
    }
    __syncthreads();
  }
  if (tid == 0) {
    const float ssim_last = (float)means[((long)(LEVELS - 1) * B + b) * 2];
    float prod = 1.0f;
    for (int l = 0; l < LEVELS - 1; ++l) {
      const float cs = (float)means[((long)l * B + b) * 2 + 1];
      prod = prod * (powf(cs, c_msssim_w[l]) * powf(ssim_last, c_msssim_w[LEVELS - 1]));
    }
    out[b] = prod;
  }
}

// Single-scale SSIM (ms_ssim_torch.py:86-120 → _ssim :36-83 with size_average=False, full=True):
// per image the means of the ssim and cs maps over C·Ho·Wo, the same fixed-order sums as above.
__global__ void __launch_bounds__(256) ssim_finish_kernel(const double* __restrict__ partial,
                                                          long tiles3, double count,
                                                          float* __restrict__ out_ssim,
                                                          float* __restrict__ out_cs) {
  __shared__ double red[2][256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const double* p = partial + 2 * (long)b * tiles3;
  double a = 0.0, c = 0.0;
  for (long t = tid; t < tiles3; t += 256) {
    a += p[2 * t];
    c += p[2 * t + 1];
  }
  red[0][tid] = a;
  red[1][tid] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      red[0][tid] += red[0][tid + s];
      red[1][tid] += red[1][tid + s];
    }
    __syncthreads();
  }
  if (tid == 0) {
    out_ssim[b] = (float)(red[0][0] / count);
    if (out_cs) out_cs[b] = (float)(red[1][0] / count);
  }
}

int level_plan(int H, int W, Level* lv, int B, long* pyr_floats, long* partial_doubles,
               int levels = LEVELS) {
  long off = 0, part = 0;
  for (int l = 0; l < levels; ++l) {
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
  ICLR17_REQUIRE(B <= 10000 && H <= 65535 * 2, ICLR17_EINVAL, "ms_ssim: B=%d H=%d exceed the grid", B, H);
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
  FinishPlan fp;
  for (int l = 0; l < LEVELS; ++l) {
    const int Hl = lv[l].H, Wl = lv[l].W;
    if (l > 0) {
      float* Xn = pyrbuf + lv[l].off;
      float* Yn = Xn + (long)B * 3 * Hl * Wl;
      const int Hp = lv[l - 1].H, Wp = lv[l - 1].W;
      hipLaunchKernelGGL(avgpool2_kernel, dim3((Wl + 255) / 256, Hl, 2 * B * 3), dim3(256), 0, st,
                         X, Y, B * 3, Hp, Wp, Xn, Yn);
      X = Xn;
      Y = Yn;
    }
    const int Ho = Hl - WIN + 1, Wo = Wl - WIN + 1;
    dim3 grid((Wo + TOW - 1) / TOW, (Ho + TOH - 1) / TOH, B * 3);
    hipLaunchKernelGGL(ssim_level_kernel, grid, dim3(256), 0, st, X, Y, Hl, Wl, c1, c2, pl);
    fp.poff[l] = pl - partial;
    fp.tiles[l] = lv[l].tiles;
    fp.count[l] = 3.0 * Ho * Wo;
    pl += 2L * B * 3 * lv[l].tiles;
  }
  hipLaunchKernelGGL(msssim_finish_kernel, dim3(B), dim3(256), 0, st, partial, fp, B, means, out);
  return check_launch("ms_ssim");
}

size_t iclr17_ssim_workspace_size(int B, int H, int W) {
  Level lv[1];
  long pyr = 0, part = 0;
  if (B <= 0 || level_plan(H, W, lv, B, &pyr, &part, 1) != 0) return 0;
  return (size_t)part * 8 + 256;
}

int iclr17_ssim(const float* x, const float* y, int B, int H, int W, float data_range,
                void* workspace, size_t workspace_bytes, float* out_ssim, float* out_cs,
                void* stream) {
  ICLR17_REQUIRE(x && y && workspace && out_ssim && B > 0, ICLR17_EINVAL, "ssim: null pointer");
  ICLR17_REQUIRE(B <= 10000 && H <= 65535 * 2, ICLR17_EINVAL, "ssim: B=%d H=%d exceed the grid", B, H);
  Level lv[1];
  long pyr = 0, part = 0;
  ICLR17_REQUIRE(level_plan(H, W, lv, B, &pyr, &part, 1) == 0, ICLR17_EINVAL,
                 "ssim: %dx%d is smaller than the 11-tap window", H, W);
  ICLR17_REQUIRE(workspace_bytes >= iclr17_ssim_workspace_size(B, H, W), ICLR17_EINVAL,
                 "ssim: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  double* partial = (double*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  const float c1 = (0.01f * data_range) * (0.01f * data_range);
  const float c2 = (0.03f * data_range) * (0.03f * data_range);
  const int Ho = H - WIN + 1, Wo = W - WIN + 1;
  dim3 grid((Wo + TOW - 1) / TOW, (Ho + TOH - 1) / TOH, B * 3);
  hipLaunchKernelGGL(ssim_level_kernel, grid, dim3(256), 0, st, x, y, H, W, c1, c2, partial);
  hipLaunchKernelGGL(ssim_finish_kernel, dim3(B), dim3(256), 0, st, partial, 3L * lv[0].tiles,
                     3.0 * Ho * Wo, out_ssim, out_cs);
  return check_launch("ssim");
}

}  // extern "C"
