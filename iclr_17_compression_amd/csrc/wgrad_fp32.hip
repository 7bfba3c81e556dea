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
#include <atomic>
#include "common.h"

namespace iclr17 {
namespace {

hipStream_t S(void* s) { return (hipStream_t)s; }

constexpr int KP = 32;  // pixels per k-step

__device__ __attribute__((aligned(16))) float g_wzero[4] = {0.f, 0.f, 0.f, 0.f};

__device__ __forceinline__ void glds16w(const float* src, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

typedef float f16w __attribute__((ext_vector_type(16)));

// GEMM: dW[m][tap, c] = Σ_p G[p][m] · X[p ⊕ tap][c] for one tap and a 64-channel tile c, over one
// split of the pixels (SQUARE: the GDN γ gradient, a 1×1 tap over X², pixel p = row p of X).
// v_mfma_f32_32x32x2_f32 (exact f32; lane l holds A[m = l&31][k = l>>5] and
// B[k = l>>5][c = l&31]): a k-step of two pixels needs one element per lane per operand, and 32
// consecutive lanes read 32 consecutive channels of one LDS pixel row — conflict-free
// ds_read_b32, the [pixel][channel] tiles need no transpose. Both tiles arrive by LDS-DMA:
// G [32 px][M] is one contiguous block of the NHWC gradient, X [32 px][64] the tap-shifted rows
// (zero line outside the image), two stages, one barrier per 32 pixels. 4 waves: wave w owns
// channels 32(w&1) .. +31 and rows 32·(3 (w>>1)) .. of M (3 tiles of 32×32 at M = 192, 2 at 128).
template <int M, bool SQUARE>
__global__ void __launch_bounds__(256) wgrad_k5_kernel(const float* __restrict__ G,
                                                       const float* __restrict__ X, int B, int Ho,
                                                       int Wo, int Hi, int Wi, int C, int ksize,
                                                       int stride, int pad, int nsplit,
                                                       float* __restrict__ part) {
  constexpr int MT = M / 64;                 // 32-row m-tiles per wave
  constexpr int SG = KP * M, SX = KP * 64;   // floats per stage
  constexpr int STAGE = SG + SX;
  constexpr int NGI = SG * 4 / 1024, NXI = SX * 4 / 1024;   // DMA wave-instructions per stage
  constexpr int NI = NGI + NXI, NI_W = NI / 4;
  static_assert(NI % 4 == 0, "uniform DMA slots");
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntap = ksize * ksize;
  const int tap = blockIdx.x % ntap, ct = blockIdx.x / ntap;
  const int kh = tap / ksize, kw = tap % ksize;
  const int split = blockIdx.y;
  const long P = (long)B * Ho * Wo;
  const long per = ((P + nsplit - 1) / nsplit + KP - 1) / KP * KP;
  const long p0 = split * per;
  const long p1 = p0 + per < P ? p0 + per : P;
  const int nsteps = p1 > p0 ? (int)((p1 - p0 + KP - 1) / KP) : 0;

  auto issue = [&](int s, int buf) {
    const long pb = p0 + (long)s * KP;
    float* st = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < NI_W; ++j) {
      const int i = wave + 4 * j;
      if (i < NGI) {   // G: contiguous [pb, pb + 32) × M
        const long e = (long)i * 256 + lane * 4;   // float offset in the tile
        const long p = pb + e / M;
        glds16w(p < p1 ? G + pb * M + e : g_wzero, st + i * 256);
      } else {         // X: 4 pixel rows of 64 channels per instruction
        const int xi = i - NGI;
        const int row = xi * 4 + (lane >> 4), piece = lane & 15;
        const long p = pb + row;
        const float* src = g_wzero;
        if (SQUARE) {   // the GDN 1×1 case: pixel p is row p of X, no spatial mapping
          if (p < p1) src = X + p * C + ct * 64 + piece * 4;
        } else if (p < p1) {
          const int ow = (int)(p % Wo);
          const long q = p / Wo;
          const int oh = (int)(q % Ho);
          const int b = (int)(q / Ho);
          const int iy = oh * stride - pad + kh, ix = ow * stride - pad + kw;
          if (iy >= 0 && iy < Hi && ix >= 0 && ix < Wi)
            src = X + (((long)b * Hi + iy) * Wi + ix) * C + ct * 64 + piece * 4;
        }
        glds16w(src, st + SG + xi * 256);
      }
    }
  };

  f16w acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[mt][r] = 0.f;
  const int mrow0 = (wave >> 1) * MT * 32;
  const int aoff = (lane >> 5) * M + mrow0 + (lane & 31);
  const int boff = (lane >> 5) * 64 + (wave & 1) * 32 + (lane & 31);

  if (nsteps > 0) issue(0, 0);
  for (int s = 0; s < nsteps; ++s) {
    dma_barrier();   // stage s landed for every wave; stage (s+1)&1 is free
    if (s + 1 < nsteps) issue(s + 1, (s + 1) & 1);
    const float* g = smem + (s & 1) * STAGE + aoff;
    const float* x = smem + (s & 1) * STAGE + SG + boff;
#pragma unroll
    for (int k2 = 0; k2 < KP / 2; ++k2) {
      float bv = x[k2 * 2 * 64];
      if (SQUARE) bv = bv * bv;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(g[k2 * 2 * M + mt * 32], bv, acc[mt], 0, 0, 0);
    }
  }
  // part[split][m][c][tap]  (the PyTorch [m][c][kh][kw] layout)
  float* out = part + (long)split * M * C * ntap;
  const int c = ct * 64 + (wave & 1) * 32 + (lane & 31);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mrow0 + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      out[((long)m * C + c) * ntap + tap] = acc[mt][r];
    }
}

// A weight gradient in the bf16x6 scheme as a 1×1 contraction over pixels, from split-form
// operands (three bf16 planes): dW[m][c] = Σ_p G[p][m]·X[p][c] with G [P][M] and X [P][C] both
// [pixel][channel] rows — the k9 weight gradients, X being the split im2col of the window.
// v_mfma_f32_16x16x32_bf16 with K = 32 pixels per step: a workgroup owns all M rows and a CB-column
// tile of C on 2×4 waves. Both tiles arrive by LDS-DMA as [pixel][channel] bf16 rows (per plane),
// and the k-strided MFMA operands (8 consecutive pixels of one channel) come out of
// ds_read_b64_tr_b16: a 16-lane group reads 4 pixel rows × 16 channels and lane i receives
// channel i of the 4 rows — two reads make the 8-deep k-group. Six part products (lo·hi, hi·lo,
// mid·mid, mid·hi, hi·mid, hi·hi) per 16×16 tile, fp32 accumulation; partials [split][m][c].
typedef short s4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint2 tr16(const unsigned short* lds) {
  const s4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)lds);
  return __builtin_bit_cast(uint2, v);
}

// The same transposed read as inline asm, which the compiler does not track: its LDS-DMA alias
// check would otherwise make every LDS read of stage s wait (vmcnt(0)) for the DMA of stage s+1
// that was just issued, serialising the copy with the MFMAs. The caller publishes the results
// with lgkm_wait, which ties each fragment to a full lgkmcnt(0) so no use can precede it.
__device__ __forceinline__ uint2 tr16a(unsigned lds_byte_addr) {
  uint2 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_byte_addr) : "memory");
  return v;
}
__device__ __forceinline__ void lgkm_wait(u4& v) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v));
}

// LDS images are XOR-swizzled by 16-byte piece: piece k of pixel row r sits at k ^ swz6(r). A
// transposed read's 32-lane half touches rows {q, 8 + q} (+4), two pieces each; swz6 gives them
// disjoint bank windows (384-byte rows: the row parity already splits the 64 banks in two).
__device__ __forceinline__ int swz6(int r, int row_elems) {
  return row_elems == 192 ? 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1))
                          : 2 * ((r & 3) | (((r >> 3) & 1) << 2));
}

// IM2COL (the k9 weight gradients): X is not read from a materialised split im2col but built
// per k-step from the 3-channel NCHW image Xi ([B][3][4·Ho][4·Wo]): each of the 512 threads owns
// one (pixel, 8-column piece) of the step's [32 px][CB] X image, loads its 8 window values for the
// NEXT step into registers before the current step's MFMAs, and splits and writes them into the
// idle stage after them (the G operand still arrives by LDS-DMA). The X image holds the same split
// values in the same swizzled layout as the DMA'd one, so the partials are bit-identical; the
// 201 MB im2col write (B=32, 256²) and its re-read leave the k9 weight gradient.
template <int M, int CB, bool IM2COL = false>
__global__ void __launch_bounds__(512) wgrad_x6_1x1_kernel(const unsigned short* __restrict__ G6,
                                                              long pg, const unsigned short* __restrict__ X6,
                                                              long pxs, long P, int C, int nsplit,
                                                              float* __restrict__ part,
                                                              const float* __restrict__ Xi = nullptr,
                                                              int Ho = 0, int Wo = 0) {
  constexpr int WM = 2, WN = 4, NW = WM * WN;        // 8 waves
  constexpr int MT = M / WM / 16, NT = CB / WN / 16; // 16×16 tiles per wave
  constexpr int GPL = KP * M, XPL = KP * CB;         // u16 per plane image
  constexpr int STAGE = 3 * GPL + 3 * XPL;           // u16 per stage
  constexpr int GPR = M / 8, XPR = CB / 8;           // 16-byte pieces per pixel row
  constexpr int NGI = KP * GPR / 64, NXI = IM2COL ? 0 : KP * XPR / 64;   // DMA wave-instructions per plane
  constexpr int NI = 3 * NGI + 3 * NXI;
  static_assert(!IM2COL || KP * XPR == NW * 64, "IM2COL: one X piece per thread and step");
  constexpr int NXD = NXI > 0 ? NXI : 1;             // divisor in the (IM2COL: dead) X-slot paths
  constexpr int NI_W = (NI + NW - 1) / NW;
  static_assert(MT * WM * 16 == M && NT * WN * 16 == CB, "tile shape");
  static_assert(KP * GPR % 64 == 0 && KP * XPR % 64 == 0, "whole DMA instructions");
  static_assert((M == 192 || M == 128) && (CB == 192 || CB == 128), "384- or 256-byte rows");
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware order: the hardware deals workgroup ids round-robin to the 8 XCDs (id % 8), so
  // logical workgroup xcd·(n/8) + id/8 puts a split's column tiles on one XCD (one G chunk).
  const int nwg = gridDim.x;                  // padded to a multiple of 8
  const int L = (blockIdx.x % 8) * (nwg / 8) + blockIdx.x / 8;
  const int tiles = C / CB;
  if (L >= tiles * nsplit) return;            // padding workgroups (before any barrier)
  const int ct = L % tiles, split = L / tiles;
  const long per = ((P + nsplit - 1) / nsplit + KP - 1) / KP * KP;
  const long p0 = split * per;
  const long p1 = p0 + per < P ? p0 + per : P;
  const int nsteps = p1 > p0 ? (int)((p1 - p0 + KP - 1) / KP) : 0;

  // DMA slot j of this wave: instruction i = wave + NW·j, a fixed plane and 16-byte piece column
  // of a contiguous [pixel][channel] row; the element offset advances by KP rows per step.
  long pj[NI_W], off[NI_W];
#pragma unroll
  for (int j = 0; j < NI_W; ++j) {
    const int i = wave + NW * j;
    const bool isg = i < 3 * NGI;
    const int pc = (isg ? (i % NGI) : ((i - 3 * NGI) % NXD)) * 64 + lane;
    const int prow = isg ? pc / GPR : pc / XPR;
    const int piece = isg ? (pc % GPR) ^ swz6(prow, M) : (pc % XPR) ^ swz6(prow, CB);
    pj[j] = p0 + prow;
    off[j] = isg ? pj[j] * M + piece * 8 : pj[j] * C + ct * CB + piece * 8;
  }
  auto issue = [&](int buf) {
    unsigned short* st = smem + buf * STAGE;
#pragma unroll
    for (int j = 0; j < NI_W; ++j) {
      const int i = wave + NW * j;
      if (NI % NW != 0 && i >= NI) break;   // wave-uniform
      const void* src = g_wzero;
      unsigned short* dst;
      if (i < 3 * NGI) {
        const int pl = i / NGI, ii = i % NGI;
        if (pj[j] < p1) src = G6 + pl * pg + off[j];
        dst = st + pl * GPL + ii * 512;
      } else {
        const int pl = (i - 3 * NGI) / NXD, ii = (i - 3 * NGI) % NXD;
        if (pj[j] < p1) src = X6 + pl * pxs + off[j];
        dst = st + 3 * GPL + pl * XPL + ii * 512;
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  auto advance = [&]() {   // every slot's pixel moves on by KP
#pragma unroll
    for (int j = 0; j < NI_W; ++j) {
      const int i = wave + NW * j;
      pj[j] += KP;
      off[j] += (long)KP * (i < 3 * NGI ? M : C);
    }
  };

  f4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
  // transposed-read lane addresses: group g = lane >> 4 takes pixel rows 8g .. 8g+7 (two reads of
  // 4); lane 4q + p of the group addresses row q, channels 4p .. 4p+3.
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int frg = swz6(8 * g + q, M), frx = swz6(8 * g + q, CB);   // both ignore row bit 2 (+4 rows)
  int aoff[MT], boff[NT];          // u16 offsets within a plane image (second read: + 4 rows)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int ch = wm * (M / WM) + mt * 16 + 4 * pp;
    aoff[mt] = (8 * g + q) * M + (((ch >> 3) ^ frg) << 3) + (ch & 7);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int ch = wn * (CB / WN) + nt * 16 + 4 * pp;
    boff[nt] = (8 * g + q) * CB + (((ch >> 3) ^ frx) << 3) + (ch & 7);
  }

  // IM2COL: this thread's X piece — pixel row xpx of the step, logical piece xpc (k = ct·CB +
  // 8·xpc + e) at its swizzled slot; the window offsets of its 8 k relative to (4·oy, 4·ox)
  const int xpx = tid / XPR, xpc = tid % XPR;
  const int xdst = xpx * CB + ((xpc ^ swz6(xpx, CB)) << 3);
  const int Hi = 4 * Ho, Wi = 4 * Wo;
  int xdy[8], xdx[8], xoff[8];
  bool xkv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = ct * CB + xpc * 8 + e;
    const int c = k / 81, kh = (k % 81) / 9, kw = k % 9;
    xkv[e] = k < 243;
    xdy[e] = kh - 4;
    xdx[e] = kw - 4;
    xoff[e] = (c * Hi + kh - 4) * Wi + kw - 4;
  }
  float xr[8];
  auto load_x = [&](int s) {
    const long p = p0 + (long)s * KP + xpx;
    const int pi = (int)(p < p1 ? p : 0);
    const int ox = pi % Wo, t2 = pi / Wo, oy = t2 % Ho, b = t2 / Ho;
    const long base = ((long)b * 3 * Hi + 4 * oy) * Wi + 4 * ox;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int iy = 4 * oy + xdy[e], ix = 4 * ox + xdx[e];
      const bool ok = p < p1 && xkv[e] && (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi;
      xr[e] = ok ? Xi[base + xoff[e]] : 0.f;
    }
  };
  auto store_x = [&](int buf) {
    u4 hi, mi, lo;
    split8(f4{xr[0], xr[1], xr[2], xr[3]}, f4{xr[4], xr[5], xr[6], xr[7]}, hi, mi, lo);
    unsigned short* d = smem + buf * STAGE + 3 * GPL + xdst;
    *(u4*)d = hi;
    *(u4*)(d + XPL) = mi;
    *(u4*)(d + 2 * XPL) = lo;
  };

  const unsigned sbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned short*)smem;
  if (nsteps > 0) {
    issue(0);
    if constexpr (IM2COL) {
      load_x(0);
      store_x(0);
    }
  }
  for (int s = 0; s < nsteps; ++s) {
    dma_barrier();   // stage s landed for every wave; stage (s+1)&1 is free
    if (s + 1 < nsteps) {
      advance();
      issue((s + 1) & 1);
      if constexpr (IM2COL) load_x(s + 1);   // under this step's MFMAs
    }
    const unsigned st = sbase + (s & 1) * STAGE * 2;   // LDS byte address of the stage
    auto frag = [&](unsigned a, int rowe) {             // 8 pixels (k) of 4 channels
      const uint2 lo = tr16a(a), hi = tr16a(a + 8 * rowe);
      return u4{lo.x, lo.y, hi.x, hi.y};
    };
    u4 Bf[3][NT], Af[2][3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) Bf[pl][nt] = frag(st + 2 * (3 * GPL + pl * XPL + boff[nt]), CB);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) Af[0][pl] = frag(st + 2 * (pl * GPL + aoff[0]), M);
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) lgkm_wait(Bf[pl][nt]);
      lgkm_wait(Af[0][pl]);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int cur = mt & 1;
      if (mt + 1 < MT) {   // the next row tile's fragments load under this one's MFMAs
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) Af[cur ^ 1][pl] = frag(st + 2 * (pl * GPL + aoff[mt + 1]), M);
      }
      const bf8 A0 = __builtin_bit_cast(bf8, Af[cur][0]), A1 = __builtin_bit_cast(bf8, Af[cur][1]),
                 A2 = __builtin_bit_cast(bf8, Af[cur][2]);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf8 B0 = __builtin_bit_cast(bf8, Bf[0][nt]), B1 = __builtin_bit_cast(bf8, Bf[1][nt]),
                  B2 = __builtin_bit_cast(bf8, Bf[2][nt]);
        f4 c = acc[mt][nt];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2, B0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B2, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B1, c, 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B0, c, 0, 0, 0);
      }
      if (mt + 1 < MT) {
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) lgkm_wait(Af[cur ^ 1][pl]);
      }
    }
    if constexpr (IM2COL) {
      if (s + 1 < nsteps) store_x((s + 1) & 1);   // published by the next dma_barrier
    }
  }
  // part[split][m][c]: lane holds rows 4(lane >> 4) + r, column lane & 15 of each tile
  float* out = part + (long)split * M * C;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * (M / WM) + mt * 16 + 4 * (lane >> 4) + r;
        const int c = ct * CB + wn * (CB / WN) + nt * 16 + (lane & 15);
        out[(long)m * C + c] = acc[mt][nt][r];
      }
}

// GDN.py:83 γ gradient in x6: dγ_eff[i][j] = Σ_p dn[p][i] · u[p][j]², straight from the fp32
// tensors. The tiles, LDS images and MFMA loop are wgrad_x6_1x1_kernel's (M = CB = C), but
// the workgroup stages the operands itself: each thread loads its fp32 pieces of the next step
// into registers while the current step computes, squares u, splits both into the three bf16
// planes and writes them to the idle LDS buffer — no split copies of dn and u² in HBM, which
// would cost more traffic than the x6 contraction saves. One workgroup per pixel split.

__device__ __forceinline__ void split4(const f4& x, uint2& hi, uint2& mi, uint2& lo) {
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h[i] = __float_as_uint(x[i]) & 0xffff0000u;
    const float r = x[i] - __uint_as_float(h[i]);
    m[i] = __float_as_uint(r) & 0xffff0000u;
    l[i] = __float_as_uint(r - __uint_as_float(m[i]));
  }
  hi = uint2{__builtin_amdgcn_perm(h[1], h[0], 0x07060302u), __builtin_amdgcn_perm(h[3], h[2], 0x07060302u)};
  mi = uint2{__builtin_amdgcn_perm(m[1], m[0], 0x07060302u), __builtin_amdgcn_perm(m[3], m[2], 0x07060302u)};
  lo = uint2{__builtin_amdgcn_perm(l[1], l[0], 0x07060302u), __builtin_amdgcn_perm(l[3], l[2], 0x07060302u)};
}

template <int C>
__global__ void __launch_bounds__(512) gdn_wgrad_x6_kernel(const float* __restrict__ G,
                                                             const float* __restrict__ X, long P,
                                                             int nsplit, float* __restrict__ part) {
  constexpr int WM = 2, WN = 4, MT = C / WM / 16, NT = C / WN / 16;
  constexpr int PL = KP * C;            // u16 per plane image
  constexpr int STAGE = 6 * PL;         // three G planes, then three X planes
  constexpr int R4 = C / 4;             // float4 pieces per pixel row
  constexpr int NV = KP * R4 / 512;     // pieces per thread per operand per step
  static_assert(C == 192 || C == 128, "C");
  static_assert(KP * R4 % 512 == 0, "whole pieces per thread");
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int split = blockIdx.x;
  const long per = ((P + nsplit - 1) / nsplit + KP - 1) / KP * KP;
  const long p0 = split * per;
  const long p1 = p0 + per < P ? p0 + per : P;
  const int nsteps = p1 > p0 ? (int)((p1 - p0 + KP - 1) / KP) : 0;

  int prow[NV], gofs[NV], wofs[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int e = tid + 512 * v;
    const int r = e / R4, ch = (e % R4) * 4;
    prow[v] = r;
    gofs[v] = r * C + ch;
    wofs[v] = r * C + (((ch >> 3) ^ swz6(r, C)) << 3) + (ch & 7);
  }
  // dn pieces run two steps ahead (two register sets), u pieces one step
  f4 rga[NV], rx[NV];
  auto load_one = [&](const float* base, int s, f4 (&r)[NV]) {
    const long pb = p0 + (long)s * KP;
    const float* b = base + pb * C;
#pragma unroll
    for (int v = 0; v < NV; ++v)
      r[v] = pb + prow[v] < p1 ? *(const f4*)(b + gofs[v]) : f4{0.f, 0.f, 0.f, 0.f};
  };
  auto convert = [&](int buf, const f4 (&rg)[NV], const f4 (&ru)[NV]) {
    unsigned short* st = smem + buf * STAGE;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      uint2 h, m, l;
      split4(rg[v], h, m, l);
      *(uint2*)(st + wofs[v]) = h;
      *(uint2*)(st + PL + wofs[v]) = m;
      *(uint2*)(st + 2 * PL + wofs[v]) = l;
      const f4 sq = ru[v] * ru[v];   // u², rounded as the fp32 reference's x ** 2
      split4(sq, h, m, l);
      *(uint2*)(st + 3 * PL + wofs[v]) = h;
      *(uint2*)(st + 4 * PL + wofs[v]) = m;
      *(uint2*)(st + 5 * PL + wofs[v]) = l;
    }
  };

  f4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int fr = swz6(8 * g + q, C);
  int aoff[MT], boff[NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int ch = wm * (C / WM) + mt * 16 + 4 * pp;
    aoff[mt] = (8 * g + q) * C + (((ch >> 3) ^ fr) << 3) + (ch & 7);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int ch = wn * (C / WN) + nt * 16 + 4 * pp;
    boff[nt] = (8 * g + q) * C + (((ch >> 3) ^ fr) << 3) + (ch & 7);
  }

  auto compute = [&](int buf) {
    const unsigned short* st = smem + buf * STAGE;
    bf8 Bf[3][NT];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const unsigned short* b = st + (3 + pl) * PL + boff[nt];
        const uint2 lo = tr16(b), hi = tr16(b + 4 * C);
        Bf[pl][nt] = __builtin_bit_cast(bf8, u4{lo.x, lo.y, hi.x, hi.y});
      }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      bf8 Af[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const unsigned short* a = st + pl * PL + aoff[mt];
        const uint2 lo = tr16(a), hi = tr16(a + 4 * C);
        Af[pl] = __builtin_bit_cast(bf8, u4{lo.x, lo.y, hi.x, hi.y});
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        f4 c = acc[mt][nt];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[2], Bf[0][nt], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[0], Bf[2][nt], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[1], Bf[1][nt], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[1], Bf[0][nt], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[0], Bf[1][nt], c, 0, 0, 0);
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[0], Bf[0][nt], c, 0, 0, 0);
      }
    }
  };

  // step s computes LDS buffer s & 1; set a holds even steps, set b odd ones
  if (nsteps > 0) {
    load_one(G, 0, rga);
    load_one(X, 0, rx);
    convert(0, rga, rx);
  }
  for (int s = 0; s < nsteps; ++s) {
    __syncthreads();   // buffer s & 1 holds step s; the other one is no longer read
    if (s + 1 < nsteps) {
      load_one(G, s + 1, rga);
      load_one(X, s + 1, rx);
    }
    compute(s & 1);
    if (s + 1 < nsteps) convert((s + 1) & 1, rga, rx);
  }
  float* out = part + (long)split * C * C;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * (C / WM) + mt * 16 + 4 * (lane >> 4) + r;
        const int c = wn * (C / WN) + nt * 16 + (lane & 15);
        out[(long)m * C + c] = acc[mt][nt][r];
      }
}

// The k5 s2 p2 weight gradient in x6 with one KERNEL ROW per workgroup: workgroup (kh, 64-channel
// block cb of C, split) accumulates dW[m][cb·64 ..][kh][0..4] for all M rows. A k-step is 32 output
// pixels — two output rows × 16 columns — whose G rows [32][M] all five taps kw share, and whose
// X operands for the five taps are columns 2ow − 2 + kw of the same two input rows: one
// [2 × 36][64] X image serves every kw (the tap picks rows 2k + kw of it). Against a workgroup per
// tap this moves 64 KB per 1440 MFMAs instead of 74 KB per 864 — the LDS-DMA stream, not the
// MFMAs, bounded the per-tap kernel. 8 waves: wave (wm, wn) owns rows wm·M/4 .. and columns
// wn·32 .. of every tap, i.e. 5 × (M/64) × 2 tiles of 16×16 (120 accumulator VGPRs at M = 192).
// X image: 128-byte rows (64 channels), row r stored at slot r ^ bit4(r) and its 32-byte column
// pairs XOR-ed with (r >> 1) & 3, so a transposed read's 32-lane half — rows r0 + 2i and
// r0 + 16 + 2i, one pair each — hits 8 distinct bank windows. Partials land as
// [split][tap][m][c] (sum_splits_tap_kernel reorders them into [m][c][tap]).
template <int M>
__global__ void __launch_bounds__(512) wgrad_x6_row_kernel(const unsigned short* __restrict__ G6,
                                                              long pg, const unsigned short* __restrict__ X6,
                                                              long pxs, int B, int Ho, int Wo, int Hi,
                                                              int Wi, int C, int nsplit,
                                                              float* __restrict__ part) {
  constexpr int NW = 8, KW = 5, CBX = 64;
  constexpr int MT = M / 64, NT = 2;                 // per wave: M/4 rows × 32 columns per tap
  constexpr int XROW = 36, XR = 2 * XROW;            // X image rows (35 used per input row)
  constexpr int GPL = KP * M, XPL = XR * CBX;        // u16 per plane image
  constexpr int STAGE = 3 * GPL + 3 * XPL;
  constexpr int GPR = M / 8;                         // 16-byte pieces per G row
  constexpr int NGI = KP * GPR / 64, NXI = XR * 8 / 64;
  constexpr int NI = 3 * NGI + 3 * NXI, NI_W = (NI + NW - 1) / NW;
  static_assert(M == 192 || M == 128, "M");
  static_assert(KP * GPR % 64 == 0 && XR * 8 % 64 == 0, "whole DMA instructions");
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 3, wn = wave >> 2;
  // XCD-aware order (as wgrad_x6_1x1_kernel): a split's 5·C/64 workgroups share one XCD's L2
  const int nwg = gridDim.x;
  const int L = (blockIdx.x % 8) * (nwg / 8) + blockIdx.x / 8;
  const int tiles = KW * (C / CBX);
  if (L >= tiles * nsplit) return;   // padding workgroups (before any barrier)
  const int tile = L % tiles, split = L / tiles;
  const int kh = tile % KW, cb = tile / KW;
  const int OHP = (Ho + 1) / 2, OWB = (Wo + 15) / 16;
  const long NSTEP = (long)B * OHP * OWB;
  const long per = (NSTEP + nsplit - 1) / nsplit;
  const long s0 = split * per;
  const long s1 = s0 + per < NSTEP ? s0 + per : NSTEP;
  const int nsteps = s1 > s0 ? (int)(s1 - s0) : 0;

  // DMA slots: G slot (row k = 16·dr + dc, physical piece) ← piece ^ swz6(k) of output pixel
  // (oh0 + dr, ow0 + dc); X slot (physical row R, 16-byte chunk J) ← chunk of logical row
  // r = R ^ bit4(R): input (2·(oh0 + r / 36) − 2 + kh, 2·ow0 − 2 + r % 36). so[j] is the slot's
  // element offset from the operand base (plane · plane stride + channel piece; 32-bit, the host
  // checks 3 planes < 2^31 elements), sa[j] its (row, column) within the step's pixel block.
  int sa[NI_W], so[NI_W];
#pragma unroll
  for (int j = 0; j < NI_W; ++j) {
    const int i = wave + NW * j;
    if (i < 3 * NGI) {
      const int pc = (i % NGI) * 64 + lane;
      const int k = pc / GPR, piece = (pc % GPR) ^ swz6(k, M);
      sa[j] = ((k >> 4) << 8) | (k & 15);
      so[j] = (i / NGI) * (int)pg + piece * 8;
    } else {
      const int ii = i - 3 * NGI;
      const int R = (ii % NXI) * 8 + (lane >> 3), J = lane & 7;
      const int r = R ^ ((R >> 4) & 1);
      const int chunk = ((((J >> 1) ^ ((r >> 1) & 3)) << 1) | (J & 1));
      sa[j] = ((r / XROW) << 8) | (r % XROW);
      so[j] = (ii / NXI) * (int)pxs + cb * CBX + chunk * 8;
    }
  }
  // position (image, output row pair, 16-column block) of the next step to issue, advanced by one
  // step per issue: no 64-bit divisions in the loop
  int owb, ohp, bimg;
  {
    const long t = s0 / OWB;
    owb = (int)(s0 - t * OWB);
    ohp = (int)(t % OHP);
    bimg = (int)(t / OHP);
  }
  // the zero line's address pinned in SGPRs: as a __device__ global it would be re-read from the
  // GOT by a scalar load at every use, and each such load delays the next lgkmcnt(0) wait
  const unsigned short* zp = (const unsigned short*)g_wzero;
  asm volatile("" : "+s"(zp));
  auto issue = [&](int buf, int j0, int j1, bool adv) {
    const int oh0 = 2 * ohp, ow0 = 16 * owb;
    const int gpix = (bimg * Ho + oh0) * Wo + ow0;            // G pixel of (oh0, ow0)
    const int xrow = bimg * Hi + 2 * oh0 - 2 + kh, xcol = 2 * ow0 - 2;
    unsigned short* st = smem + buf * STAGE;
#pragma unroll
    for (int j = j0; j < j1; ++j) {
      const int i = wave + NW * j;
      if (NI % NW != 0 && i >= NI) break;   // wave-uniform
      const unsigned short* src;
      unsigned short* dst;
      const int dr = sa[j] >> 8, dc = sa[j] & 255;
      if (i < 3 * NGI) {   // wave-uniform; the bounds checks below are selects, not branches
        const unsigned short* p = G6 + (unsigned)(so[j] + (gpix + dr * Wo + dc) * M);
        src = oh0 + dr < Ho && ow0 + dc < Wo ? p : zp;
        dst = st + (i / NGI) * GPL + (i % NGI) * 512;
      } else {
        const int ii = i - 3 * NGI;
        const int iy = 2 * (oh0 + dr) - 2 + kh, ix = xcol + dc;
        const unsigned short* p = X6 + (unsigned)(so[j] + ((xrow + 2 * dr) * Wi + ix) * C);
        src = dc < 2 * 16 + 3 && (unsigned)iy < (unsigned)Hi && (unsigned)ix < (unsigned)Wi ? p : zp;
        dst = st + 3 * GPL + (ii / NXI) * XPL + (ii % NXI) * 512;
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
    if (adv && ++owb == OWB) {
      owb = 0;
      if (++ohp == OHP) { ohp = 0; ++bimg; }
    }
  };

  f4 acc[KW][MT][NT];
#pragma unroll
  for (int kw = 0; kw < KW; ++kw)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[kw][mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
  // transposed-read lanes: group g = lane >> 4 takes k-rows 8g .. 8g+7 (two reads of 4); lane
  // 4q + p of the group addresses k-row q (+4), channels 4p .. 4p+3 of its 16-column block
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int frg = swz6(8 * g + q, M);
  int aoff[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int ch = wm * (M / 4) + mt * 16 + 4 * pp;
    aoff[mt] = (8 * g + q) * M + (((ch >> 3) ^ frg) << 3) + (ch & 7);
  }
  // X row of k-row k for tap kw: (k >> 4)·36 + 2·(k & 15) + kw
  const int k0 = 8 * g + q;
  const int xr0 = (k0 >> 4) * XROW + 2 * (k0 & 15), xr1 = xr0 + 8;   // k0 + 4 stays in its half
  auto xoff = [&](int r, int nt) {   // u16 offset in a plane image
    const int R = r ^ ((r >> 4) & 1);
    return R * CBX + ((((2 * wn + nt) ^ ((r >> 1) & 3))) << 4) + 4 * pp;
  };
  const unsigned sbase = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned short*)smem;
  auto frag = [&](unsigned lo_addr, unsigned hi_addr) {
    const uint2 lo = tr16a(lo_addr), hi = tr16a(hi_addr);
    return u4{lo.x, lo.y, hi.x, hi.y};
  };

  if (nsteps > 0) issue(0, 0, NI_W, true);
  for (int s = 0; s < nsteps; ++s) {
    dma_barrier();   // stage s landed for every wave; stage (s+1)&1 is free
    const unsigned st = sbase + (s & 1) * STAGE * 2;
    const unsigned sx = st + 3 * GPL * 2;
    u4 Af[MT][3], Bf[2][NT][3];
    auto load_b = [&](int kw, int buf) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int o0 = xoff(xr0 + kw, nt), o1 = xoff(xr1 + kw, nt);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          Bf[buf][nt][pl] = frag(sx + 2 * (pl * XPL + o0), sx + 2 * (pl * XPL + o1));
      }
    };
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        Af[mt][pl] = frag(st + 2 * (pl * GPL + aoff[mt]), st + 2 * (pl * GPL + aoff[mt] + 4 * M));
    load_b(0, 0);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) lgkm_wait(Af[mt][pl]);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) lgkm_wait(Bf[0][nt][pl]);
#pragma unroll
    for (int kw = 0; kw < KW; ++kw) {
      const int cur = kw & 1;
      if (kw + 1 < KW) load_b(kw + 1, cur ^ 1);   // the next tap's X fragments under these MFMAs
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf8 A0 = __builtin_bit_cast(bf8, Af[mt][0]), A1 = __builtin_bit_cast(bf8, Af[mt][1]),
                   A2 = __builtin_bit_cast(bf8, Af[mt][2]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const bf8 B0 = __builtin_bit_cast(bf8, Bf[cur][nt][0]),
                    B1 = __builtin_bit_cast(bf8, Bf[cur][nt][1]),
                    B2 = __builtin_bit_cast(bf8, Bf[cur][nt][2]);
          f4 c = acc[kw][mt][nt];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A2, B0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B2, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B1, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A1, B0, c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B1, c, 0, 0, 0);
          acc[kw][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A0, B0, c, 0, 0, 0);
        }
      }
      // the next stage's DMA goes out two slots per tap behind the MFMAs of taps 0-3: its address
      // arithmetic fills MFMA gaps instead of delaying the step's first fragment reads after the
      // barrier, where all 8 waves would run it at once (wgrad_check B=32: 0.405 -> 0.375 ms)
      if (kw < 4 && s + 1 < nsteps) issue((s + 1) & 1, 2 * kw, 2 * kw + 2 < NI_W ? 2 * kw + 2 : NI_W, kw == 3);
      if (kw + 1 < KW) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) lgkm_wait(Bf[cur ^ 1][nt][pl]);
      }
    }
  }
  // part[split][tap][m][c]: a store instruction writes four 64-byte runs of c (the [m][c][tap]
  // order of the per-tap kernels scattered every lane 100 bytes apart); sum_splits_tap_kernel
  // adds the splits and writes PyTorch's [m][c][kh][kw]
  float* out = part + (long)split * M * C * 25;
#pragma unroll
  for (int kw = 0; kw < KW; ++kw)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = wm * (M / 4) + mt * 16 + 4 * (lane >> 4) + r;
          const int c = cb * CBX + wn * 32 + nt * 16 + (lane & 15);
          out[((long)(kh * 5 + kw) * M + m) * C + c] = acc[kw][mt][nt][r];
        }
}


// Σ over splits of part[s][m][256] → dW[m][243] (fixed split order, 8 loads in flight).
__global__ void sum_splits_k9_kernel(const float* __restrict__ part, int nsplit, int M,
                                     float* __restrict__ out) {
  const long n = (long)M * 243;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long src = (i / 243) * 256 + i % 243;
    const long stride = (long)M * 256;
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= nsplit; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long)(k + j) * stride + src];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < nsplit; ++k) s += part[(long)k * stride + src];
    out[i] = s;
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

// Up to two independent [T][C] matrices per launch pair (blockIdx.z / blockIdx.y picks one).
struct Rows2 {
  const float* part[2];
  float* ws[2];
  float* out[2];
};
// sum_splits_kernel over the workspace of matrix blockIdx.y of a Rows2 (nsplit rows of n)
__global__ void sum_splits2_kernel(const Rows2 r, int nsplit, long n) {
  const float* __restrict__ part = r.ws[blockIdx.y];
  float* __restrict__ out = r.out[blockIdx.y];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= nsplit; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long)(k + j) * n + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < nsplit; ++k) s += part[(long)k * n + i];
    out[i] = s;
  }
}

// Σ over many splits (≥ 64) of few elements: 4 lanes per element each add a quarter of the splits
// in order, then the quarters are added in order ((q0 + q1) + q2) + q3 — a fixed tree, so the
// result is reproducible — on 4× the workgroups of sum_splits_kernel.
__global__ void __launch_bounds__(256) sum_splits4_kernel(const float* __restrict__ part,
                                                          int nsplit, long n,
                                                          float* __restrict__ out) {
  __shared__ float red[4][64];
  const int el = threadIdx.x & 63, g = threadIdx.x >> 6;
  const long i = (long)blockIdx.x * 64 + el;
  const int q = (nsplit + 3) / 4, k0 = g * q, k1 = k0 + q < nsplit ? k0 + q : nsplit;
  float s = 0.f;
  if (i < n) {
    int k = k0;
    for (; k + 8 <= k1; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long)(k + j) * n + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < k1; ++k) s += part[(long)k * n + i];
  }
  red[g][el] = s;
  __syncthreads();
  if (g == 0 && i < n) out[i] = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
}

// out[i] = Σ_s part[s][i], fixed order.
__global__ void sum_splits_kernel(const float* __restrict__ part, int nsplit, long n,
                                  float* __restrict__ out) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= nsplit; k += 8) {   // 8 loads in flight, added in split order
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long)(k + j) * n + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < nsplit; ++k) s += part[(long)k * n + i];
    out[i] = s;
  }
}

// dW[m][c][tap] = Σ_s part[s][tap][m][c] (wgrad_x6_row_kernel's partials), the splits added in
// order as sum_splits_kernel does: reads coalesced along c, one scattered write per element.
__global__ void sum_splits_tap_kernel(const float* __restrict__ part, int nsplit, int M, int C,
                                      float* __restrict__ out) {
  const long n = (long)M * C * 25;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    int k = 0;
    for (; k + 8 <= nsplit; k += 8) {   // 8 loads in flight, added in split order
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(long)(k + j) * n + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; k < nsplit; ++k) s += part[(long)k * n + i];
    const long mc = i % ((long)M * C);
    out[mc * 25 + i / ((long)M * C)] = s;
  }
}

// out[c] = Σ_t part[t][c] in two fixed-order levels (bitwise reproducible): workgroup (column
// block, split s) sums rows [s·per, (s+1)·per) — 4 lane groups strided, combined in order — into
// ws[s][c]; then sum_splits adds the splits in order. Enough workgroups to be bandwidth-bound
// (one workgroup per 64 columns walked thousands of rows serially).
constexpr int SUM_ROWS_SPLITS = 64;

// Split s of matrix blockIdx.z, columns blockIdx.x·64 ..: ws[s][c] = Σ_t part[t][c] over the split's
// rows. The split rows go out write-through (sc1) and the workgroup of a (column block, matrix)
// whose arrival on a device-global counter comes last adds them in split order — the order of
// sum_splits2_kernel, which this folds in (one launch instead of two): the counter's slot is dealt
// round-robin by the host and reset by that last workgroup (zero when the code object loads).
constexpr unsigned kRowSlots = 256;
__device__ unsigned g_rows_done[kRowSlots][8];   // [slot][column block + 4 · matrix]
static std::atomic<unsigned> g_rows_slot{0};

__global__ void sum_rows2_kernel(const Rows2 r, int T, int C, int per, unsigned slot) {
  const float* __restrict__ part = r.part[blockIdx.z];
  float* __restrict__ ws = r.ws[blockIdx.z];
  __shared__ float red[4][64];
  __shared__ bool last;
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int t0 = blockIdx.y * per, t1 = t0 + per < T ? t0 + per : T;
  float s = 0.f;
  if (c < C)
    for (int t = t0 + g; t < t1; t += 4) s += part[(long)t * C + c];
  red[g][cl] = s;
  __syncthreads();
  if (slot == ~0u) {   // C > 256: sum_splits2_kernel adds the splits
    if (g == 0 && c < C)
      ws[(long)blockIdx.y * C + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
    return;
  }
  unsigned* done = &g_rows_done[slot][blockIdx.x + 4 * blockIdx.z];
  if (g == 0) {
    if (c < C)
      __hip_atomic_store(&ws[(long)blockIdx.y * C + c],
                         ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    // the arrival is an agent-scope acq_rel read-modify-write: its release orders the wave's
    // split row (and the other waves' rows, behind the barrier below the stores) before the count,
    // its acquire orders the last workgroup's loads of every split row after it (the memory
    // model's guarantee, not the store-ack timing a bare s_waitcnt gives)
    if (cl == 0)
      last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.y - 1;
  }
  __syncthreads();
  if (!last) return;
  if (g == 0 && c < C) {   // eight loads in flight at a time, added in split order
    const int ns = gridDim.y;
    float o = 0.f;
    int k = 0;
    for (; k + 8 <= ns; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = __hip_atomic_load(&ws[(long)(k + j) * C + c], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int j = 0; j < 8; ++j) o += v[j];
    }
    for (; k < ns; ++k)
      o += __hip_atomic_load(&ws[(long)k * C + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    r.out[blockIdx.z][c] = o;
  }
  if (threadIdx.x == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// Per-channel sums of an NCHW tensor [B][C][HW] over fixed PLANE_CHUNK-element chunks of each
// plane: part[b·K + k][c], K = ⌈HW / PLANE_CHUNK⌉ (one workgroup per (b, c, k)); summed over the
// B·K rows by iclr17_sum_rows in a fixed order.
constexpr long PLANE_CHUNK = 4096;
__global__ void plane_sum_kernel(const float* __restrict__ A, int C, long HW, int K,
                                 float* __restrict__ part) {
  __shared__ float red[4];
  const int bc = blockIdx.x, k = blockIdx.y;
  const long base = (long)bc * HW;
  const long lo = k * PLANE_CHUNK, hi = lo + PLANE_CHUNK < HW ? lo + PLANE_CHUNK : HW;
  float s = 0.f;
  for (long i = lo + threadIdx.x; i < hi; i += 256) s += A[base + i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int b = bc / C, c = bc % C;
    part[((long)b * K + k) * C + c] = ((red[0] + red[1]) + red[2]) + red[3];
  }
}

// x6 wgrad: one workgroup per CU
int wgrad6_splits(long P, int tiles) {   // one round of 256 workgroup slots (1 per CU)
  int s = 256 / tiles;
  const long maxs = P / 256 > 1 ? P / 256 : 1;
  if (s > maxs) s = (int)maxs;
  return s < 1 ? 1 : s;
}
int wgrad9_splits(int ntiles) { return ntiles < 128 ? ntiles : 128; }
int gdn6_splits(long P) {   // one workgroup per CU, at least 4 steps of 32 pixels each
  const long s = P / 128;
  return s > 256 ? 256 : s < 1 ? 1 : (int)s;
}

int wgrad_splits(long P, int tiles) {
  // as many splits as fit ONE round of 512 workgroup slots (256 CUs × 2): a grid just over 512
  // (75 tiles × 7 = 525) would run a second round for 13 workgroups and double the time;
  // at least ~256 pixels per split
  int s = 512 / tiles;
  const long maxs = P / 256 > 1 ? P / 256 : 1;
  if (s > maxs) s = (int)maxs;
  if (s < 1) s = 1;
  return s;
}

}  // namespace
}  // namespace iclr17

using namespace iclr17;

extern "C" {

int iclr17_sum_rows(const float* part, int T, int C, float* workspace, float* out, void* stream);

size_t iclr17_wgrad_workspace_size(int kind, int B, int Ho, int Wo, int M, int C) {
  const long P = (long)B * Ho * Wo;
  if (kind == 9) return (size_t)wgrad9_splits(B * ((Wo + 7) / 8) * ((Ho + 7) / 8)) * M * 243;
  if (kind == 6) return (size_t)wgrad6_splits(P, 5 * (C / 64)) * M * C * 25;
  if (kind == 7)   // k9 x6: partials [ns][M][256]
    return (size_t)wgrad6_splits(P, 2) * M * 256;
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

int iclr17_wgrad_k5_x6(const uint16_t* G_split, const uint16_t* X_split, int B, int Ho, int Wo,
                       int M, int C, float* workspace, float* dW, void* stream) {
  ICLR17_REQUIRE(B > 0 && Ho > 0 && Wo > 0, ICLR17_EINVAL, "wgrad_k5_x6: bad shape");
  ICLR17_REQUIRE((M == 128 || M == 192) && C % 64 == 0 && C > 0, ICLR17_EUNSUPPORTED,
                 "wgrad_k5_x6: M=%d C=%d unsupported", M, C);
  ICLR17_REQUIRE(G_split && X_split && workspace && dW, ICLR17_EINVAL, "wgrad_k5_x6: null pointer");
  const long P = (long)B * Ho * Wo;
  ICLR17_REQUIRE(M == C, ICLR17_EUNSUPPORTED, "wgrad_k5_x6: M=%d C=%d (square layers only)", M, C);
  const int tiles = 5 * (C / 64);   // (kernel row, 64-channel block)
  const int ns = wgrad6_splits(P, tiles);
  const long pg = P * M, pxs = (long)B * 4 * Ho * Wo * C;
  ICLR17_REQUIRE(3 * pg < (1L << 31) && 3 * pxs < (1L << 31), ICLR17_EUNSUPPORTED,
                 "wgrad_k5_x6: split operands of %ld / %ld elements exceed 32-bit offsets", 3 * pg, 3 * pxs);
  hipStream_t st = S(stream);
  dim3 grid((tiles * ns + 7) / 8 * 8);   // 1-D, padded to whole XCD rounds (see the kernel)
  const unsigned short* g6 = (const unsigned short*)G_split;
  const unsigned short* x6 = (const unsigned short*)X_split;
  if (M == 192)
    hipLaunchKernelGGL((wgrad_x6_row_kernel<192>), grid, dim3(512), 0, st, g6, pg, x6, pxs, B, Ho, Wo, 2 * Ho, 2 * Wo, C, ns, workspace);
  else
    hipLaunchKernelGGL((wgrad_x6_row_kernel<128>), grid, dim3(512), 0, st, g6, pg, x6, pxs, B, Ho, Wo, 2 * Ho, 2 * Wo, C, ns, workspace);
  int rc = check_launch("wgrad_k5_x6");
  if (rc) return rc;
  const long n = (long)M * C * 25;
  hipLaunchKernelGGL(sum_splits_tap_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, workspace, ns, M, C, dW);
  return check_launch("wgrad_k5_x6_sum");
}
int iclr17_wgrad_k9_x6(const uint16_t* G_split, const float* X, int B, int Ho, int Wo, int M,
                       float* workspace, float* dW, void* stream) {
  ICLR17_REQUIRE(B > 0 && Ho > 0 && Wo > 0 && (long)B * Ho <= 65535, ICLR17_EINVAL,
                 "wgrad_k9_x6: bad shape");
  ICLR17_REQUIRE(M == 128 || M == 192, ICLR17_EUNSUPPORTED, "wgrad_k9_x6: M=%d unsupported", M);
  ICLR17_REQUIRE(G_split && X && workspace && dW, ICLR17_EINVAL, "wgrad_k9_x6: null pointer");
  const long P = (long)B * Ho * Wo;
  const int tiles = 2;   // 256 columns (243 used) in two 128-column tiles
  const int ns = wgrad6_splits(P, tiles);
  float* part = workspace;
  hipStream_t st = S(stream);
  dim3 grid((tiles * ns + 7) / 8 * 8);
  const unsigned short* g6 = (const unsigned short*)G_split;
  int rc;
  if (M == 192) {
    hipLaunchKernelGGL((wgrad_x6_1x1_kernel<192, 128, true>), grid, dim3(512), 0, st, g6, P * M, nullptr, 0L, P, 256, ns, part, X, Ho, Wo);
  } else {
    hipLaunchKernelGGL((wgrad_x6_1x1_kernel<128, 128, true>), grid, dim3(512), 0, st, g6, P * M, nullptr, 0L, P, 256, ns, part, X, Ho, Wo);
  }
  rc = check_launch("wgrad_k9_x6");
  if (rc) return rc;
  const long n = (long)M * 243;
  hipLaunchKernelGGL(sum_splits_k9_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, ns, M, dW);
  return check_launch("wgrad_k9_x6_sum");
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

size_t iclr17_gdn_wgrad_x6_workspace_size(long P, int C) {
  return (size_t)gdn6_splits(P) * C * C;
}

// iclr17_gdn_wgrad in the x6 scheme (fp32 dn and u in, split by the kernel).
int iclr17_gdn_wgrad_x6(const float* dn, const float* u, long P, int C, float* workspace,
                        float* dgamma_eff, void* stream) {
  ICLR17_REQUIRE(P > 0 && (C == 128 || C == 192), ICLR17_EUNSUPPORTED, "gdn_wgrad_x6: C=%d", C);
  ICLR17_REQUIRE(dn && u && workspace && dgamma_eff, ICLR17_EINVAL, "gdn_wgrad_x6: null pointer");
  const int ns = gdn6_splits(P);
  hipStream_t st = S(stream);
  if (C == 192)
    hipLaunchKernelGGL(gdn_wgrad_x6_kernel<192>, dim3(ns), dim3(512), 0, st, dn, u, P, ns, workspace);
  else
    hipLaunchKernelGGL(gdn_wgrad_x6_kernel<128>, dim3(ns), dim3(512), 0, st, dn, u, P, ns, workspace);
  int rc = check_launch("gdn_wgrad_x6");
  if (rc) return rc;
  const long n = (long)C * C;
  hipLaunchKernelGGL(sum_splits4_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, st, workspace, ns, n, dgamma_eff);
  return check_launch("gdn_wgrad_x6_sum");
}

size_t iclr17_sum_rows_workspace_size(int C) { return (size_t)SUM_ROWS_SPLITS * C; }

// out[c] = Σ_t part[t][c] (fixed order). workspace: iclr17_sum_rows_workspace_size(C) floats.
static int sum_rows_n(const Rows2& r, int nm, int T, int C, void* stream) {
  const int per = (T + SUM_ROWS_SPLITS - 1) / SUM_ROWS_SPLITS;
  const int ns = (T + per - 1) / per;
  const bool fused = C <= 256;   // g_rows_done holds 4 column blocks per matrix
  hipLaunchKernelGGL(sum_rows2_kernel, dim3((C + 63) / 64, ns, nm), dim3(256), 0, S(stream), r, T,
                     C, per, fused ? g_rows_slot.fetch_add(1) % kRowSlots : ~0u);
  int rc = check_launch("sum_rows");
  if (rc || fused) return rc;
  hipLaunchKernelGGL(sum_splits2_kernel, dim3((C + 255) / 256, nm), dim3(256), 0, S(stream), r, ns,
                     (long)C);
  return check_launch("sum_rows_splits");
}

int iclr17_sum_rows(const float* part, int T, int C, float* workspace, float* out, void* stream) {
  ICLR17_REQUIRE(part && workspace && out && T > 0 && C > 0, ICLR17_EINVAL,
                 "sum_rows: bad arguments");
  const Rows2 r{{part, nullptr}, {workspace, nullptr}, {out, nullptr}};
  return sum_rows_n(r, 1, T, C, stream);
}

// iclr17_sum_rows of two [T][C] matrices in one launch pair; workspace: twice
// iclr17_sum_rows_workspace_size(C) floats.
int iclr17_sum_rows2(const float* part_a, const float* part_b, int T, int C, float* workspace,
                     float* out_a, float* out_b, void* stream) {
  ICLR17_REQUIRE(part_a && part_b && workspace && out_a && out_b && T > 0 && C > 0, ICLR17_EINVAL,
                 "sum_rows2: bad arguments");
  const Rows2 r{{part_a, part_b}, {workspace, workspace + (long)SUM_ROWS_SPLITS * C}, {out_a, out_b}};
  return sum_rows_n(r, 2, T, C, stream);
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
  return iclr17_sum_rows(workspace, 1024, C, workspace + 1024L * C, db, stream);
}

// Bias gradient from an NCHW gradient [B][C][HW] (deconv3 output): workspace (B + 64)*C floats.
int iclr17_bias_grad_nchw(const float* G, int B, int C, long HW, float* workspace, float* db,
                          void* stream) {
  ICLR17_REQUIRE(B > 0 && C > 0 && HW > 0 && G && workspace && db, ICLR17_EINVAL, "bias_grad_nchw: bad arguments");
  hipStream_t st = S(stream);
  const int K = (int)((HW + PLANE_CHUNK - 1) / PLANE_CHUNK);
  hipLaunchKernelGGL(plane_sum_kernel, dim3(B * C, K), dim3(256), 0, st, G, C, HW, K, workspace);
  int rc = check_launch("bias_grad_nchw");
  if (rc) return rc;
  // part is [B·K][C] → sum over the rows for each c
  return iclr17_sum_rows(workspace, B * K, C, workspace + (long)B * K * C, db, stream);
}

}  // extern "C"
