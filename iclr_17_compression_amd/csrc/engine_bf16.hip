// bf16 throughput mode of the Ballé-2017 codec forward on gfx950.
//
// Activations between layers are bf16 NHWC ([B][h][w][N], round-to-nearest-even from fp32), the
// weights and the GDN γ are bf16, every contraction is ONE v_mfma_f32_16x16x32_bf16 product per
// MAC with fp32 accumulation, and the epilogues (bias, GDN/IGDN normalisation, quantiser, rate,
// clamp) run in fp32. This is the mode the north_star's "≥ 40 % of the bf16 MFMA peak" bar is
// quoted on; the parity modes (exact-f32 and x6) stay the default.
//
// The k5 engine (conv2, conv3 + quantiser + rate, deconv1, deconv2), analysis_17.py:18-23 and
// synthesis_17.py:15-22:
//   * Tile: TH × 16 output pixels of the base grid (conv: the output grid; deconv: one stride
//     phase of the input grid) × NB output channels per workgroup of WM × WN waves. MFMA
//     orientation C[channel][pixel]: A = weights (16 channels × 8 k per lane), B = pixels (one
//     pixel's 8 consecutive input channels per lane), so a lane's accumulator holds 4
//     consecutive channels of one pixel and the epilogue stores 8 bytes per lane.
//   * Input: per 16-channel chunk the halo patch of the tile (conv: (2·TH+3) × 35 pixels, stored
//     as even / odd column planes so a stride-2 tap reads consecutive 32-byte pixel slots; deconv:
//     (TH+2) × 18) is staged ONCE by LDS-DMA and every tap reads a shifted window of it — 4.8×
//     (conv) / 1.3× (deconv) the tile's pixels instead of 25× / 6.25×. Double buffered: chunk
//     c+1's patch streams in during chunk c's steps. Fragment reads are conflict-free (a 16-lane
//     group reads 16 consecutive pixel slots, the two 16-byte halves in alternate slots).
//   * K order: one k32 step = two taps × the chunk's 16 channels (lane groups 0/1: tap 2s,
//     channel halves; 2/3: tap 2s+1); an odd tap count is padded with a zero-weight tap.
//   * Weights: the step's [4 k-groups][NB][8] bf16 slice (12 KB at NB = 192) by LDS-DMA into a
//     two-stage ring, one barrier per step.
//   * Epilogues: GDN / IGDN (x² → bf16 tile in LDS, the channel contraction n = γ·x² on the same
//     MFMA with γ bf16 from L2, then x/√(β+n) or x·√(β+n) in fp32), and the quantiser + rate of
//     conv3 (round half-to-even, the factorised CDF twice, −log₂, per-workgroup bit sums).
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "k5_common.h"

namespace iclr17 {
namespace bfm {

constexpr int kC3KS = 2;   // conv3: input-channel halves per tile, one 4-wave group each
constexpr int kNST = 4;    // weight ring stages (F + 2 for F DMA groups in flight)
__device__ __attribute__((aligned(16))) unsigned g_zero16[4] = {0u, 0u, 0u, 0u};

// A padding ("sink") load of the counted-vmcnt DMA schedule: one vector-memory instruction like
// any other, but 4 bytes per lane (256 B into the sink) instead of a 16-byte piece (1 KB)
__device__ __forceinline__ void sink_load(void* lds_sink) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g_zero16,
                                   (__attribute__((address_space(3))) void*)lds_sink,
                                   4, 0, 0);
}

enum BEpi : int { BE_GDN = 0, BE_IGDN = 1, BE_QUANT = 2 };

__device__ __forceinline__ f4 mfma_bf16(const u4& a, const u4& b, const f4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a),
                                                 __builtin_bit_cast(bf8, b), c, 0, 0, 0);
}

struct K5Args {
  const u16* in;        // bf16 NHWC [B][Hin][Win][CI]
  const u16* w;         // packed bf16 weights (iclr17_pack_bf16 ICLR17_BF_CONV5 / _DECONV5)
  const float* bias;    // [CO] or null
  const float* beta;    // GDN: β_eff [CO]
  const u16* gamma;     // GDN: γ_eff bf16 in the A-fragment layout [CO/8][CO][8]
  u16* out;             // bf16 NHWC [B][Hout][Wout][CO]
  float* out_f32;       // QUANT: ŷ fp32 NHWC
  float* y_f32;         // QUANT: y (before rounding) fp32 NHWC, or null
  const float* rate;    // QUANT: packed rate table [11][CO]
  const float* rtab;    // QUANT: element_bits(v, c) for integer v ∈ [−RT_K, RT_K] ([CO][2·RT_K+1])
  double* partial;      // QUANT: bit sums [B][ppi]
  int ppi;              // QUANT: partials per image
  int B, Hin, Win, Hout, Wout;
  int gh, gw;           // base grid (conv: output grid; deconv: input grid)
  int tiles_x, tiles_y;
};

// ------------------------------------------------------------------------- rate table
// element_bits(v, c) (model.py:71-73 per element) for the integer latents v ∈ [−RT_K, RT_K] of
// each channel: the round-mode quantiser epilogue looks them up instead of evaluating the
// 4-layer factorised CDF twice (tanh ×3, sigmoid, log) per element.
constexpr int RT_K = 32, RT_W = 2 * RT_K + 1;

__global__ void __launch_bounds__(256) rate_table_kernel(const float* __restrict__ rate, int C,
                                                         float* __restrict__ table) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C * RT_W) return;
  const int c = i / RT_W, v = i - c * RT_W - RT_K;
  table[i] = element_bits((float)v, rate, C, c);
}

// ---------------------------------------------------------------- x² / output tile layout
// [R pixels][CO] bf16 rows of stride CO·2 + 16 bytes (≡ 4 dwords mod 64 banks at N = 128 and
// 192): the 16-byte fragment reads of 16 consecutive pixels hit 16 distinct 4-bank slots, and
// the 8-byte writes of 16 pixels are at most 2-way (CO·2 + 32 had 2-way reads, 4-way writes:
// 34 % of conv1p's LDS cycles were conflicts, profiles/r05_bf16_traffic.json)
constexpr int kEpiPad = 16;
template <int CO>
__device__ __forceinline__ int epi_off(int p, int ch) {   // byte offset of (pixel, channel)
  return p * (CO * 2 + kEpiPad) + ch * 2;
}

template <int CO>
constexpr int epi_tile_bytes(int R) { return R * (CO * 2 + kEpiPad); }

// ------------------------------------------------------------------------------ kernel
// One workgroup: a TH × 16 tile of base pixels (conv: output pixels; deconv: input pixels of
// one stride phase) × NB output channels on TH / 2 waves. Wave w owns the 32 pixels of tile
// rows 2w and 2w + 1 and all NB channels: NB / 32 accumulators of v_mfma_f32_32x32x16_bf16,
// C[channel][pixel]. The 32×32 tile leaves 24 of every 32 issue cycles beside the MFMA (the
// 16×16×32 form leaves 8 of 16), room for the fragment reads and the DMA issue of a step.
// conv3 (the quantiser epilogue) splits K: KS groups of TH / 2 waves in one workgroup each run
// the whole main loop on their share of the input channels with their own patch buffers and
// weight ring (the groups' barriers line up: equal step counts), then group 0 adds the other
// groups' accumulators from LDS in a fixed order and runs the epilogue. conv3's 256 tiles at B=64
// otherwise hold one wave per SIMD.
constexpr int k5_threads(int TH, int EPI) { return TH / 2 * 64 * (EPI == BE_QUANT ? kC3KS : 1); }

template <int MODE, int TH, int NB, int CO, int CI, int EPI>
struct K5 {
  static constexpr int KS = EPI == BE_QUANT ? kC3KS : 1;   // K-split groups
  static_assert(k5_threads(TH, EPI) == KS * (TH / 2) * 64, "threads");
  static constexpr int NW = TH / 2, NT_ = NW * 64;   // waves / threads of one group
  static constexpr int NT = NB / 32;            // 32-channel accumulator tiles per wave
  static constexpr int R = TH * 16;             // pixels per tile
  static constexpr int NCH = CI / 16 / KS;      // 16-channel chunks per group
  static constexpr int SB = 4 * NB * 16;        // weight stage bytes
  static constexpr int NBI = SB / 1024;         // weight DMA wave-instructions per step
  using P = Patch<MODE, TH>;
  static constexpr int NST = kNST;              // weight stages (ring)
  static constexpr int MAIN_LDS = 2 * P::BUF + NST * SB + 1024;
  static constexpr int GBLK = (CO / 32) * (CO / 16);   // GDN: γ fragment blocks, 1 KB each
  static constexpr int OS = CO * 2 + 16;               // GDN: output tile row stride (bytes)
  // γ staged beside the main-loop buffers, by DMAs issued in the prologue, where that still
  // fits one workgroup per CU (the 8-wave tiles run one per CU anyway); else after the loop
  static constexpr bool EARLY_G = EPI != BE_QUANT && NW == 8 && MAIN_LDS + GBLK * 1024 <= 160 * 1024;
  static constexpr int GOFF = EARLY_G ? MAIN_LDS : 0;
  static constexpr int EPI_LDS = EPI == BE_QUANT ? 64
                                 : (GOFF + GBLK * 1024 > R * OS ? GOFF + GBLK * 1024 : R * OS);
  static constexpr int LDS0 = KS * MAIN_LDS > EPI_LDS ? KS * MAIN_LDS : EPI_LDS;
  // GDN: each wave stores its own y rows, a channel pair of tiles at a time, through a private
  // 4 KB [32 px][64 ch] image (no workgroup barrier: the stores overlap other waves' contraction)
  static constexpr int YOFF = EARLY_G ? 0 : GBLK * 1024;
  static constexpr bool DIRECT_Y = EPI != BE_QUANT && NT % 2 == 0 && YOFF + NW * 4096 <= LDS0 &&
                                   (EARLY_G ? NW * 4096 <= MAIN_LDS : true);
  // GDN: bias and β_eff staged by two prologue DMAs into their own 2 KB (an epilogue global load
  // of them waited out a full L2 round trip after the main loop)
  static constexpr int BBOFF = (LDS0 + 1023) / 1024 * 1024;
  static constexpr int LDS = EPI == BE_QUANT ? LDS0 : BBOFF + 2048;
  static_assert(KS == 1 || (KS - 1) * NW * NT * 16 * 64 * 4 <= KS * MAIN_LDS, "K-split exchange");
  static_assert(TH % 2 == 0 && NB % 32 == 0 && SB % 1024 == 0 && CI % (16 * KS) == 0, "tile shape");
  static_assert(EPI == BE_QUANT || NB == CO, "GDN needs every channel of a pixel in the tile");
};

template <int MODE, int TH, int NB, int CO, int CI, int EPI, int PH>
__device__ __forceinline__ void k5_body(const K5Args& a, unsigned char* smem, int b, int ty, int tx,
                                        int nb) {
  using KK = K5<MODE, TH, NB, CO, CI, EPI>;
  using P = typename KK::P;
  using TP = Taps<MODE, PH>;
  constexpr int NT = KK::NT, NW = KK::NW, S = TP::S, NCH = KK::NCH;
  constexpr int SB = KK::SB, NBI = KK::NBI;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = wv / NW, wave = wv - kg * NW;   // K-split group, wave within the group
  unsigned char* const gsmem = smem + kg * KK::MAIN_LDS;
  const int r32 = lane & 31, h = lane >> 5;
  // LDS-DMA schedule. Every step every wave issues exactly K DMA instructions (weights of step
  // g+F+1 into a four-stage ring, pieces of the next chunk's patch, 1 KB sink loads as padding),
  // so a counted `s_waitcnt vmcnt(F·K)` before the step's barrier retires everything but the
  // last F steps' groups: the weights of step g and, at a chunk start, the whole patch (its
  // pieces go out in the previous chunk's steps 0 .. S-F-1). F = 2 groups stay in flight where
  // a chunk has ≥ 4 steps, else 1.
  constexpr int NST = KK::NST;
  constexpr int F = (S >= 6 && NST >= 5) ? 3 : (S >= 3 ? 2 : 1), SI = S - F;
  static_assert(F >= 1 && SI >= 1, "DMA schedule");
  static_assert(NST >= F + 2, "ring depth");
  constexpr int PS = (P::NQI + SI - 1) / SI;          // patch pieces per issuing step
  constexpr int K = (NBI + PS + NW - 1) / NW;         // DMA instructions per wave per step
  constexpr int GS = NCH * S;                         // steps
  unsigned char* const sP = gsmem;                    // two patch buffers
  unsigned char* const sB = gsmem + 2 * P::BUF;       // NST weight stages
  unsigned char* const sD = sB + NST * SB;   // sink of the padding loads
  const long img = (long)b * a.Hin * a.Win;
  const int iy0 = MODE == BM_CONV ? 2 * ty * TH - 2 : ty * TH - 1;
  const int ix0 = MODE == BM_CONV ? 2 * tx * 16 - 2 : tx * 16 - 1;
  const u16* __restrict__ inb = a.in + img * CI + kg * (CI / KK::KS);
  // patch piece (wave-instruction) `piece`: this lane's 16-byte slot → source u16 offset or -1
  auto piece_src = [&](int piece) -> int {
    const int byte = (piece * 64 + lane) * 16;
    const int pr = byte / P::ROWB, rem = byte - pr * P::ROWB;
    int pc, hh;
    bool ok;
    if (MODE == BM_CONV) {
      const int par = rem / (2 * P::HALF), r2 = rem - par * 2 * P::HALF;
      hh = r2 / P::HALF;
      pc = 2 * ((r2 - hh * P::HALF) / 16) + par;
      ok = pc < 35;
    } else {
      hh = rem / P::HALF;
      pc = (rem - hh * P::HALF) / 16;
      ok = true;
    }
    const int iy = iy0 + pr, ix = ix0 + pc;
    ok = ok && pr < P::ROWS && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
    return ok ? (iy * a.Win + ix) * CI + 8 * hh : -1;
  };
  // patch piece of chunk c1 (valid) or a sink load (not valid: same instruction count)
  auto issue_piece = [&](int c1, int piece, bool valid) {
    if (!valid) {
      sink_load(sD);
      return;
    }
    const int src = piece_src(piece);
    glds16(src >= 0 ? (const void*)(inb + src + c1 * 16) : (const void*)g_zero16,
           sP + (c1 & 1) * P::BUF + piece * 1024);
  };
  // weight slots: slot k·NW + wave < NBI of a group copies 1 KB of the step's [4][NB][8] slice
  const long wstep = 4L * CO * 8;                     // u16 per (chunk, step) of the packing
  int wsrc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int q = (k * NW + wave) * 64 + lane;
    const int g = q / NB, col = q - g * NB;
    wsrc[k] = (g * CO + nb * NB + col) * 8;
  }
  // packed weights of this phase: [NCH·KS][S][4][CO][8]; K-split group kg starts at chunk kg·NCH
  const u16* __restrict__ wph = a.w + (long)kg * NCH * S * wstep;
  if (MODE == BM_DECONV) {
    long off = 0;
#pragma unroll
    for (int p = 0; p < PH; ++p) {
      const int ny = (p >> 1) == 0 ? 3 : 2, nx = (p & 1) == 0 ? 3 : 2;
      off += (long)NCH * ((ny * nx + 1) / 2) * wstep;
    }
    wph += off;
  }
  // weight slot k of step wg; past the last step a load of the last step into the sink
  auto issue_w = [&](int k, int wg) {
    const int slot = k * NW + wave;
    if (wg >= GS) {
      sink_load(sD);
      return;
    }
    glds16(wph + (long)wg * wstep + wsrc[k], sB + (wg % NST) * SB + slot * 1024);
  };

  // ---- per-lane fragment addresses
  // B (pixels): pixel (tile row 2·wave + (r32 >> 4), column r32 & 15), channel half h
  const int prow = 2 * wave + (r32 >> 4), pcol = r32 & 15;
  const int tpix = prow * 16 + pcol;   // tile pixel of this lane's accumulator column
  const int pbase = (MODE == BM_CONV ? P::off(2 * prow, 2 * pcol) : P::off(prow, pcol)) + h * P::HALF;
  // A (weights): stage [4][NB][8]: lane (k-group 2·tap + h, channel 32·i + r32)
  const int abase = (h * NB + r32) * 16;

  f16v acc[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;

  constexpr int KB16 = CO / 16;   // GDN: 16-channel k-blocks
  // γ fragments into LDS: block (i, kb) = the A operand of output tile i, k-block kb; lane
  // (r32, h) ← γ[32i + r32][16kb + 8h .. +7], 16 contiguous bytes of the [CO/8][CO][8] packing
  auto stage_gamma = [&]() {
    for (int blk = wave; blk < KK::GBLK; blk += NW) {
      const int i = blk / KB16, kb = blk - i * KB16;
      glds16(a.gamma + ((long)(2 * kb + h) * CO + 32 * i + r32) * 8, smem + KK::GOFF + blk * 1024);
    }
  };
  float* const sbb = (float*)(smem + KK::BBOFF);   // GDN: [bias CO | pad][β_eff CO | pad]
  if constexpr (EPI != BE_QUANT) {
    // waves 0 / 1: one 16-byte piece per lane (CO ≤ 256 floats); retired by the first counted wait
    static_assert(CO <= 256, "bias / β stage");
    if (wave < 2) {
      const float* src = wave == 0 ? a.bias : a.beta;
      glds16(lane * 4 < CO ? (const void*)(src + lane * 4) : (const void*)g_zero16, sbb + wave * 256);
    }
  }
  if constexpr (KK::EARLY_G) stage_gamma();   // retired by the loop's first counted wait
  // prologue: chunk 0's patch and the weights of steps 0 .. F-1 (any count per wave), then
  // step F's weights as a full K-group, so the loop's first wait leaves exactly F groups
  for (int piece = wave; piece < P::NQI; piece += NW) issue_piece(0, piece, true);
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k * NW + wave < NBI) issue_w(k, f);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k * NW + wave < NBI) issue_w(k, F);
    else sink_load(sD);
  }
#pragma unroll
  for (int f = 1; f < F; ++f)   // F−1 more full groups: the first wait keeps F in flight
#pragma unroll
    for (int k = 0; k < K; ++k) sink_load(sD);

  typedef const __attribute__((address_space(3))) u4* lu4p;
  int stage = 0;   // g % NST
  for (int c = 0; c < NCH; ++c) {
    const unsigned char* pbuf = sP + (c & 1) * P::BUF + pbase;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int g = c * S + s;
      wait_vm_barrier<F * K>();   // all but the last F groups landed: weights of step g and,
                                  // at s = 0, chunk c's patch; stage (g+F+1) % NST is free
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int slot = k * NW + wave;
        if ((k + 1) * NW <= NBI || slot < NBI) {
          issue_w(k, g + F + 1);
        } else if (s < SI) {
          const int piece = s * PS + slot - NBI;
          issue_piece(c + 1, piece, c + 1 < NCH && piece < P::NQI);
        } else {
          sink_load(sD);
        }
      }
      // taps 2s and 2s+1 (the second absent in the last step of an odd tap count): one k16
      // MFMA per tap and channel tile
      const bool two = 2 * s + 1 < TP::T;
      const unsigned char* wb = sB + stage * SB + abase;
      stage = stage + 1 == NST ? 0 : stage + 1;
      const u4 p0 = *(lu4p)(pbuf + P::template tap_off<PH>(2 * s));
      u4 w0[NT], w1[NT], p1;
#pragma unroll
      for (int i = 0; i < NT; ++i) w0[i] = *(lu4p)(wb + i * 512);
      if (two) {
        p1 = *(lu4p)(pbuf + P::template tap_off<PH>(2 * s + 1));
#pragma unroll
        for (int i = 0; i < NT; ++i) w1[i] = *(lu4p)(wb + 2 * NB * 16 + i * 512);
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) acc[i] = mfma32(w0[i], p0, acc[i]);
      if (two) {
#pragma unroll
        for (int i = 0; i < NT; ++i) acc[i] = mfma32(w1[i], p1, acc[i]);
      }
    }
  }
  vm_barrier();   // the trailing sink loads landed and every wave is done with the stages

  // ---- epilogue. acc[i][4m + j]: channel nb·NB + 32i + 8m + 4h + j of tile pixel tpix
  auto out_pixel = [&](int p) -> long {   // NHWC pixel index, or -1 outside the grid
    const int gy = ty * TH + (p >> 4), gx = tx * 16 + (p & 15);
    if (gy >= a.gh || gx >= a.gw) return -1;
    if (MODE == BM_CONV) return ((long)b * a.Hout + gy) * a.Wout + gx;
    return ((long)b * a.Hout + 2 * gy + (PH >> 1)) * a.Wout + 2 * gx + (PH & 1);
  };
  const long o = out_pixel(tpix);
  if constexpr (EPI == BE_GDN || EPI == BE_IGDN) {
    // GDN / IGDN (models/GDN.py:64-94): n[i][p] = Σ_j γ[i][j]·x²[j][p] with γ_eff in bf16 as
    // the A operand from LDS and x² (bias added, squared, rounded to bf16) as the B operand
    // straight from the accumulators, then y = x·rsqrt(β + n) | x·sqrt(β + n) in fp32.
    constexpr int KB = KB16;
    if constexpr (!KK::EARLY_G) stage_gamma();
    // x² as B fragments: k-block 2i + q holds channels 32i + 16q + 8h + 0..7 in lanes h. The
    // accumulator rows a lane holds are 4h + 0..3 and 8 + 4h + 0..3 of each 16-channel block;
    // one permlane32 swap per register pair hands lanes h the 8 consecutive channels.
    u4 xb[KB];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const f4 bv = *(const f4*)(sbb + 32 * i + 8 * m + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][4 * m + j] += bv[j];
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int r0 = 8 * q;
        float sq[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) sq[j] = acc[i][r0 + j] * acc[i][r0 + j];
        const unsigned lo0 = pack_bf2(sq[0], sq[1]), lo1 = pack_bf2(sq[2], sq[3]);
        const unsigned hi0 = pack_bf2(sq[4], sq[5]), hi1 = pack_bf2(sq[6], sq[7]);
        const auto s0 = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
        xb[2 * i + q] = u4{s0[0], s1[0], s0[1], s1[1]};
      }
    }
    if constexpr (!KK::EARLY_G) vm_barrier();   // γ of every wave landed
    const unsigned char* sg = smem + KK::GOFF + lane * 16;
    // DIRECT_Y: this wave's [32 px][64 ch] bf16 image, 128-byte rows, 16-byte piece pc of pixel
    // p at slot pc ^ (p & 7) (the 4×16-lane read groups cover the 64 banks; the 8-byte writes
    // are 2-way)
    unsigned char* const yb = smem + KK::YOFF + wave * 4096;
    auto yswz = [](int p, int pc) { return p * 128 + ((pc ^ (p & 7)) << 4); };
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      f16v n;
#pragma unroll
      for (int j = 0; j < 16; ++j) n[j] = 0.f;
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
        const u4 g = *(lu4p)(sg + (i * KB + kb) * 1024);
        n = mfma32(g, xb[kb], n);
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int ch = 32 * i + 8 * m + 4 * h;
        const f4 be = *(const f4*)(sbb + 256 + ch);
        f4 y;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float t = n[4 * m + j] + be[j];
          y[j] = acc[i][4 * m + j] * (EPI == BE_IGDN ? __builtin_amdgcn_sqrtf(t)
                                                     : __builtin_amdgcn_rsqf(t));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][4 * m + j] = y[j];
      }
      if constexpr (KK::DIRECT_Y) {
        if (i & 1) {   // tiles i − 1, i: channels 32(i − 1) .. 32i + 31, 8 pieces of 16 bytes
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
#pragma unroll
            for (int m = 0; m < 4; ++m) {
              const f16v& v = acc[i - 1 + tt];
              *(uint2*)(yb + yswz(r32, 4 * tt + m) + 8 * h) =
                  uint2{pack_bf2(v[4 * m], v[4 * m + 1]), pack_bf2(v[4 * m + 2], v[4 * m + 3])};
            }
          wave_lds_sync();   // the image's writes before any lane's reads (cross-lane exchange)
          // wave-local: LDS keeps one wave's accesses in order. Pixel px = (lane >> 3) + 8j of
          // the wave: tile row 2·wave + (j >> 1), column (lane >> 3) + 8·(j & 1); a uniform image
          // base and 32-bit offsets (recomputed here, not held through the loop)
          const int fl = fresh_tid() & 63;
          u16* const ob = a.out + (long)b * a.Hout * a.Wout * CO;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int px = (fl >> 3) + 8 * j, pc = fl & 7;
            const u4 v = *(lu4p)(yb + yswz(px, pc));
            const int gy = ty * TH + 2 * wave + (j >> 1), gx = tx * 16 + (fl >> 3) + 8 * (j & 1);
            const int oy = MODE == BM_CONV ? gy : 2 * gy + (PH >> 1);
            const int ox = MODE == BM_CONV ? gx : 2 * gx + (PH & 1);
            if (gy < a.gh && gx < a.gw) *(u4*)(ob + (oy * a.Wout + ox) * CO + 32 * (i - 1) + 8 * pc) = v;
          }
          wave_lds_sync();   // every lane's reads before the next tile pair's writes (WAR)
        }
      }
    }
    if constexpr (!KK::DIRECT_Y) {
    // y through an LDS tile [pixel][channel] (row stride OS) to whole-row 16-byte stores
    __syncthreads();   // every wave's γ reads done: the tile reuses the γ blocks
    constexpr int OS = KK::OS;
    unsigned char* const row = smem + tpix * OS + 8 * h;
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        *(uint2*)(row + (32 * i + 8 * m) * 2) =
            uint2{pack_bf2(acc[i][4 * m], acc[i][4 * m + 1]), pack_bf2(acc[i][4 * m + 2], acc[i][4 * m + 3])};
    __syncthreads();
    constexpr int PCS = CO * 2 / 16;   // 16-byte pieces per pixel row
    for (int idx = tid; idx < KK::R * PCS; idx += KK::NT_) {
      const int p = idx / PCS, pc = idx - p * PCS;
      const long op = out_pixel(p);
      if (op >= 0) *(u4*)(a.out + op * CO + pc * 8) = *(lu4p)(smem + p * OS + pc * 16);
    }
    }
  } else {
    static_assert(EPI == BE_QUANT, "epilogue");
    // conv3 + model.py:56 round (half to even) + model.py:71-73 rate: rows 8m .. 8m + 7 of every
    // accumulator tile (registers 4m .. 4m + 3 of the lane's half h)
    float bits = 0.f;
    // the rate table rows of this tile's NB channels: staged in LDS after the K-split exchange
    // area (KS == 2, the rate table rows) or read from L2
    constexpr bool RT_LDS = KK::KS == 2;
    constexpr int XS_BYTES = (KK::KS * NW * NT * 8 * 64 * 4 + 1023) / 1024 * 1024;
    constexpr int RTU = NB * RT_W / 4, RTP = (RTU + 63) / 64;   // 16-byte units, 1 KB pieces
    static_assert(!RT_LDS || (NB * RT_W % 4 == 0 && XS_BYTES + RTP * 1024 <= KK::KS * KK::MAIN_LDS),
                  "rate table stage");
    const float* const stab = (const float*)(smem + XS_BYTES);
    auto rtab_at = [&](int cl, int v, int c) -> float {
      if constexpr (RT_LDS) return stab[cl * RT_W + v + RT_K];
      else return a.rtab[c * RT_W + v + RT_K];
    };
    // ŷ through an LDS tile [R px][NB ch] (row stride NB + 4 floats: a 16-lane b128 write group
    // covers 64 distinct banks), then stored by every wave as 16-byte chunks of contiguous
    // pixel rows: the accumulator layout would store 32 pixels × 32 bytes per wave-instruction
    constexpr bool QST = RT_LDS;
    constexpr int QS = NB + 4, QOFF = XS_BYTES + RTP * 1024;
    static_assert(!QST || QOFF + KK::R * QS * 4 <= KK::KS * KK::MAIN_LDS, "ŷ tile");
    float* const sq = (float*)(smem + QOFF);
    // Every element's table entry is read unconditionally (index clamped), and the elements
    // outside the table (|ŷ| > RT_K, or NaN) are recomputed in ONE rarely-taken block after them:
    // a per-element `lookup ? table : element_bits` put 2 KB of inlined element_bits between
    // consecutive lookups, and every skip over it missed the instruction cache (≈ 10k cycles of
    // the epilogue). The bits are then added in the same element order as before.
    auto quant_rows = [&](int m) {
      if (o < 0) return;
      f4 qv[NT], bv[NT];
      bool slow = false;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int ch = nb * NB + 32 * i + 8 * m + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float q = rintf(acc[i][4 * m + j]);
          qv[i][j] = q;
          const float qc = fminf(fmaxf(q, -(float)RT_K), (float)RT_K);
          bv[i][j] = rtab_at(ch - nb * NB + j, (int)qc, ch + j);
          slow |= !(fabsf(q) <= (float)RT_K);
        }
      }
      if (slow) {
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (!(fabsf(qv[i][j]) <= (float)RT_K))
              bv[i][j] = element_bits(qv[i][j], a.rate, CO, nb * NB + 32 * i + 8 * m + 4 * h + j);
      }
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int ch = nb * NB + 32 * i + 8 * m + 4 * h;
        const f4 y = f4{acc[i][4 * m], acc[i][4 * m + 1], acc[i][4 * m + 2], acc[i][4 * m + 3]};
        const f4 q = qv[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) bits += bv[i][j];
        if (a.y_f32) *(f4*)(a.y_f32 + o * CO + ch) = y;
        if constexpr (QST) {
          *(f4*)(sq + tpix * QS + (ch - nb * NB)) = q;
        } else {
          *(f4*)(a.out_f32 + o * CO + ch) = q;
          *(uint2*)(a.out + o * CO + ch) = uint2{pack_bf2(q[0], q[1]), pack_bf2(q[2], q[3])};
        }
      }
    };
    auto store_tile = [&]() {   // QST: after the barrier that publishes sq
      constexpr int NCK = NB / 4, TOT = KK::R * NCK, NTH = KK::KS * KK::NT_;
      static_assert(TOT % NTH == 0, "ŷ store split");
#pragma unroll
      for (int it = 0; it < TOT / NTH; ++it) {
        const int idx = it * NTH + tid, p = idx / NCK, k = idx - p * NCK;
        const long op = out_pixel(p);
        if (op < 0) continue;
        const f4 q = *(const f4*)(sq + p * QS + 4 * k);
        const long e = op * CO + nb * NB + 4 * k;
        *(f4*)(a.out_f32 + e) = q;
        *(uint2*)(a.out + e) = uint2{pack_bf2(q[0], q[1]), pack_bf2(q[2], q[3])};
      }
    };
    int nred = NW;   // bit partials to add, one per finishing wave
    if constexpr (KK::KS == 2) {
      // K-split halves exchange HALF their accumulators through LDS (the main-loop buffers are
      // free after the trailing vm_barrier): group g finalises rows m ∈ {2g, 2g + 1} of every
      // tile with the other group's partial of those rows (x0 + x1, exact either way round), so
      // both groups run the quantiser on half the elements
      float* xs = (float*)smem;   // [group][wave][tile][8][lane]
      auto put = [&](int r0) {
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) xs[(((kg * NW + wave) * NT + i) * 8 + j) * 64 + lane] = acc[i][r0 + j];
      };
      auto add = [&](int r0) {
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][r0 + j] += xs[((((1 - kg) * NW + wave) * NT + i) * 8 + j) * 64 + lane];
      };
      if (kg == 0) put(8); else put(0);   // the rows the other group finalises
      __syncthreads();
      if constexpr (RT_LDS) {   // no DMA in flight at the barrier above; landed by the one below
        for (int pc = wv; pc < RTP; pc += KK::KS * NW) {
          const int u = pc * 64 + lane;
          glds16(u < RTU ? (const void*)(a.rtab + (long)nb * NB * RT_W + u * 4) : (const void*)g_zero16,
                 smem + XS_BYTES + pc * 1024);
        }
      }
      if (kg == 0) add(0); else add(8);
      if constexpr (RT_LDS) vm_barrier();   // table landed; exchange reads done before red[] reuse
      else __syncthreads();                 // exchange reads done before red[] reuses the area
      if (kg == 0) {
        quant_rows(0);
        quant_rows(1);
      } else {
        quant_rows(2);
        quant_rows(3);
      }
      if constexpr (QST) {
        __syncthreads();   // ŷ tile complete
        store_tile();
      }
      nred = 2 * NW;
    } else {
      static_assert(KK::KS == 1, "K split");
#pragma unroll
      for (int m = 0; m < 4; ++m) quant_rows(m);
    }
    bits = wave_sum(bits);
    float* red = (float*)smem;
    if (lane == 0) red[kg * NW + wave] = bits;
    __syncthreads();
    if (tid == 0) {
      double sum = 0.0;
      for (int w = 0; w < nred; ++w) sum += (double)red[w];
      const int tile = ty * a.tiles_x + tx;
      a.partial[(long)b * a.ppi + tile * (CO / NB) + nb] = sum;
    }
  }
}

template <int MODE, int TH, int NB, int CO, int CI, int EPI>
__global__ void __launch_bounds__(k5_threads(TH, EPI), (TH == 8 && EPI != BE_QUANT) ? 2 : 1)   // 8-row deconv tiles: two per CU
k5_bf16_kernel(const K5Args a) {
  using KK = K5<MODE, TH, NB, CO, CI, EPI>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[KK::LDS];
  int bid = blockIdx.x;
  const int per_ph = a.tiles_x * a.tiles_y * a.B;
  const int q = MODE == BM_DECONV ? bid / per_ph : 0;   // phases dispatched phase-major
  bid -= q * per_ph;
  const int ph = q;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int b = bid / a.tiles_y;
  const int nb = blockIdx.y;
  if constexpr (MODE == BM_CONV) {
    k5_body<MODE, TH, NB, CO, CI, EPI, 0>(a, smem, b, ty, tx, nb);
  } else {
    switch (ph) {   // wave-uniform: the tap lists are compile-time per phase
      case 0: k5_body<MODE, TH, NB, CO, CI, EPI, 0>(a, smem, b, ty, tx, nb); break;
      case 1: k5_body<MODE, TH, NB, CO, CI, EPI, 1>(a, smem, b, ty, tx, nb); break;
      case 2: k5_body<MODE, TH, NB, CO, CI, EPI, 2>(a, smem, b, ty, tx, nb); break;
      default: k5_body<MODE, TH, NB, CO, CI, EPI, 3>(a, smem, b, ty, tx, nb); break;
    }
  }
}

// ------------------------------------------------------------------------------ conv1
// analysis_17.py:14-17 conv1 (3→N, k9 s4 p4) + GDN1 in bf16 on 8×8 output blocks. The 37×37×3
// input patch is rounded once into one bf16 plane [3·37][40]. K = 243 is reordered
// (ICLR17_W_CONV1_X6 packing): k-group g = 4s + (lane >> 4) is 8 consecutive patch columns of
// one (channel, kernel row) pair for g < 27, zero for g = 27, and for g = 28..31 the kw = 8
// column of 8 pairs gathered element-wise; weight fragments [32][N][8] bf16.
constexpr int C1P = 37;                       // patch side: 8·4 + 9 − 4
constexpr int C1RS = 40;                      // row stride (elements): 10 16-byte fp32 pieces
constexpr int C1PIECES = 3 * C1P * 10;        // fp32 16-byte pieces of the patch (1110)
constexpr int C1U = 3 * C1P * C1RS;           // u16 elements of the bf16 plane (4440)

// ---------------------------------------------------------------- conv1, persistent form
// One 8×8 block: 64 pixels × CO channels on 8 waves, v_mfma_f32_16x16x32_bf16 (A = weights,
// B = pixels), the GDN contraction n = γ·x² on the same MFMA through an x² tile in LDS. Round 3
// made it persistent (bit-identical to the round-2 one-block-per-workgroup kernel, 0.091 →
// 0.080 ms at B=64) so that nothing per block waits on L2 or HBM. One 8-wave workgroup per CU walks the 8×8 output blocks t = blockIdx.x,
// + gridDim.x, …:
//   * each wave holds its weight slice in registers for the whole kernel (wave w: channels
//     (w & 3)·CO/4 .. +CO/4 of pixel half w >> 2; 8 steps × CO/64 fragments, 96 VGPRs at N = 192)
//     and γ_eff (bf16, 72 KB) sits in LDS, both loaded once: no per-block weight or γ refetch
//     from L2 (165 KB per 64-pixel block in the one-block-per-workgroup form);
//   * the next block's 37×37×3 fp32 patch is loaded into registers while this block computes,
//     and rounded into the idle bf16 plane after this block's epilogue (double-buffered plane);
//   * the output rows leave as 16-byte stores that drain during the next block.
// analysis_17.py:14-17 (conv1) + models/GDN.py:64-94 (GDN1).
constexpr int C1P_WAVES = 8;
constexpr int C1P_LOADS = (C1PIECES + C1P_WAVES * 64 - 1) / (C1P_WAVES * 64);   // 3 per thread

template <int CO>
struct C1PL {
  static constexpr int G = CO * CO * 2;                   // γ_eff bf16 [CO/8][CO][8]
  static constexpr int PL = C1U * 2;                      // one bf16 plane
  static constexpr int SQ = epi_tile_bytes<CO>(64);       // x² / output tile
  static constexpr int BB = CO * 8;                       // bias, β_eff (fp32)
  static constexpr int LDS = G + 2 * PL + SQ + BB;
  static_assert(G % 1024 == 0 && LDS <= 160 * 1024, "conv1p LDS");
};


template <int CO, bool FULL>   // FULL: the output grid is whole 8×8 blocks (no store guard)
__global__ void __launch_bounds__(C1P_WAVES * 64, 1)
conv1p_bf16_kernel(const float* __restrict__ x, int H, int W, const u16* __restrict__ wbf,
                   const float* __restrict__ bias, const float* __restrict__ beta,
                   const u16* __restrict__ gamma, u16* __restrict__ out, int tiles_x, int tiles_y,
                   int ntiles) {
  constexpr int MT = 2, NT = CO / 4 / 16, KB = CO / 32, NTHR = C1P_WAVES * 64;
  using L = C1PL<CO>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[L::LDS];
  typedef const __attribute__((address_space(3))) u4* lu4p;
  unsigned char* const sg = smem;                          // γ
  u16* const sp0 = (u16*)(smem + L::G);                    // planes 0, 1
  unsigned char* const sq = smem + L::G + 2 * L::PL;       // x² / output tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wave & 3, half = wave >> 2;
  const int ncol = cg * (CO / 4), kg = lane >> 4;
  // bias and β_eff in LDS: a global load of them inside the block loop would be younger than the
  // next block's patch loads, and its use would wait (in-order vmcnt) for those HBM reads
  float* const sbias = (float*)(sq + L::SQ);
  float* const sbeta = sbias + CO;
  if (tid < CO) {
    sbias[tid] = bias[tid];
    sbeta[tid] = beta[tid];
  }

  // γ into LDS (1 KB per wave-instruction), retired by the first vm_barrier
  for (int blk = wave; blk < L::G / 1024; blk += C1P_WAVES) glds16(gamma + blk * 512 + lane * 8, sg + blk * 1024);
  // this wave's weight fragments: step s, channel tile nt (k-group 4s + kg, channel ncol + nt·16 + lane & 15)
  u4 wr[8][NT];
  {
    const u16* gb = wbf + (kg * CO + ncol + (lane & 15)) * 8;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) wr[s][nt] = *(const u4*)(gb + (long)s * 4 * CO * 8 + nt * 128);
  }
  // patch pieces of block t into registers: piece (c, r, q) = columns 4q .. 4q+3 of patch row r
  // of channel c; the patch origin ≡ 0 (mod 4) and W ≡ 0 (mod 16): a piece is wholly in or out
  f4 pr[C1P_LOADS];
  int okm = 0;   // bit j: piece j is inside the image
  // (uniform image base + 32-bit lane offsets: no 64-bit per-lane addresses to hold or spill)
  // per-lane piece geometry, computed once: offset within the image and (row, column) in the patch
  int poff[C1P_LOADS], prc[C1P_LOADS];
#pragma unroll
  for (int j = 0; j < C1P_LOADS; ++j) {
    const int pc = tid + j * NTHR;
    const int cr = pc / 10, q = pc - cr * 10;
    const int c = cr / C1P, r = cr - c * C1P;
    poff[j] = (c * H + r) * W + 4 * q;
    prc[j] = pc < C1PIECES ? r | (4 * q) << 8 : -1;
  }
  auto load_patch = [&](int t) {
    const int tx = t % tiles_x, ty = (t / tiles_x) % tiles_y, b = t / (tiles_x * tiles_y);
    const int iy0 = ty * 32 - 4, ix0 = tx * 32 - 4;
    const float* __restrict__ xb = x + (long)b * 3 * H * W;
    const int o0 = iy0 * W + ix0;
#pragma unroll
    for (int j = 0; j < C1P_LOADS; ++j) {
      const bool ok = prc[j] >= 0 && (unsigned)(iy0 + (prc[j] & 255)) < (unsigned)H &&
                      (unsigned)(ix0 + (prc[j] >> 8)) < (unsigned)W;
      // no branch, and no use of the value before store_plane (a select here made the compiler
      // wait for the load in the middle of this block's main loop)
      pr[j] = *(const f4*)(xb + (ok ? poff[j] + o0 : 0));
      okm = j == 0 ? (int)ok : okm | ((int)ok << j);
    }
  };
  auto store_plane = [&](u16* sp) {   // round once into the bf16 plane
    const int ft = fresh_tid();
#pragma unroll
    for (int j = 0; j < C1P_LOADS; ++j) {
      const int pc = ft + j * NTHR;
      const f4 v = (okm >> j) & 1 ? pr[j] : f4{0.f, 0.f, 0.f, 0.f};
      if (pc < C1PIECES) *(uint2*)(sp + pc * 4) = uint2{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
    }
  };
  int t = blockIdx.x;
  load_patch(t);
  store_plane(sp0);
  vm_barrier();   // γ landed, plane 0 written

  int pix[MT];   // output pixel (my, mx) → patch row 4·my, column 4·mx
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = (MT * half + mt) * 16 + (lane & 15);
    pix[mt] = (m >> 3) * 4 * C1RS + (m & 7) * 4;
  }
  auto pair_off = [](int p) { return ((p / 9) * C1P + p % 9) * C1RS; };
  const int ho = H / 4, wo = W / 4;
  // Per block: main loop (MFMA, A = the weights in registers, B = the bf16 plane), GDN
  // epilogue (each pixel half on its 4 waves: x² rows, contraction with γ from LDS, output rows),
  // next plane, output stores by all waves.
  f4 acc[NT][MT];
  auto main_tile = [&](const u16* sp) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[nt][mt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      const int g = 4 * s + kg;
      const int po = pair_off(g < 27 ? g : 26);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const u16* e = sp + po + pix[mt];
        const uint2 lo2 = *(const uint2*)e, hi2 = *(const uint2*)(e + 4);
        const u4 px = u4{lo2.x, lo2.y, hi2.x, hi2.y};
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[nt][mt] = mfma_bf16(wr[s][nt], px, acc[nt][mt]);
      }
      __builtin_amdgcn_sched_barrier(0);   // one step's fragments live at a time (register budget)
    }
    int po8[8];   // kw = 8 column: pair offsets of k-group 28 + kg
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int p = 8 * kg + e;
      po8[e] = pair_off(p < 27 ? p : 26) + 8;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      u4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned lo = sp[po8[2 * i] + pix[mt]], hi = sp[po8[2 * i + 1] + pix[mt]];
        v[i] = lo | (hi << 16);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt][mt] = mfma_bf16(wr[7][nt], v, acc[nt][mt]);
    }
  };
  // GDN epilogue of this half's 32 pixels (bias, x² rows in bf16, n = γ·x² with γ from LDS,
  // x·rsqrt(β + n)); this half's rows of the x² / output tile
  const int pix0 = MT * 16 * half;
  auto epi_tile = [&]() {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int ch = ncol + nt * 16 + 4 * kg;
      const f4 bv = *(const f4*)(sbias + ch);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[nt][mt] += bv;
        const f4 v = acc[nt][mt];
        const int p = pix0 + mt * 16 + (lane & 15);
        *(uint2*)(sq + epi_off<CO>(p, ch)) = uint2{pack_bf2(v[0] * v[0], v[1] * v[1]),
                                                   pack_bf2(v[2] * v[2], v[3] * v[3])};
      }
    }
    __syncthreads();   // x² rows of this half complete
    const int pl = pix0 + (lane & 15);
    const unsigned char* ga = sg + ((kg * CO + ncol + (lane & 15)) * 8) * 2;
    // k-block outer: each x² fragment is read once for all NT channel tiles (not once per
    // tile); the same per-accumulator k order, so the same bits
    f4 nacc[NT][MT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) nacc[nt][mt] = f4{0.f, 0.f, 0.f, 0.f};
    u4 xs[2][MT], gc[2][NT];
    auto rd = [&](int kb, int q) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) xs[q][mt] = *(lu4p)(sq + epi_off<CO>(pl + mt * 16, 32 * kb + 8 * kg));
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) gc[q][nt] = *(lu4p)(ga + (kb * 4 * CO * 8 + nt * 128) * 2);
    };
    rd(0, 0);
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      if (kb + 1 < KB) rd(kb + 1, (kb + 1) & 1);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) nacc[nt][mt] = mfma_bf16(gc[kb & 1][nt], xs[kb & 1][mt], nacc[nt][mt]);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int ch = ncol + nt * 16 + 4 * kg;
      const f4 be = *(const f4*)(sbeta + ch);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[nt][mt][j] *= __builtin_amdgcn_rsqf(nacc[nt][mt][j] + be[j]);
    }
    __syncthreads();   // x² reads done: the rows are rewritten with the output
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int ch = ncol + nt * 16 + 4 * kg;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f4 y = acc[nt][mt];
        const int p = pix0 + mt * 16 + (lane & 15);
        *(uint2*)(sq + epi_off<CO>(p, ch)) = uint2{pack_bf2(y[0], y[1]), pack_bf2(y[2], y[3])};
      }
    }
    __syncthreads();   // output rows complete (stored by copy_out after the segment barrier)
  };
  // the block's output rows by all 512 threads, 16 bytes per piece, the same count on every
  // wave: the stores sit on the common path, so the vmcnt waits of the next plane count them
  // exactly and never wait for them
  auto copy_out = [&](int t) {
    const int tx = t % tiles_x, ty = (t / tiles_x) % tiles_y, b = t / (tiles_x * tiles_y);
    u16* __restrict__ ob = out + (long)b * ho * wo * CO;
    constexpr int Q = CO / 8;                 // 16-byte pieces per pixel row
    static_assert((64 * Q) % NTHR == 0, "copy_out pieces");
    const int ft = fresh_tid();
#pragma unroll
    for (int j = 0; j < 64 * Q / NTHR; ++j) {
      const int i = ft + j * NTHR;
      const int p = i / Q, c8 = i % Q;
      const int oy = ty * 8 + (p >> 3), ox = tx * 8 + (p & 7);
      const u4 v = *(lu4p)(sq + epi_off<CO>(p, c8 * 8));
      if (FULL || (oy < ho && ox < wo)) *(u4*)(ob + (oy * wo + ox) * CO + c8 * 8) = v;
    }
  };
  const int G = gridDim.x;
  {
    int k = 0;
    for (int t = blockIdx.x; t < ntiles; t += G, ++k) {
      const int tn = t + G;
      // the next block's patch, in flight during this block (past the last block: a repeat of
      // this one), rounded into the idle plane after the epilogue
      load_patch(tn < ntiles ? tn : t);
      main_tile(sp0 + (k & 1) * C1U);
      epi_tile();
      store_plane(sp0 + ((k + 1) & 1) * C1U);
      copy_out(t);
      __syncthreads();   // next plane written, output rows read
    }
    return;
  }
}

// ------------------------------------------------------------------------------ packing
// conv (ICLR17_BF_CONV5), W[co][ci][5][5] → [CI/16][S=13][4][CO][8]: k-group kg of step s is tap
// 2s + (kg >> 1), channels 16c + 8·(kg & 1) + e; tap 25 (the pad) is zero.
// deconv (ICLR17_BF_DECONV5), W[ci][co][5][5] → the four phases back to back, phase p:
// [CI/16][S_p][4][CO][8] with the phase's taps in Taps<BM_DECONV, p> order.
__global__ void __launch_bounds__(256) pack_k5_bf16_kernel(const float* __restrict__ w, int N,
                                                           int deconv, u16* __restrict__ out,
                                                           long total) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int e = (int)(i & 7);
    long r = i >> 3;
    const int co = (int)(r % N);
    r /= N;
    const int kg = (int)(r & 3);
    r >>= 2;
    const int nch = N / 16;
    int ph = 0, ny = 5, nx = 5, S = 13;
    if (deconv) {   // phase blocks of nch·S_p·4·N·8
      for (ph = 0; ph < 4; ++ph) {
        ny = (ph >> 1) == 0 ? 3 : 2;
        nx = (ph & 1) == 0 ? 3 : 2;
        S = (ny * nx + 1) / 2;
        if (r < (long)nch * S) break;
        r -= (long)nch * S;
      }
    }
    const int c = (int)(r / S), s = (int)(r % S);
    const int t = 2 * s + (kg >> 1);
    const int ci = 16 * c + 8 * (kg & 1) + e;
    float v = 0.f;
    if (t < ny * nx) {
      int ky, kx;
      if (!deconv) {
        ky = t / 5;
        kx = t % 5;
      } else {
        ky = (ph >> 1) == 0 ? 2 * (t / nx) : 2 * (t / nx) + 1;
        kx = (ph & 1) == 0 ? 2 * (t % nx) : 2 * (t % nx) + 1;
      }
      v = deconv ? w[(((long)ci * N + co) * 5 + ky) * 5 + kx] : w[(((long)co * N + ci) * 5 + ky) * 5 + kx];
    }
    out[i] = __builtin_bit_cast(u16, (__bf16)v);
  }
}

// packed fp32 operand [taps][K/4][N][4] → bf16 (round to nearest even) [taps][K/8][N][8]:
// the 16x16x32 fragment layout (conv1's reordered weights, the GDN γ)
__global__ void __launch_bounds__(256) round_packed_kernel(const float* __restrict__ w, int K, int N,
                                                           long groups, u16* __restrict__ out) {
  for (long g = (long)blockIdx.x * 256 + threadIdx.x; g < groups; g += (long)gridDim.x * 256) {
    const long tk = g / N;
    const int col = (int)(g - tk * N);
    const long tap = tk / (K / 8);
    const int k8 = (int)(tk - tap * (K / 8));
    const float* src = w + ((tap * (K / 4) + 2 * k8) * N + col) * 4;
    const f4 lo = *(const f4*)src, hi = *(const f4*)(src + (long)N * 4);
    *(u4*)(out + g * 8) = u4{pack_bf2(lo[0], lo[1]), pack_bf2(lo[2], lo[3]), pack_bf2(hi[0], hi[1]),
                             pack_bf2(hi[2], hi[3])};
  }
}

// fp32 → bf16 (round to nearest even), 8 per thread
__global__ void __launch_bounds__(256) to_bf16_kernel(const float* __restrict__ x, long n8,
                                                      u16* __restrict__ out) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const f4 a = *(const f4*)(x + 8 * i), b = *(const f4*)(x + 8 * i + 4);
    *(u4*)(out + 8 * i) = u4{pack_bf2(a[0], a[1]), pack_bf2(a[2], a[3]), pack_bf2(b[0], b[1]),
                             pack_bf2(b[2], b[3])};
  }
}

// ------------------------------------------------------------------------------ launchers
// compute units of the current device (persistent grids), cached per device
static int cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

template <int N>
int launch_conv2(const K5Args& a0, hipStream_t st) {
  K5Args a = a0;
  a.tiles_y = (a.gh + 15) / 16;
  a.tiles_x = (a.gw + 15) / 16;
  hipLaunchKernelGGL((k5_bf16_kernel<BM_CONV, 16, N, N, N, BE_GDN>),
                     dim3(a.tiles_x * a.tiles_y * a.B, 1), dim3(512), 0, st, a);
  return check_launch("conv2_gdn_bf16");
}

template <int N>
int launch_conv3(const K5Args& a0, hipStream_t st) {
  K5Args a = a0;
  a.tiles_y = (a.gh + 7) / 8;
  a.tiles_x = (a.gw + 15) / 16;
  constexpr int NB = N / 2;
  a.ppi = a.tiles_x * a.tiles_y * 2;
  hipLaunchKernelGGL((k5_bf16_kernel<BM_CONV, 8, NB, N, N, BE_QUANT>),
                     dim3(a.tiles_x * a.tiles_y * a.B, 2), dim3(k5_threads(8, BE_QUANT)), 0, st, a);
  return check_launch("conv3_quant_rate_bf16");
}

template <int N, int TH>
int launch_deconv(const K5Args& a0, hipStream_t st) {
  K5Args a = a0;
  a.tiles_y = (a.gh + TH - 1) / TH;
  a.tiles_x = (a.gw + 15) / 16;
  const int tiles = a.tiles_x * a.tiles_y * a.B * 4;
  hipLaunchKernelGGL((k5_bf16_kernel<BM_DECONV, TH, N, N, N, BE_IGDN>),
                     dim3(tiles, 1), dim3(TH / 2 * 64), 0, st, a);
  return check_launch("deconv_igdn_bf16");
}

}  // namespace bfm
}  // namespace iclr17

using namespace iclr17;
using namespace iclr17::bfm;

extern "C" {



size_t iclr17_bf16_weight_size(int which, int N) {
  if (N != 128 && N != 192) return 0;
  switch (which) {
    case ICLR17_BF_CONV5: return (size_t)(N / 16) * 13 * 4 * N * 8;
    case ICLR17_BF_DECONV5: return (size_t)(N / 16) * (5 + 3 + 3 + 2) * 4 * N * 8;
    default: return 0;
  }
}

int iclr17_pack_bf16(int which, const float* w, uint16_t* out, int N, void* stream) {
  const size_t total = iclr17_bf16_weight_size(which, N);
  ICLR17_REQUIRE(total > 0, ICLR17_EUNSUPPORTED, "pack_bf16: kind %d, N=%d unsupported", which, N);
  ICLR17_REQUIRE(w && out, ICLR17_EINVAL, "pack_bf16: null pointer");
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  hipLaunchKernelGGL(pack_k5_bf16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, N,
                     which == ICLR17_BF_DECONV5 ? 1 : 0, out, (long)total);
  return check_launch("pack_bf16");
}

int iclr17_round_packed(const float* packed, int taps, int K, int N, uint16_t* out, void* stream) {
  ICLR17_REQUIRE(packed && out && taps > 0 && K % 8 == 0 && N > 0, ICLR17_EINVAL,
                 "round_packed: bad arguments");
  const long groups = (long)taps * (K / 8) * N;
  const int blocks = (int)((groups + 255) / 256 < 4096 ? (groups + 255) / 256 : 4096);
  hipLaunchKernelGGL(round_packed_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, packed,
                     K, N, groups, out);
  return check_launch("round_packed");
}

int iclr17_to_bf16(const float* x, long n, uint16_t* out, void* stream) {
  ICLR17_REQUIRE(x && out && n >= 0 && n % 8 == 0, ICLR17_EINVAL,
                 "to_bf16: null pointer or n (%ld) not a multiple of 8", n);
  if (n == 0) return ICLR17_OK;
  const long n8 = n / 8;
  const int blocks = (int)((n8 + 255) / 256 < 8192 ? (n8 + 255) / 256 : 8192);
  hipLaunchKernelGGL(to_bf16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, n8, out);
  return check_launch("to_bf16");
}

int iclr17_analysis_conv1_gdn_bf16(const float* x, int B, int H, int W, int N,
                                   const uint16_t* w_bf16, const float* bias,
                                   const float* beta_eff, const uint16_t* gamma_bf16,
                                   uint16_t* out, void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "conv1_gdn_bf16: N=%d", N);
  ICLR17_REQUIRE(x && w_bf16 && bias && beta_eff && gamma_bf16 && out && B > 0 && H > 0 && W > 0 &&
                     H % 16 == 0 && W % 16 == 0,
                 ICLR17_EINVAL, "conv1_gdn_bf16: bad arguments (H, W multiples of 16)");
  const int tiles_y = (H / 4 + 7) / 8, tiles_x = (W / 4 + 7) / 8;
  hipStream_t st = (hipStream_t)stream;
  // persistent: one 8-wave workgroup per CU (LDS-bound), walking the blocks
  const int ntiles = tiles_x * tiles_y * B, ncu = cu_count();
  const dim3 pgrid(ntiles < ncu ? ntiles : ncu);
  const bool full = (H / 4) % 8 == 0 && (W / 4) % 8 == 0;
  auto kern = N == 192 ? (full ? conv1p_bf16_kernel<192, true> : conv1p_bf16_kernel<192, false>)
                       : (full ? conv1p_bf16_kernel<128, true> : conv1p_bf16_kernel<128, false>);
  hipLaunchKernelGGL(kern, pgrid, dim3(C1P_WAVES * 64), 0, st, x, H, W, w_bf16, bias, beta_eff,
                     gamma_bf16, out, tiles_x, tiles_y, ntiles);
  return check_launch("conv1_gdn_bf16");
}

int iclr17_analysis_conv2_gdn_bf16(const uint16_t* in, int B, int H, int W, int N,
                                   const uint16_t* w_bf16, const float* bias, const float* beta_eff,
                                   const uint16_t* gamma_bf16, uint16_t* out, void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "conv2_gdn_bf16: N=%d", N);
  ICLR17_REQUIRE(in && w_bf16 && bias && beta_eff && gamma_bf16 && out && B > 0 && H % 16 == 0 &&
                     W % 16 == 0 && H > 0 && W > 0,
                 ICLR17_EINVAL, "conv2_gdn_bf16: bad arguments (H, W multiples of 16)");
  K5Args a;
  memset(&a, 0, sizeof(a));
  a.in = in; a.w = w_bf16; a.bias = bias; a.beta = beta_eff; a.gamma = gamma_bf16; a.out = out;
  a.B = B; a.Hin = H / 4; a.Win = W / 4; a.Hout = H / 8; a.Wout = W / 8;
  a.gh = a.Hout; a.gw = a.Wout;
  hipStream_t st = (hipStream_t)stream;
  return N == 192 ? launch_conv2<192>(a, st) : launch_conv2<128>(a, st);
}

int iclr17_bf16_rate_partials_per_image(int H, int W, int N) {
  (void)N;
  return ((H / 16 + 7) / 8) * ((W / 16 + 15) / 16) * 2;
}

size_t iclr17_rate_table_size(int N) { return (size_t)N * RT_W; }

int iclr17_rate_table(const float* rate_packed, int N, float* table, void* stream) {
  ICLR17_REQUIRE(rate_packed && table && N > 0, ICLR17_EINVAL, "rate_table: bad arguments");
  hipLaunchKernelGGL(rate_table_kernel, dim3((N * RT_W + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, rate_packed, N, table);
  return check_launch("rate_table");
}

int iclr17_analysis_conv3_quant_rate_bf16(const uint16_t* in, int B, int H, int W, int N,
                                          const uint16_t* w_bf16, const float* rate_packed,
                                          const float* rate_table, float* y_out, float* y_hat,
                                          uint16_t* y_hat_bf16, double* bits_partial,
                                          void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "conv3_quant_rate_bf16: N=%d", N);
  ICLR17_REQUIRE(in && w_bf16 && rate_packed && rate_table && y_hat && y_hat_bf16 && bits_partial && B > 0 &&
                     H % 16 == 0 && W % 16 == 0 && H > 0 && W > 0,
                 ICLR17_EINVAL, "conv3_quant_rate_bf16: bad arguments");
  K5Args a;
  memset(&a, 0, sizeof(a));
  a.in = in; a.w = w_bf16; a.rate = rate_packed; a.rtab = rate_table; a.y_f32 = y_out; a.out_f32 = y_hat;
  a.out = y_hat_bf16; a.partial = bits_partial;
  a.B = B; a.Hin = H / 8; a.Win = W / 8; a.Hout = H / 16; a.Wout = W / 16;
  a.gh = a.Hout; a.gw = a.Wout;
  hipStream_t st = (hipStream_t)stream;
  return N == 192 ? launch_conv3<192>(a, st) : launch_conv3<128>(a, st);
}

int iclr17_synthesis_deconv_igdn_bf16(const uint16_t* in, int B, int h, int w, int N,
                                      const uint16_t* w_bf16, const float* bias,
                                      const float* beta_eff, const uint16_t* gamma_bf16,
                                      uint16_t* out, void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "deconv_igdn_bf16: N=%d", N);
  ICLR17_REQUIRE(in && w_bf16 && bias && beta_eff && gamma_bf16 && out && B > 0 && h > 0 && w > 0,
                 ICLR17_EINVAL, "deconv_igdn_bf16: bad arguments");
  K5Args a;
  memset(&a, 0, sizeof(a));
  a.in = in; a.w = w_bf16; a.bias = bias; a.beta = beta_eff; a.gamma = gamma_bf16; a.out = out;
  a.B = B; a.Hin = h; a.Win = w; a.Hout = 2 * h; a.Wout = 2 * w;
  a.gh = h; a.gw = w;
  hipStream_t st = (hipStream_t)stream;
  // 16-row tiles where the grid stays ≥ 2 rounds of workgroups (deconv2), 8 rows otherwise
  const bool big = (long)((h + 15) / 16) * ((w + 15) / 16) * B * 4 >= 512;
  if (N == 192) return big ? launch_deconv<192, 16>(a, st) : launch_deconv<192, 8>(a, st);
  return big ? launch_deconv<128, 16>(a, st) : launch_deconv<128, 8>(a, st);
}

}  // extern "C"
