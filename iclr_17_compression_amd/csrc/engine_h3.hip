// The k5 layers in the h3 form (common.h): three fp16 part products per MAC on
// v_mfma_f32_32x32x16_f16, half the x6 mode's six bf16 ones, at the same fp32-level accuracy.
// synthesis_17.py:15-22 (deconv1/2 + IGDN), analysis_17.py:18-21 (conv2 + GDN),
// models/GDN.py:64-94.
//
// Form (the bf16 throughput engine's, engine_bf16.hip):
//   * a workgroup of TH/2 waves covers TH × 16 base pixels; wave w owns the 32 pixels of tile rows
//     2w, 2w+1 and every output channel (NT = CO/32 accumulators of 32×32), so the GDN / IGDN
//     channel contraction runs straight from the accumulators;
//   * the input arrives in the h3 form (two fp16 planes, written by the producing layer's
//     epilogue) and is staged per 16-channel chunk as ONE halo patch by LDS-DMA; every tap of the
//     chunk reads its fragment at a shifted offset;
//   * the weights arrive pre-split (iclr17_pack_h3k: hi and lo planes of w·σ_w in the A-fragment
//     layout), streamed through a 4-stage LDS ring with counted DMA waits; hi·2¹¹ is formed in
//     registers (4 packed fp16 multiplies per fragment) instead of being a third plane.
// One k16 step = one tap × the chunk's 16 channels: per 32-channel tile three MFMAs, small terms
// first: hi_w·lo_a, lo_w·hi_a, (hi_w·2¹¹)·hi_a, in place on the accumulator (the h3 chain's
// rounding error is 0.7× the x6 chain's: common.h).
//
// INT_IN (deconv1 on ŷ: integers, exact in the hi plane while |ŷ| < 2048): the lo plane is zero,
// only the hi plane is staged and the two products with hi_a run. INT_OK kernels check this per
// workgroup over the input window and fall back to the full body otherwise.
//
// Epilogue: x = acc·2⁻¹¹/(σ_a·σ_w) + bias (a power-of-two scale: exact), then the GDN / IGDN
// contraction n = Σ_j γ[i][j]·x_j² in the h3 form (γ split into two fp16 planes, staged in LDS
// half the output channels at a time; x² scaled per pixel by a power of two and split in
// registers), y = x·√(β + n) | x / √(β + n), and y stored
// as fp32 and/or in the h3 form (NHWC, or chunk-major [2][B][N/32][h][w][32]) and/or the x6
// split form.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <type_traits>

#include "common.h"
#include "k5_common.h"

namespace iclr17 {
namespace h3k {
using namespace bfm;

// One zero line for the padding loads and the zero pieces of the halo patches. (Measured: every
// wave reading its own 1 KB of a 64 KB zero table instead made conv2 0.345 → 0.46 ms and deconv2
// 0.415 → 0.45 ms — the one hot, coalesced line is effectively free.)
__device__ __attribute__((aligned(16))) unsigned g_zero16h[4] = {0u, 0u, 0u, 0u};
__device__ __forceinline__ const void* zero16(int) { return g_zero16h; }

// padding load of the counted-vmcnt DMA schedule (4 bytes per lane into the sink)
__device__ __forceinline__ void sink4(void* lds_sink) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g_zero16h,
                                   (__attribute__((address_space(3))) void*)lds_sink, 4, 0, 0);
}

__device__ __forceinline__ f16v mfma32h(const u4& a, const u4& b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8v, a),
                                                __builtin_bit_cast(h8v, b), c, 0, 0, 0);
}

// HE_QUANT: conv3 (analysis_17.py:22, no bias) + the quantiser and rate of model.py:48-56,71-73
// (the engine_fp32.hip EPI_QUANT epilogue's arithmetic), on an output-channel slice of COT channels
enum HEpi : int { HE_GDN = 0, HE_IGDN = 1, HE_QUANT = 2 };

struct HArgs {
  const u16* in;        // h3 input [2][B][Hin][Win][CI] (fp16 bits)
  const float* img;     // HM_CONV1: the fp32 NCHW image [B][3][Hin][Win]
  long in_plane;
  const u16* w;         // iclr17_pack_h3k weights, [2][…] (plane stride w_plane) + trailer
  long w_plane;
  const float* wscale;  // the packing's trailer: [0] max|w|, [1] 2⁻¹¹/(σ_a·σ_w)
  const float* bias;    // [CO]
  const float* beta;    // β_eff [CO]
  const u16* gamma_h3;  // γ_eff in the h3 form (iclr17_split_packed_h3, taps 1): [2][CO/8][CO][8]
                        // + trailer (gamma_scale: [1] = 2⁻¹¹/(σ_a·σ_γ))
  const float* gamma_scale;
  float* out;           // fp32 NHWC [B][Hout][Wout][CO] or null
  float* pre;           // the GDN / IGDN input x = conv + bias, fp32 NHWC, or null (training)
  u16* out_h3;          // h3 output: NHWC [2][B][Hout][Wout][CO] or chunk-major (out_cm)
  long out_h3_plane;    //   [2][B][CO/out_cm][Hout][Wout][out_cm]
  u16* out_x6;          // x6 split output (NHWC, 3 planes) or null
  long out_x6_plane;
  int out_cm;           // the h3 output's chunk-major chunk: 0 (NHWC), 8, 16 or 32
  int* range;           // set to 1 when a value does not fit the h3 form (nullable)
  // HE_QUANT (conv3 + quantiser + rate): out = y (nullable), yhat = ŷ | ỹ fp32 NHWC, out_h3 = ŷ in
  // the h3 form (nullable), bits partial sums [B][T] (T = tiles · channel groups)
  int qmode;
  const float* noise;   // NCHW [B][CO][Hout][Wout] (noise mode)
  const float* rate;    // packed [11][CO]
  const float* rtab;    // round mode, nullable: element_bits of −32..32 [CO][65]
  float* yhat;
  double* partial;
  int T;
  int B, Hin, Win, Hout, Wout;
  int gh, gw;           // base grid (conv: output grid; deconv: input grid)
  int tiles_x, tiles_y;
};

// conv2 (k5 s2 p2) in this engine: 8-channel chunks and two taps per 16-deep step — lane half h of
// a fragment holds tap 2s + h — so that a chunk's 35×35-pixel patch (both h3 planes) stays at
// 45 KB and double-buffers beside the weight ring (16-channel chunks would need 157 KB).
constexpr int HM_CONV8 = 2;
constexpr int kConv8Steps = 13;   // tap pairs (25 taps + one zero-weight pad)

// Patch of HM_CONV8: per row [column parity 2][20 slots] × 16 bytes (8 channels) — 640-byte rows,
// so the two rows of a 32-pixel fragment half are 1280 bytes (a multiple of 256) apart and its
// ds_read_b128 lane groups hit 16 distinct 16-byte slots
template <int TH>
struct PatchC8 {
  static constexpr int ROWS = 2 * TH + 3;
  static constexpr int ROWB = 640;
  static constexpr int BYTES = ROWS * ROWB;
  __host__ __device__ static constexpr int off(int pr, int pc) {
    return pr * ROWB + (pc & 1) * 320 + (pc >> 1) * 16;
  }
  __host__ __device__ static constexpr int tap8(int t) {   // tap t = 5·ky + kx; 25 = the pad
    return t < 25 ? off(t / 5, t % 5) : 0;
  }
};
// conv1 (k9 s4 p4, 3 input channels) in this engine: the whole 3 × 69 × 69 input window of a
// 16 × 16-pixel output tile split once into the two h3 planes, [channel][row][80 columns] fp16
// (160-byte rows: the two pixel rows of a fragment half, 4 input rows apart, land 128 bytes apart
// mod 256 — their ds_read_b64 lane groups cover all 64 banks); K = 243 reordered as in the x6
// conv1 kernel (csrc/engine_fp32.hip conv1_x6_kernel): k-group g < 27 = 8 consecutive columns of
// one (channel, kernel row), g = 27 .. 30 = column 8 of (channel, kernel row) pairs 8(g − 27) + e,
// g = 31 zero; 16 steps of 16 (lane half h: g = 2s + h).
constexpr int HM_CONV1 = 3;
constexpr int kConv1Steps = 16;
template <int TH>
struct PatchC1 {
  static constexpr int ROWS = 4 * TH + 5;
  static constexpr int ROWB = 160;
  static constexpr int BYTES = 3 * ROWS * ROWB;   // one plane
  // byte offset of k-group g's (channel, kernel row) row, g < 27
  __host__ __device__ static constexpr int rowoff(int g) { return ((g / 9) * ROWS + g % 9) * ROWB; }
  // byte offset of pair q's column-8 element (−1: a zero-weight pad)
  __host__ __device__ static constexpr int gath(int q) {
    return q < 27 ? ((q / 9) * ROWS + q % 9) * ROWB + 16 : -1;
  }
};

template <int MODE, int TH>
struct HPatch {
  using type = Patch<MODE, TH>;
};
template <int TH>
struct HPatch<HM_CONV8, TH> {
  using type = PatchC8<TH>;
};
template <int TH>
struct HPatch<HM_CONV1, TH> {
  using type = PatchC1<TH>;
};

// NS: weight-ring stages (F + 2 for F DMA groups in flight)
template <int MODE, int TH, int CO, int CI, bool INT_IN, int NS = 4>
struct HK {
  static constexpr int NW = TH / 2, NTHR = NW * 64;
  static constexpr int NT = CO / 32;           // 32-channel accumulator tiles per wave
  static constexpr bool C1 = MODE == HM_CONV1;
  static constexpr int CCH = MODE == HM_CONV8 ? 8 : 16;   // channels per chunk
  static constexpr int NCH = C1 ? 1 : CI / CCH;  // chunks (conv1: the whole window, once)
  using P = typename HPatch<MODE, TH>::type;
  static constexpr int PL = INT_IN ? 1 : 2;    // input planes staged
  static constexpr int PB = PL * P::BYTES;     // patch bytes (planes back to back)
  static constexpr int NQI = C1 ? 0 : (PB + 1023) / 1024;   // patch DMA pieces per chunk
  static constexpr int PBUF = (PB + 1023) / 1024 * 1024;
  static constexpr int NPB = C1 ? 1 : 2;       // patch buffers
  static constexpr int SB = 2 * 2 * CO * 16;   // weight stage: [plane 2][half 2][CO][8] fp16
  static constexpr int NBI = SB / 1024;
  static constexpr int NST = NS;
  static constexpr int MAIN = NPB * PBUF + NST * SB + 1024;
  static constexpr int NTH = NT / 2;           // epilogue: output tiles per pass
  static constexpr int KB = CO / 16;           // epilogue: 16-channel k-blocks
  static constexpr int GBL = 2 * NTH * KB;     // epilogue: γ fragment blocks per pass (1 KB)
  static constexpr int LDS0 = MAIN > GBL * 1024 ? MAIN : GBL * 1024;
  static constexpr int BBOFF = (LDS0 + 1023) / 1024 * 1024;
  static constexpr int LDS = BBOFF + 2048 + 256;   // + bias, β_eff, the epilogue's sink
  static_assert(SB % 1024 == 0, "weight stage");
  static_assert(C1 || CI % CCH == 0, "tile shape");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// COT: the output channels of this workgroup (channel group cg: cg·COT .. cg·COT + COT − 1 of CO;
// COT < CO only for HE_QUANT, whose epilogue needs no other channel of the pixel). SEP: two-level
// accumulation — each input chunk's K = 200 products summed from zero in a chain of their own and
// added to the total with one VALU add (the MFMA chain rounds at the scale of its running sum;
// conv3's output is rounded into ŷ).
// u16 offset (within a plane) of 8 channels ch .. ch + 7 of output pixel (oy, ox) of image b in the
// h3 output's layout: NHWC (out_cm = 0) or chunk-major [B][CO/out_cm][Hout][Wout][out_cm]
// (cm is a power of two: shifts and masks, not the integer divisions a runtime divisor compiles to)
__device__ __forceinline__ long h3_out_off(const HArgs& a, int b, int oy, int ox, int CO, int ch) {
  const int cm = a.out_cm;
  if (cm == 0) return (((long)b * a.Hout + oy) * a.Wout + ox) * CO + ch;
  const int sh = __builtin_ctz(cm);
  return ((((long)b * (CO >> sh) + (ch >> sh)) * a.Hout + oy) * a.Wout + ox << sh) + (ch & (cm - 1));
}
// h3_out_off(…, ch + 32i) − h3_out_off(…, ch) for ch % 32 + 8 ≤ 32: the same for every lane (cm ≤ 32
// divides 32), so the epilogues compute a lane's two offsets once and step them by i times this
__device__ __forceinline__ long h3_out_step32(const HArgs& a) {
  return a.out_cm == 0 ? 32L : 32L * a.Hout * a.Wout;
}

// conv3's epilogue (HE_QUANT): y = acc·2⁻¹¹/(σ_a·σ_w) (no bias, analysis_17.py:22), then
// model.py:48-56 — ŷ = rint(y) (round) or ỹ = y + u (noise, u from the NCHW noise tensor) — and
// the rate of model.py:71-73 per element (the rate table's lookup for integers |ŷ| ≤ 32 in round
// mode; element_bits otherwise, evaluated after the lookups as in engine_fp32.hip's EPI_QUANT: a
// per-element branch inlines 2 KB of element_bits per element). Outputs: ŷ fp32 NHWC, y fp32
// (nullable), ŷ in the h3 form (nullable; 16-byte stores after permlane32 swaps as the GDN
// epilogue's), and the workgroup's bit sum — lanes in (tile, register) order, the xor tree of
// wave_sum, the waves in order in double — at partial[b][tile · (CO / COT) + cg].
// The range flag: bit 0 is set by the chain's earlier kernels (conv1 / conv2 / the h3 split of an
// input) — read here, it makes every output of this kernel NaN (y, ŷ, its h3 form, the bits), so
// the encoder's own results are loud too, not only the chain's last kernel's; this kernel's own
// overflow (ŷ's h3 form, deconv1's input) sets bit 1, which it does not read (another workgroup's
// result would otherwise depend on timing) and deconv3 does.
template <int TH, int CO, int COT>
__device__ __forceinline__ void quant_epilogue(const HArgs& a, f16v (&acc)[COT / 32],
                                               unsigned char* lds0, unsigned char* scratch, int b,
                                               int ty, int tx, int cg) {
  constexpr int NT = COT / 32, NW = TH / 2;
  const int etid = fresh_tid(), elane = etid & 63, er32 = elane & 31, eh = elane >> 5;
  const int ewave = __builtin_amdgcn_readfirstlane(etid >> 6);
  const int gy = ty * TH + 2 * ewave + (er32 >> 4), gx = tx * 16 + (er32 & 15);
  const bool inside = gy < a.gh && gx < a.gw;
  const long o = ((long)b * a.Hout + gy) * a.Wout + gx;
  const float dsc = a.wscale[1];
  const bool round = a.qmode == ICLR17_QUANT_ROUND;
  const bool table = a.rtab != nullptr && round;
  // the slow path's lane-private rows in LDS (the main loop's stages, free now): 16 latents and
  // their bits (128 bytes per lane), so that element_bits sits in a rolled loop (one inlined copy
  // per tile, not one per element)
  float* const lq = (float*)lds0 + etid * 32;
  float bits = 0.f;
  bool ovf = false;
  const bool poison = a.range != nullptr && (*(const volatile int*)a.range & 1) != 0;
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const int c0 = cg * COT + 32 * i;
    float q[16], bv[16];
    bool slow = false;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = c0 + 8 * (r >> 2) + 4 * eh + (r & 3);
      const float y = poison ? __builtin_nanf("") : acc[i][r] * dsc;   // a power of two: exact
      acc[i][r] = y;
      const float yh = round ? rintf(y)
                             : y + (inside ? a.noise[(((long)b * CO + c) * a.Hout + gy) * a.Wout + gx] : 0.f);
      q[r] = yh;
      bv[r] = table ? a.rtab[c * 65 + (int)fminf(fmaxf(yh, -32.f), 32.f) + 32] : 0.f;
      slow |= inside && !(table && fabsf(yh) <= 32.f);
    }
    if (slow) {
#pragma unroll
      for (int r = 0; r < 16; ++r) lq[r] = q[r];
#pragma unroll 1
      for (int r = 0; r < 16; ++r) {
        const float v = lq[r];
        if (!(table && fabsf(v) <= 32.f))
          lq[16 + r] = element_bits(v, a.rate, CO, c0 + 8 * (r >> 2) + 4 * eh + (r & 3));
      }
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (!(table && fabsf(q[r]) <= 32.f)) bv[r] = lq[16 + r];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) bits += inside ? bv[r] : 0.f;
    f4 yq[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      yq[m] = f4{q[4 * m], q[4 * m + 1], q[4 * m + 2], q[4 * m + 3]};
      if (inside) {
        *(f4*)(a.yhat + o * CO + c0 + 8 * m + 4 * eh) = yq[m];
        if (a.out)
          *(f4*)(a.out + o * CO + c0 + 8 * m + 4 * eh) =
              f4{acc[i][4 * m], acc[i][4 * m + 1], acc[i][4 * m + 2], acc[i][4 * m + 3]};
      }
    }
    if (a.out_h3) {
      uint2 hb[4], lb[4];
      bool ov = false;
#pragma unroll
      for (int m = 0; m < 4; ++m) h3_split4(yq[m], hb[m], lb[m], ov);
      ovf |= inside && ov;
      u4 sv[2][2];
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const uint2 A = pl ? lb[k] : hb[k], Bv = pl ? lb[k + 2] : hb[k + 2];
          const auto sx = __builtin_amdgcn_permlane32_swap(A.x, Bv.x, false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(A.y, Bv.y, false, false);
          sv[pl][k] = u4{sx[0], sy[0], sx[1], sy[1]};
        }
      if (inside) {
        const long s0 = h3_out_off(a, b, gy, gx, CO, c0 + 16 * eh);
        const long s1 = h3_out_off(a, b, gy, gx, CO, c0 + 16 * eh + 8);
        *(u4*)(a.out_h3 + s0) = sv[0][0];
        *(u4*)(a.out_h3 + s1) = sv[0][1];
        *(u4*)(a.out_h3 + a.out_h3_plane + s0) = sv[1][0];
        *(u4*)(a.out_h3 + a.out_h3_plane + s1) = sv[1][1];
      }
    }
  }
  if (ovf && a.range) atomicOr(a.range, 2);   // vector atomic, per offending lane (rare)
  bits = wave_sum(poison ? __builtin_nanf("") : bits);
  float* sw = (float*)scratch;
  if (elane == 0) sw[ewave] = bits;
  __syncthreads();
  if (etid == 0) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += (double)sw[w];
    a.partial[(long)b * a.T + (ty * a.tiles_x + tx) * (CO / COT) + cg] = t;
  }
}

// ICM: the input's chunk-major chunk (the layout of the h3 form below; 0: NHWC, conv1's image).
template <int MODE, int TH, int CO, int CI, int EPI, bool INT_IN, int PH, int COT = CO,
          bool SEP = false, int ICM = 0>
__device__ __forceinline__ void h3k_body(const HArgs& a, unsigned char* smem, int b, int ty, int tx,
                                         int cg = 0) {
  static_assert(CO % COT == 0 && (COT == CO || EPI == HE_QUANT), "channel groups: conv3 only");
  // conv3's short steps (9 MFMAs per wave, one wave per SIMD) keep four DMA groups in flight, so
  // a weight slot has four steps to arrive instead of two (the other layers' 18-MFMA steps on two
  // waves per SIMD cover the latency with two)
  constexpr int NSG = EPI == HE_QUANT ? 6 : 4;
  using KK = HK<MODE, TH, COT, CI, INT_IN, NSG>;
  using P = typename KK::P;
  constexpr bool CONV = MODE != BM_DECONV, C8 = MODE == HM_CONV8, C1 = MODE == HM_CONV1;
  using TP = Taps<CONV ? BM_CONV : BM_DECONV, PH>;
  // one tap per step (HM_CONV8: a tap pair; HM_CONV1: two k-groups)
  constexpr int NT = KK::NT, NW = KK::NW, NCH = KK::NCH;
  constexpr int S = C1 ? kConv1Steps : C8 ? kConv8Steps : TP::T;
  constexpr int SB = KK::SB, NBI = KK::NBI, NST = KK::NST;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  // counted DMA schedule (engine_bf16.hip k5_body): every wave issues exactly K DMA instructions
  // per step — weight slots of step g+F+1, pieces of the next chunk's patch during steps
  // 0 .. S-F-1, sink loads as padding — so `s_waitcnt vmcnt((F-1)·K)` + barrier at step g retires
  // all but the newest F-1 groups: step g+1's stage is complete when step g reads it ahead
  constexpr int F = NSG - 2 < S - 1 ? NSG - 2 : (S >= 3 ? 2 : 1), SI = S - F;
  static_assert(SI >= 1 && NST >= F + 2, "DMA schedule");
  constexpr int PS = (KK::NQI + SI - 1) / SI;
  constexpr int K = (NBI + PS + NW - 1) / NW;
  static_assert(F * K < 64, "vmcnt");
  constexpr int GS = NCH * S;
  unsigned char* const sP = smem;
  unsigned char* const sB = smem + KK::NPB * KK::PBUF;
  unsigned char* const sD = sB + NST * SB;
  float* const sbb = (float*)(smem + KK::BBOFF);   // [bias | pad][β_eff | pad]
  const long img = (long)b * a.Hin * a.Win;
  const int iy0 = CONV ? 2 * ty * TH - 2 : ty * TH - 1;
  const int ix0 = CONV ? 2 * tx * 16 - 2 : tx * 16 - 1;
  // input layout: chunk-major [2][B][CI/ICM][h][w][ICM] with ICM = the chunk's channels, so a
  // patch piece (one pixel's 8 channels) is 16 bytes of a contiguous run of pixels, not 16 bytes
  // of a 384-byte NHWC pixel (a cache line per piece: conv2 −8 %, conv3 −23 % measured)
  static_assert(ICM == 0 || ICM == KK::CCH, "chunk-major input: one chunk per layout chunk");
  const long cstride = ICM ? (long)a.Hin * a.Win * ICM : KK::CCH;   // u16 per chunk
  constexpr int PXS = ICM ? ICM : CI;                                 // u16 per pixel
  const u16* __restrict__ inb = a.in + img * CI;
  // patch piece `piece` (1 KB): this lane's 16-byte slot → source u16 offset, or -1 (zeros)
  auto piece_src = [&](int piece) -> long {
    const int byte = (piece * 64 + lane) * 16;
    const int pl = byte / P::BYTES, rem = byte - pl * P::BYTES;
    const int pr = rem / P::ROWB, r1 = rem - pr * P::ROWB;
    int pc, hh = 0;
    bool ok;
    if constexpr (C1) {   // conv1 stages its window without pieces
      pc = 0;
      ok = false;
    } else if constexpr (C8) {
      const int par = r1 / 320, slot = (r1 - par * 320) / 16;
      pc = 2 * slot + par;
      ok = slot < 18 && pc < 35;
    } else if constexpr (MODE == BM_CONV) {
      const int par = r1 / (2 * P::HALF), r2 = r1 - par * 2 * P::HALF;
      hh = r2 / P::HALF;
      pc = 2 * ((r2 - hh * P::HALF) / 16) + par;
      ok = pc < 35;
    } else {
      hh = r1 / P::HALF;
      pc = (r1 - hh * P::HALF) / 16;
      ok = true;
    }
    const int iy = iy0 + pr, ix = ix0 + pc;
    ok = ok && pl < KK::PL && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
    return ok ? pl * a.in_plane + (long)(iy * a.Win + ix) * PXS + 8 * hh : -1;
  };
  auto issue_piece = [&](int c1, int piece, bool valid) {
    if (!valid) {
      sink4(sD);
      return;
    }
    const long src = piece_src(piece);
    glds16(src >= 0 ? (const void*)(inb + src + c1 * cstride) : zero16(lane),
           sP + (c1 & 1) * KK::PBUF + piece * 1024);
  };
  // weights of this phase: per plane [NCH][S][2][CO][8]; the step's stage [plane][2][CO][8]
  constexpr long WSTEP = 2L * CO * 8;   // u16 per (chunk, tap) block of one plane
  const u16* __restrict__ wph = a.w;
  if (MODE == BM_DECONV) {
    long off = 0;
#pragma unroll
    for (int p = 0; p < PH; ++p) {
      const int ny = (p >> 1) == 0 ? 3 : 2, nx = (p & 1) == 0 ? 3 : 2;
      off += (long)NCH * ny * nx * WSTEP;
    }
    wph += off;
  }
  int wsrc[K];   // slot k of a step: plane + unit offset (16-byte units of [2][CO]; the stage
                // holds units (half, cg·COT .. cg·COT + COT − 1) as [2][COT]); < 2^31 elements
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int q = (k * NW + wave) * 64 + lane;
    const int pl = q / (2 * COT), u = q - pl * (2 * COT), hu = u / COT;
    wsrc[k] = (int)(pl * a.w_plane) + (hu * CO + cg * COT + (u - hu * COT)) * 8;
  }
  auto issue_w = [&](int k, int wg) {
    const int slot = k * NW + wave;
    if (wg >= GS) {
      sink4(sD);
      return;
    }
    glds16(wph + (long)wg * WSTEP + wsrc[k], sB + (wg % NST) * SB + slot * 1024);
  };

  // ---- per-lane fragment addresses
  // B (pixels): pixel (tile row 2·wave + (r32 >> 4), column r32 & 15), channel half h
  const int prow = 2 * wave + (r32 >> 4), pcol = r32 & 15;
  const int tpix = prow * 16 + pcol;
  int pbase;
  if constexpr (C1) pbase = 4 * prow * P::ROWB + 8 * pcol;
  else if constexpr (C8) pbase = P::off(2 * prow, 2 * pcol);
  else pbase = (MODE == BM_CONV ? P::off(2 * prow, 2 * pcol) : P::off(prow, pcol)) + h * P::HALF;
  // the step's tap offset: one tap for every lane, or (HM_CONV8) tap 2s + h for lane half h
  auto tap_of = [&](int s) -> int {
    if constexpr (C8) return h ? P::tap8(2 * s + 1) : P::tap8(2 * s);
    else if constexpr (C1) return 0;
    else return P::template tap_off<PH>(s);
  };
  // A (weights): stage [plane][2][CO][8]: lane (k-group h, channel 32·i + r32)
  const int abase = (h * COT + r32) * 16;
  constexpr int APL = 2 * COT * 16;   // stage bytes per plane

  f16v acc[NT], cacc[NT];   // cacc: SEP's chunk sums (unused otherwise)
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = 0.f;

  // prologue: bias and β_eff (waves 0 / 1), chunk 0's patch, the weights of steps 0 .. F-1, then
  // step F's weights as a full K-group and F-1 sink groups (the first wait keeps F in flight)
  static_assert(CO <= 256, "bias / β stage");
  if (EPI != HE_QUANT && wave < 2) {
    const float* src = wave == 0 ? a.bias : a.beta;
    glds16(lane * 4 < CO ? (const void*)(src + lane * 4) : zero16(lane), sbb + wave * 256);
  }
  for (int piece = wave; piece < KK::NQI; piece += NW) issue_piece(0, piece, true);
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k * NW + wave < NBI) issue_w(k, f);
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k * NW + wave < NBI) issue_w(k, F);
    else sink4(sD);
  }
#pragma unroll
  for (int f = 1; f < F; ++f)
#pragma unroll
    for (int k = 0; k < K; ++k) sink4(sD);
  if constexpr (C1) {
    // the input window (fp32 NCHW image a.img) → the two h3 planes, once: 18 float4 per patch
    // row (72 columns ≥ 69), every load issued before the first split
    constexpr int QR = 18, NU = 3 * P::ROWS * QR, IT = (NU + KK::NTHR - 1) / KK::NTHR;
    const int jy0 = 4 * TH * ty - 4, jx0 = 64 * tx - 4;
    const float* __restrict__ xb = a.img + (long)b * 3 * a.Hin * a.Win;
    f4 v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int u = tid + it * KK::NTHR;
      const int q = u % QR, cr = u / QR, c = cr / P::ROWS, r = cr - c * P::ROWS;
      const int iy = jy0 + r, ix = jx0 + 4 * q;
      const bool ok = u < NU && (unsigned)iy < (unsigned)a.Hin && (unsigned)ix < (unsigned)a.Win;
      v[it] = ok ? *(const f4*)(xb + ((long)c * a.Hin + iy) * a.Win + ix) : f4{0.f, 0.f, 0.f, 0.f};
    }
    bool povf = false;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int u = tid + it * KK::NTHR;
      if (u >= NU) break;
      const int q = u % QR, cr = u / QR;
      uint2 hb, lb;
      h3_split4(v[it], hb, lb, povf);
      *(uint2*)(sP + cr * P::ROWB + 8 * q) = hb;
      *(uint2*)(sP + P::BYTES + cr * P::ROWB + 8 * q) = lb;
    }
    if (povf && a.range) atomicOr(a.range, 1);   // vector atomic, per offending lane (rare)
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the planes written before the first barrier
  }

  typedef const __attribute__((address_space(3))) u4* lu4p;
  // slot k of step g's DMA group: weights of step g+F+1, the next chunk's patch, or a sink load
  auto dma_k = [&](int k, int c, int s, int g) {
    const int slot = k * NW + wave;
    if ((k + 1) * NW <= NBI || slot < NBI) {
      issue_w(k, g + F + 1);
    } else if (s < SI) {
      const int piece = s * PS + slot - NBI;
      issue_piece(c + 1, piece, c + 1 < NCH && piece < KK::NQI);
    } else {
      sink4(sD);
    }
  };
  // fragments one step ahead: the barrier of step g retires all but the newest F-1 DMA groups,
  // so step g+1's weights (and at s = S-1 the next chunk's patch) are visible; its fragment reads
  // go out before step g's MFMAs and the LDS latency hides behind them (deconv1 0.128 -> 0.109 ms)
  struct Frag {
    u4 bh, bl, wh[NT], wl[NT];
  };
  typedef unsigned u2e __attribute__((ext_vector_type(2)));
  typedef const __attribute__((address_space(3))) u2e* lu2p;
  typedef const __attribute__((address_space(3))) unsigned short* lu16p;
  // conv1's B fragment of step s from one plane (lane half h: k-group g = 2s + h)
  auto conv1_b = [&](const unsigned char* pp, int s) -> u4 {
    u4 v = u4{0u, 0u, 0u, 0u};
    if constexpr (!C1) return v;
    else {
    const int g0 = 2 * s, g1 = 2 * s + 1;
    if (g0 < 27) {   // 8 columns of one (channel, kernel row): two 8-byte reads
      const int ro = h ? (g1 < 27 ? P::rowoff(g1) : P::rowoff(g0)) : P::rowoff(g0);
      const u2e x0 = *(lu2p)(pp + ro), x1 = *(lu2p)(pp + ro + 8);
      v = u4{x0.x, x0.y, x1.x, x1.y};
    }
    if (g1 >= 27) {   // column 8 of eight (channel, kernel row) pairs, element-wise
      unsigned e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int oa = g0 >= 27 ? P::gath(8 * (g0 - 27) + j) : -1;
        const int ob = P::gath(8 * (g1 - 27) + j);
        const int o = h ? ob : oa;
        const unsigned x = *(lu16p)(pp + (o >= 0 ? o : 0));
        e[j] = o >= 0 ? x : 0u;
      }
      const u4 w = u4{e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16), e[6] | (e[7] << 16)};
      if (g0 >= 27) v = w;
      else if (h) v = w;   // g0 = 26: the lower half keeps its row read
    }
    return v;
    }
  };
  auto read_frag = [&](Frag& f, const unsigned char* pb, int to, const unsigned char* wb, int s) {
    if constexpr (C1) {
      f.bh = conv1_b(sP + pbase, s);
      f.bl = conv1_b(sP + P::BYTES + pbase, s);
    } else {
      f.bh = *(lu4p)(pb + to);
      if constexpr (!INT_IN) f.bl = *(lu4p)(pb + P::BYTES + to);
      else f.bl = u4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      f.wh[i] = *(lu4p)(wb + i * 512);
      f.wl[i] = *(lu4p)(wb + APL + i * 512);
    }
  };
  Frag cur;
  int stage = 1;   // stage of step g+1
  for (int c = 0; c < NCH; ++c) {
    if constexpr (SEP) {
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < 16; ++j) cacc[i][j] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int g = c * S + s;
      wait_vm_barrier<(F - 1) * K>();   // step g+1's weights (and patch) landed (at g = 0 the
                                        // prologue's padding tail is all that may be in flight);
                                        // stage (g+F+1) % NST is free
      if (s == 0 && c == 0) read_frag(cur, sP + pbase, tap_of(0), sB + abase, 0);
      Frag nxt;
      read_frag(nxt, sP + ((s + 1 < S ? c : c + 1) & 1) * KK::PBUF + pbase,
                tap_of(s + 1 < S ? s + 1 : 0), sB + stage * SB + abase, s + 1 < S ? s + 1 : 0);
      stage = stage + 1 == NST ? 0 : stage + 1;
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        f16v t = SEP ? cacc[i] : acc[i];
        if constexpr (!INT_IN) t = mfma32h(cur.wh[i], cur.bl, t);
        t = mfma32h(cur.wl[i], cur.bh, t);
        t = mfma32h(h3_x2048(cur.wh[i]), cur.bh, t);
        if constexpr (SEP) cacc[i] = t;
        else acc[i] = t;
      }
      // the step's DMA group after the fragment reads: an LDS read after an LDS-DMA of unknown
      // destination makes the compiler wait for that DMA (s_waitcnt vmcnt(0)) first. (Spread
      // between the tiles' MFMAs instead: no faster.)
#pragma unroll
      for (int k = 0; k < K; ++k) dma_k(k, c, s, g);
      cur = nxt;
    }
    if constexpr (SEP) {   // the chunk's sum into the total (correctly rounded VALU adds)
#pragma unroll
      for (int i = 0; i < NT; ++i) acc[i] += cacc[i];
    }
  }
  vm_barrier();   // trailing sink loads landed; every wave is done with the stages
  if constexpr (EPI == HE_QUANT) {
    // (the kernel's LDS is sized by the full-input form: HK<…, false>)
    using KF = HK<MODE, TH, COT, CI, false, NSG>;
    static_assert(TH / 2 * 64 * 128 <= KF::BBOFF, "the epilogue's lane rows fit the stages");
    quant_epilogue<TH, CO, COT>(a, acc, smem, smem + KF::BBOFF, b, ty, tx, cg);
    return;
  } else {

  // ---- epilogue. acc[i][4m + j]: channel 32i + 8m + 4h + j of tile pixel tpix. The lane
  // indices are re-derived from a fresh threadIdx.x: the main loop's copies otherwise stay live
  // through it, and the INT_OK kernel spilled them (a scratch op would break the counted vmcnt
  // groups that tools/dma_sync_check.py proves)
  const int etid = fresh_tid(), elane = etid & 63, er32 = elane & 31, eh = elane >> 5;
  const int ewave = __builtin_amdgcn_readfirstlane(etid >> 6);
  const int etpix = (2 * ewave + (er32 >> 4)) * 16 + (er32 & 15);
  const int gy = ty * TH + (etpix >> 4), gx = tx * 16 + (etpix & 15);
  const bool inside = gy < a.gh && gx < a.gw;
  const int oy = CONV ? gy : 2 * gy + (PH >> 1);
  const int ox = CONV ? gx : 2 * gx + (PH & 1);
  const long o = ((long)b * a.Hout + oy) * a.Wout + ox;
  const float dsc = a.wscale[1];   // 2⁻¹¹/(σ_a·σ_w): exact
  const long hb0 = h3_out_off(a, b, oy, ox, CO, 16 * eh), hb1 = h3_out_off(a, b, oy, ox, CO, 16 * eh + 8);
  const long hstep = h3_out_step32(a);
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f4 bv = *(const f4*)(sbb + 32 * i + 8 * m + 4 * eh);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][4 * m + j] = acc[i][4 * m + j] * dsc + bv[j];   // x = conv + bias
    }
  constexpr int NTH = KK::NTH, KB = KK::KB;
  static_assert(NT % 2 == 0, "GDN epilogue: pairs of 32-channel tiles");
  bool ovf = false;
  // The channel contraction n_i = Σ_j γ_ij·x_j² in the h3 form. x² of a pixel (rounded to fp32,
  // as conv2d(x², γ) sees it) is scaled by a power of two s_p that puts the pixel's largest x²
  // in [2¹³, 2¹⁴) — the pixel is this elane's MFMA column, so the scale is undone per elane — and
  // split into hi / lo fp16 planes; γ arrives split with its own per-tensor power of two. The
  // pixel's 192 channels sit in this elane (96) and elane er32 + 32·(1 − eh) (the other 96).
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) mx = fmaxf(mx, fabsf(acc[i][j]));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  int ep = 0;   // s_p = 2^ep
  {
    const float m2 = mx * mx;
    if (m2 > 0.f && m2 <= 3.40282347e38f) {
      int e;
      frexpf(m2, &e);   // m2 ∈ [2^(e−1), 2^e)
      // at most 2^100: a pixel whose largest x² is below 2^-86 (a near-zero pixel, or an x² that
      // underflowed) keeps s_p and the n scale finite (2^(14−e) overflowed to inf for x² < 2^-113
      // and made the pixel NaN); its x²·s_p then stays below 2^14 and its n is negligible
      ep = 14 - e < 100 ? 14 - e : 100;
    }
  }
  const float sp = ldexpf(1.0f, ep);
  // n = acc_n · 2⁻¹¹ / (σ_γ · s_p) = acc_n · gamma_scale[1] · σ_a / s_p (powers of two: exact)
  const float nsc = ldexpf(a.gamma_scale[1] * kH3Sa, -ep);
  // γ staged in four half-passes q = (pass hf, k-half kh) into two alternating 36-KB buffers: the
  // rows 32·(hf·NTH + il) .. of both planes for k-blocks kh·KH .. kh·KH + KH − 1; block (plane, il,
  // kk) ← elane (er32, eh) γ_p[32(hf·NTH + il) + er32][16kb + 8eh .. +7] (the [CO/8][CO][8]
  // packing). Each wave issues GK pieces per stage (sink loads as padding), so vmcnt(GK) leaves
  // exactly the newer stage in flight. Stage q+1 lands while stage q is contracted.
  constexpr int KH = KB / 2, HBL = 2 * NTH * KH, GK = (HBL + NW - 1) / NW;
  static_assert(KB % 2 == 0 && 2 * HBL * 1024 <= KK::LDS0, "γ half-stages");
  auto stage_g = [&](int q) {
    const int hf = q >> 1, kh = q & 1;
#pragma unroll
    for (int k = 0; k < GK; ++k) {
      const int blk = k * NW + ewave;
      if (blk >= HBL) {   // the epilogue's own sink: the main loop's may lie under a γ buffer
        sink4((unsigned char*)sbb + 2048);
        continue;
      }
      const int p = blk / (NTH * KH), rem = blk - p * NTH * KH;
      const int il = rem / KH, kb = kh * KH + rem - il * KH;
      glds16(a.gamma_h3 + (long)p * CO * CO + ((2 * kb + eh) * CO + 32 * (hf * NTH + il) + er32) * 8,
             smem + (q & 1) * HBL * 1024 + blk * 1024);
    }
  };
  stage_g(0);
  stage_g(1);
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    // opaque to the optimiser: pass 1 recomputes the x² planes instead of keeping pass 0's
    // (12 k-blocks × 2 planes × 4 registers) alive across the passes
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(acc[i][j]));
    f16v n[NTH];
#pragma unroll
    for (int il = 0; il < NTH; ++il)
#pragma unroll
      for (int j = 0; j < 16; ++j) n[il][j] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int q = 2 * hf + kh;
      if (q == 0) {
        wait_vm_barrier<GK>();   // stage 0 landed (stage 1 in flight)
      } else {
        vm_barrier();            // stage q landed (and pass 0's stores), every wave done with
                                 // the buffer stage q+1 refills
        if (q + 1 < 4 && q >= 1) stage_g(q + 1);
      }
      const unsigned char* sg = smem + (q & 1) * HBL * 1024 + elane * 16;
#pragma unroll
      for (int kk = 0; kk < KH; ++kk) {
        const int kb = kh * KH + kk;
        // x²·s_p of channels 16kb .. 16kb + 15 as the hi / lo B planes: the accumulator rows a
        // lane holds are 4h + 0..3 and 8 + 4h + 0..3 of the 16-channel block; one permlane32 swap
        // per register pair and plane hands lane half eh the 8 consecutive channels 8eh .. 8eh + 7
        const int i = kb >> 1, r0 = 8 * (kb & 1);
        unsigned hv[4], lv[4];   // channel pairs (2q, 2q + 1) of the lane's 8, packed fp16
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          typedef float f2 __attribute__((ext_vector_type(2)));
          const f2 v = f2{acc[i][r0 + 2 * qq] * acc[i][r0 + 2 * qq], acc[i][r0 + 2 * qq + 1] * acc[i][r0 + 2 * qq + 1]} * sp;
          const h2v hh = __builtin_convertvector(v, h2v);
          const h2v ll = __builtin_convertvector((v - __builtin_convertvector(hh, f2)) * 2048.0f, h2v);
          hv[qq] = __builtin_bit_cast(unsigned, hh);
          lv[qq] = __builtin_bit_cast(unsigned, ll);
        }
        u4 xp[2];
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const unsigned* v = pl == 0 ? hv : lv;
          const auto s0 = __builtin_amdgcn_permlane32_swap(v[0], v[2], false, false);
          const auto s1 = __builtin_amdgcn_permlane32_swap(v[1], v[3], false, false);
          xp[pl] = u4{s0[0], s1[0], s0[1], s1[1]};
        }
#pragma unroll
        for (int il = 0; il < NTH; ++il) {
          const u4 gh = *(lu4p)(sg + ((0 * NTH + il) * KH + kk) * 1024);
          const u4 gl = *(lu4p)(sg + ((1 * NTH + il) * KH + kk) * 1024);
          f16v t = mfma32h(gh, xp[1], n[il]);
          t = mfma32h(gl, xp[0], t);
          n[il] = mfma32h(h3_x2048(gh), xp[0], t);
        }
        __builtin_amdgcn_sched_barrier(0);   // one k-block's operands live at a time
      }
    }
#pragma unroll
    for (int il = 0; il < NTH; ++il)
#pragma unroll
      for (int j = 0; j < 16; ++j) n[il][j] = n[il][j] * nsc;
    // y = x·√(β + n) (IGDN) | x / √(β + n) (GDN); stores
#pragma unroll
    for (int il = 0; il < NTH; ++il) {
      const int i = hf * NTH + il;
      f4 y[4], bes[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) bes[m] = *(const f4*)(sbb + 256 + 32 * i + 8 * m + 4 * eh);   // one wait
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int ch = 32 * i + 8 * m + 4 * eh;
        if (inside && a.pre)
          *(f4*)(a.pre + o * CO + ch) = f4{acc[i][4 * m], acc[i][4 * m + 1], acc[i][4 * m + 2], acc[i][4 * m + 3]};
        const f4 be = bes[m];
        // the hardware square root / reciprocal square root (v_sqrt_f32, v_rsq_f32: within an ulp
        // or two, far inside the h3 form's own 2⁻²² — and a sixth of the IEEE sequences' VALU
        // work, which set the epilogue's length); n ≥ β_min > 0
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float nn = n[il][4 * m + j] + be[j];
          const float x = acc[i][4 * m + j];
          y[m][j] = EPI == HE_IGDN ? x * __builtin_amdgcn_sqrtf(nn) : x * __builtin_amdgcn_rsqf(nn);
        }
        if (inside && a.out) *(f4*)(a.out + o * CO + ch) = y[m];
      }
      if (a.out_h3) {
        // the tile's 32 channels of this pixel in the h3 form, as two 16-byte stores per plane:
        // lanes eh hold channels 8m + 4eh + 0..3; one permlane32 swap per dword pair (m, m + 2)
        // hands lane half 0 channels 0 .. 15 and half 1 channels 16 .. 31 (half the store
        // instructions of 8-byte stores; the epilogue's stores were issue-bound)
        uint2 hb[4], lb[4];
        bool ov = false;
#pragma unroll
        for (int m = 0; m < 4; ++m) h3_split4(y[m], hb[m], lb[m], ov);
        ovf |= inside && ov;
        u4 sv[2][2];
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const uint2 A = pl ? lb[k] : hb[k], B = pl ? lb[k + 2] : hb[k + 2];
            const auto sx = __builtin_amdgcn_permlane32_swap(A.x, B.x, false, false);
            const auto sy = __builtin_amdgcn_permlane32_swap(A.y, B.y, false, false);
            sv[pl][k] = u4{sx[0], sy[0], sx[1], sy[1]};
          }
        if (inside) {
          const long s0 = hb0 + i * hstep, s1 = hb1 + i * hstep;
          *(u4*)(a.out_h3 + s0) = sv[0][0];
          *(u4*)(a.out_h3 + s1) = sv[0][1];
          *(u4*)(a.out_h3 + a.out_h3_plane + s0) = sv[1][0];
          *(u4*)(a.out_h3 + a.out_h3_plane + s1) = sv[1][1];
        }
      }
      if (a.out_x6) {
        // the x6 split (training's weight-gradient operand), stored like the h3 output: 16 bytes
        // per lane and plane after the same permlane32 swaps
        uint2 xp[3][4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          unsigned hb[4], mb[4], lb[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            hb[j] = __float_as_uint(y[m][j]) & 0xffff0000u;
            const float r = y[m][j] - __uint_as_float(hb[j]);
            mb[j] = __float_as_uint(r) & 0xffff0000u;
            lb[j] = __float_as_uint(r - __uint_as_float(mb[j]));
          }
          xp[0][m] = uint2{__builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u), __builtin_amdgcn_perm(hb[3], hb[2], 0x07060302u)};
          xp[1][m] = uint2{__builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u), __builtin_amdgcn_perm(mb[3], mb[2], 0x07060302u)};
          xp[2][m] = uint2{__builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u), __builtin_amdgcn_perm(lb[3], lb[2], 0x07060302u)};
        }
        u4 sv6[3][2];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const auto sx = __builtin_amdgcn_permlane32_swap(xp[pl][k].x, xp[pl][k + 2].x, false, false);
            const auto sy = __builtin_amdgcn_permlane32_swap(xp[pl][k].y, xp[pl][k + 2].y, false, false);
            sv6[pl][k] = u4{sx[0], sy[0], sx[1], sy[1]};
          }
        if (inside) {
          const long so = o * CO + 32 * i + 16 * eh;
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            *(u4*)(a.out_x6 + pl * a.out_x6_plane + so) = sv6[pl][0];
            *(u4*)(a.out_x6 + pl * a.out_x6_plane + so + 8) = sv6[pl][1];
          }
        }
      }
    }
  }
  if (ovf && a.range) atomicOr(a.range, 1);   // vector atomic, per offending lane (rare)
  }
}

// INT_OK: the caller guarantees an integer-valued input (ŷ). A workgroup then checks that the lo
// plane of its input window is zero (every value exact in the hi plane) and runs the INT_IN body;
// otherwise the full body.
template <int MODE, int TH, int CO, int CI, int EPI, bool INT_OK, int COT = CO, bool SEP = false,
          int ICM = 0>
// two waves per SIMD: TH = 16 (8 waves) one workgroup per CU, TH = 8 (4 waves) two — except the
// 8-row deconv, which runs where 16-row tiles would leave CUs idle (one workgroup per CU either
// way) and at N = 192 spilled under the two-workgroup register budget
__global__ void __launch_bounds__(TH / 2 * 64, TH == 8 && MODE != BM_DECONV ? 2 : 1)
h3k_kernel(const HArgs a) {
  constexpr int NSG = EPI == HE_QUANT ? 6 : 4;   // as h3k_body's
  using KK = HK<MODE, TH, COT, CI, false, NSG>;
  static_assert(KK::LDS >= HK<MODE, TH, COT, CI, true, NSG>::LDS, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[KK::LDS];
  int bid = blockIdx.x;
  const int per_ph = a.tiles_x * a.tiles_y * a.B;
  const int ph = MODE == BM_DECONV ? bid / per_ph : 0;   // phases dispatched phase-major
  bid -= ph * per_ph;
  // channel groups innermost: consecutive workgroups (dealt round-robin to the 8 XCDs) take
  // consecutive groups, so an XCD's L2 serves one group's weight slice to all its workgroups
  const int cg = bid % (CO / COT);
  bid /= CO / COT;
  const int tx = bid % a.tiles_x;
  bid /= a.tiles_x;
  const int ty = bid % a.tiles_y;
  const int b = bid / a.tiles_y;
  bool small = false;
  if constexpr (INT_OK) {
    static_assert(MODE == BM_DECONV, "INT_OK: deconv1");
    // the lo plane of the window the patch stages, all CI channels, 8 values per 16-byte load
    using P = Patch<MODE, TH>;
    constexpr int COLS = MODE == BM_CONV ? 35 : 18, PER = COLS * CI / 8;
    const int iy0 = MODE == BM_CONV ? 2 * ty * TH - 2 : ty * TH - 1;
    const int ix0 = MODE == BM_CONV ? 2 * tx * 16 - 2 : tx * 16 - 1;
    const u16* inb = a.in + a.in_plane + (long)b * a.Hin * a.Win * CI;
    // the loads issued in batches of 8 before their compares (one memory latency per batch, not
    // one per load; all of them at once held 17 × 4 registers at TH = 8 and spilled)
    constexpr int NTHR = TH / 2 * 64, IT = (P::ROWS * PER + NTHR - 1) / NTHR, IB = 8;
    unsigned bad = 0;
#pragma unroll
    for (int i0 = 0; i0 < IT; i0 += IB) {
      u4 v[IB];
#pragma unroll
      for (int k = 0; k < IB; ++k) {
        const int u = threadIdx.x + (i0 + k) * NTHR;
        int r, c;
        long off;
        if constexpr (ICM != 0) {   // chunk-major: (chunk, row, column, 8-channel half) order
          constexpr int PR = COLS * ICM / 8;
          const int q = u / (P::ROWS * PR), rem = u - q * (P::ROWS * PR);
          r = rem / PR;
          const int rem2 = rem - r * PR;
          c = rem2 / (ICM / 8);
          off = (((long)q * a.Hin + iy0 + r) * a.Win + ix0 + c) * ICM + 8 * (rem2 - c * (ICM / 8));
        } else {
          r = u / PER;
          const int rem = u - r * PER;
          c = rem / (CI / 8);
          off = ((long)(iy0 + r) * a.Win + ix0 + c) * CI + 8 * (rem - c * (CI / 8));
        }
        const int iy = iy0 + r, ix = ix0 + c;
        const bool ok = i0 + k < IT && u < P::ROWS * PER && (unsigned)iy < (unsigned)a.Hin &&
                        (unsigned)ix < (unsigned)a.Win;
        v[k] = ok ? *(const u4*)(inb + off) : u4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int k = 0; k < IB; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) bad |= v[k][e] & 0x7fff7fffu;   // ±0 only
    }
    small = __syncthreads_or(bad) == 0;
  }
  auto run = [&](auto int_in) {
    constexpr bool II = decltype(int_in)::value;
    if constexpr (MODE != BM_DECONV) {
      h3k_body<MODE, TH, CO, CI, EPI, II, 0, COT, SEP, ICM>(a, smem, b, ty, tx, cg);
    } else {
      switch (ph) {   // wave-uniform: the tap lists are compile-time per phase
        case 0: h3k_body<MODE, TH, CO, CI, EPI, II, 0, CO, false, ICM>(a, smem, b, ty, tx); break;
        case 1: h3k_body<MODE, TH, CO, CI, EPI, II, 1, CO, false, ICM>(a, smem, b, ty, tx); break;
        case 2: h3k_body<MODE, TH, CO, CI, EPI, II, 2, CO, false, ICM>(a, smem, b, ty, tx); break;
        default: h3k_body<MODE, TH, CO, CI, EPI, II, 3, CO, false, ICM>(a, smem, b, ty, tx); break;
      }
    }
  };
  if (INT_OK && small) run(std::true_type{});
  else run(std::false_type{});
}

// ---------------------------------------------------------------------------- packing
// max|w| over the tensor into trailer[0]: a grid-stride reduction, one vector atomicMax per wave
// on the bits of the non-negative float (ordered like the values) into a slot of a device-global
// table, whose last workgroup to finish (a counter beside the slot) writes the maximum to the
// trailer and zeroes the slot again. The table starts zeroed when the code object loads, so no
// launch clears it (a memset per pack was ten fill launches per training step); the host deals
// the slots round-robin, so launches in flight on different streams use different slots. One
// workgroup took 69 µs for conv2's 0.9 M weights, ten of them per training step.
constexpr unsigned kAbsmaxSlots = 256;
__device__ unsigned g_absmax_slot[kAbsmaxSlots][2];   // [0] max bits, [1] workgroups done

// workgroup bx of nbx serving one tensor (the single kernel, or one job of the batch kernel)
__device__ __forceinline__ void absmax_body(const float* __restrict__ w, long n,
                                            float* __restrict__ trailer, unsigned slot, int bx,
                                            int nbx) {
  __shared__ bool last;
  __shared__ float wmax[4];
  float m = 0.f;
  const long n4 = ((uintptr_t)w & 15) == 0 ? n / 4 : 0;   // 16-byte loads, then the tail
  for (long i = (long)bx * 256 + threadIdx.x; i < n4; i += (long)nbx * 256) {
    const f4 v = *(const f4*)(w + 4 * i);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  for (long i = 4 * n4 + (long)bx * 256 + threadIdx.x; i < n; i += (long)nbx * 256)
    m = fmaxf(m, fabsf(w[i]));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  // one atomic per workgroup: same-address atomics serialise at the L2 (one per wave of 1024
  // workgroups made the pass 13 µs)
  unsigned* s = g_absmax_slot[slot];
  if (threadIdx.x == 0) {
    atomicMax(&s[0], __float_as_uint(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]))));
    // the arrival count is an agent-scope acq_rel read-modify-write: its release orders this
    // workgroup's max before the count, its acquire orders the last workgroup's read of the
    // maximum after every other arrival (the memory model's guarantee)
    last = __hip_atomic_fetch_add(&s[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
           (unsigned)nbx - 1;
  }
  __syncthreads();
  if (last && threadIdx.x == 0) {
    trailer[0] = __uint_as_float(atomicExch(&s[0], 0u));
    __hip_atomic_store(&s[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void __launch_bounds__(256) absmax_kernel(const float* __restrict__ w, long n,
                                                     float* __restrict__ trailer, unsigned slot) {
  absmax_body(w, n, trailer, slot, blockIdx.x, gridDim.x);
}

static std::atomic<unsigned> g_next_slot{0};
static int absmax_blocks(long n) {
  const long blocks = (n + 16383) / 16384;   // ≥ 16 values per thread
  return (int)(blocks < 256 ? (blocks > 0 ? blocks : 1) : 256);
}

static int launch_absmax(const float* w, long n, float* trailer, hipStream_t st) {
  hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)absmax_blocks(n)), dim3(256), 0, st, w, n,
                     trailer, g_next_slot.fetch_add(1) % kAbsmaxSlots);
  return check_launch("absmax");
}

// σ_w = 2^(3 − ⌊log2 max|w|⌋) (max|w|·σ_w ∈ [8, 16), so hi·2¹¹ < 2¹⁵); 1 for an all-zero or
// non-finite tensor (whose products are then what fp32 makes of them)
__device__ __forceinline__ int h3_weight_exp(float mx) {
  if (!(mx > 0.f) || !(mx <= 3.40282347e38f)) return 0;
  int e;
  frexpf(mx, &e);   // mx = f·2^e, f ∈ [0.5, 1)
  // at most 2^100 (a tensor with max|w| < 2^-97: σ_w = 2^(4−e) would overflow to inf below
  // 2^-124; its scaled weights then stay below 8 and every scale finite)
  return 4 - e < 100 ? 4 - e : 100;
}

// W → two planes, per plane [blocks][2][CO][8] fp16:
// conv (W[co][ci][5][5], HM_CONV8): block c·13 + p over 8-channel chunks c and tap pairs p;
// element (block, h, co, j) = W[co][8c + j] at tap t = 2p + h = 5·ky + kx (zero for t = 25);
// deconv (W[ci][co][5][5]): the four stride phases back to back, phase p's blocks c·T_p + t over
// 16-channel chunks c with the tap order of Taps<BM_DECONV, p>; element (block, h, co, j) = W at
// input channel 16c + 8h + j.
__device__ __forceinline__ void pack_h3k_body(const float* __restrict__ w, int N, int deconv,
                                              long groups, u16* __restrict__ out,
                                              float* __restrict__ trailer, int bx, int nbx) {
  const int se = h3_weight_exp(trailer[0]);
  const float sw = ldexpf(1.0f, se);
  if (bx == 0 && threadIdx.x == 0) trailer[1] = ldexpf(1.0f, -11 - kH3SaLog2 - se);
  const int nch = N / 16;
  for (long g = (long)bx * 256 + threadIdx.x; g < groups; g += (long)nbx * 256) {
    const int co = (int)(g % N);
    long r = g / N;
    const int h = (int)(r % 2);
    int u = (int)(r / 2);   // block index
    int c, ky, kx, ci0;
    bool zero = false;
    if (deconv == 2) {   // conv1 (W[co][3][9][9]): block = step s, k-group g = 2s + h
      // (kx is the element j, or 8 for the column-8 groups; ci0 + j carries the channel instead)
      c = 0;
      ci0 = 0;
      ky = kx = 0;
      zero = true;   // resolved per element below
    } else if (!deconv) {
      c = u / kConv8Steps;
      const int t = 2 * (u - c * kConv8Steps) + h;
      zero = t >= 25;
      ky = zero ? 0 : t / 5;
      kx = zero ? 0 : t % 5;
      ci0 = 8 * c;
    } else {
      int p = 0, T = 9;
      while (true) {
        const int ny = (p >> 1) == 0 ? 3 : 2, nx = (p & 1) == 0 ? 3 : 2;
        T = ny * nx;
        if (u < nch * T) break;
        u -= nch * T;
        ++p;
      }
      const int nx = (p & 1) == 0 ? 3 : 2;
      c = u / T;
      const int t = u - c * T;
      ky = (p >> 1) == 0 ? 2 * (t / nx) : 2 * (t / nx) + 1;
      kx = (p & 1) == 0 ? 2 * (t % nx) : 2 * (t % nx) + 1;
      ci0 = 16 * c + 8 * h;
    }
    unsigned short hv[8], lv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ci = ci0 + j;
      float v;
      if (deconv == 2) {
        const int g = 2 * u + h;
        int cc = -1, yy = 0, xx = 0;
        if (g < 27) {
          cc = g / 9; yy = g % 9; xx = j;
        } else {
          const int q = 8 * (g - 27) + j;
          if (q < 27) { cc = q / 9; yy = q % 9; xx = 8; }
        }
        v = cc < 0 ? 0.f : w[(((long)co * 3 + cc) * 9 + yy) * 9 + xx] * sw;
      } else {
        v = zero ? 0.f
                 : (deconv ? w[(((long)ci * N + co) * 5 + ky) * 5 + kx]
                           : w[(((long)co * N + ci) * 5 + ky) * 5 + kx]) * sw;
      }
      const _Float16 hh = (_Float16)v;
      hv[j] = h16_bits(hh);
      lv[j] = h16_bits((_Float16)((v - (float)hh) * 2048.0f));
    }
    u4 H, L;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      H[i] = hv[2 * i] | ((unsigned)hv[2 * i + 1] << 16);
      L[i] = lv[2 * i] | ((unsigned)lv[2 * i + 1] << 16);
    }
    *(u4*)(out + g * 8) = H;
    *(u4*)(out + groups * 8 + g * 8) = L;
  }
}

__global__ void __launch_bounds__(256) pack_h3k_kernel(const float* __restrict__ w, int N, int deconv,
                                                       long groups, u16* __restrict__ out,
                                                       float* __restrict__ trailer) {
  pack_h3k_body(w, N, deconv, groups, out, trailer, blockIdx.x, gridDim.x);
}

// A packed operand [taps][K/4][N][4] fp32 → two fp16 planes [2][taps][K/8][N][8] of w·σ_w (the
// H3 engine's B-fragment layout, the x6 split_packed's with two planes), trailer after them
__device__ __forceinline__ void split_packed_h3_body(const float* __restrict__ w, int K, int N,
                                                     long groups, u16* __restrict__ out,
                                                     float* __restrict__ trailer, int bx, int nbx) {
  const int se = h3_weight_exp(trailer[0]);
  const float sw = ldexpf(1.0f, se);
  if (bx == 0 && threadIdx.x == 0) trailer[1] = ldexpf(1.0f, -11 - kH3SaLog2 - se);
  for (long g = (long)bx * 256 + threadIdx.x; g < groups; g += (long)nbx * 256) {
    const long tk = g / N;
    const int col = (int)(g - tk * N);
    const long tap = tk / (K / 8);
    const int k8 = (int)(tk - tap * (K / 8));
    const float* src = w + ((tap * (K / 4) + 2 * k8) * N + col) * 4;
    const f4 x0 = *(const f4*)src, x1 = *(const f4*)(src + (long)N * 4);
    const float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    u4 H, L;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      unsigned short hv[2], lv[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float x = v[2 * i + e] * sw;
        const _Float16 hh = (_Float16)x;
        hv[e] = h16_bits(hh);
        lv[e] = h16_bits((_Float16)((x - (float)hh) * 2048.0f));
      }
      H[i] = hv[0] | ((unsigned)hv[1] << 16);
      L[i] = lv[0] | ((unsigned)lv[1] << 16);
    }
    *(u4*)(out + g * 8) = H;
    *(u4*)(out + groups * 8 + g * 8) = L;
  }
}

__global__ void __launch_bounds__(256) split_packed_h3_kernel(const float* __restrict__ w, int K,
                                                              int N, long groups,
                                                              u16* __restrict__ out,
                                                              float* __restrict__ trailer) {
  split_packed_h3_body(w, K, N, groups, out, trailer, blockIdx.x, gridDim.x);
}

// A batch of h3 packs (iclr17_pack_h3_batch): job j owns workgroups [begin[j], begin[j+1]) of
// each launch — the absmax pass first, then the packing pass, both the single kernels' bodies.
struct H3Job {
  const float* src;
  u16* out;
  float* trailer;
  long n, groups;      // absmax values; 16-byte packing groups
  int kind, N, K, deconv;
  unsigned slot;
};
struct H3Batch {
  int n;
  int begin[ICLR17_PACK_H3_MAXJ + 1];
  H3Job job[ICLR17_PACK_H3_MAXJ];
};

__device__ __forceinline__ int h3_batch_job(const H3Batch& b, int& bx, int& nbx) {
  int j = 0;
  while (j + 1 < b.n && (int)blockIdx.x >= b.begin[j + 1]) ++j;
  bx = blockIdx.x - b.begin[j];
  nbx = b.begin[j + 1] - b.begin[j];
  return j;
}

__global__ void __launch_bounds__(256) absmax_batch_kernel(const H3Batch b) {
  int bx, nbx;
  const H3Job& J = b.job[h3_batch_job(b, bx, nbx)];
  absmax_body(J.src, J.n, J.trailer, J.slot, bx, nbx);
}

__global__ void __launch_bounds__(256) pack_h3_batch_kernel(const H3Batch b) {
  int bx, nbx;
  const H3Job& J = b.job[h3_batch_job(b, bx, nbx)];
  if (J.kind == ICLR17_PACK_H3K) pack_h3k_body(J.src, J.N, J.deconv, J.groups, J.out, J.trailer, bx, nbx);
  else split_packed_h3_body(J.src, J.K, J.N, J.groups, J.out, J.trailer, bx, nbx);
}

// fp32 → h3 planes (x·σ_a split): iclr17_h3_planes
__global__ void __launch_bounds__(256) h3_planes_kernel(const float* __restrict__ x, long n4,
                                                        long plane, u16* __restrict__ out,
                                                        int* range) {
  bool ovf = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    uint2 hb, lb;
    h3_split4(*(const f4*)(x + 4 * i), hb, lb, ovf);
    *(uint2*)(out + 4 * i) = hb;
    *(uint2*)(out + plane + 4 * i) = lb;
  }
  if (ovf && range) atomicOr(range, 1);
}

// fp32 NHWC [B][h][w][N] → the h3 form chunk-major [2][B][N/cm][h][w][cm] (iclr17_h3_planes_cm):
// a thread per 4 consecutive channels of a pixel
__global__ void __launch_bounds__(256) h3_planes_cm_kernel(const float* __restrict__ x, long n4,
                                                           int N, int cm, long hw, long plane,
                                                           u16* __restrict__ out, int* range) {
  bool ovf = false;
  const int q4 = N / 4;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const long p = i / q4;
    const int ch = 4 * (int)(i - p * q4);
    const long b = p / hw, pix = p - b * hw;
    const long o = ((b * (N / cm) + ch / cm) * hw + pix) * cm + ch % cm;
    uint2 hb, lb;
    h3_split4(*(const f4*)(x + 4 * i), hb, lb, ovf);
    *(uint2*)(out + o) = hb;
    *(uint2*)(out + plane + o) = lb;
  }
  if (ovf && range) atomicOr(range, 1);
}

// The chain's h3 layouts (the consumer's patch chunk): conv1 → conv2 and conv2 →
// conv3 chunk-major 8 (HM_CONV8's 8-channel chunks), conv3's ŷ → deconv1 and deconv1 → deconv2
// chunk-major 16 (the deconv mode's 16-channel chunks), deconv2 → deconv3 chunk-major 32.
constexpr int kConvCM = 8, kDeconvCM = 16;

// Tile height of a conv2 / deconv launch: 16 rows (8 waves, one workgroup per CU) unless that
// leaves CUs idle (fewer workgroups than the 256 CUs: training's B = 32 conv2 and deconv1), then
// 8 rows (4 waves), twice the workgroups. A pixel's arithmetic does not depend on the tile (the
// same chunk and tap order, the same per-pixel epilogue), so the results are bitwise the same.
constexpr int kCUs = 256;
inline int h3_tile_rows(int gh, int gw, int B, int phases = 1) {
  return (long)((gh + 15) / 16) * ((gw + 15) / 16) * B * phases < kCUs ? 8 : 16;
}

template <int N, bool INT_OK, int TH>
int launch_deconv_th(const HArgs& a0, hipStream_t st) {
  HArgs a = a0;
  a.tiles_y = (a.gh + TH - 1) / TH;
  a.tiles_x = (a.gw + 15) / 16;
  hipLaunchKernelGGL((h3k_kernel<BM_DECONV, TH, N, N, HE_IGDN, INT_OK, N, false, kDeconvCM>),
                     dim3(a.tiles_x * a.tiles_y * a.B * 4), dim3(TH / 2 * 64), 0, st, a);
  return check_launch("deconv_igdn_h3");
}

template <int N, bool INT_OK>
int launch_deconv(const HArgs& a, hipStream_t st) {
  return h3_tile_rows(a.gh, a.gw, a.B, 4) == 8 ? launch_deconv_th<N, INT_OK, 8>(a, st)
                                               : launch_deconv_th<N, INT_OK, 16>(a, st);
}

// conv3 + quantiser + rate on the h3 engine: 8 × 16-pixel tiles of 4 waves, each workgroup one
// 64-channel slice of the output channels (B = 64 at N = 192: 384 workgroups; conv3's 16 × 16
// output per 256² image is one 16 × 16 tile, 64 workgroups without the split), two-level sums per
// 8-channel chunk, and four DMA groups in flight (h3k_body: NSG). The slice does not change an
// element's summation order, and it does not depend on the batch, so an image's results do not
// depend on the batch it is in. Measured (B = 64 eval / B = 32 noise, one box): 64-channel slices
// 0.114 / 0.119 ms, 96-channel 0.116 / 0.166, 32-channel 0.146 / 0.111; left out earlier: 16 × 16
// tiles with 64 / 96 / 192 channels and split-K over 2 / 4 / 8 workgroups per tile with a second
// reducing launch (0.16–0.44 ms).
constexpr int kC3TH = 8, kC3COT = 64;

template <int N>
static void launch_conv3(const HArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((h3k_kernel<HM_CONV8, kC3TH, N, N, HE_QUANT, false, kC3COT, true, kConvCM>),
                     dim3(a.tiles_x * a.tiles_y * a.B * (N / kC3COT)), dim3(kC3TH / 2 * 64), 0, st, a);
}

static bool valid_cm(int cm, int N) { return cm == 0 || ((cm == 8 || cm == 16 || cm == 32) && N % cm == 0); }

}  // namespace h3k
}  // namespace iclr17

using namespace iclr17;
using namespace iclr17::h3k;

extern "C" {

size_t iclr17_h3k_weight_size(int which, int N) {
  if (N != 128 && N != 192) return 0;
  if (which == ICLR17_H3K_CONV1) return (size_t)2 * kConv1Steps * 2 * N * 8 + 8;
  if (which != ICLR17_H3K_CONV5 && which != ICLR17_H3K_DECONV5) return 0;
  // two planes of 25 (chunk, tap) blocks per 16-channel chunk (deconv) or 13 (chunk, tap pair)
  // blocks per 8-channel chunk (conv), + the 16-byte trailer
  return which == ICLR17_H3K_DECONV5 ? (size_t)2 * (N / 16) * 25 * 2 * N * 8 + 8
                                     : (size_t)2 * (N / 8) * kConv8Steps * 2 * N * 8 + 8;
}

int iclr17_pack_h3k(int which, const float* w, uint16_t* out, int N, void* stream) {
  const size_t total = iclr17_h3k_weight_size(which, N);
  ICLR17_REQUIRE(total > 0, ICLR17_EUNSUPPORTED, "pack_h3k: kind %d, N=%d unsupported", which, N);
  ICLR17_REQUIRE(w && out, ICLR17_EINVAL, "pack_h3k: null pointer");
  const long groups = (long)((total - 8) / 16);
  float* trailer = (float*)(out + (total - 8));
  hipStream_t st = (hipStream_t)stream;
  const long nw = which == ICLR17_H3K_CONV1 ? (long)N * 3 * 81 : (long)N * N * 25;
  int rc = launch_absmax(w, nw, trailer, st);
  if (rc) return rc;
  const int blocks = (int)((groups + 255) / 256 < 4096 ? (groups + 255) / 256 : 4096);
  hipLaunchKernelGGL(pack_h3k_kernel, dim3(blocks), dim3(256), 0, st, w, N,
                     which == ICLR17_H3K_DECONV5 ? 1 : which == ICLR17_H3K_CONV1 ? 2 : 0, groups,
                     out, trailer);
  return check_launch("pack_h3k");
}

size_t iclr17_split_packed_h3_size(int taps, int K, int N) {
  if (taps <= 0 || K <= 0 || K % 8 || N <= 0) return 0;
  return (size_t)2 * taps * K * N + 8;
}

int iclr17_split_packed_h3(const float* packed, int taps, int K, int N, uint16_t* planes,
                           void* stream) {
  const size_t total = iclr17_split_packed_h3_size(taps, K, N);
  ICLR17_REQUIRE(packed && planes && total > 0, ICLR17_EINVAL, "split_packed_h3: bad arguments");
  const long groups = (long)taps * (K / 8) * N;
  float* trailer = (float*)(planes + (total - 8));
  hipStream_t st = (hipStream_t)stream;
  int rc = launch_absmax(packed, (long)taps * K * N, trailer, st);
  if (rc) return rc;
  const int blocks = (int)((groups + 255) / 256 < 4096 ? (groups + 255) / 256 : 4096);
  hipLaunchKernelGGL(split_packed_h3_kernel, dim3(blocks), dim3(256), 0, st, packed, K, N, groups,
                     planes, trailer);
  return check_launch("split_packed_h3");
}

int iclr17_pack_h3_batch(const iclr17_pack_job* jobs, int n, void* stream) {
  ICLR17_REQUIRE(jobs && n >= 0 && n <= ICLR17_PACK_H3_MAXJ, ICLR17_EINVAL,
                 "pack_h3_batch: bad arguments (n=%d)", n);
  if (n == 0) return ICLR17_OK;
  H3Batch b;
  memset(&b, 0, sizeof(b));
  b.n = n;
  int pack_begin[ICLR17_PACK_H3_MAXJ + 1];
  pack_begin[0] = 0;
  for (int j = 0; j < n; ++j) {
    const iclr17_pack_job& q = jobs[j];
    H3Job& J = b.job[j];
    J.kind = q.kind;
    J.N = q.N;
    J.K = q.K;
    J.src = q.src0;
    J.out = (u16*)q.dst0;
    size_t total = 0;
    if (q.kind == ICLR17_PACK_H3K) {
      total = iclr17_h3k_weight_size(q.K, q.N);
      ICLR17_REQUIRE(total > 0, ICLR17_EUNSUPPORTED, "pack_h3_batch: job %d: kind %d, N=%d", j, q.K, q.N);
      J.n = q.K == ICLR17_H3K_CONV1 ? (long)q.N * 3 * 81 : (long)q.N * q.N * 25;
      J.deconv = q.K == ICLR17_H3K_DECONV5 ? 1 : q.K == ICLR17_H3K_CONV1 ? 2 : 0;
    } else if (q.kind == ICLR17_PACK_SPLIT_H3) {
      total = iclr17_split_packed_h3_size(q.taps, q.K, q.N);
      ICLR17_REQUIRE(total > 0, ICLR17_EINVAL, "pack_h3_batch: bad split job %d", j);
      J.n = (long)q.taps * q.K * q.N;
    } else {
      ICLR17_REQUIRE(false, ICLR17_EINVAL, "pack_h3_batch: unknown job kind %d", q.kind);
    }
    ICLR17_REQUIRE(q.src0 && q.dst0, ICLR17_EINVAL, "pack_h3_batch: null pointer (job %d)", j);
    J.groups = (long)((total - 8) / 16);
    J.trailer = (float*)(J.out + (total - 8));
    J.slot = g_next_slot.fetch_add(1) % kAbsmaxSlots;
    b.begin[j + 1] = b.begin[j] + absmax_blocks(J.n);
    const long pb = (J.groups + 255) / 256;
    pack_begin[j + 1] = pack_begin[j] + (int)(pb < 4096 ? pb : 4096);
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(absmax_batch_kernel, dim3((unsigned)b.begin[n]), dim3(256), 0, st, b);
  int rc = check_launch("absmax_batch");
  if (rc) return rc;
  memcpy(b.begin, pack_begin, sizeof(pack_begin));
  hipLaunchKernelGGL(pack_h3_batch_kernel, dim3((unsigned)b.begin[n]), dim3(256), 0, st, b);
  return check_launch("pack_h3_batch");
}

int iclr17_h3_planes(const float* x, long n, uint16_t* planes, int* range_flag, void* stream) {
  ICLR17_REQUIRE(x && planes && n >= 0 && n % 4 == 0, ICLR17_EINVAL, "h3_planes: bad arguments");
  if (n == 0) return ICLR17_OK;
  const long n4 = n / 4;
  const int blocks = (int)((n4 + 255) / 256 < 8192 ? (n4 + 255) / 256 : 8192);
  hipLaunchKernelGGL(h3_planes_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, n4, n,
                     planes, range_flag);
  return check_launch("h3_planes");
}

int iclr17_h3_planes_cm(const float* x, int B, int h, int w, int N, int cm, uint16_t* planes,
                        int* range_flag, void* stream) {
  ICLR17_REQUIRE(x && planes && B > 0 && h > 0 && w > 0 && N > 0 && N % 4 == 0 && valid_cm(cm, N) &&
                     cm != 0,
                 ICLR17_EINVAL, "h3_planes_cm: bad arguments (N=%d, cm=%d)", N, cm);
  const long n = (long)B * h * w * N, n4 = n / 4;
  const int blocks = (int)((n4 + 255) / 256 < 8192 ? (n4 + 255) / 256 : 8192);
  hipLaunchKernelGGL(h3_planes_cm_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, n4, N,
                     cm, (long)h * w, n, planes, range_flag);
  return check_launch("h3_planes_cm");
}

int iclr17_analysis_conv1_gdn_h3(const float* x, int B, int H, int W, int N,
                                 const uint16_t* w_h3k, const float* bias, const float* beta_eff,
                                 const uint16_t* gamma_h3, float* out, float* pre_out,
                                 uint16_t* out_h3, int out_cm, uint16_t* out_x6, int* range_flag,
                                 void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "conv1_gdn_h3: N=%d", N);
  ICLR17_REQUIRE(x && w_h3k && bias && beta_eff && gamma_h3 && (out || out_h3 || out_x6) && B > 0 &&
                     H > 0 && W > 0 && H % 16 == 0 && W % 16 == 0 && valid_cm(out_cm, N),
                 ICLR17_EINVAL, "conv1_gdn_h3: bad arguments");
  HArgs a;
  memset(&a, 0, sizeof(a));
  a.img = x;
  const size_t wsz = iclr17_h3k_weight_size(ICLR17_H3K_CONV1, N);
  a.w = w_h3k; a.w_plane = (long)(wsz - 8) / 2;
  a.wscale = (const float*)(w_h3k + (wsz - 8));
  a.bias = bias; a.beta = beta_eff; a.gamma_h3 = gamma_h3;
  a.gamma_scale = (const float*)(gamma_h3 + 2L * N * N);
  a.out = out;
  a.pre = pre_out;
  a.out_h3 = out_h3; a.out_h3_plane = (long)B * (H / 4) * (W / 4) * N; a.out_cm = out_cm;
  a.out_x6 = out_x6; a.out_x6_plane = a.out_h3_plane;
  a.range = range_flag;
  a.B = B; a.Hin = H; a.Win = W; a.Hout = H / 4; a.Wout = W / 4;
  a.gh = H / 4; a.gw = W / 4;
  constexpr int TH = 16;
  a.tiles_y = (a.gh + TH - 1) / TH;
  a.tiles_x = (a.gw + 15) / 16;
  const dim3 grid(a.tiles_x * a.tiles_y * B);
  if (N == 192)
    hipLaunchKernelGGL((h3k_kernel<HM_CONV1, TH, 192, 3, HE_GDN, false>), grid, dim3(TH / 2 * 64), 0,
                       (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL((h3k_kernel<HM_CONV1, TH, 128, 3, HE_GDN, false>), grid, dim3(TH / 2 * 64), 0,
                       (hipStream_t)stream, a);
  return check_launch("conv1_gdn_h3");
}

int iclr17_analysis_conv2_gdn_h3(const uint16_t* in_h3, int B, int H, int W, int N,
                                 const uint16_t* w_h3k, const float* bias, const float* beta_eff,
                                 const uint16_t* gamma_h3, float* out, float* pre_out,
                                 uint16_t* out_h3, int out_cm, uint16_t* out_x6, int* range_flag,
                                 void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "conv2_gdn_h3: N=%d", N);
  ICLR17_REQUIRE(in_h3 && w_h3k && bias && beta_eff && gamma_h3 && (out || out_h3 || out_x6) &&
                     B > 0 && H > 0 && W > 0 && H % 16 == 0 && W % 16 == 0 && valid_cm(out_cm, N),
                 ICLR17_EINVAL, "conv2_gdn_h3: bad arguments");
  HArgs a;
  memset(&a, 0, sizeof(a));
  const int h = H / 4, w = W / 4;
  a.in = in_h3; a.in_plane = (long)B * h * w * N;
  const size_t wsz = iclr17_h3k_weight_size(ICLR17_H3K_CONV5, N);
  a.w = w_h3k; a.w_plane = (long)(wsz - 8) / 2;
  a.wscale = (const float*)(w_h3k + (wsz - 8));
  a.bias = bias; a.beta = beta_eff; a.gamma_h3 = gamma_h3;
  a.gamma_scale = (const float*)(gamma_h3 + 2L * N * N);
  a.out = out;
  a.pre = pre_out;
  a.out_h3 = out_h3; a.out_h3_plane = (long)B * (h / 2) * (w / 2) * N; a.out_cm = out_cm;
  a.out_x6 = out_x6; a.out_x6_plane = a.out_h3_plane;
  a.range = range_flag;
  a.B = B; a.Hin = h; a.Win = w; a.Hout = h / 2; a.Wout = w / 2;
  a.gh = h / 2; a.gw = w / 2;
  const int TH = h3_tile_rows(a.gh, a.gw, B);
  a.tiles_y = (a.gh + TH - 1) / TH;
  a.tiles_x = (a.gw + 15) / 16;
  const dim3 grid(a.tiles_x * a.tiles_y * B), block(TH / 2 * 64);
  hipStream_t st = (hipStream_t)stream;
  if (TH == 8) {
    if (N == 192)
      hipLaunchKernelGGL((h3k_kernel<HM_CONV8, 8, 192, 192, HE_GDN, false, 192, false, kConvCM>), grid, block, 0, st, a);
    else
      hipLaunchKernelGGL((h3k_kernel<HM_CONV8, 8, 128, 128, HE_GDN, false, 128, false, kConvCM>), grid, block, 0, st, a);
  } else if (N == 192) {
    hipLaunchKernelGGL((h3k_kernel<HM_CONV8, 16, 192, 192, HE_GDN, false, 192, false, kConvCM>), grid, block, 0, st, a);
  } else {
    hipLaunchKernelGGL((h3k_kernel<HM_CONV8, 16, 128, 128, HE_GDN, false, 128, false, kConvCM>), grid, block, 0, st, a);
  }
  return check_launch("conv2_gdn_h3");
}

int iclr17_synthesis_deconv_igdn_h3(const uint16_t* in_h3, int B, int h, int w, int N,
                                    const uint16_t* w_h3k, const float* bias,
                                    const float* beta_eff, const uint16_t* gamma_h3,
                                    float* out, float* pre_out, uint16_t* out_h3, uint16_t* out_x6,
                                    int out_cm, int int_in, int* range_flag, void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "deconv_igdn_h3: N=%d", N);
  ICLR17_REQUIRE(in_h3 && w_h3k && bias && beta_eff && gamma_h3 && (out || out_h3 || out_x6) &&
                     B > 0 && h > 0 && w > 0 && valid_cm(out_cm, N),
                 ICLR17_EINVAL, "deconv_igdn_h3: bad arguments");
  HArgs a;
  memset(&a, 0, sizeof(a));
  a.in = in_h3; a.in_plane = (long)B * h * w * N;
  const size_t wsz = iclr17_h3k_weight_size(ICLR17_H3K_DECONV5, N);
  a.w = w_h3k; a.w_plane = (long)(wsz - 8) / 2;
  a.wscale = (const float*)(w_h3k + (wsz - 8));
  a.bias = bias; a.beta = beta_eff; a.gamma_h3 = gamma_h3;
  a.gamma_scale = (const float*)(gamma_h3 + 2L * N * N);
  a.out = out;
  a.pre = pre_out;
  a.out_h3 = out_h3; a.out_h3_plane = (long)B * 4 * h * w * N;
  a.out_x6 = out_x6; a.out_x6_plane = (long)B * 4 * h * w * N;
  a.out_cm = out_cm;
  a.range = range_flag;
  a.B = B; a.Hin = h; a.Win = w; a.Hout = 2 * h; a.Wout = 2 * w;
  a.gh = h; a.gw = w;
  hipStream_t st = (hipStream_t)stream;
  if (int_in) return N == 192 ? launch_deconv<192, true>(a, st) : launch_deconv<128, true>(a, st);
  return N == 192 ? launch_deconv<192, false>(a, st) : launch_deconv<128, false>(a, st);
}

int iclr17_conv3_h3_partials_per_image(int B, int H, int W, int N, int quant_mode) {
  (void)quant_mode;
  if (B <= 0 || H <= 0 || W <= 0 || H % 16 || W % 16 || (N != 128 && N != 192)) return 0;
  return ((H / 16 + kC3TH - 1) / kC3TH) * ((W / 16 + 15) / 16) * (N / kC3COT);
}

int iclr17_analysis_conv3_quant_rate_h3(const uint16_t* in_h3, int B, int H, int W, int N,
                                        const uint16_t* w_h3k, int quant_mode, const float* noise,
                                        const float* rate_packed, const float* rate_table,
                                        float* y_out, float* y_hat, uint16_t* y_hat_h3, int out_cm,
                                        double* bits_partial, int* range_flag, void* stream) {
  ICLR17_REQUIRE(N == 128 || N == 192, ICLR17_EUNSUPPORTED, "conv3_quant_rate_h3: N=%d", N);
  ICLR17_REQUIRE(B > 0 && H > 0 && W > 0 && H % 16 == 0 && W % 16 == 0 && valid_cm(out_cm, N),
                 ICLR17_EINVAL, "conv3_quant_rate_h3: bad shape %dx%d / layout %d", H, W, out_cm);
  ICLR17_REQUIRE(in_h3 && w_h3k && rate_packed && y_hat && bits_partial, ICLR17_EINVAL,
                 "conv3_quant_rate_h3: null pointer");
  ICLR17_REQUIRE(quant_mode == ICLR17_QUANT_ROUND || (quant_mode == ICLR17_QUANT_NOISE && noise),
                 ICLR17_EINVAL, "conv3_quant_rate_h3: bad quant mode %d / missing noise", quant_mode);
  HArgs a;
  memset(&a, 0, sizeof(a));
  const int h = H / 8, w = W / 8;
  a.in = in_h3; a.in_plane = (long)B * h * w * N;
  const size_t wsz = iclr17_h3k_weight_size(ICLR17_H3K_CONV5, N);
  a.w = w_h3k; a.w_plane = (long)(wsz - 8) / 2;
  a.wscale = (const float*)(w_h3k + (wsz - 8));
  a.out = y_out;
  a.out_h3 = y_hat_h3; a.out_h3_plane = (long)B * (h / 2) * (w / 2) * N; a.out_cm = out_cm;
  a.range = range_flag;
  a.qmode = quant_mode; a.noise = noise; a.rate = rate_packed;
  a.rtab = rate_table; a.yhat = y_hat; a.partial = bits_partial;
  a.B = B; a.Hin = h; a.Win = w; a.Hout = h / 2; a.Wout = w / 2;
  a.gh = h / 2; a.gw = w / 2;
  a.tiles_y = (a.gh + kC3TH - 1) / kC3TH;
  a.tiles_x = (a.gw + 15) / 16;
  a.T = iclr17_conv3_h3_partials_per_image(B, H, W, N, quant_mode);
  hipStream_t st = (hipStream_t)stream;
  if (N == 192) launch_conv3<192>(a, st);
  else launch_conv3<128>(a, st);
  return check_launch("conv3_quant_rate_h3");
}

}  // extern "C"
