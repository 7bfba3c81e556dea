// Shared device/host helpers for the iclr17 gfx950 kernels.
//
// Numerics contract (fp32 parity mode): every contraction runs on the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32: a k-ordered fmaf chain, no reduced-precision internals); every
// elementwise step the reference evaluates as separate PyTorch ops (mul, add, sqrt, div …)
// is evaluated as separate correctly-rounded ops here too — the library is compiled with
// -ffp-contract=off so no mul+add pair is silently fused.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/iclr17.h"

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));   // 8 packed bf16
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));

namespace iclr17 {

// ----------------------------------------------------------------------------- errors
void set_error(int code, const char* fmt, ...);
int check_launch(const char* what);

#define ICLR17_REQUIRE(cond, code, ...)          \
  do {                                           \
    if (!(cond)) {                               \
      ::iclr17::set_error((code), __VA_ARGS__);  \
      return (code);                             \
    }                                            \
  } while (0)

// ----------------------------------------------------------------------------- LDS-DMA sync
// Publishes LDS-DMA (global_load_lds) data to the whole workgroup: this wave's DMAs landed
// (s_waitcnt vmcnt(0)), then the barrier. A bare __syncthreads() is NOT enough: the workgroup
// release fence waits only for lgkmcnt, and the compiler adds a vmcnt wait before a barrier only
// when it proves that this wave's own LDS reads after it may alias the DMA. conv1_gdn_kernel's
// main loop compiled to `s_waitcnt lgkmcnt(0); s_barrier` with the previous step's weight DMA in
// flight, and one run in ~20 read a stale B stage (a rare run-to-run difference in fp32 conv1).
__device__ __forceinline__ void dma_barrier() {
  __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8));   // vmcnt(0), exp/lgkm untouched
  __syncthreads();
}

// ----------------------------------------------------------------------------- MFMA
__device__ __forceinline__ f4 mfma16(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Two-level accumulation . A long MFMA accumulation chain puts every
// rounding at the scale of the whole running sum: for conv2 (K = 4800) the exact-f32 16x16x4
// chain lands ~10x farther from the exact value than the reference's oneDNN conv, and
// v_mfma_f32_16x16x32_bf16 is not a single correctly rounded C + Σ a·b (tools/mfma_numerics.hip:
// ~0.6-1.5 ulp of C per instruction, unbiased), so the x6 mode's six part products per k-block
// landed ~6x farther still. Each 32-deep k-block is therefore summed from zero in a short chain of
// its own and added to the accumulator with one correctly rounded VALU add; the block sums are
// ~1/sqrt(K/32) of the total, so their own rounding is small. conv2+GDN2 pre-activations: rms
// error vs fp64 2e-5 (fp32) / 1.1e-4 (x6) → below oneDNN's 2.1e-6.
constexpr bool kSepAcc = true;

// x6 product of one 32-deep k-block (lo·hi + hi·lo + mid·mid + mid·hi + hi·mid + hi·hi, small
// terms first) onto acc[mt][nt]. With two-level accumulation (SEP) the block sum is a fresh six-MFMA chain
// whose add into acc is deferred to the NEXT call (X6Acc holds it), so the add never waits on
// its own chain, and a scheduling barrier keeps the chains in program order: at most two block
// sums are live (letting the scheduler interleave every chain of a k-step, as it does with
// in-place accumulation, doubled the accumulator registers). Call x6_flush after the last one.
struct X6Acc {
  f4 pend;
  int pm = -1, pn = -1;   // compile-time constants once the callers' loops are unrolled
};
// instruction classes that may still move across the barrier (SALU, VMEM, DS)
constexpr int kX6SchedMask = 0x0004 | 0x0010 | 0x0080;

template <bool SEP, int MT, int NT>
__device__ __forceinline__ void mfma_x6(f4 (&acc)[MT][NT], X6Acc& st, int mt, int nt,
                                        const bf8& Ah, const bf8& Am, const bf8& Al,
                                        const bf8& Bh, const bf8& Bm, const bf8& Bl) {
  f4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Al, Bh, SEP ? f4{0.f, 0.f, 0.f, 0.f} : acc[mt][nt],
                                                 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Am, Bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Am, Bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah, Bh, c, 0, 0, 0);
  if constexpr (SEP) {
    if (st.pm >= 0) acc[st.pm][st.pn] += st.pend;
    st.pend = c;
    st.pm = mt;
    st.pn = nt;
    if constexpr (kX6SchedMask >= 0) __builtin_amdgcn_sched_barrier(kX6SchedMask);
  } else {
    acc[mt][nt] = c;
  }
}

template <bool SEP, int MT, int NT>
__device__ __forceinline__ void x6_flush(f4 (&acc)[MT][NT], X6Acc& st) {
  if constexpr (SEP) {
    if (st.pm >= 0) acc[st.pm][st.pn] += st.pend;
    st.pm = -1;
  }
}

// ----------------------------------------------------------------------------- rate model
// Packed per-channel BitEstimator parameters, rows of C floats:
//   0..2  softplus(h1), b1, tanh(a1)     3..5  layer 2     6..8  layer 3
//   9,10  softplus(h4), b4
constexpr int kRateRows = 11;

__device__ __forceinline__ float bitparm_cdf(float v, const float* __restrict__ rp, int C, int c) {
  // models/bitEstimator.py:20-25, evaluated as the reference's separate fp32 ops
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float sp = rp[(3 * k + 0) * C + c];
    const float bb = rp[(3 * k + 1) * C + c];
    const float ta = rp[(3 * k + 2) * C + c];
    const float t = v * sp + bb;          // x * softplus(h) + b
    v = t + tanhf(t) * ta;                // x + tanh(x) * tanh(a)
  }
  const float t = v * rp[9 * C + c] + rp[10 * C + c];
  return 1.0f / (1.0f + expf(-t));        // torch.sigmoid
}

// model.py:71-73 per element: clamp(-log(F(z+.5) - F(z-.5) + 1e-10) / ln 2, 0, 50)
__device__ __forceinline__ float element_bits(float z, const float* __restrict__ rp, int C, int c) {
  const float hi = bitparm_cdf(z + 0.5f, rp, C, c);
  const float lo = bitparm_cdf(z - 0.5f, rp, C, c);
  const float prob = hi - lo;
  float bits = (-1.0f * logf(prob + 1e-10f)) / 0.693147182464599609375f;  // float(math.log(2))
  bits = fminf(fmaxf(bits, 0.0f), 50.0f);
  return bits;
}

// Exact three-way bf16 split of 8 floats: x = hi + mid + lo, each part a bf16 (truncation
// split: hi = the top 8 significand bits, mid the next 8, lo the last 8, all exact in fp32).
// Packed as bf16x8 fragments (u4 = 8 × 16 bits).
__device__ __forceinline__ void split8(const f4& x0, const f4& x1, u4& hi, u4& mi, u4& lo) {
  const float x[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  unsigned h[8], m[8], l[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = __float_as_uint(x[i]) & 0xffff0000u;
    const float r = x[i] - __uint_as_float(h[i]);
    m[i] = __float_as_uint(r) & 0xffff0000u;
    l[i] = __float_as_uint(r - __uint_as_float(m[i]));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    hi[i] = __builtin_amdgcn_perm(h[2 * i + 1], h[2 * i], 0x07060302u);
    mi[i] = __builtin_amdgcn_perm(m[2 * i + 1], m[2 * i], 0x07060302u);
    lo[i] = __builtin_amdgcn_perm(l[2 * i + 1], l[2 * i], 0x07060302u);
  }
}

// Group g (8 consecutive k of one column) of a packed operand [taps][K/4][N][4] fp32 → planes
// [3][taps][K/8][N][8] (plane = taps·K·N uint16): iclr17_split_packed.
__device__ __forceinline__ void split_packed_group(const float* __restrict__ w, int K, int N,
                                                   long plane, unsigned short* __restrict__ planes,
                                                   long g) {
  const long tk = g / N;
  const int col = (int)(g - tk * N);
  const long tap = tk / (K / 8);
  const int k8 = (int)(tk - tap * (K / 8));
  const float* src = w + ((tap * (K / 4) + 2 * k8) * N + col) * 4;
  u4 hi, mi, lo;
  split8(*(const f4*)src, *(const f4*)(src + (long)N * 4), hi, mi, lo);
  *(u4*)(planes + g * 8) = hi;
  *(u4*)(planes + plane + g * 8) = mi;
  *(u4*)(planes + 2 * plane + g * 8) = lo;
}

// ----------------------------------------------------------------------------- h3 form
// The h3 operand form: three fp16 part products per MAC on the f16 MFMA instead of the x6 mode's
// six bf16 ones. An activation x is stored as two fp16 planes of a = x·σ_a (σ_a = 2^kH3SaLog2):
//   hi = rne16(a),  lo = rne16((a − hi)·2¹¹)      (22 significant bits; a − hi is exact in fp32)
// a weight w the same way with its own power-of-two σ_w (max|w|·σ_w ∈ [8, 16), chosen per tensor
// at packing), and a product as
//   2¹¹·a·v ≈ (hi_w·2¹¹)·hi_a + lo_w·hi_a + hi_w·lo_a                 (lo·lo, < 2⁻²², dropped)
// accumulated in fp32 and scaled back by 2⁻¹¹/(σ_a·σ_w), a power of two. The lo plane keeps 11
// more binades below hi, so values down to 2⁻¹³/σ_a keep all 22 bits and smaller ones an absolute
// error below 2⁻³⁶/σ_a; a ≥ 65520 (|x| ≥ 2^22 at σ_a = 2⁻⁶) does not fit and is reported through
// the caller's range flag. The f16 MFMA keeps fp16 subnormal operands (tools/h3_numerics.hip) and
// runs at the bf16 rate; against float64 a K = 1728 / 4800 dot product lands at 0.7× the x6 chain's
// rms error (fewer roundings of the running sum; profiles/r05_h3_numerics.txt).
constexpr int kH3SaLog2 = -6;
constexpr float kH3Sa = 1.0f / 64.0f;
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned short h16_bits(_Float16 v) {
  return __builtin_bit_cast(unsigned short, v);
}

// 4 consecutive values x → 8 bytes of each plane of a = x·σ_a: hi = rne16(a), lo = rne16((a − hi)·2¹¹),
// converted two at a time (v_cvt_pk_f16_f32); ovf |= one of the four does not fit (|a| ≥ 65520 — an
// infinite value counts too: its results are not finite either way). The check is one compare on
// the largest |a| of the four (NaN ignored by the max), not two per value: in the GDN epilogues
// the per-value compares were a tenth of the VALU work
__device__ __forceinline__ void h3_split4(const f4& x, uint2& hi, uint2& lo, bool& ovf) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 a0 = f2{x[0], x[1]} * kH3Sa, a1 = f2{x[2], x[3]} * kH3Sa;
  const h2v h0 = __builtin_convertvector(a0, h2v), h1 = __builtin_convertvector(a1, h2v);
  const h2v l0 = __builtin_convertvector((a0 - __builtin_convertvector(h0, f2)) * 2048.0f, h2v);
  const h2v l1 = __builtin_convertvector((a1 - __builtin_convertvector(h1, f2)) * 2048.0f, h2v);
  hi = uint2{__builtin_bit_cast(unsigned, h0), __builtin_bit_cast(unsigned, h1)};
  lo = uint2{__builtin_bit_cast(unsigned, l0), __builtin_bit_cast(unsigned, l1)};
  const float m = fmaxf(fmaxf(fabsf(a0.x), fabsf(a0.y)), fmaxf(fabsf(a1.x), fabsf(a1.y)));
  ovf |= m >= 65520.0f;
}

// 8 fp16 values × 2¹¹ (exact while they stay below 32: the weight scaling guarantees it)
// (one 8-wide vector multiply: the per-dword form of this compiled to one v_pk_mul_f16 whose
// result was copied into all four dwords)
__device__ __forceinline__ u4 h3_x2048(const u4& v) {
  const h8v k = {(_Float16)2048.0f, (_Float16)2048.0f, (_Float16)2048.0f, (_Float16)2048.0f,
                 (_Float16)2048.0f, (_Float16)2048.0f, (_Float16)2048.0f, (_Float16)2048.0f};
  return __builtin_bit_cast(u4, __builtin_bit_cast(h8v, v) * k);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace iclr17
