// Helpers shared by the k5 engines on v_mfma_f32_32x32x16_bf16: the bf16 throughput engine
// (engine_bf16.hip) and its x6 form (engine_x6k.hip). Tap geometry of the k5 s2 convs and
// transposed convs, the halo-patch layout, LDS-DMA and counted-wait helpers.
#pragma once

#include "common.h"

namespace iclr17 {
namespace bfm {

typedef unsigned short u16;

enum BMode : int { BM_CONV = 0, BM_DECONV = 1 };
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  const bf2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// threadIdx.x re-materialised where it is used: keeps the compiler from hoisting per-lane
// address arithmetic out of a loop into registers it then spills (a scratch reload is a VMEM op,
// and its vmcnt wait would also wait for every load in flight)
__device__ __forceinline__ int fresh_tid() {
  int v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"((int)threadIdx.x));
  return v;
}

// Orders one wave's LDS accesses across its lanes (a lane reading what another lane wrote): a
// wavefront-scope acquire/release fence, which the memory model needs for the cross-lane
// exchange, plus a wave barrier so the scheduler moves no LDS op across it. DS instructions of
// one wave already execute in order, so this emits no instruction.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

typedef float f16v __attribute__((ext_vector_type(16)));

// C[32][32] += A[32][16]·B[16][32]: lane l (r = l & 31, h = l >> 5) holds A[r][8h + j] and
// B[8h + j][r] (j = 0..7); C register i is C[(i & 3) + 8·(i >> 2) + 4h][r]
__device__ __forceinline__ f16v mfma32(const u4& a, const u4& b, const f16v& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, a),
                                                 __builtin_bit_cast(bf8, b), c, 0, 0, 0);
}

// s_waitcnt vmcnt(N) (lgkm / exp untouched) + workgroup barrier
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void vm_barrier() {
  // every LDS-DMA of this wave landed (vmcnt(0)), then the workgroup barrier
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------- tap geometry
// conv (k5 s2 p2): tap t = 5·ky + kx reads patch row 2·r + ky, column 2·m + kx.
// deconv (k5 s2 p2 op1), stride phase (py, px): output (2g + p) sums k ≡ p (mod 2), input
// g + (p + 2 − k)/2, i.e. offsets d ∈ {1, 0, −1} (p = 0: k = 0, 2, 4) or {1, 0} (p = 1: k = 1, 3).
template <int MODE, int PH>
struct Taps {
  static constexpr int NY = MODE == BM_CONV ? 5 : ((PH >> 1) == 0 ? 3 : 2);
  static constexpr int NX = MODE == BM_CONV ? 5 : ((PH & 1) == 0 ? 3 : 2);
  static constexpr int T = NY * NX;
  static constexpr int S = (T + 1) / 2;   // k32 steps per chunk
  __host__ __device__ static constexpr int ky(int t) {
    return MODE == BM_CONV ? t / 5 : ((PH >> 1) == 0 ? 2 * (t / NX) : 2 * (t / NX) + 1);
  }
  __host__ __device__ static constexpr int kx(int t) {
    return MODE == BM_CONV ? t % 5 : ((PH & 1) == 0 ? 2 * (t % NX) : 2 * (t % NX) + 1);
  }
};

template <int MODE, int TH>
struct Patch {
  // A patch row holds, per column plane (conv: even / odd input columns; deconv: one), the two
  // 8-channel halves of the chunk as separate runs of 18 16-byte slots: consecutive pixels of a
  // fragment read are 16 bytes apart (conflict-free ds_read_b128).
  // conv: rows 2·TH+3, [plane 2][half 2][slot 18]; deconv: rows TH+2, [half 2][slot 18]
  static constexpr int ROWS = MODE == BM_CONV ? 2 * TH + 3 : TH + 2;
  static constexpr int HALF = 18 * 16;                 // bytes of one half-run
  static constexpr int ROWB = MODE == BM_CONV ? 4 * HALF : 2 * HALF;
  static constexpr int BYTES = ROWS * ROWB;
  static constexpr int NQI = (BYTES + 1023) / 1024;   // LDS-DMA wave-instructions per chunk
  static constexpr int BUF = NQI * 1024;               // buffer bytes (tail slots load zeros)
  // byte offset of (patch row pr, patch column pc), half 0
  __host__ __device__ static constexpr int off(int pr, int pc) {
    return MODE == BM_CONV ? pr * ROWB + (pc & 1) * 2 * HALF + (pc >> 1) * 16 : pr * ROWB + pc * 16;
  }
  // tap offset relative to tile pixel (r, m) = (0, 0)
  template <int PH>
  __host__ __device__ static constexpr int tap_off(int t) {
    using TP = Taps<MODE, PH>;
    if (t >= TP::T) return 0;   // the zero-weight pad tap reads any valid slot
    if (MODE == BM_CONV) return off(TP::ky(t), TP::kx(t));
    const int dy = ((PH >> 1) + 2 - TP::ky(t)) / 2, dx = ((PH & 1) + 2 - TP::kx(t)) / 2;
    return off(dy + 1, dx + 1);
  }
};

}  // namespace bfm
}  // namespace iclr17
