// Diagnostic (GPU): can three fp16 part products stand in for the x6 mode's six bf16 ones?
//
// The "h3" operand form: a = x·σ is split as hi = rne16(a), lo = rne16((a − hi)·2¹¹) (two fp16
// planes, 22 significant bits), the weights the same way with their own power-of-two σ_w, and
//   2¹¹·a·w ≈ hi_a·(hi_w·2¹¹) + hi_a·lo_w + lo_a·hi_w
// on v_mfma_f32_32x32x16_f16 (lo·lo, ~2⁻²² of a product, dropped). This tool checks on gfx950:
//   1. fp16 subnormal operands are not flushed by the f16 MFMA (lo of small values lives there);
//   2. the error against float64 of K-deep dot products in four forms: x6 (six bf16 MFMAs in place,
//      the engine's order), h3 (three f16 MFMAs in place), bf16 (one product), and the exact-f32
//      16x16x4 chain — rms and max relative to the rms of the outputs, over activations spread
//      over many binades (log-uniform magnitudes) and Gaussian weights.
//   hipcc --offload-arch=gfx950 -O2 tools/h3_numerics.hip -o /tmp/h3n && /tmp/h3n
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// one wave: C[32][32] = Σ_k A[r][k]·B[k][c]; planes are [P][32][K] (A) and [P][K][32] (B) u16
// mode 0: x6 (bf16 planes hi, mid, lo), 1: h3 (A planes hi·2¹¹, lo, hi; B planes hi, lo),
// 2: bf16 (one plane each)
__global__ void dot_kernel(const uint16_t* A, const uint16_t* B, int K, int mode, float* C) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  f16v acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const long pa = 32L * K, pb = 32L * K;
  for (int k0 = 0; k0 < K; k0 += 16) {
    u4 a[3], b[3];
    for (int p = 0; p < 3; ++p) {
      uint16_t va[8], vb[8];
      for (int j = 0; j < 8; ++j) {
        va[j] = A[p * pa + (long)r * K + k0 + 8 * h + j];
        vb[j] = B[p * pb + (long)(k0 + 8 * h + j) * 32 + r];
      }
      memcpy(&a[p], va, 16);
      memcpy(&b[p], vb, 16);
    }
    if (mode == 0) {
      auto m = [](const u4& x, const u4& y, f16v c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8, x), __builtin_bit_cast(b8, y), c, 0, 0, 0);
      };
      f16v t = m(a[2], b[0], acc);   // lo·hi, hi·lo, mid·mid, mid·hi, hi·mid, hi·hi
      t = m(a[0], b[2], t);
      t = m(a[1], b[1], t);
      t = m(a[1], b[0], t);
      t = m(a[0], b[1], t);
      acc = m(a[0], b[0], t);
    } else if (mode == 1) {
      auto m = [](const u4& x, const u4& y, f16v c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, x), __builtin_bit_cast(h8, y), c, 0, 0, 0);
      };
      f16v t = m(a[2], b[1], acc);   // hi_w·lo_a, lo_w·hi_a, (hi_w·2¹¹)·hi_a
      t = m(a[1], b[0], t);
      acc = m(a[0], b[0], t);
    } else {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(b8, a[0]), __builtin_bit_cast(b8, b[0]), acc, 0, 0, 0);
    }
  }
  for (int i = 0; i < 16; ++i) C[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = acc[i];
}

// exact-f32 reference chain on the f32 MFMA: one k at a time per lane group
__global__ void f32_kernel(const float* A, const float* B, int K, float* C) {
  // 16x16x4: lane l: A[l&15][k0 + (l>>4)], B[k0 + (l>>4)][l&15]; four 16×16 quadrants
  const int l = threadIdx.x;
  for (int q = 0; q < 4; ++q) {
    const int r0 = 16 * (q >> 1), c0 = 16 * (q & 1);
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < K; k0 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[(long)(r0 + (l & 15)) * K + k0 + (l >> 4)],
                                                 B[(long)(k0 + (l >> 4)) * 32 + c0 + (l & 15)], acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[(r0 + (l >> 4) * 4 + i) * 32 + c0 + (l & 15)] = acc[i];
  }
}

// subnormal probe: A row 0 = s (fp16 bits), B = 1.0; C[0][c] = 16·s if subnormals are kept
__global__ void denorm_kernel(uint16_t s, float* out) {
  const int l = threadIdx.x;
  uint16_t va[8], vb[8];
  for (int j = 0; j < 8; ++j) { va[j] = s; vb[j] = 0x3c00; }
  u4 a, b;
  memcpy(&a, va, 16);
  memcpy(&b, vb, 16);
  f16v acc;
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), acc, 0, 0, 0);
  if (l == 0) out[0] = acc[0];
}

static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; }
static float h2f(uint16_t u) { _Float16 h; memcpy(&h, &u, 2); return (float)h; }
static uint16_t bf_hi(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
static float bf(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }

static void split_x6(float x, uint16_t p[3]) {
  p[0] = bf_hi(x);
  const float r = x - bf(p[0]);
  p[1] = bf_hi(r);
  const float r2 = r - bf(p[1]);
  uint32_t u; memcpy(&u, &r2, 4);
  p[2] = (uint16_t)(u >> 16);
}
// h3: a = x·σ (exact, pow2), hi = rne16(a), lo = rne16((a − hi)·2¹¹)
static void split_h3(float x, float sigma, uint16_t& hi, uint16_t& lo) {
  const float a = x * sigma;
  hi = f2h(a);
  lo = f2h((a - h2f(hi)) * 2048.f);
}

int main() {
  float* dd;
  CK(hipMalloc(&dd, 4));
  printf("f16 MFMA subnormal operands (A = s, B = 1, sum of 16 products):\n");
  const uint16_t probes[] = {0x0001, 0x0010, 0x0200, 0x03ff, 0x0400};
  for (uint16_t s : probes) {
    hipLaunchKernelGGL(denorm_kernel, dim3(1), dim3(64), 0, 0, s, dd);
    float v;
    CK(hipMemcpy(&v, dd, 4, hipMemcpyDeviceToHost));
    printf("  s = 0x%04x (%.6g): got %.9g, expected %.9g -> %s\n", s, h2f(s), v, 16.0 * h2f(s),
           v == (float)(16.0 * h2f(s)) ? "kept" : "FLUSHED/DIFFERENT");
  }

  std::mt19937_64 rng(1234);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::uniform_real_distribution<float> ud(-1.f, 1.f);
  const int Ks[] = {1728, 4800};
  for (int K : Ks) {
    for (int dist = 0; dist < 3; ++dist) {
      // activations B[K][32]: dist 0 Gaussian, 1 log-uniform over 2^-12 .. 2^4 with random sign,
      // 2 ReLU-like (half zeros) Gaussian ×8
      std::vector<float> A(32L * K), B(32L * K);
      for (auto& v : A) v = 0.05f * nd(rng);
      for (auto& v : B) {
        if (dist == 0) v = nd(rng);
        else if (dist == 1) v = (ud(rng) < 0 ? -1.f : 1.f) * std::exp2(-12.f + 16.f * (0.5f + 0.5f * ud(rng)));
        else { const float g = nd(rng); v = g > 0 ? 8.f * g : 0.f; }
      }
      std::vector<double> ref(1024);
      double rms = 0;
      for (int r = 0; r < 32; ++r)
        for (int c = 0; c < 32; ++c) {
          double s = 0;
          for (int k = 0; k < K; ++k) s += (double)A[(long)r * K + k] * (double)B[(long)k * 32 + c];
          ref[r * 32 + c] = s;
          rms += s * s;
        }
      rms = std::sqrt(rms / 1024);
      // weight σ_w: max|w|·σ_w in [8, 16); activation σ_a = 2^-4
      float mw = 0;
      for (float v : A) mw = std::fmax(mw, std::fabs(v));
      const float sw = std::exp2(3.f - std::floor(std::log2(mw))), sa = 0.0625f;
      std::vector<uint16_t> A6(3 * 32L * K), B6(3 * 32L * K), AH(3 * 32L * K), BH(3 * 32L * K, 0);
      for (int r = 0; r < 32; ++r)
        for (int k = 0; k < K; ++k) {
          const long i = (long)r * K + k, pl = 32L * K;
          uint16_t p[3];
          split_x6(A[i], p);
          for (int q = 0; q < 3; ++q) A6[q * pl + i] = p[q];
          uint16_t hi, lo;
          split_h3(A[i], sw, hi, lo);
          AH[i] = f2h(h2f(hi) * 2048.f);
          AH[pl + i] = lo;
          AH[2 * pl + i] = hi;
        }
      for (long i = 0; i < 32L * K; ++i) {
        const long pl = 32L * K;
        uint16_t p[3];
        split_x6(B[i], p);
        for (int q = 0; q < 3; ++q) B6[q * pl + i] = p[q];
        uint16_t hi, lo;
        split_h3(B[i], sa, hi, lo);
        BH[i] = hi;
        BH[pl + i] = lo;
      }
      uint16_t *dA, *dB;
      float *dC, *dAf, *dBf;
      CK(hipMalloc(&dA, 6 * 32L * K));
      CK(hipMalloc(&dB, 6 * 32L * K));
      CK(hipMalloc(&dC, 4096));
      CK(hipMalloc(&dAf, 4 * 32L * K));
      CK(hipMalloc(&dBf, 4 * 32L * K));
      std::vector<float> C(1024);
      const char* names[] = {"x6 (6 bf16)", "h3 (3 f16)", "bf16 (1)", "f32 chain"};
      const char* dn[] = {"gaussian", "log-uniform 2^-12..2^4", "relu-like x8"};
      printf("K = %d, activations %s (output rms %.3g):\n", K, dn[dist], rms);
      for (int mode = 0; mode < 4; ++mode) {
        double scale = 1.0;
        if (mode == 0 || mode == 2) {
          CK(hipMemcpy(dA, A6.data(), 6 * 32L * K, hipMemcpyHostToDevice));
          CK(hipMemcpy(dB, B6.data(), 6 * 32L * K, hipMemcpyHostToDevice));
          hipLaunchKernelGGL(dot_kernel, dim3(1), dim3(64), 0, 0, dA, dB, K, mode == 0 ? 0 : 2, dC);
        } else if (mode == 1) {
          CK(hipMemcpy(dA, AH.data(), 6 * 32L * K, hipMemcpyHostToDevice));
          CK(hipMemcpy(dB, BH.data(), 6 * 32L * K, hipMemcpyHostToDevice));
          hipLaunchKernelGGL(dot_kernel, dim3(1), dim3(64), 0, 0, dA, dB, K, 1, dC);
          scale = 1.0 / (2048.0 * sw * sa);
        } else {
          CK(hipMemcpy(dAf, A.data(), 4 * 32L * K, hipMemcpyHostToDevice));
          CK(hipMemcpy(dBf, B.data(), 4 * 32L * K, hipMemcpyHostToDevice));
          hipLaunchKernelGGL(f32_kernel, dim3(1), dim3(64), 0, 0, dAf, dBf, K, dC);
        }
        CK(hipMemcpy(C.data(), dC, 4096, hipMemcpyDeviceToHost));
        double e2 = 0, emax = 0;
        for (int i = 0; i < 1024; ++i) {
          const double e = (double)C[i] * scale - ref[i];
          e2 += e * e;
          emax = std::fmax(emax, std::fabs(e));
        }
        printf("  %-12s rms err / rms %.3e   max err / rms %.3e\n", names[mode], std::sqrt(e2 / 1024) / rms,
               emax / rms);
      }
      hipFree(dA); hipFree(dB); hipFree(dC); hipFree(dAf); hipFree(dBf);
    }
  }
  return 0;
}
