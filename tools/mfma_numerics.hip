// Diagnostic (GPU): what v_mfma_f32_16x16x32_bf16 does to C + Σ a·b, on gfx950.
// Random trials, each one MFMA of a wave; the host compares D with models of the hardware:
//   rne1   exact C + Σ_k a_k b_k, rounded once to nearest-even
//   rz1    the same, truncated toward zero
//   chain  k-ordered fmaf chain starting at C (the f32 MFMA's documented behaviour)
// and reports how often each model matches bit for bit, plus the signed error of D in units of
// the ulp of the exact result (mean = bias, rms). Also the f32 MFMA (16x16x4) as a control.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_numerics.hip -o /tmp/mfma_numerics && /tmp/mfma_numerics
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

using frag_ab = __attribute__((ext_vector_type(8))) short;
using frag_cd = __attribute__((ext_vector_type(4))) float;

// A [T][16][32] bf16, B [T][32][16] bf16, C/D [T][16][16] fp32; one wave per trial
__global__ void mfma_bf16(const uint16_t* A, const uint16_t* B, const float* C, float* D) {
  int t = blockIdx.x, l = threadIdx.x;
  const uint16_t* a = A + t * 512;
  const uint16_t* b = B + t * 512;
  frag_ab fa, fb;
  for (int j = 0; j < 8; ++j) {
    fa[j] = (short)a[(l & 15) * 32 + 8 * (l >> 4) + j];
    fb[j] = (short)b[(8 * (l >> 4) + j) * 16 + (l & 15)];
  }
  frag_cd c;
  for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)];
  frag_cd d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[t * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)] = d[r];
}

// A [T][16][4] f32, B [T][4][16] f32
__global__ void mfma_f32(const float* A, const float* B, const float* C, float* D) {
  int t = blockIdx.x, l = threadIdx.x;
  float fa = A[t * 64 + (l & 15) * 4 + (l >> 4)];
  float fb = B[t * 64 + (l >> 4) * 16 + (l & 15)];
  frag_cd c;
  for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)];
  frag_cd d = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[t * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)] = d[r];
}

static float bf(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }
static uint16_t to_bf_trunc(float f) { uint32_t u; memcpy(&u, &f, 4); return (uint16_t)(u >> 16); }
static float rz(double x) {
  float f = (float)x;   // RNE
  if (std::fabs((double)f) > std::fabs(x)) f = std::nextafter(f, 0.0f);
  return f;
}
static double ulp_of(double x) {
  float f = (float)std::fabs(x);
  return (double)std::nextafter(f, INFINITY) - (double)f;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct Stats { long n = 0, rne = 0, rz = 0, chain = 0; double s = 0, s2 = 0; };

static void report(const char* what, const Stats& st) {
  double mean = st.s / st.n, rms = std::sqrt(st.s2 / st.n);
  printf("%-44s n=%ld  rne1 %.4f  rz1 %.4f  chain %.4f  err/ulp mean %+.4f rms %.4f\n", what, st.n,
         (double)st.rne / st.n, (double)st.rz / st.n, (double)st.chain / st.n, mean, rms);
}

int main() {
  const int T = 4096;
  std::mt19937_64 rng(12345);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<uint16_t> A(T * 512), B(T * 512);
  std::vector<float> C(T * 256), D(T * 256);
  uint16_t *dA, *dB; float *dC, *dD;
  CK(hipMalloc(&dA, A.size() * 2)); CK(hipMalloc(&dB, B.size() * 2));
  CK(hipMalloc(&dC, C.size() * 4)); CK(hipMalloc(&dD, D.size() * 4));
  // cases: C scale relative to a typical |Σ a·b| (≈ sqrt(32)); "mixed" draws per-element exponents
  struct Case { const char* name; float cscale; int mixed; int same_sign; };
  Case cases[] = {{"bf16 C~0 (C=0)", 0.f, 0, 0}, {"bf16 C~sum", 6.f, 0, 0}, {"bf16 C 100x sum", 600.f, 0, 0},
                  {"bf16 C 1e4x sum", 6e4f, 0, 0}, {"bf16 mixed exponents, C~sum", 6.f, 1, 0},
                  {"bf16 positive products, C 100x", 600.f, 0, 1}};
  for (const Case& cs : cases) {
    for (int i = 0; i < T * 512; ++i) {
      float a = nd(rng), b = nd(rng);
      if (cs.mixed) { a = std::ldexp(a, (int)(rng() % 24) - 12); b = std::ldexp(b, (int)(rng() % 24) - 12); }
      if (cs.same_sign) { a = std::fabs(a); b = std::fabs(b); }
      A[i] = to_bf_trunc(a); B[i] = to_bf_trunc(b);
    }
    for (int i = 0; i < T * 256; ++i) C[i] = nd(rng) * cs.cscale;
    CK(hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(mfma_bf16, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
    Stats st;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double ex = C[t * 256 + i * 16 + j];
          float ch = C[t * 256 + i * 16 + j];
          for (int k = 0; k < 32; ++k) {
            float a = bf(A[t * 512 + i * 32 + k]), b = bf(B[t * 512 + k * 16 + j]);
            ex += (double)a * (double)b;
            ch = std::fmaf(a, b, ch);
          }
          float d = D[t * 256 + i * 16 + j];
          st.n++;
          st.rne += d == (float)ex;
          st.rz += d == rz(ex);
          st.chain += d == ch;
          double e = ((double)d - ex) / ulp_of(ex) * (ex < 0 ? -1.0 : 1.0);   // + = away from zero
          st.s += e; st.s2 += e * e;
        }
    report(cs.name, st);
  }
  // control: f32 MFMA
  {
    std::vector<float> Af(T * 64), Bf(T * 64);
    for (auto& v : Af) v = nd(rng);
    for (auto& v : Bf) v = nd(rng);
    for (int i = 0; i < T * 256; ++i) C[i] = nd(rng) * 2.f;
    float *dAf, *dBf;
    CK(hipMalloc(&dAf, Af.size() * 4)); CK(hipMalloc(&dBf, Bf.size() * 4));
    CK(hipMemcpy(dAf, Af.data(), Af.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dBf, Bf.data(), Bf.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(mfma_f32, dim3(T), dim3(64), 0, 0, dAf, dBf, dC, dD);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
    Stats st;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double ex = C[t * 256 + i * 16 + j];
          float ch = C[t * 256 + i * 16 + j];
          for (int k = 0; k < 4; ++k) {
            float a = Af[t * 64 + i * 4 + k], b = Bf[t * 64 + k * 16 + j];
            ex += (double)a * (double)b;
            ch = std::fmaf(a, b, ch);
          }
          float d = D[t * 256 + i * 16 + j];
          st.n++;
          st.rne += d == (float)ex; st.rz += d == rz(ex); st.chain += d == ch;
          double e = ((double)d - ex) / ulp_of(ex) * (ex < 0 ? -1.0 : 1.0);
          st.s += e; st.s2 += e * e;
        }
    report("f32 16x16x4 (control)", st);
  }
  return 0;
}
