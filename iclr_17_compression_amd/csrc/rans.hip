// Entropy coding of the quantised latent ŷ with the factorised BitEstimator — SURVEY §8(f) row 4.
// The reference only ESTIMATES the rate (model.py:71-78: bits = Σ −log2(F(ŷ+½) − F(ŷ−½))); this
// turns the same per-channel distribution into a real bitstream and back, bit-exactly.
//
// Alphabet per channel: values v ∈ [−K, K] (symbol v + K) and one escape symbol (2K + 1) for
// |v| > K, followed by v + 32768 as one uniform 16-bit symbol (|v| ≤ 32767). Probabilities:
// p(v) = F(v + ½) − F(v − ½) with F the BitEstimator CDF evaluated exactly as the rate kernel
// does (common.h bitparm_cdf), p(escape) = F(−K − ½) + (1 − F(K + ½)); quantised to 16-bit
// frequencies (each ≥ 1, summing to 2^16).
//
// Coder: interleaved rANS, 32-bit states in [2^16, 2^32), 16-bit renormalisation words, 16-bit
// probability precision. Streams: each image's channels are cut into P contiguous groups, one
// stream per (image, group), symbols in (channel, row, column) order. One wave codes a stream:
// lane l owns symbols l, l + 64, … with its own state; a block's renormalisation words are
// ordered by lane (ballot + prefix count), so the stream stays one word sequence. The encoder
// writes back to front into its own scratch slot; the offsets scan and the pack kernel then
// concatenate the streams. The CDF tables are staged in LDS.
#include "common.h"

namespace iclr17 {
namespace {

constexpr unsigned kProbBits = 16;
constexpr unsigned kProbScale = 1u << kProbBits;   // Σ freq
constexpr unsigned kL = 1u << 16;                   // state lower bound

// cum[c][0 .. 2K+2]: symbol i covers [cum[i], cum[i+1]) of the 2^16 slots
__global__ void __launch_bounds__(256) tables_kernel(const float* __restrict__ rp, int N, int K,
                                                     int* __restrict__ cum) {
  const int c = blockIdx.x;
  const int NS = 2 * K + 2;   // symbols incl. escape
  extern __shared__ int tsh[];
  float* sc = (float*)tsh;   // [2K + 2] CDF values, then [NS] freqs (as int)
  for (int j = threadIdx.x; j < 2 * K + 2; j += blockDim.x)
    sc[j] = bitparm_cdf((float)(j - K) - 0.5f, rp, N, c);
  __syncthreads();
  if (threadIdx.x != 0) return;
  int* freq = (int*)(sc + 2 * K + 2);
  const float spread = (float)(kProbScale - (unsigned)NS);
  int total = 0, imax = 0;
  float pmax = -1.f;
  for (int i = 0; i < NS; ++i) {
    float p = i < NS - 1 ? sc[i + 1] - sc[i] : sc[0] + (1.0f - sc[2 * K + 1]);
    p = fmaxf(p, 0.f);
    const int f = 1 + (int)floorf(p * spread);
    freq[i] = f;
    total += f;
    if (p > pmax) { pmax = p; imax = i; }
  }
  freq[imax] += (int)kProbScale - total;   // exact sum; the most probable symbol absorbs it
  int* cc = cum + (long)c * (NS + 1);
  int acc = 0;
  for (int i = 0; i < NS; ++i) {
    cc[i] = acc;
    acc += freq[i];
  }
  cc[NS] = acc;
}

struct StreamGeo {
  int HW, N, cpg;   // pixels per channel, channels, channels per stream group
  int P;            // streams per image
};

constexpr int W = 64;   // interleaved lanes per stream (one wave)

__device__ __forceinline__ long sym_index(const StreamGeo& g, int b, int grp, int i) {
  const int cl = i / g.HW, pix = i - cl * g.HW;
  return ((long)b * g.HW + pix) * g.N + grp * g.cpg + cl;   // NHWC element
}

// status bits
enum : int { ST_NONINT = 1, ST_RANGE = 2, ST_OVERRUN = 4, ST_TRAIL = 8 };

// every channel's table into LDS (N·(2K + 3) ints)
__device__ __forceinline__ void load_tables(const int* __restrict__ cum, int n, int* sc) {
  for (int i = threadIdx.x; i < n; i += W) sc[i] = cum[i];
  __syncthreads();
}

__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v |= __shfl_xor(v, off, 64);
  return v;
}

// lanes with `need` get consecutive ranks in lane order; returns (rank, count)
__device__ __forceinline__ int2 lane_rank(bool need, int lane) {
  const unsigned long long m = __ballot(need);
  return make_int2(__popcll(m & ((1ull << lane) - 1ull)), __popcll(m));
}

// One wave per stream; lane l codes symbols l, l + 64, … with its own state. Blocks of 64
// symbols are encoded last to first; inside a block the escape payloads go first, then the
// symbols (the decoder's reverse). Renormalisation words of a (block, sub-round) are placed
// back to front as a group, lane order ascending, so the decoder reading forward hands each
// lane its own word. The 64 final states (high word first) lead the stream.
__global__ void __launch_bounds__(W) encode_kernel(const float* __restrict__ y, StreamGeo g,
                                                   const int* __restrict__ cum, int K,
                                                   unsigned short* __restrict__ scratch, long cap,
                                                   unsigned* __restrict__ lengths,
                                                   int* __restrict__ status) {
  extern __shared__ int sc[];
  const int NS = 2 * K + 2, TS = NS + 1;
  load_tables(cum, g.N * TS, sc);
  const int s = blockIdx.x, lane = threadIdx.x;
  const int b = s / g.P, grp = s - b * g.P;
  unsigned short* out = scratch + (long)s * cap;
  long ptr = cap;
  unsigned x = kL;
  int bad = 0;
  const int nsym = g.cpg * g.HW;
  const int nblk = (nsym + W - 1) / W;
  for (int blk = nblk - 1; blk >= 0; --blk) {
    const int i = blk * W + lane;
    const bool act = i < nsym;
    int sym = 0, pay = -1;
    const int* cc = sc;
    if (act) {
      const long e = sym_index(g, b, grp, i);
      const float v = y[e];
      cc = sc + (grp * g.cpg + i / g.HW) * TS;
      const float r = rintf(v);
      if (!(r == v)) { bad |= ST_NONINT; sym = K; }   // NaN / non-integer
      else if (fabsf(v) > 32767.f) { bad |= ST_RANGE; sym = K; }
      else {
        const int iv = (int)v;
        sym = (iv >= -K && iv <= K) ? iv + K : NS - 1;
        if (sym == NS - 1) pay = iv + 32768;
      }
    }
    // sub-round B: escape payloads (uniform, freq 1: always one word out)
    {
      const bool need = pay >= 0;
      const int2 rc = lane_rank(need, lane);
      if (need) {
        out[ptr - rc.y + rc.x] = (unsigned short)(x & 0xffffu);
        x = ((x >> 16) << 16) + (unsigned)pay;
      }
      ptr -= rc.y;
    }
    // sub-round A: the symbols
    {
      const unsigned start = (unsigned)cc[sym], f = (unsigned)(cc[sym + 1] - cc[sym]);
      const bool need = act && x >= (f << 16);
      const int2 rc = lane_rank(need, lane);
      if (need) {
        out[ptr - rc.y + rc.x] = (unsigned short)(x & 0xffffu);
        x >>= 16;
      }
      ptr -= rc.y;
      if (act) x = ((x / f) << 16) + (x % f) + start;
    }
  }
  ptr -= 2 * W;
  out[ptr + 2 * lane] = (unsigned short)(x >> 16);
  out[ptr + 2 * lane + 1] = (unsigned short)(x & 0xffffu);
  if (lane == 0) lengths[s] = (unsigned)(cap - ptr);
  bad = wave_or(bad);
  if (lane == 0 && bad) atomicOr(status, bad);
}

// offsets[0] = 0, offsets[i + 1] = offsets[i] + lengths[i]   (one workgroup; n ≤ a few 10^5)
__global__ void __launch_bounds__(1024) offsets_kernel(const unsigned* __restrict__ len, int n,
                                                       long* __restrict__ offsets) {
  __shared__ long part[1024];
  const int t = threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int i0 = t * per, i1 = min(n, i0 + per);
  long s = 0;
  for (int i = i0; i < i1; ++i) s += len[i];
  part[t] = s;
  __syncthreads();
  if (t == 0) {
    long a = 0;
    for (int k = 0; k < 1024; ++k) {
      const long v = part[k];
      part[k] = a;
      a += v;
    }
  }
  __syncthreads();
  long a = part[t];
  for (int i = i0; i < i1; ++i) {
    offsets[i] = a;
    a += len[i];
  }
  if (i1 == n && i0 < i1) offsets[n] = a;
  if (n == 0 && t == 0) offsets[0] = 0;
}

__global__ void __launch_bounds__(256) pack_kernel(const unsigned short* __restrict__ scratch,
                                                   long cap, const long* __restrict__ offsets,
                                                   unsigned short* __restrict__ words) {
  const int s = blockIdx.x;
  const long o = offsets[s], n = offsets[s + 1] - o;
  const unsigned short* src = scratch + (long)s * cap + (cap - n);
  for (long i = threadIdx.x; i < n; i += 256) words[o + i] = src[i];
}

__global__ void __launch_bounds__(W) decode_kernel(const unsigned short* __restrict__ words,
                                                   const long* __restrict__ offsets, StreamGeo g,
                                                   const int* __restrict__ cum, int K,
                                                   float* __restrict__ y, int* __restrict__ status) {
  extern __shared__ int sc[];
  const int NS = 2 * K + 2, TS = NS + 1;
  load_tables(cum, g.N * TS, sc);
  const int s = blockIdx.x, lane = threadIdx.x;
  const int b = s / g.P, grp = s - b * g.P;
  const unsigned short* in = words + offsets[s];
  const long n = offsets[s + 1] - offsets[s];
  int bad = 0;
  if (n < 2 * W) {
    if (lane == 0) atomicOr(status, ST_OVERRUN);
    return;
  }
  unsigned x = ((unsigned)in[2 * lane] << 16) | in[2 * lane + 1];
  long ptr = 2 * W;
  auto word = [&](bool need, int& fail) -> unsigned {
    const int2 rc = lane_rank(need, lane);
    unsigned w = 0;
    if (need) {
      if (ptr + rc.x < n) w = in[ptr + rc.x];
      else fail |= ST_OVERRUN;
    }
    ptr += rc.y;
    return w;
  };
  const int nsym = g.cpg * g.HW;
  const int nblk = (nsym + W - 1) / W;
  for (int blk = 0; blk < nblk; ++blk) {
    const int i = blk * W + lane;
    const bool act = i < nsym;
    int v = 0;
    bool esc = false;
    if (act) {
      const int* cc = sc + (grp * g.cpg + i / g.HW) * TS;
      const unsigned slot = x & 0xffffu;
      int lo = 0, hi = NS;   // cc[lo] ≤ slot < cc[hi]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if ((unsigned)cc[mid] <= slot) lo = mid; else hi = mid;
      }
      const unsigned start = (unsigned)cc[lo], f = (unsigned)(cc[lo + 1] - cc[lo]);
      x = f * (x >> 16) + slot - start;
      v = lo - K;
      esc = lo == NS - 1;
    }
    {   // sub-round A: renormalise after the symbols
      const bool need = act && x < kL;
      const unsigned w = word(need, bad);
      if (need) x = (x << 16) | w;
    }
    {   // sub-round B: escape payloads
      unsigned u = 0;
      if (esc) {
        u = x & 0xffffu;
        x >>= 16;
      }
      const unsigned w = word(esc, bad);
      if (esc) {
        x = (x << 16) | w;
        v = (int)u - 32768;
      }
    }
    if (act) y[sym_index(g, b, grp, i)] = (float)v;
  }
  if (x != kL) bad |= ST_TRAIL;
  if (lane == 0 && ptr != n) bad |= ST_TRAIL;
  bad = wave_or(bad);
  if (lane == 0 && bad) atomicOr(status, bad);
}

}  // namespace
}  // namespace iclr17

using namespace iclr17;

extern "C" {

int iclr17_entropy_tables(const float* rate_packed, int N, int K, int32_t* cum, void* stream) {
  ICLR17_REQUIRE(rate_packed && cum && N > 0 && K >= 1 && K <= 1024, ICLR17_EINVAL,
                 "entropy_tables: bad arguments (K=%d)", K);
  const size_t shm = (size_t)(2 * K + 2) * 4 + (size_t)(2 * K + 2) * 4;
  hipLaunchKernelGGL(tables_kernel, dim3(N), dim3(256), shm, (hipStream_t)stream, rate_packed,
                     N, K, (int*)cum);
  return check_launch("entropy_tables");
}

long iclr17_rans_capacity(int h, int w, int N, int streams_per_image) {
  if (h <= 0 || w <= 0 || N <= 0 || streams_per_image <= 0 || N % streams_per_image) return 0;
  return 2L * W + 2L * (N / streams_per_image) * h * w;
}

int iclr17_rans_encode(const float* y_hat, int B, int h, int w, int N, int streams_per_image,
                       const int32_t* cum, int K, uint16_t* scratch, long scratch_words,
                       uint32_t* lengths, int32_t* status, void* stream) {
  const long cap = iclr17_rans_capacity(h, w, N, streams_per_image);
  ICLR17_REQUIRE(y_hat && cum && scratch && lengths && status && B > 0 && cap > 0 && K >= 1,
                 ICLR17_EINVAL, "rans_encode: bad arguments");
  const size_t shm = (size_t)N * (2 * K + 3) * sizeof(int);
  ICLR17_REQUIRE(shm <= 64 * 1024, ICLR17_EINVAL, "rans_encode: tables of %zu bytes exceed LDS", shm);
  const int ns = B * streams_per_image;
  ICLR17_REQUIRE(scratch_words >= cap * ns, ICLR17_EINVAL,
                 "rans_encode: scratch of %ld words < %ld", scratch_words, cap * ns);
  StreamGeo g{h * w, N, N / streams_per_image, streams_per_image};
  hipLaunchKernelGGL(encode_kernel, dim3(ns), dim3(W), shm, (hipStream_t)stream, y_hat, g,
                     (const int*)cum, K, (unsigned short*)scratch, cap, (unsigned*)lengths,
                     (int*)status);
  return check_launch("rans_encode");
}

int iclr17_rans_offsets(const uint32_t* lengths, int n, int64_t* offsets, void* stream) {
  ICLR17_REQUIRE(lengths && offsets && n >= 0, ICLR17_EINVAL, "rans_offsets: bad arguments");
  hipLaunchKernelGGL(offsets_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                     (const unsigned*)lengths, n, (long*)offsets);
  return check_launch("rans_offsets");
}

int iclr17_rans_pack(const uint16_t* scratch, long cap, const int64_t* offsets, int n,
                     uint16_t* words, void* stream) {
  ICLR17_REQUIRE(scratch && offsets && words && n > 0 && cap > 0, ICLR17_EINVAL,
                 "rans_pack: bad arguments");
  hipLaunchKernelGGL(pack_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream,
                     (const unsigned short*)scratch, cap, (const long*)offsets,
                     (unsigned short*)words);
  return check_launch("rans_pack");
}

int iclr17_rans_decode(const uint16_t* words, const int64_t* offsets, int B, int h, int w, int N,
                       int streams_per_image, const int32_t* cum, int K, float* y_hat,
                       int32_t* status, void* stream) {
  ICLR17_REQUIRE(words && offsets && cum && y_hat && status && B > 0 && h > 0 && w > 0 &&
                     N > 0 && streams_per_image > 0 && N % streams_per_image == 0 && K >= 1,
                 ICLR17_EINVAL, "rans_decode: bad arguments");
  const size_t shm = (size_t)N * (2 * K + 3) * sizeof(int);
  ICLR17_REQUIRE(shm <= 64 * 1024, ICLR17_EINVAL, "rans_decode: tables of %zu bytes exceed LDS", shm);
  const int ns = B * streams_per_image;
  StreamGeo g{h * w, N, N / streams_per_image, streams_per_image};
  hipLaunchKernelGGL(decode_kernel, dim3(ns), dim3(W), shm, (hipStream_t)stream,
                     (const unsigned short*)words, (const long*)offsets, g, (const int*)cum, K,
                     y_hat, (int*)status);
  return check_launch("rans_decode");
}

}  // extern "C"
