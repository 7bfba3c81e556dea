// Training data path on the GPU — datasets.py:14-37 (Datasets.__getitem__):
//   RandomResizedCrop(256) → RandomHorizontalFlip → RandomVerticalFlip → ToTensor
// The host decodes each image to uint8 RGB (PIL), draws the crop box and flips, and computes
// PIL's resampling taps; this file does the pixel work on uint8 images uploaded as they are
// (a quarter of the fp32 bytes over PCIe):
//   pass 1: horizontal resample of the crop's rows to S columns (uint8 result, as PIL keeps it)
//   pass 2: vertical resample to S rows, then the flips, then /255 into an NCHW fp32 batch.
// Both passes are PIL's 8-bit bilinear resampling (Resample.c: 22-bit fixed-point taps, a
// rounding offset of 2^21, >> 22, clip to 0..255), so the batch equals torchvision's PIL path bit
// for bit (tests/test_gpu_datapath.py).
#include "common.h"

namespace iclr17 {
namespace {

constexpr int PREC = 22;   // PIL: PRECISION_BITS = 32 - 8 - 2

// int64 descriptor row per image
enum : int {
  D_SRC = 0,    // byte offset of the image in the uint8 HWC source buffer
  D_H, D_W,     // source size
  D_CI, D_CJ,   // crop top, left
  D_CH, D_CW,   // crop height, width
  D_FH, D_FV,   // horizontal / vertical flip
  D_TMP,        // byte offset of the image's pass-1 buffer [CH][S][3]
  D_CX, D_KX,   // x taps: int32 offset in the tap table, taps per output
  D_CY, D_KY,   // y taps
  D_N = 16
};

__device__ __forceinline__ int clip8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

__global__ void __launch_bounds__(256) resample_h_kernel(const unsigned char* __restrict__ src,
                                                         const long* __restrict__ desc,
                                                         const int* __restrict__ taps, int S,
                                                         unsigned char* __restrict__ tmp) {
  const long* d = desc + (long)blockIdx.x * D_N;
  const int W = (int)d[D_W], ci = (int)d[D_CI], cj = (int)d[D_CJ], ch = (int)d[D_CH];
  const int kx = (int)d[D_KX];
  const unsigned char* img = src + d[D_SRC];
  unsigned char* out = tmp + d[D_TMP];
  const int* tx = taps + d[D_CX];
  for (int r = blockIdx.y; r < ch; r += gridDim.y) {
    const unsigned char* row = img + ((long)(ci + r) * W + cj) * 3;
    for (int x = threadIdx.x; x < S; x += 256) {
      const int* t = tx + x * (2 + kx);
      const int xmin = t[0], n = t[1];
      int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
      for (int k = 0; k < n; ++k) {
        const int w = t[2 + k];
        const unsigned char* p = row + (xmin + k) * 3;
        s0 += p[0] * w;
        s1 += p[1] * w;
        s2 += p[2] * w;
      }
      unsigned char* o = out + ((long)r * S + x) * 3;
      o[0] = (unsigned char)clip8(s0 >> PREC);
      o[1] = (unsigned char)clip8(s1 >> PREC);
      o[2] = (unsigned char)clip8(s2 >> PREC);
    }
  }
}

__global__ void __launch_bounds__(256) resample_v_kernel(const unsigned char* __restrict__ tmp,
                                                         const long* __restrict__ desc,
                                                         const int* __restrict__ taps, int S,
                                                         float* __restrict__ out) {
  const int b = blockIdx.x, y = blockIdx.y;
  const long* d = desc + (long)b * D_N;
  const int fh = (int)d[D_FH], fv = (int)d[D_FV], ky = (int)d[D_KY];
  const unsigned char* in = tmp + d[D_TMP];
  const int yy = fv ? S - 1 - y : y;   // output row y shows resampled row yy
  const int* t = taps + d[D_CY] + yy * (2 + ky);
  const int ymin = t[0], n = t[1];
  const long plane = (long)S * S;
  for (int x = threadIdx.x; x < S; x += 256) {
    const int xx = fh ? S - 1 - x : x;
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    for (int k = 0; k < n; ++k) {
      const int w = t[2 + k];
      const unsigned char* p = in + ((long)(ymin + k) * S + xx) * 3;
      s0 += p[0] * w;
      s1 += p[1] * w;
      s2 += p[2] * w;
    }
    float* o = out + (long)b * 3 * plane + (long)y * S + x;
    o[0] = (float)clip8(s0 >> PREC) / 255.0f;   // ToTensor: uint8 / 255
    o[plane] = (float)clip8(s1 >> PREC) / 255.0f;
    o[2 * plane] = (float)clip8(s2 >> PREC) / 255.0f;
  }
}

}  // namespace
}  // namespace iclr17

using namespace iclr17;

extern "C" {

int iclr17_resized_crop_batch(const uint8_t* src, const int64_t* desc, int B, int S, int max_ch,
                              const int32_t* taps, uint8_t* tmp, float* out, void* stream) {
  ICLR17_REQUIRE(src && desc && taps && tmp && out && B > 0 && S > 0 && max_ch > 0,
                 ICLR17_EINVAL, "resized_crop_batch: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const int gy = max_ch < 256 ? max_ch : 256;
  hipLaunchKernelGGL(resample_h_kernel, dim3(B, gy), dim3(256), 0, st,
                     (const unsigned char*)src, (const long*)desc, (const int*)taps, S,
                     (unsigned char*)tmp);
  hipLaunchKernelGGL(resample_v_kernel, dim3(B, S), dim3(256), 0, st, (const unsigned char*)tmp,
                     (const long*)desc, (const int*)taps, S, out);
  return check_launch("resized_crop_batch");
}

}  // extern "C"
