/*
 * iclr17.h — C ABI of libiclr17.so, the gfx950 (MI355X) kernels of the Ballé-2017 codec
 * hot path of Yuval-H/iclr_17_compression (analysis conv+GDN → quantiser + factorised
 * rate → synthesis deconv+IGDN).
 *
 * The reference is pure PyTorch and binds no FFI; each entry point below replaces the
 * stock PyTorch ops of one reference layer (or a fused run of them), cited per function
 * as reference-file:line. The Python host layer (iclr_17_compression_amd/) keeps the
 * reference nn.Module surface and calls these through ctypes; INTEGRATION.md shows the
 * binding.
 *
 * Conventions
 *  - Plain pointers to device memory (hipMalloc / PyTorch caching allocator); the caller
 *    owns every buffer, including the packed-parameter caches and partial-sum buffers.
 *    The library allocates nothing and keeps no global mutable state except a
 *    thread-local last-error string.
 *  - All work is enqueued on `stream` (a hipStream_t; NULL = the default stream). No call
 *    synchronises the host, so every call may be captured in a hipGraph.
 *  - Activations between layers are fp32 NHWC ("channels-last"); the codec input image
 *    and the reconstruction are fp32 NCHW, exactly the reference's tensors.
 *  - Return 0 on success or a negative ICLR17_E* code; iclr17_last_error() explains.
 *  - Supported channel counts N: 128 (ImageCompressor default, model.py:39) and
 *    192 (Analysis_net_17 / Synthesis_net_17 default, analysis_17.py:12). Image height and
 *    width must be positive multiples of 16 (model.py:48).
 */
#ifndef ICLR17_H_
#define ICLR17_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ICLR17_OK 0
#define ICLR17_EINVAL (-1)       /* bad pointer / shape / argument */
#define ICLR17_EUNSUPPORTED (-2) /* shape or mode this build does not implement */
#define ICLR17_ELAUNCH (-3)      /* HIP launch / runtime error */

#define ICLR17_QUANT_ROUND 0 /* eval: ŷ = round(y), half-to-even (model.py:56) */
#define ICLR17_QUANT_NOISE 1 /* train: ỹ = y + u, u caller-supplied (model.py:48-54) */

#define ICLR17_LAYOUT_NCHW 0
#define ICLR17_LAYOUT_NHWC 1

/* Which weight tensor a packing call converts (see iclr17_pack_weight). */
#define ICLR17_W_CONV1 0   /* Analysis conv1  [N,3,9,9]   analysis_17.py:14 */
#define ICLR17_W_CONV5 1   /* Analysis conv2/conv3 [N,N,5,5] analysis_17.py:18,22 */
#define ICLR17_W_DECONV5 2 /* Synthesis deconv1/deconv2 [N,N,5,5] synthesis_17.py:15,19 */
#define ICLR17_W_DECONV9 3 /* Synthesis deconv3 [N,3,9,9] synthesis_17.py:23 */

int iclr17_version(void);
/* Copies the calling thread's last error message (NUL-terminated); returns its length. */
int iclr17_last_error(char* buf, size_t len);

/* ------------------------------------------------------------------ parameter packing
 * Packed layouts are derived caches of the fp32 module parameters; repack after every
 * parameter update. Sizes are in floats. */
size_t iclr17_packed_weight_size(int which, int N);
/* w: the reference weight tensor, contiguous fp32 in its PyTorch layout. */
int iclr17_pack_weight(int which, const float* w, float* packed, int N, void* stream);
/* GDN.py:46-49,73-83: beta_eff[C] = max(beta, beta_bound)² − pedestal and
 * gamma_eff = max(gamma, gamma_bound)² − pedestal, the latter packed for the channel
 * contraction ([C/4][C][4]: packed[q][i][e] = gamma_eff[i][4q+e]); gamma_packed holds C*C
 * floats. Bounds/pedestal are the fp32 values the reference's ones_like(x)*bound produce
 * (defaults: float(sqrt(1e-6 + 2^-36)), 2^-18, 2^-36). */
int iclr17_pack_gdn(const float* beta, const float* gamma, float* beta_eff, float* gamma_packed,
                    int C, float beta_bound, float gamma_bound, float pedestal, void* stream);
/* bitEstimator.py:13-25: rows softplus(h_k), b_k, tanh(a_k) for k = 1..3 then softplus(h_4),
 * b_4 → packed[11][C]. h/b/a are the (1,C,1,1) parameters of f1..f4 (a4 absent). */
int iclr17_pack_rate(const float* h1, const float* b1, const float* a1, const float* h2,
                     const float* b2, const float* a2, const float* h3, const float* b3,
                     const float* a3, const float* h4, const float* b4, float* packed, int C,
                     void* stream);

/* ------------------------------------------------------------------ fused codec layers
 * Shapes: B images, input image H×W (multiples of 16), N channels.
 * pre_out (nullable) receives the layer's pre-GDN / pre-IGDN activation (needed only by
 * backward). */

/* analysis_17.py:14-17,33 : gdn1(conv1(x)); x NCHW [B,3,H,W] → out NHWC [B,H/4,W/4,N]. */
int iclr17_analysis_conv1_gdn(const float* x, int B, int H, int W, int N, const float* w_packed,
                              const float* bias, const float* beta_eff, const float* gamma_packed,
                              float* out, float* pre_out, void* stream);
/* analysis_17.py:18-21,34 : gdn2(conv2(h)); in NHWC [B,H/4,W/4,N] → out [B,H/8,W/8,N]. */
int iclr17_analysis_conv2_gdn(const float* in, int B, int H, int W, int N, const float* w_packed,
                              const float* bias, const float* beta_eff, const float* gamma_packed,
                              float* out, float* pre_out, void* stream);
/* analysis_17.py:22,35 + model.py:48-56,71-73 : y = conv3(h) (no bias); ŷ = round(y) or y+noise;
 * per-element rate bits summed per tile. in NHWC [B,H/8,W/8,N]; y_out, y_hat NHWC
 * [B,H/16,W/16,N] (y_out nullable); noise NCHW [B,N,H/16,W/16] (QUANT_NOISE only);
 * bits_partial[B * iclr17_rate_partials_per_image(H,W,N)] doubles. */
int iclr17_analysis_conv3_quant_rate(const float* in, int B, int H, int W, int N,
                                     const float* w_packed, int quant_mode, const float* noise,
                                     const float* rate_packed, float* y_out, float* y_hat,
                                     double* bits_partial, void* stream);
int iclr17_rate_partials_per_image(int H, int W, int N);
/* analysis_17.py:22,35 alone (Analysis_net_17.forward without the quantiser): y NHWC. */
int iclr17_analysis_conv3(const float* in, int B, int H, int W, int N, const float* w_packed,
                          float* y_out, void* stream);
/* synthesis_17.py:15-18,28 / :19-22,29 : igdn(deconv(h)), stride 2, k5, p2, op1.
 * in NHWC [B,h,w,N] → out NHWC [B,2h,2w,N]; (h,w) are the INPUT spatial dims. */
int iclr17_synthesis_deconv_igdn(const float* in, int B, int h, int w, int N,
                                 const float* w_packed, const float* bias, const float* beta_eff,
                                 const float* gamma_packed, float* out, float* pre_out,
                                 void* stream);
/* synthesis_17.py:23-25,30 + model.py:59 : deconv3 (N→3, k9, s4, p4, op3) + bias, clamp[0,1].
 * in NHWC [B,H/4,W/4,N] → clipped NCHW [B,3,H,W]; recon (nullable) gets the unclipped
 * output; if x (NCHW image, nullable) is given, Σ(clipped−x)² per tile goes to
 * sse_partial[B * iclr17_output_partials_per_image(H,W)]. */
int iclr17_synthesis_deconv3(const float* in, int B, int H, int W, int N, const float* w_packed,
                             const float* bias, const float* x, float* clipped, float* recon,
                             double* sse_partial, void* stream);
int iclr17_output_partials_per_image(int H, int W);

/* Deterministic fixed-order sums: per_image[b] = Σ_t partial[b*T + t] (nullable);
 * *total = (float)(scale · Σ_b per_image[b]) (nullable). model.py:73,78 bits→bpp. */
int iclr17_reduce_partials(const double* partial, int B, int T, double* per_image, float* total,
                           double scale, void* stream);

/* ------------------------------------------------------------------ stand-alone modules */
/* GDN.forward (GDN.py:64-94) on a [B,C,H,W] tensor in NCHW or NHWC memory layout. */
int iclr17_gdn(const float* x, int B, int C, int H, int W, int layout, int inverse,
               const float* beta_eff, const float* gamma_packed, float* y, void* stream);
/* BitEstimator.forward (bitEstimator.py:38-42): out = F(x) elementwise; channel of flat
 * element i is (i / inner) % C (inner = H*W for NCHW, 1 for NHWC). */
int iclr17_bit_estimator(const float* x, int64_t n, int C, int64_t inner,
                         const float* rate_packed, float* out, void* stream);
/* One Bitparm layer (bitEstimator.py:20-25) on raw h, b, a (a == NULL → final sigmoid layer);
 * work holds 2*C floats of scratch. */
int iclr17_bitparm(const float* x, int64_t n, int C, int64_t inner, const float* h,
                   const float* b, const float* a, float* work, float* out, void* stream);
/* model.py:71-73 on an arbitrary latent z ([B,C,h,w], layout as above): Σ bits per image →
 * bits_partial[B * iclr17_rate_bits_partials(C,h,w)]. */
int iclr17_rate_bits(const float* z, int B, int C, int h, int w, int layout,
                     const float* rate_packed, double* bits_partial, void* stream);
int iclr17_rate_bits_partials(int C, int h, int w);

#ifdef __cplusplus
}
#endif
#endif /* ICLR17_H_ */
