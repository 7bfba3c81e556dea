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
#define ICLR17_W_CONV1_X6 4 /* Analysis conv1 in the k order of iclr17_analysis_conv1x6_gdn */

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
 * floats; gamma_packed_t (nullable, backward only) the transpose (packed[q][j][e] =
 * gamma_eff[4q+e][j]). Bounds/pedestal are the fp32 values the reference's ones_like(x)*bound
 * produce (defaults: float(sqrt(1e-6 + 2^-36)), 2^-18, 2^-36). */
int iclr17_pack_gdn(const float* beta, const float* gamma, float* beta_eff, float* gamma_packed,
                    float* gamma_packed_t, int C, float beta_bound, float gamma_bound,
                    float pedestal, void* stream);
/* bitEstimator.py:13-25: rows softplus(h_k), b_k, tanh(a_k) for k = 1..3 then softplus(h_4),
 * b_4 → packed[11][C]. h/b/a are the (1,C,1,1) parameters of f1..f4 (a4 absent). */
int iclr17_pack_rate(const float* h1, const float* b1, const float* a1, const float* h2,
                     const float* b2, const float* a2, const float* h3, const float* b3,
                     const float* a3, const float* h4, const float* b4, float* packed, int C,
                     void* stream);

/* A batch of packs in two launches (all non-split jobs, then the splits, which may read packs
 * made by the first launch): the derived layouts of a training step's parameter update without
 * ~25 separate small launches. kind: an ICLR17_W_* weight layout (src0 = w, dst0 = packed, N),
 * ICLR17_PACK_GDN (src0 = beta, src1 = gamma, dst0/1/2 = beta_eff, gamma_packed,
 * gamma_packed_t (nullable), N = C, f0/f1/f2 = beta_bound, gamma_bound, pedestal: as
 * iclr17_pack_gdn), ICLR17_PACK_RATE (dst0 = packed, N = C; the 11 parameters in rate_params,
 * as iclr17_pack_rate; at most one rate job per call) or ICLR17_PACK_SPLIT (src0 = packed,
 * dst0 = planes (uint16), taps, K, N: as iclr17_split_packed). Results are bitwise those of
 * the single-pack entry points. */
#define ICLR17_PACK_GDN 16
#define ICLR17_PACK_RATE 17
#define ICLR17_PACK_SPLIT 18
typedef struct iclr17_pack_job {
  int kind, N, taps, K;
  const float* src0;
  const float* src1;
  void* dst0;
  void* dst1;
  void* dst2;
  float f0, f1, f2;
} iclr17_pack_job;
int iclr17_pack_batch(const iclr17_pack_job* jobs, int n, const float* const* rate_params,
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
 * bits_partial[B * iclr17_rate_partials_per_image(H,W,N)] doubles. rate_table (nullable;
 * iclr17_rate_table of rate_packed): in round mode the bits of |ŷ| ≤ 32 are looked up instead
 * of evaluating the factorised model (the same fp32 function, so the same values). */
int iclr17_analysis_conv3_quant_rate(const float* in, int B, int H, int W, int N,
                                     const float* w_packed, int quant_mode, const float* noise,
                                     const float* rate_packed, const float* rate_table,
                                     float* y_out, float* y_hat, double* bits_partial,
                                     void* stream);
int iclr17_rate_partials_per_image(int H, int W, int N);
/* Bit partials per image of the x6 and h3 conv3 entries (…_x6, …_x6w, …_h3): as above, except that in noise
 * mode on fewer than 256 tiles·images (training at B=32, 256²) the kernel runs 48-column tiles
 * and writes tiles × N/48 partials. */
int iclr17_conv3_x6_partials_per_image(int B, int H, int W, int N, int quant_mode);
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
 * output; if x (NCHW image, nullable) is given, Σ(clipped−x)² per tile (Σ(recon−x)² with
 * sse_unclipped, the training MSE of model.py:61) goes to
 * sse_partial[B * iclr17_output_partials_per_image(H,W)]. */
int iclr17_synthesis_deconv3(const float* in, int B, int H, int W, int N, const float* w_packed,
                             const float* bias, const float* x, float* clipped, float* recon,
                             double* sse_partial, int sse_unclipped, void* stream);
int iclr17_output_partials_per_image(int H, int W);

/* ------------------------------------------------------------------ x6 precision mode
 * The same layers with the conv contractions on v_mfma_f32_16x16x32_bf16 in the bf16x6 scheme:
 * every fp32 operand is split exactly into three bf16 parts (x = hi + mid + lo; truncation
 * split) and each product is formed from the six significant part products (hi·hi, hi·mid,
 * mid·hi, hi·lo, mid·mid, lo·hi — the dropped terms are below 2^-24 of the product), with
 * fp32 accumulation. Activations travel between layers in "split form": three bf16 planes
 * [3][B][h][w][N] (uint16 bf16 bits, plane stride B·h·w·N), written by the producing layer's
 * epilogue. conv1 (3-channel NCHW image) keeps exact-f32 products. out / out_split
 * are each nullable, not both. The GDN/IGDN channel contraction runs in x6 as well when given
 * gamma_split (required by conv2/deconv; nullable for conv1: then exact-f32). */
/* x[n] (n % 8 == 0) → planes[3][n]. */
int iclr17_split_planes(const float* x, long n, uint16_t* planes, void* stream);
/* A packed operand [taps][K/4][N][4] fp32 → planes [3][taps][K/8][N][8] (3·taps·K·N uint16). The
 * x6 GDN/IGDN channel contraction takes gamma_packed split this way (taps = 1, K = N = C):
 * the gamma_split argument below. */
int iclr17_split_packed(const float* packed, int taps, int K, int N, uint16_t* planes,
                        void* stream);
/* iclr17_analysis_conv1_gdn with the output also (or only) in split form. */
int iclr17_analysis_conv1_gdn_x6(const float* x, int B, int H, int W, int N,
                                 const float* w_packed, const float* bias, const float* beta_eff,
                                 const float* gamma_packed, const uint16_t* gamma_split,
                                 float* out, uint16_t* out_split, float* pre_out, void* stream);
/* analysis_17.py:14-17,33 with BOTH contractions in x6 (conv1's patch contraction too): the
 * weights are packed with ICLR17_W_CONV1_X6 and split by iclr17_split_packed(taps = 1, K = 256,
 * N) into w_split [3][32][N][8]; gamma_split as above. out / out_split / pre_out as
 * iclr17_analysis_conv1_gdn_x6. */
int iclr17_analysis_conv1x6_gdn(const float* x, int B, int H, int W, int N,
                                const uint16_t* w_split, const float* bias, const float* beta_eff,
                                const uint16_t* gamma_split, float* out, uint16_t* out_split,
                                float* pre_out, void* stream);
/* iclr17_analysis_conv2_gdn on a split-form input. */
int iclr17_analysis_conv2_gdn_x6(const uint16_t* in_split, int B, int H, int W, int N,
                                 const float* w_packed, const float* bias, const float* beta_eff,
                                 const float* gamma_packed, const uint16_t* gamma_split,
                                 float* out, uint16_t* out_split, float* pre_out, void* stream);
/* iclr17_analysis_conv3_quant_rate on a split-form input; ŷ also in split form (nullable).
 * The packed fp32 weights are split in the loop. */
int iclr17_analysis_conv3_quant_rate_x6(const uint16_t* in_split, int B, int H, int W, int N,
                                        const float* w_packed, int quant_mode, const float* noise,
                                        const float* rate_packed, const float* rate_table,
                                        float* y_out, float* y_hat, uint16_t* y_hat_split,
                                        double* bits_partial, void* stream);
/* The same with the weights pre-split: w_split = iclr17_split_packed(w_packed, 25, N, N, …)
 * ([3][25][N/8][N][8] bf16). Bit-identical to iclr17_analysis_conv3_quant_rate_x6 (the same
 * split, done once per weight update instead of per k-step in the loop). */
int iclr17_analysis_conv3_quant_rate_x6w(const uint16_t* in_split, int B, int H, int W, int N,
                                         const float* w_packed, const uint16_t* w_split,
                                         int quant_mode, const float* noise,
                                         const float* rate_packed, const float* rate_table,
                                         float* y_out, float* y_hat, uint16_t* y_hat_split,
                                         double* bits_partial, void* stream);
/* iclr17_synthesis_deconv_igdn on a split-form input. */
int iclr17_synthesis_deconv_igdn_x6(const uint16_t* in_split, int B, int h, int w, int N,
                                    const float* w_packed, const float* bias,
                                    const float* beta_eff, const float* gamma_packed,
                                    const uint16_t* gamma_split, float* out, uint16_t* out_split,
                                    float* pre_out, void* stream);
/* iclr17_synthesis_deconv_igdn_x6 writing the split output in the CHUNK-MAJOR split form
 * [3][B][N/32][2h][2w][32] (the fp32 out / pre_out stay NHWC), the input layout of
 * iclr17_synthesis_deconv3_x6_cm: a 32-channel chunk of a patch row is then contiguous, so
 * deconv3's per-chunk patch reads do not share 128-byte lines with the next chunk's (the NHWC
 * planes hold two chunks per line, and the second was refetched from HBM: 2.3x the bytes).
 * Replaces the same reference lines (synthesis_17.py:19-22). */
int iclr17_synthesis_deconv_igdn_x6_cm(const uint16_t* in_split, int B, int h, int w, int N,
                                       const float* w_packed, const float* bias,
                                       const float* beta_eff, const float* gamma_packed,
                                       const uint16_t* gamma_split, float* out,
                                       uint16_t* out_split_cm, float* pre_out, void* stream);
/* iclr17_synthesis_deconv3 on a split-form input (the same outputs and sse_partial layout:
 * iclr17_output_partials_per_image(H, W) doubles per image). w_split: the ICLR17_W_DECONV9
 * packing split by iclr17_split_packed(taps = 9, K = N, N = 48) — [3][9][N/8][48][8]. */
int iclr17_synthesis_deconv3_x6(const uint16_t* in_split, int B, int H, int W, int N,
                                const uint16_t* w_split, const float* bias, const float* x,
                                float* clipped, float* recon, double* sse_partial,
                                int sse_unclipped, void* stream);
/* iclr17_synthesis_deconv3_x6 reading the chunk-major split form of
 * iclr17_synthesis_deconv_igdn_x6_cm (synthesis_17.py:23-25); bit-identical results. */
int iclr17_synthesis_deconv3_x6_cm(const uint16_t* in_split_cm, int B, int H, int W, int N,
                                   const uint16_t* w_split, const float* bias, const float* x,
                                   float* clipped, float* recon, double* sse_partial,
                                   int sse_unclipped, void* stream);
/* iclr17_synthesis_deconv3_x6_cm that also performs iclr17_reduce_partials(bits_partial, B,
 * bits_T, bits_per_image, bpp_total, bits_scale) of conv3's bit partials (model.py:71-78: the
 * per-image bits and bpp = scale·Σ), in its workgroup 0 with reduce_partials' arithmetic and order
 * (bit-identical): the eval chain ends on deconv3 instead of one more launch. bits_per_image may
 * be NULL. */
int iclr17_synthesis_deconv3_x6_cm_bits(const uint16_t* in_split_cm, int B, int H, int W, int N,
                                        const uint16_t* w_split, const float* bias, const float* x,
                                        float* clipped, float* recon, double* sse_partial,
                                        int sse_unclipped, const double* bits_partial, int bits_T,
                                        double* bits_per_image, float* bpp_total, double bits_scale,
                                        void* stream);

/* ---------------------------------------------------------------- entropy coding (§8 f4)
 * A real bitstream for ŷ with the factorised model the reference only uses to ESTIMATE the rate
 * (model.py:71-78 / bitEstimator.py). Per channel c, symbols v ∈ [−K, K] plus an escape (the
 * value then follows as one uniform 16-bit symbol, |v| ≤ 32767); frequencies quantised to 16
 * bits from F_c(v ± ½) (the rate kernel's own CDF evaluation). Interleaved rANS: 64 32-bit
 * states per stream (state l owns symbols l, l + 64, …), 16-bit words ordered by lane within
 * each block of 64 symbols; each image's channels are cut into P contiguous groups ("streams",
 * N % P == 0), symbols in (channel, row, column) order; one wave per stream. A stream is its 64
 * final states (128 words) followed by the renormalisation words (oracle/rans_ref.py spells
 * out the order). */
/* cum: int32 [N][2K + 3] cumulative frequencies (cum[c][2K + 2] = 65536). */
int iclr17_entropy_tables(const float* rate_packed, int N, int K, int32_t* cum, void* stream);
/* Words of per-stream scratch: 128 + 2·(N/P)·h·w (0: bad arguments). */
long iclr17_rans_capacity(int h, int w, int N, int streams_per_image);
/* ŷ NHWC [B][h][w][N] (integer-valued fp32) → each stream's words at the END of its scratch
 * slot s·capacity (s = b·P + group), its word count in lengths[s]. status |= 1 non-integer or
 * NaN, 2 |v| > 32767 (int32 on the device, caller-zeroed). */
int iclr17_rans_encode(const float* y_hat, int B, int h, int w, int N, int streams_per_image,
                       const int32_t* cum, int K, uint16_t* scratch, long scratch_words,
                       uint32_t* lengths, int32_t* status, void* stream);
/* offsets[0] = 0, offsets[i + 1] = offsets[i] + lengths[i] (int64 [n + 1]). */
int iclr17_rans_offsets(const uint32_t* lengths, int n, int64_t* offsets, void* stream);
/* Concatenate the n streams: words[offsets[s] .. offsets[s + 1]) = stream s. */
int iclr17_rans_pack(const uint16_t* scratch, long capacity, const int64_t* offsets, int n,
                     uint16_t* words, void* stream);
/* Inverse of encode + pack → ŷ NHWC. status |= 4 a stream ran past its words, 8 a stream did
 * not end in the encoder's initial state with every word consumed (corrupt input). */
int iclr17_rans_decode(const uint16_t* words, const int64_t* offsets, int B, int h, int w, int N,
                       int streams_per_image, const int32_t* cum, int K, float* y_hat,
                       int32_t* status, void* stream);

/* testKodak's MS-SSIM (train.py:178 → models/ms_ssim_torch.py:123-196): per-image
 * ms_ssim(x, y, data_range) of NCHW [B,3,H,W] fp32 images, 11-tap σ=1.5 window, 5 levels (each
 * level must be ≥ 11×11: H, W ≥ 161 or so), the reference's level weights and final product.
 * workspace: iclr17_ms_ssim_workspace_size(B,H,W) bytes (0 = shape unsupported). out: [B]. */
size_t iclr17_ms_ssim_workspace_size(int B, int H, int W);
int iclr17_ms_ssim(const float* x, const float* y, int B, int H, int W, float data_range,
                   void* workspace, size_t workspace_bytes, float* out, void* stream);

/* Single-scale SSIM, models/ms_ssim_torch.py:86-120 (ssim → _ssim :36-83, size_average=False,
 * full=True): per image the means over C·Ho·Wo of the ssim map (out_ssim [B]) and the cs map
 * (out_cs [B], may be null) of NCHW [B,3,H,W] fp32 images, 11-tap σ=1.5 window, H, W ≥ 11.
 * workspace: iclr17_ssim_workspace_size(B,H,W) bytes (0 = shape unsupported). */
size_t iclr17_ssim_workspace_size(int B, int H, int W);
int iclr17_ssim(const float* x, const float* y, int B, int H, int W, float data_range,
                void* workspace, size_t workspace_bytes, float* out_ssim, float* out_cs,
                void* stream);

/* datasets.py:27-33 training transform on the GPU: per image, PIL-exact bilinear resize of its
 * crop box to S×S (two passes, 8-bit fixed point), horizontal / vertical flips, /255 → out NCHW
 * fp32 [B,3,S,S]. src: uint8 HWC images back to back; desc: int64 [B][16] = {src byte offset, H,
 * W, crop top, left, height, width, flip_h, flip_v, tmp byte offset, x-tap offset, x taps per
 * output, y-tap offset, y taps per output, 0, 0}; taps: int32 rows [S][2 + k] = {first, count,
 * k 22-bit taps} per axis (iclr_17_compression_amd/data.py builds them); tmp: Σ crop_h·S·3 bytes;
 * max_ch: the largest crop height. */
int iclr17_resized_crop_batch(const uint8_t* src, const int64_t* desc, int B, int S, int max_ch,
                              const int32_t* taps, uint8_t* tmp, float* out, void* stream);

/* train.py:106-112: element-wise gradient clamp to ±grad_clip (≤ 0: none; written back to the
 * gradient) fused with one torch.optim.Adam step (no weight decay, no amsgrad) over n_tensors
 * parameter tensors in one launch. desc: device int64 [n_tensors][5] = {param, grad, exp_avg,
 * exp_avg_sq, numel} (pointers as integers); step = the 1-based step count after the increment;
 * max_numel = the largest numel. */
int iclr17_adam_step(const int64_t* desc, int n_tensors, long max_numel, double lr, double beta1,
                     double beta2, double eps, long step, float grad_clip, void* stream);

/* Deterministic fixed-order sums: per_image[b] = Σ_t partial[b*T + t] (nullable);
 * *total = (float)(scale · Σ_b per_image[b]) (nullable). model.py:73,78 bits→bpp. */
int iclr17_reduce_partials(const double* partial, int B, int T, double* per_image, float* total,
                           double scale, void* stream);

/* ------------------------------------------------------------------ stand-alone modules */
/* GDN.py:64-94 backward of the stand-alone module (autograd of gdn(x)): from x and g = ∂L/∂y
 * (both in `layout`), writes ∂x (same layout), dn = ∂L/∂n NHWC [B·H·W][C] and, when u_nhwc is
 * non-NULL, x as NHWC [B·H·W][C]. Parameter gradients: ∂β_eff = Σ_p dn (iclr17_bias_grad_nhwc),
 * ∂γ_eff = iclr17_gdn_wgrad(dn, u), then iclr17_gdn_param_chain. */
int iclr17_gdn_bwd(const float* x, const float* g, int B, int C, int H, int W, int layout,
                   int inverse, const float* beta_eff, const float* gamma_packed,
                   const float* gamma_packed_t, float* dx, float* dn, float* u_nhwc,
                   void* stream);
/* bitEstimator.py:20-42 backward of the stand-alone modules for an upstream gradient g (same
 * shape as x; channel of flat element i is (i / inner) % C): ∂x, and per-channel parameter
 * partials partial[iclr17_bitest_bwd_chunks(n, C)][11][C] in the rate-table slots (reduce and
 * chain to ∂h, ∂b, ∂a with iclr17_rate_param_grad). bitparm_bwd: one Bitparm (a == NULL: the
 * final layer, slots 9-10; else slots 0-2); work: 11·C floats. */
int iclr17_bitest_bwd_chunks(int64_t n, int C);
int iclr17_bit_estimator_bwd(const float* x, const float* g, int64_t n, int C, int64_t inner,
                             const float* rate_packed, float* dx, float* partial, void* stream);
int iclr17_bitparm_bwd(const float* x, const float* g, int64_t n, int C, int64_t inner,
                       const float* h, const float* b, const float* a, float* work, float* dx,
                       float* partial, void* stream);
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

/* ------------------------------------------------------------------ backward (training)
 * The autograd of the reference hot path (train.py:105 rd_loss.backward()) as fused kernels.
 * Input gradients reuse the forward engine (conv dgrad = transposed conv and vice versa), each
 * fused with the backward of the GDN/IGDN that precedes it; dn = ∂L/∂n (the GDN norm pool)
 * feeds the GDN parameter gradients. Weight packing for the dgrads: deconv weights with
 * ICLR17_W_CONV5 (deconv1/2) or ICLR17_W_CONV1 (deconv3), conv weights with ICLR17_W_DECONV5.
 * In the three GDN-backward entries the fp32 input gradient (g_v / g_v_prev / g_u_prev) may be
 * NULL when its split form is requested: the x6 backward hands only the split to the next kernel. */

/* ∂recon of λ·mean((recon−x)²) (model.py:61) and/or of a gradient on clamp(recon,0,1)
 * (model.py:59): g_mse, g_clip nullable (device scalar / NCHW tensor). */
int iclr17_grad_recon(const float* recon, const float* x, const float* g_mse, const float* g_clip,
                      int64_t n, float* g_recon, void* stream);
/* synthesis_17.py:23,30 + :22,29 backward: g_v = IGDN2ᵀ(conv2d(g_recon, W3, s4, p4)).
 * g_recon NCHW [B,3,H,W]; v_saved = deconv2 output (pre-IGDN2) NHWC [B,H/4,W/4,N]. */
int iclr17_bwd_deconv3_igdn(const float* g_recon, int B, int H, int W, int N,
                            const float* w_packed, const uint16_t* w_split, const float* v_saved,
                            const float* beta_eff, const float* gamma_packed,
                            const float* gamma_packed_t,
                            const uint16_t* gamma_split, const uint16_t* gamma_t_split, float* g_v, uint16_t* g_v_split,
                            float* dn, float* colsum_gv, float* colsum_dn, void* stream);
/* synthesis_17.py:19-22 / :18 backward: g_v_prev = IGDNᵀ(conv2d(g_v, Wd, s2, p2)).
 * g_v NHWC [B,2h,2w,N]; v_prev = the previous deconv's pre-IGDN output NHWC [B,h,w,N]. */
int iclr17_bwd_deconv_igdn(const float* g_v, const uint16_t* g_v_split, int B, int h, int w,
                           int N, const float* w_packed, const float* v_prev,
                           const float* beta_eff, const float* gamma_packed,
                           const float* gamma_packed_t,
                            const uint16_t* gamma_split, const uint16_t* gamma_t_split, float* g_v_prev, uint16_t* g_v_prev_split,
                           float* dn, float* colsum_gv, float* colsum_dn, void* stream);
/* synthesis_17.py:15 backward + model.py:71-78 rate backward:
 * g_y = conv2d(g_v1, Wd1, s2, p2) + (*g_bpp / count)·∂bits/∂ỹ; per-tile rate parameter partials
 * rate_partial[B * iclr17_rate_bwd_partials(h,w)][11][N]. g_bpp == NULL → no rate term. */
int iclr17_bwd_deconv_rate(const float* g_v, const uint16_t* g_v_split, int B, int h, int w,
                           int N, const float* w_packed, const float* y_tilde,
                           const float* rate_packed, const float* g_bpp, float count, float* g_y,
                           uint16_t* g_y_split, float* rate_partial, void* stream);
int iclr17_rate_bwd_partials(int h, int w);
/* analysis_17.py:22 / :18 backward fused with GDN2 / GDN1 backward:
 * g_u_prev = GDNᵀ(conv_transpose2d(g_u, W, s2, p2, op1)); g_u NHWC [B,h,w,N] (conv output grid),
 * u_prev = the previous conv's pre-GDN output NHWC [B,2h,2w,N]. */
int iclr17_bwd_conv_gdn(const float* g_u, const uint16_t* g_u_split, int B, int h, int w, int N,
                        const float* w_packed, const float* u_prev, const float* beta_eff,
                        const float* gamma_packed, const float* gamma_packed_t,
                            const uint16_t* gamma_split, const uint16_t* gamma_t_split, float* g_u_prev,
                        uint16_t* g_u_prev_split, float* dn, float* colsum_gu, float* colsum_dn,
                        void* stream);
/* x6 backward: the four GDN/rate backward kernels above take their incoming gradient in split
 * form (g_*_split, [3][B][..][N] bf16 planes) when it is non-NULL — the contraction then runs on
 * v_mfma_f32_16x16x32_bf16 in the bf16x6 scheme; the fp32 gradient pointer is then unused and
 * may be NULL — and additionally write their outgoing gradient in split form when
 * *_prev_split / g_y_split / g_v_split is non-NULL. bwd_deconv3_igdn runs x6 when w_split (the
 * deconv3 weight packed ICLR17_W_CONV1_X6 and split by iclr17_split_packed(1, 256, N)) is
 * non-NULL; w_packed may then be NULL. gamma_split / gamma_t_split (nullable: iclr17_split_packed
 * of gamma_packed and gamma_packed_t) run the two GDN-backward channel contractions in x6. */
/* The three GDN-backward kernels above also emit (nullable) per-workgroup column sums of their
 * two outputs, [B * iclr17_bwd_tiles(kind, h, w)][N] floats: Σ ∂u is the preceding layer's bias
 * gradient and Σ dn is ∂β_eff. kind 0 (bwd_deconv3_igdn with (H/4, W/4), bwd_deconv_igdn with
 * (h, w)), kind 1 (bwd_conv_gdn with (h, w)). Reduce them with iclr17_sum_rows. */
int iclr17_bwd_tiles(int kind, int h, int w);
/* iclr17_sum_rows of two [T][C] matrices in one launch pair (each bitwise as iclr17_sum_rows);
 * workspace: 2 · iclr17_sum_rows_workspace_size(C) floats. */
int iclr17_sum_rows2(const float* part_a, const float* part_b, int T, int C, float* workspace,
                     float* out_a, float* out_b, void* stream);
int iclr17_sum_rows(const float* part, int T, int C, float* workspace, float* out, void* stream);
size_t iclr17_sum_rows_workspace_size(int C);   /* floats */
/* Weight gradients in PyTorch layout [m][c][kh][kw] (split-K, fixed-order reduction):
 * k5: G NHWC [B,Ho,Wo,M], X NHWC [B,2Ho,2Wo,C], kind 5 (k5 s2 p2) — conv2/conv3 (G=∂u, X=input)
 *     and deconv1/deconv2 (G=input, X=∂output);
 * k9: G NHWC [B,Ho,Wo,M], X NCHW [B,3,4Ho,4Wo] (k9 s4 p4) — conv1 (G=∂u1, X=image) and
 *     deconv3 (G=s2, X=∂recon). Workspace sizes in floats (kind 5, 9; 1 = GDN). */
size_t iclr17_wgrad_workspace_size(int kind, int B, int Ho, int Wo, int M, int C);
int iclr17_wgrad_k5(const float* G, const float* X, int B, int Ho, int Wo, int M, int C,
                    float* workspace, float* dW, void* stream);
/* wgrad_k5 in the bf16x6 scheme from split-form operands: G_split [3][B][Ho][Wo][M], X_split
 * [3][B][2Ho][2Wo][C] (the x6 activation format); workspace: iclr17_wgrad_workspace_size(6, ...)
 * floats. */
int iclr17_wgrad_k5_x6(const uint16_t* G_split, const uint16_t* X_split, int B, int Ho, int Wo,
                       int M, int C, float* workspace, float* dW, void* stream);
/* wgrad_k9 in the bf16x6 scheme: G_split [3][B][Ho][Wo][M] (split form), X NCHW fp32 [B,3,4Ho,4Wo];
 * the 243-wide window of every output pixel is formed split (im2col, inside the workspace) and
 * contracted as a 1×1 weight gradient. workspace: iclr17_wgrad_workspace_size(7, ...) floats. */
int iclr17_wgrad_k9_x6(const uint16_t* G_split, const float* X, int B, int Ho, int Wo, int M,
                       float* workspace, float* dW, void* stream);
int iclr17_wgrad_k9(const float* G, const float* X, int B, int Ho, int Wo, int M,
                    float* workspace, float* dW, void* stream);
/* GDN.py:83 weight gradient: dgamma_eff[i][j] = Σ_p dn[p][i]·u[p][j]² (dβ_eff = Σ_p dn comes
 * from the backward kernels' column sums). */
size_t iclr17_gdn_wgrad_workspace_size(long P, int C);
int iclr17_gdn_wgrad(const float* dn, const float* u, long P, int C, float* workspace,
                     float* dgamma_eff, void* stream);
/* The same gradient in the x6 scheme: dn and u² split into three bf16 parts inside the kernel,
 * six part products per MAC on the bf16 MFMA, fp32 accumulation. */
size_t iclr17_gdn_wgrad_x6_workspace_size(long P, int C);
int iclr17_gdn_wgrad_x6(const float* dn, const float* u, long P, int C, float* workspace,
                        float* dgamma_eff, void* stream);
/* GDN.py:10-24,73-79 chain: dβ = LowerBoundᵀ(dβ_eff · 2·max(β, bβ)), same for γ. */
int iclr17_gdn_param_chain(const float* beta, const float* gamma, const float* dbeta_eff,
                           const float* dgamma_eff, int C, float beta_bound, float gamma_bound,
                           float* dbeta, float* dgamma, void* stream);
/* Bias gradients: Σ over pixels of an NHWC [P][C] or NCHW [B][C][HW] gradient.
 * Workspace: (1024 + 64)*C floats (NHWC), (B·⌈HW/4096⌉ + 64)*C floats (NCHW). */
int iclr17_bias_grad_nhwc(const float* G, long P, int C, float* workspace, float* db, void* stream);
int iclr17_bias_grad_nchw(const float* G, int B, int C, long HW, float* workspace, float* db,
                          void* stream);
/* BitEstimator parameter gradients (bitEstimator.py:13-25) from the rate partials [T][11][C]. */
int iclr17_rate_param_grad(const float* partial, int T, int C, const float* h1, const float* a1,
                           const float* h2, const float* a2, const float* h3, const float* a3,
                           const float* h4, float* dh1, float* db1, float* da1, float* dh2,
                           float* db2, float* da2, float* dh3, float* db3, float* da3, float* dh4,
                           float* db4, void* stream);

/* ------------------------------------------------------------------ h3 form (32x32x16 f16)
 * The parity mode's k5 layers with THREE fp16 part products per MAC on v_mfma_f32_32x32x16_f16
 * (csrc/engine_h3.hip, csrc/common.h "h3 form"): an activation is stored as two fp16 planes
 * [2][…] of a = x·2^-6, hi = rne16(a) and lo = rne16((a − hi)·2^11); weights the same way with a
 * per-tensor power-of-two scale chosen at packing. Against float64 its dot products land closer
 * than the x6 chain's (tools/h3_numerics.hip). |x| ≥ 2^22 does not fit the form: the kernels then
 * set *range_flag (nullable) to 1 (conv3_quant_rate_h3: 2). Halo patch of the h3 input per 16-channel chunk, a wave owns 32
 * pixels × all N channels, GDN/IGDN contraction (in the h3 form) from the accumulators.
 * Replaces iclr17_synthesis_deconv_igdn_x6[_cm] on the parity path
 * (synthesis_17.py:15-22; models/GDN.py:64-94, inverse). */
#define ICLR17_H3K_CONV5 42   /* conv2 W[co][ci][5][5] → [2][N/8·13][2][N][8] fp16 planes + trailer */
#define ICLR17_H3K_DECONV5 43 /* deconv1/2 W[ci][co][5][5] → [2][4 phases: N/16·T_p][2][N][8] + trailer */
#define ICLR17_H3K_CONV1 44   /* conv1 W[co][3][9][9] → [2][16 steps][2][N][8] (reordered K) + trailer */
/* uint16 elements: two planes + an 8-element (16-byte) trailer {max|w|, 2^-11/(σ_a·σ_w)}; 0 =
 * unsupported */
size_t iclr17_h3k_weight_size(int which, int N);
int iclr17_pack_h3k(int which, const float* w, uint16_t* out, int N, void* stream);
/* fp32 x[n] (n % 4 == 0) → h3 planes [2][n] */
int iclr17_h3_planes(const float* x, long n, uint16_t* planes, int* range_flag, void* stream);
/* fp32 NHWC x [B][h][w][N] → h3 planes chunk-major [2][B][N/cm][h][w][cm] (cm 8, 16 or 32): the
 * layout each h3 layer reads (conv2 / conv3: cm 8; deconv1 / deconv2: cm 16; deconv3: cm 32) */
int iclr17_h3_planes_cm(const float* x, int B, int h, int w, int N, int cm, uint16_t* planes,
                        int* range_flag, void* stream);
/* A packed operand [taps][K/4][N][4] fp32 → two fp16 planes [2][taps][K/8][N][8] of w·σ_w + the
 * trailer (the h3 conv3 weights: the ICLR17_W_CONV5 packing with taps 25, K = N; deconv3's
 * ICLR17_W_DECONV9 packing with taps 9, 48 columns; a GDN γ_eff packing with taps 1, K = N).
 * iclr17_split_packed_h3_size() uint16 elements (0 = bad arguments). */
size_t iclr17_split_packed_h3_size(int taps, int K, int N);
int iclr17_split_packed_h3(const float* packed, int taps, int K, int N, uint16_t* planes,
                           void* stream);
/* A batch of h3 packs in two launches (every job's max|w|, then every job's planes), bitwise
 * those of the single-pack entry points: a training step's h3 layouts without two launches per
 * pack. jobs (iclr17_pack_job above): ICLR17_PACK_H3K (src0 = w, dst0 = out, N, K = the
 * ICLR17_H3K_* kind: as iclr17_pack_h3k) or ICLR17_PACK_SPLIT_H3 (src0 = packed, dst0 = planes,
 * taps, K, N: as iclr17_split_packed_h3). At most ICLR17_PACK_H3_MAXJ jobs. */
#define ICLR17_PACK_H3K 19
#define ICLR17_PACK_SPLIT_H3 20
#define ICLR17_PACK_H3_MAXJ 16
int iclr17_pack_h3_batch(const iclr17_pack_job* jobs, int n, void* stream);
/* analysis_17.py:14-17 conv1 + GDN1 on the h3 engine (csrc/engine_h3.hip): 16×16-pixel output
 * tiles of 8 waves; the tile's 3 × 69 × 69 input window split once into the two h3 planes in LDS,
 * K = 243 reordered into 16 steps of 16, three f16 part products per MAC, GDN contraction in the
 * h3 form. Outputs (each nullable, not all): fp32 NHWC, the h3 form [2][B][H/4][W/4][N] (out_cm
 * 0) or chunk-major [2][B][N/out_cm][H/4][W/4][out_cm] (out_cm 8, 16, 32; conv2 reads 8), the x6
 * split [3][B][H/4][W/4][N]; pre_out (nullable): GDN1's input conv1 + bias, fp32 NHWC (training).
 * w_h3k: iclr17_pack_h3k(ICLR17_H3K_CONV1); gamma_h3: iclr17_split_packed_h3(γ_eff packing, 1, N, N). */
int iclr17_analysis_conv1_gdn_h3(const float* x, int B, int H, int W, int N,
                                 const uint16_t* w_h3k, const float* bias, const float* beta_eff,
                                 const uint16_t* gamma_h3, float* out, float* pre_out,
                                 uint16_t* out_h3, int out_cm, uint16_t* out_x6, int* range_flag,
                                 void* stream);
/* analysis_17.py:18-21 conv2 + GDN2 on the h3 engine: 16×16-pixel tiles of 8 waves, 8-channel
 * chunks with two taps per 16-deep MFMA step, three f16 part products per MAC; input the h3 form
 * chunk-major 8, [2][B][N/8][H/4][W/4][8] (a patch piece is 16 contiguous bytes). Outputs as
 * conv1_gdn_h3 at [B][H/8][W/8][N] (conv3 reads out_cm 8). w_h3k:
 * iclr17_pack_h3k(ICLR17_H3K_CONV5); gamma_h3 as above. */
int iclr17_analysis_conv2_gdn_h3(const uint16_t* in_h3, int B, int H, int W, int N,
                                 const uint16_t* w_h3k, const float* bias, const float* beta_eff,
                                 const uint16_t* gamma_h3, float* out, float* pre_out,
                                 uint16_t* out_h3, int out_cm, uint16_t* out_x6, int* range_flag,
                                 void* stream);
/* analysis_17.py:22 + model.py:48-56,71-73 on the h3 engine (csrc/engine_h3.hip): as
 * iclr17_analysis_conv3_quant_rate (round or noise mode, rate_table nullable; y_out nullable), ŷ
 * also in the h3 form (y_hat_h3 nullable; layout out_cm as conv1_gdn_h3, deconv1 reads 16). Input
 * the h3 form chunk-major 8 (conv2_gdn_h3 with out_cm 8). 8 × 16-pixel output tiles of 4 waves,
 * each workgroup one 64-channel slice of the output channels, 8-channel input chunks summed
 * two-level. w_h3k: iclr17_pack_h3k(ICLR17_H3K_CONV5) of conv3's weights. Bit partials
 * [B][iclr17_conv3_h3_partials_per_image(B, H, W, N, quant_mode)]. range_flag: when bit 0 is set
 * on entry (an earlier h3 kernel of the chain met |x| ≥ 2^22) every output — y, ŷ, its h3 form,
 * the bit partials — is NaN; this kernel's own overflow (ŷ's h3 form) sets bit 1. */
int iclr17_conv3_h3_partials_per_image(int B, int H, int W, int N, int quant_mode);
int iclr17_analysis_conv3_quant_rate_h3(const uint16_t* in_h3, int B, int H, int W, int N,
                                        const uint16_t* w_h3k, int quant_mode, const float* noise,
                                        const float* rate_packed, const float* rate_table,
                                        float* y_out, float* y_hat, uint16_t* y_hat_h3, int out_cm,
                                        double* bits_partial, int* range_flag, void* stream);
/* synthesis_17.py:23-25 deconv3 + model.py:59 clamp on the h3 form: the chunk-major h3 input
 * [2][B][N/32][H/4][W/4][32] (iclr17_synthesis_deconv_igdn_h3 with out_cm) → clipped NCHW fp32
 * (+ unclipped, + SSE partials as iclr17_synthesis_deconv3); w_h3: iclr17_split_packed_h3 of the
 * ICLR17_W_DECONV9 packing (taps 9, K N, columns 48). bits_partial non-NULL: the bit reduction
 * folded in as iclr17_synthesis_deconv3_x6_cm_bits (bits_per_image nullable). range_flag
 * (nullable, read only): the chain's h3 range flag; when it is set (an upstream h3 kernel met
 * |x| ≥ 2^22) every output of this call — clipped, recon, SSE partials, bit totals — is NaN, so
 * the out-of-range result is loud without a host synchronisation. */
int iclr17_synthesis_deconv3_h3(const uint16_t* in_h3_cm, int B, int H, int W, int N,
                                const uint16_t* w_h3, const float* bias, const float* x,
                                float* clipped, float* recon, double* sse_partial,
                                int sse_unclipped, const double* bits_partial, int bits_T,
                                double* bits_per_image, float* bpp_total, double bits_scale,
                                const int* range_flag, void* stream);
/* synthesis_17.py:15-22 deconv + IGDN on the h3 engine: input the h3 form chunk-major 16,
 * [2][B][N/16][h][w][16] → fp32 NHWC [B][2h][2w][N] and/or the h3 output (layout out_cm as
 * conv1_gdn_h3: deconv2 reads 16, deconv3 32) and/or the x6 split output [3][B][2h][2w][N] (NHWC
 * always) — each nullable, not all; pre_out (nullable): the IGDN input deconv + bias, fp32 NHWC
 * (training). int_in: the input is integer-valued (ŷ): a workgroup
 * whose input window has an all-zero lo plane (every value exact in the hi plane: integers with
 * |ŷ| < 2¹¹) runs the two products with hi_a only (same result); any other workgroup runs
 * the full three. w_h3k: iclr17_pack_h3k(ICLR17_H3K_DECONV5); gamma_h3:
 * iclr17_split_packed_h3(γ_eff packing, 1, N, N). */
int iclr17_synthesis_deconv_igdn_h3(const uint16_t* in_h3, int B, int h, int w, int N,
                                    const uint16_t* w_h3k, const float* bias,
                                    const float* beta_eff, const uint16_t* gamma_h3,
                                    float* out, float* pre_out, uint16_t* out_h3, uint16_t* out_x6,
                                    int out_cm, int int_in, int* range_flag, void* stream);

/* ------------------------------------------------------------------ bf16 throughput mode
 * The codec forward with bf16 activations (NHWC [B][h][w][N], round to nearest even), bf16
 * weights and γ, ONE v_mfma_f32_16x16x32_bf16 product per MAC with fp32 accumulation, fp32
 * epilogues (csrc/engine_bf16.hip). Same layers and arguments as the fp32 / x6 entry points
 * above; no bit-identity claim (flip rate, Δbpp and ΔPSNR are reported instead).
 * Weight layouts: iclr17_pack_bf16 (k5 layers), iclr17_round_packed of the fp32 packings
 * (conv1: ICLR17_W_CONV1_X6 with taps 1, K 256; GDN γ: iclr17_pack_gdn's gp with taps 1, K = N). */
#define ICLR17_BF_CONV5 32   /* conv2/conv3 W[co][ci][5][5] → [N/16][13][4][N][8] bf16 */
#define ICLR17_BF_DECONV5 33 /* deconv1/2 W[ci][co][5][5] → 4 phases [N/16][S_p][4][N][8] bf16 */
size_t iclr17_bf16_weight_size(int which, int N);   /* uint16 elements; 0 = unsupported */
int iclr17_pack_bf16(int which, const float* w, uint16_t* out, int N, void* stream);
/* packed fp32 [taps][K/4][N][4] → bf16 [taps][K/8][N][8] (round to nearest even) */
int iclr17_round_packed(const float* packed, int taps, int K, int N, uint16_t* out, void* stream);
/* fp32 → bf16 (round to nearest even), n a multiple of 8 */
int iclr17_to_bf16(const float* x, long n, uint16_t* out, void* stream);
/* analysis_17.py:14-17 conv1 + GDN1: x NCHW fp32 → out bf16 NHWC [B,H/4,W/4,N] */
int iclr17_analysis_conv1_gdn_bf16(const float* x, int B, int H, int W, int N,
                                   const uint16_t* w_bf16, const float* bias,
                                   const float* beta_eff, const uint16_t* gamma_bf16,
                                   uint16_t* out, void* stream);
/* analysis_17.py:18-21 conv2 + GDN2: bf16 NHWC [B,H/4,W/4,N] → bf16 NHWC [B,H/8,W/8,N] */
int iclr17_analysis_conv2_gdn_bf16(const uint16_t* in, int B, int H, int W, int N,
                                   const uint16_t* w_bf16, const float* bias, const float* beta_eff,
                                   const uint16_t* gamma_bf16, uint16_t* out, void* stream);
/* model.py:71-73 per element for the integer latents v ∈ [−32, 32] of each channel:
 * table[c][v + 32] = clamp(−log2(F_c(v+½) − F_c(v−½) + 1e-10), 0, 50) from the packed rate
 * parameters (iclr17_pack_rate); iclr17_rate_table_size(N) floats. */
size_t iclr17_rate_table_size(int N);
int iclr17_rate_table(const float* rate_packed, int N, float* table, void* stream);
/* analysis_17.py:22 + model.py:56,71-73 (round mode): → ŷ fp32 NHWC, ŷ bf16 NHWC, optional y
 * fp32 NHWC, bit partials [B][iclr17_bf16_rate_partials_per_image] (float64); rate_table from
 * iclr17_rate_table of the same rate_packed (|ŷ| > 32 evaluates the model directly). */
int iclr17_bf16_rate_partials_per_image(int H, int W, int N);
int iclr17_analysis_conv3_quant_rate_bf16(const uint16_t* in, int B, int H, int W, int N,
                                          const uint16_t* w_bf16, const float* rate_packed,
                                          const float* rate_table, float* y_out, float* y_hat,
                                          uint16_t* y_hat_bf16, double* bits_partial,
                                          void* stream);
/* synthesis_17.py:15-22 deconv + IGDN: bf16 NHWC [B,h,w,N] → bf16 NHWC [B,2h,2w,N] */
int iclr17_synthesis_deconv_igdn_bf16(const uint16_t* in, int B, int h, int w, int N,
                                      const uint16_t* w_bf16, const float* bias,
                                      const float* beta_eff, const uint16_t* gamma_bf16,
                                      uint16_t* out, void* stream);
/* synthesis_17.py:23-25 deconv3 + model.py:59 clamp: bf16 NHWC [B,H/4,W/4,N] → clipped NCHW
 * fp32 (+ unclipped, + SSE partials as iclr17_synthesis_deconv3). w_bf16: iclr17_round_packed
 * (taps 9, K N, columns 48) of the ICLR17_W_DECONV9 packing. */
int iclr17_synthesis_deconv3_bf16(const uint16_t* in, int B, int H, int W, int N,
                                  const uint16_t* w_bf16, const float* bias, const float* x_ref,
                                  float* clipped, float* recon, double* sse_partial,
                                  int sse_unclipped, void* stream);
/* iclr17_synthesis_deconv3_bf16 with the bit reduction folded in, as
 * iclr17_synthesis_deconv3_x6_cm_bits. */
int iclr17_synthesis_deconv3_bf16_bits(const uint16_t* in, int B, int H, int W, int N,
                                       const uint16_t* w_bf16, const float* bias, const float* x_ref,
                                       float* clipped, float* recon, double* sse_partial,
                                       int sse_unclipped, const double* bits_partial, int bits_T,
                                       double* bits_per_image, float* bpp_total, double bits_scale,
                                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ICLR17_H_ */
