// Fused gradient clamp + Adam step over all parameter tensors in one launch — train.py:106-112
// (clip_gradient: element-wise clamp to ±grad_clip, then optimizer.step() of torch.optim.Adam
// with the defaults the reference uses: betas (0.9, 0.999), eps 1e-8, no weight decay, no
// amsgrad).
//
// Per element, in torch's single-tensor Adam order (torch/optim/adam.py, _single_tensor_adam):
//   g  = clamp(g, −c, c)                 (written back: the reference clamps p.grad in place)
//   m  = m + (1−β1)·(g − m)              lerp_, fused as torch's CPU kernel does: fma(w, g−m, m)
//   v  = v·β2 + (1−β2)·g·g               mul_ + addcmul_: fma((1−β2)·g, g, v·β2)
//   d  = √v / √bc2 + ε                   bc2 = 1 − β2^t, from double scalars cast to fp32
//   p  = p + (−lr/bc1 · m) / d           addcdiv_(m, d, value=−lr/bc1), bc1 = 1 − β1^t
// The library is built with -ffp-contract=off, so the two fmas are explicit and nothing else
// fuses.
#include "common.h"

namespace iclr17 {
namespace {

struct AdamTensor {   // mirrors the int64 [5] rows of the descriptor table
  float* p;
  float* g;
  float* m;
  float* v;
  long n;
};

__global__ void __launch_bounds__(256) adam_step_kernel(const AdamTensor* __restrict__ desc,
                                                        float neg_step_size, float bc2_sqrt,
                                                        float w1, float beta2, float c2, float eps,
                                                        float clip) {
  const AdamTensor t = desc[blockIdx.y];
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < t.n; i += (long)gridDim.x * 256) {
    float g = t.g[i];
    if (clip > 0.f) {
      g = fminf(fmaxf(g, -clip), clip);
      t.g[i] = g;
    }
    const float m = fmaf(w1, g - t.m[i], t.m[i]);
    const float v = fmaf(c2 * g, g, t.v[i] * beta2);
    t.m[i] = m;
    t.v[i] = v;
    const float d = sqrtf(v) / bc2_sqrt + eps;
    t.p[i] = t.p[i] + (neg_step_size * m) / d;
  }
}

}  // namespace
}  // namespace iclr17

using namespace iclr17;

extern "C" {

int iclr17_adam_step(const int64_t* desc, int n_tensors, long max_numel, double lr, double beta1,
                     double beta2, double eps, long step, float grad_clip, void* stream) {
  ICLR17_REQUIRE(desc && n_tensors > 0 && max_numel > 0 && step >= 1, ICLR17_EINVAL,
                 "adam_step: bad arguments");
  ICLR17_REQUIRE(sizeof(AdamTensor) == 5 * sizeof(int64_t), ICLR17_EINVAL, "adam_step: layout");
  // the Python-float scalars of _single_tensor_adam, then fp32 as the tensor ops see them
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  const double step_size = lr / bc1;
  const double bc2_sqrt = pow(bc2, 0.5);
  const long per_block = 256L * 4;
  const long bx = (max_numel + per_block - 1) / per_block;
  dim3 grid((unsigned)(bx < 1024 ? bx : 1024), (unsigned)n_tensors);
  hipLaunchKernelGGL(adam_step_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                     (const AdamTensor*)desc, (float)(-step_size), (float)bc2_sqrt,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps,
                     grad_clip);
  return check_launch("adam_step");
}

}  // extern "C"
