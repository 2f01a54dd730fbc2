// adam_update.h — the per-element Adam arithmetic shared by adam_kernel (adam.hip) and the fused
// update + operand prep of the prototype layer (l2_adam_prep_kernel, l2_bf16.hip), so both give
// the same bits: torch.optim.Adam (reference segmentation/module.py:391; amsgrad and maximize
// off, L2 weight decay), f32, bias corrections from the tensor's device step count.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace protoseg {

struct AdamCorr {
  int t;               // this step's count (state[0] + 1)
  float step_size;     // lr / (1 - beta1^t)
  float bc2_sqrt;      // sqrt(1 - beta2^t)
};

// Bias corrections of step t = state[0] + 1: beta^t by squaring in f64 (one thread per tensor).
__device__ inline AdamCorr adam_corr(const int* state, float lr, float beta1, float beta2) {
  const int t = __atomic_load_n(state, __ATOMIC_RELAXED) + 1;
  double p1 = 1.0, p2 = 1.0, s1 = beta1, s2 = beta2;
  for (int e = t; e > 0; e >>= 1, s1 *= s1, s2 *= s2)
    if (e & 1) p1 *= s1, p2 *= s2;
  AdamCorr c;
  c.t = t;
  c.step_size = lr / static_cast<float>(1.0 - p1);
  c.bc2_sqrt = static_cast<float>(sqrt(1.0 - p2));
  return c;
}

//   g = grad + wd p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g
//   p -= step_size m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// No contraction: the compiler's choice of fused multiply-adds would otherwise depend on the
// calling kernel, and the two kernels must give the same bits (the weight-decay fma is explicit).
__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float grad, float step_size, float bc2_sqrt,
                                            float beta1, float beta2, float eps, float wd) {
#pragma clang fp contract(off)
  float gr = grad;
  if (wd != 0.f) gr = fmaf(wd, p, gr);
  m = beta1 * m + (1.f - beta1) * gr;
  v = beta2 * v + (1.f - beta2) * gr * gr;
  p = p - step_size * m / (sqrtf(v) / bc2_sqrt + eps);
}

}  // namespace protoseg
