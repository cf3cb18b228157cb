// pkc_optim.h — element update of the multi-tensor optimizer, shared by pkc_optim_step and the
// matmul epilogue that fuses the weight update into the dW product (pkc_gemm_grouped).
#pragma once
#include "pkc_common.h"

namespace pkc {

struct OptState {
  float p, g, s1, s2, s3, m;
};

// one element of torch.optim SGD / RMSprop / Adam + mask + clamp (see file header)
__device__ __forceinline__ void opt_update(const pkc_opt_tensor& t, OptState& e) {
  float p = e.p;
  float g = e.g;
  if (t.wd != 0.f) g = g + t.wd * p;
  if (t.kind == PKC_OPT_SGD) {
    // torch/optim/sgd.py: buf = g (first step) | momentum*buf + (1-dampening)*g
    if (t.momentum != 0.f) {
      const float buf = (t.step <= 1) ? g : t.momentum * e.s1 + (1.f - t.dampening) * g;
      e.s1 = buf;
      g = t.nesterov ? g + t.momentum * buf : buf;
    }
    p = p + (-t.lr) * g;
  } else if (t.kind == PKC_OPT_RMSPROP) {
    // torch/optim/rmsprop.py: sq = alpha*sq + (1-alpha)*g^2; avg = sqrt(sq) + eps
    const float sq = e.s1 * t.alpha + (1.f - t.alpha) * g * g;
    e.s1 = sq;
    float avg;
    if (t.centered) {
      const float ga = e.s2 * t.alpha + (1.f - t.alpha) * g;
      e.s2 = ga;
      avg = sqrtf(sq - ga * ga) + t.eps;
    } else {
      avg = sqrtf(sq) + t.eps;
    }
    if (t.momentum > 0.f) {
      const float buf = e.s3 * t.momentum + g / avg;
      e.s3 = buf;
      p = p + (-t.lr) * buf;
    } else {
      p = p + (-t.lr) * (g / avg);
    }
  } else {
    // torch/optim/adam.py (non-foreach math)
    const float m = e.s1 + (g - e.s1) * (1.f - t.beta1);
    const float v = e.s2 * t.beta2 + (1.f - t.beta2) * g * g;
    e.s1 = m;
    e.s2 = v;
    const float bc1 = 1.f - powf(t.beta1, (float)t.step);
    const float bc2 = 1.f - powf(t.beta2, (float)t.step);
    float vv = v;
    if (t.amsgrad) {
      vv = fmaxf(e.s3, v);
      e.s3 = vv;
    }
    const float denom = sqrtf(vv) / sqrtf(bc2) + t.eps;
    p = p + (-(t.lr / bc1)) * (m / denom);
  }
  if (t.mask) p *= e.m;
  if (t.clampv > 0.f) p = fminf(fmaxf(p, -t.clampv), t.clampv);
  e.p = p;
}

__device__ __forceinline__ float quant_w(float p, int bits) {
  // Quantize(balanced=False) of the clamped weight (quantized_modules.py:91-96)
  const float sc = ldexpf(1.f, bits - 1);
  const float sg = p > 0.f ? 1.f : (p < 0.f ? -1.f : 0.f);
  return ceilf(fabsf(p) * sc) / sc * sg;
}

}  // namespace pkc
