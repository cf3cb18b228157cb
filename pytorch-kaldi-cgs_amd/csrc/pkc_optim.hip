// pkc_optim.hip — one launch steps every parameter tensor of every architecture.
//
// Restates torch.optim SGD / RMSprop / Adam (the optimizers utils.optimizer_init builds,
// utils.py:1833-1881, stepped per architecture at core.py:230-232) elementwise, and fuses the
// weight preparation the reference performs at the start of the NEXT forward:
//   HCGS / pattern masks multiplied into W in place (neural_networks.py:258, 858-861, 980-983)
//   QuantizeLinear's in-place clamp of W to [-1, 1] (quantized_modules.py:79).
// Masked entries only ever feed the optimizer through the (dense) gradient, never through W, so
// storing W*mask here is numerically identical to the reference's mask-at-forward order.
#include "pkc_common.h"

namespace pkc {

constexpr int OPT_T = 256, OPT_PER = 8, OPT_CHUNK = OPT_T * OPT_PER;

__global__ __launch_bounds__(OPT_T) void optim_kernel(const pkc_opt_tensor* ts, const int32_t* map) {
  const int ti = map[2 * blockIdx.x];
  const int64_t start = (int64_t)map[2 * blockIdx.x + 1] * OPT_CHUNK;
  const pkc_opt_tensor t = ts[ti];
  for (int j = 0; j < OPT_PER; ++j) {
    const int64_t i = start + threadIdx.x + (int64_t)j * OPT_T;
    if (i >= t.n) return;
    float p = t.p[i];
    float g = t.g[i];
    if (t.wd != 0.f) g = g + t.wd * p;
    if (t.kind == PKC_OPT_SGD) {
      // torch/optim/sgd.py: buf = g (first step) | momentum*buf + (1-dampening)*g
      if (t.momentum != 0.f) {
        float buf = (t.step <= 1) ? g : t.momentum * t.s1[i] + (1.f - t.dampening) * g;
        t.s1[i] = buf;
        g = t.nesterov ? g + t.momentum * buf : buf;
      }
      p = p + (-t.lr) * g;
    } else if (t.kind == PKC_OPT_RMSPROP) {
      // torch/optim/rmsprop.py: sq = alpha*sq + (1-alpha)*g^2; avg = sqrt(sq) + eps
      const float sq = t.s1[i] * t.alpha + (1.f - t.alpha) * g * g;
      t.s1[i] = sq;
      float avg;
      if (t.centered) {
        const float ga = t.s2[i] * t.alpha + (1.f - t.alpha) * g;
        t.s2[i] = ga;
        avg = sqrtf(sq - ga * ga) + t.eps;
      } else {
        avg = sqrtf(sq) + t.eps;
      }
      if (t.momentum > 0.f) {
        const float buf = t.s3[i] * t.momentum + g / avg;
        t.s3[i] = buf;
        p = p + (-t.lr) * buf;
      } else {
        p = p + (-t.lr) * (g / avg);
      }
    } else {
      // torch/optim/adam.py (non-foreach math)
      const float m = t.s1[i] + (g - t.s1[i]) * (1.f - t.beta1);
      const float v = t.s2[i] * t.beta2 + (1.f - t.beta2) * g * g;
      t.s1[i] = m;
      t.s2[i] = v;
      const float bc1 = 1.f - powf(t.beta1, (float)t.step);
      const float bc2 = 1.f - powf(t.beta2, (float)t.step);
      float vv = v;
      if (t.amsgrad) {
        vv = fmaxf(t.s3[i], v);
        t.s3[i] = vv;
      }
      const float denom = sqrtf(vv) / sqrtf(bc2) + t.eps;
      p = p + (-(t.lr / bc1)) * (m / denom);
    }
    if (t.mask) p *= t.mask[i];
    if (t.clampv > 0.f) p = fminf(fmaxf(p, -t.clampv), t.clampv);
    t.p[i] = p;
    if (t.qbits > 0) {   // Quantize(balanced=False) of the clamped weight (quantized_modules.py:91-96)
      const float sc = ldexpf(1.f, t.qbits - 1);
      const float sg = p > 0.f ? 1.f : (p < 0.f ? -1.f : 0.f);
      t.qout[i] = ceilf(fabsf(p) * sc) / sc * sg;
    }
  }
}

__global__ void apply_mask_kernel(float* p, const float* mask, int64_t n, float clampv) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = p[i];
    if (mask) v *= mask[i];
    if (clampv > 0.f) v = fminf(fmaxf(v, -clampv), clampv);
    p[i] = v;
  }
}

}  // namespace pkc

extern "C" int pkc_optim_chunks(const int64_t* sizes, int ntensors, int32_t* map_out, int cap) {
  using namespace pkc;
  int n = 0;
  for (int t = 0; t < ntensors; ++t) {
    const int64_t nc = (sizes[t] + OPT_CHUNK - 1) / OPT_CHUNK;
    for (int64_t c = 0; c < nc; ++c) {
      if (map_out && n < cap) {
        map_out[2 * n] = t;
        map_out[2 * n + 1] = (int32_t)c;
      }
      ++n;
    }
  }
  return n;
}

extern "C" int pkc_optim_step(const pkc_opt_tensor* tensors_dev, int ntensors,
                              const int32_t* chunk_map_dev, int nchunks, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(tensors_dev && chunk_map_dev && ntensors > 0, "pkc_optim_step: bad arguments");
  if (nchunks <= 0) return PKC_OK;
  hipLaunchKernelGGL(optim_kernel, dim3(nchunks), dim3(OPT_T), 0, S(stream), tensors_dev,
                     chunk_map_dev);
  PKC_LAUNCH_CHECK("pkc_optim_step");
  return PKC_OK;
}

extern "C" int pkc_apply_mask(float* p, const float* mask, int64_t n, float clampv, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(p && n >= 0, "pkc_apply_mask: bad arguments");
  if (n == 0) return PKC_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(apply_mask_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), p, mask, n,
                     clampv);
  PKC_LAUNCH_CHECK("pkc_apply_mask");
  return PKC_OK;
}
