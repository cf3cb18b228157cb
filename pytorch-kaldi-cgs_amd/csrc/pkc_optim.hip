// pkc_optim.hip — one launch steps every parameter tensor of every architecture.
//
// Restates torch.optim SGD / RMSprop / Adam (the optimizers utils.optimizer_init builds,
// utils.py:1833-1881, stepped per architecture at core.py:230-232) elementwise, and fuses the
// weight preparation the reference performs at the start of the NEXT forward:
//   HCGS / pattern masks multiplied into W in place (neural_networks.py:258, 858-861, 980-983)
//   QuantizeLinear's in-place clamp of W to [-1, 1] (quantized_modules.py:79).
// Masked entries only ever feed the optimizer through the (dense) gradient, never through W, so
// storing W*mask here is numerically identical to the reference's mask-at-forward order.
#include "pkc_optim.h"

namespace pkc {


__global__ __launch_bounds__(OPT_T) void optim_kernel(const pkc_opt_tensor* ts, const int32_t* map) {
  optim_wg(ts, map, blockIdx.x);
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
