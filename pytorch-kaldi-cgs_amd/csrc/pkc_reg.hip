// pkc_reg.hip — the [model] regularisers cost_l1 / cost_l2 / cost_gl (utils.py:24-60, 1954-1991):
//   l1: lam * sum_p ||p||_1                 d/dp = lam * sign(p)
//   l2: lam * sum_p ||p||_2   (NOT squared)  d/dp = lam * p / ||p||_2
//   gl: lam * sum_p sum_blk ||blk||_2        d/dp = lam * p / ||blk||_2
// over every dim > 1 parameter of the archs without skip_regularization.  gl blocks are the
// torch.chunk(p, nblk, 1) x torch.chunk(., nblk, 0) grid; l1/l2 have one block per parameter.
//
// A block is cut into row slices ("items", a few thousand elements each) so that the reduction is
// spread over many CUs and stays deterministic: pkc_reg_partial writes one partial per item,
// pkc_reg_finalize sums each block's items in order (one workgroup), turns the block norms into
// the loss term and the per-block gradient coefficients, and pkc_reg_grad adds the gradient into
// the parameters' dW buffers (after any gradient all-reduce: the term is the same on every rank).
#include "pkc_common.h"

namespace pkc {

constexpr int RT = 256;

__device__ __forceinline__ float block_reduce(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < RT / 64; ++i) t += red[i];
  return t;
}

__global__ __launch_bounds__(RT) void reg_partial_kernel(int kind, const pkc_reg_item* items,
                                                         float* partial) {
  __shared__ float red[RT / 64];
  const pkc_reg_item it = items[blockIdx.x];
  const int w = it.c1 - it.c0;
  const int64_t n = (int64_t)(it.r1 - it.r0) * w;
  float acc = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += RT) {
    const int64_t r = it.r0 + e / w, c = it.c0 + e % w;
    const float x = it.p[r * it.ld + c];
    acc += kind == PKC_REG_L1 ? fabsf(x) : x * x;
  }
  const float t = block_reduce(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ __launch_bounds__(RT) void reg_finalize_kernel(int kind, const int32_t* bstart, int nblocks,
                                                          const float* partial, float lam,
                                                          float* coef, float* rows, int nrows) {
  __shared__ float red[RT / 64];
  __shared__ float total;
  // one thread per block (blocks are few: parameters x nblk^2); items of a block in order
  float mine = 0.f;
  for (int b = threadIdx.x; b < nblocks; b += RT) {
    float s = 0.f;
    for (int i = bstart[b]; i < bstart[b + 1]; ++i) s += partial[i];
    const float nrm = kind == PKC_REG_L1 ? s : sqrtf(s);
    coef[b] = kind == PKC_REG_L1 ? lam : (nrm > 0.f ? lam / nrm : 0.f);
    mine += nrm;
  }
  // the reference adds the norms in parameter order in fp32; a tree sum differs by rounding only
  const float t = block_reduce(mine, red);
  if (threadIdx.x == 0) total = t * lam;
  __syncthreads();
  for (int i = threadIdx.x; i < nrows; i += RT) rows[i] = total;
}

__global__ __launch_bounds__(RT) void reg_grad_kernel(int kind, const pkc_reg_item* items,
                                                      const float* coef) {
  const pkc_reg_item it = items[blockIdx.x];
  if (!it.g) return;
  const float k = coef[it.block];
  const int w = it.c1 - it.c0;
  const int64_t n = (int64_t)(it.r1 - it.r0) * w;
  for (int64_t e = threadIdx.x; e < n; e += RT) {
    const int64_t i = (it.r0 + e / w) * it.ld + it.c0 + e % w;
    const float x = it.p[i];
    const float d = kind == PKC_REG_L1 ? k * (x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f)) : k * x;
    it.g[i] = it.assign ? d : it.g[i] + d;
  }
}

}  // namespace pkc

extern "C" int pkc_reg_partial(int kind, const pkc_reg_item* items, int nitems, float* partial,
                               void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG((kind == PKC_REG_L1 || kind == PKC_REG_L2) && items && partial && nitems > 0,
                "pkc_reg_partial: bad arguments");
  hipLaunchKernelGGL(reg_partial_kernel, dim3(nitems), dim3(RT), 0, S(stream), kind, items, partial);
  PKC_LAUNCH_CHECK("pkc_reg_partial");
  return PKC_OK;
}

extern "C" int pkc_reg_finalize(int kind, const int32_t* block_start, int nblocks,
                                const float* partial, float lam, float* coef, float* loss_rows,
                                int nrows, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG((kind == PKC_REG_L1 || kind == PKC_REG_L2) && block_start && nblocks > 0 &&
                    partial && coef && (loss_rows || nrows == 0),
                "pkc_reg_finalize: bad arguments");
  hipLaunchKernelGGL(reg_finalize_kernel, dim3(1), dim3(RT), 0, S(stream), kind, block_start,
                     nblocks, partial, lam, coef, loss_rows, nrows);
  PKC_LAUNCH_CHECK("pkc_reg_finalize");
  return PKC_OK;
}

extern "C" int pkc_reg_grad(int kind, const pkc_reg_item* items, int nitems, const float* coef,
                            void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG((kind == PKC_REG_L1 || kind == PKC_REG_L2) && items && coef && nitems > 0,
                "pkc_reg_grad: bad arguments");
  hipLaunchKernelGGL(reg_grad_kernel, dim3(nitems), dim3(RT), 0, S(stream), kind, items, coef);
  PKC_LAUNCH_CHECK("pkc_reg_grad");
  return PKC_OK;
}
