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

constexpr int OPT_T = 256, OPT_PER = 8, OPT_CHUNK = OPT_T * OPT_PER;

// Every operand of a thread's OPT_PER elements is requested before any is used (independent
// loads in flight instead of one round trip per element); states the optimizer does not keep are
// never touched.  VEC: the tensor's pointers are 16-byte aligned and n % 4 == 0.
template <bool VEC>
__device__ __forceinline__ void optim_chunk(const pkc_opt_tensor& t, int64_t start) {
  constexpr int V = 4, NV = OPT_PER / V;
  const bool st1 = t.kind != PKC_OPT_SGD || t.momentum != 0.f;
  const bool st2 = t.s2 != nullptr, st3 = t.s3 != nullptr, msk = t.mask != nullptr;
  if (VEC) {
    float4 P[NV], G[NV], S1[NV], S2[NV], S3[NV], MK[NV];
    int64_t idx[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      idx[j] = start + ((int64_t)threadIdx.x + (int64_t)j * OPT_T) * V;
      const int64_t i = idx[j] < t.n ? idx[j] : 0;
      P[j] = *reinterpret_cast<const float4*>(t.p + i);
      G[j] = *reinterpret_cast<const float4*>(t.g + i);
      if (st1) S1[j] = *reinterpret_cast<const float4*>(t.s1 + i);
      if (st2) S2[j] = *reinterpret_cast<const float4*>(t.s2 + i);
      if (st3) S3[j] = *reinterpret_cast<const float4*>(t.s3 + i);
      if (msk) MK[j] = *reinterpret_cast<const float4*>(t.mask + i);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      if (idx[j] >= t.n) break;
      float* pp = &P[j].x; float* gg = &G[j].x; float* a1 = &S1[j].x; float* a2 = &S2[j].x;
      float* a3 = &S3[j].x; float* mm = &MK[j].x;
      float4 Q;
      float* qq = &Q.x;
#pragma unroll
      for (int l = 0; l < V; ++l) {
        OptState e{pp[l], gg[l], st1 ? a1[l] : 0.f, st2 ? a2[l] : 0.f, st3 ? a3[l] : 0.f,
                   msk ? mm[l] : 1.f};
        opt_update(t, e);
        pp[l] = e.p; a1[l] = e.s1; a2[l] = e.s2; a3[l] = e.s3;
        if (t.qbits > 0) qq[l] = quant_w(e.p, t.qbits);
      }
      const int64_t i = idx[j];
      *reinterpret_cast<float4*>(t.p + i) = P[j];
      if (st1) *reinterpret_cast<float4*>(t.s1 + i) = S1[j];
      if (st2) *reinterpret_cast<float4*>(t.s2 + i) = S2[j];
      if (st3) *reinterpret_cast<float4*>(t.s3 + i) = S3[j];
      if (t.qbits > 0) *reinterpret_cast<float4*>(t.qout + i) = Q;
      if (t.bout) {
        __bf16* bo = reinterpret_cast<__bf16*>(t.bout) + i;
        bo[0] = (__bf16)P[j].x; bo[1] = (__bf16)P[j].y; bo[2] = (__bf16)P[j].z; bo[3] = (__bf16)P[j].w;
      }
    }
  } else {
    OptState e[OPT_PER];
#pragma unroll
    for (int j = 0; j < OPT_PER; ++j) {
      const int64_t i0 = start + threadIdx.x + (int64_t)j * OPT_T;
      const int64_t i = i0 < t.n ? i0 : 0;
      e[j].p = t.p[i];
      e[j].g = t.g[i];
      e[j].s1 = st1 ? t.s1[i] : 0.f;
      e[j].s2 = st2 ? t.s2[i] : 0.f;
      e[j].s3 = st3 ? t.s3[i] : 0.f;
      e[j].m = msk ? t.mask[i] : 1.f;
    }
#pragma unroll
    for (int j = 0; j < OPT_PER; ++j) {
      const int64_t i = start + threadIdx.x + (int64_t)j * OPT_T;
      if (i >= t.n) break;
      opt_update(t, e[j]);
      t.p[i] = e[j].p;
      if (st1) t.s1[i] = e[j].s1;
      if (st2) t.s2[i] = e[j].s2;
      if (st3) t.s3[i] = e[j].s3;
      if (t.qbits > 0) t.qout[i] = quant_w(e[j].p, t.qbits);
      if (t.bout) reinterpret_cast<__bf16*>(t.bout)[i] = (__bf16)e[j].p;
    }
  }
}

__global__ __launch_bounds__(OPT_T) void optim_kernel(const pkc_opt_tensor* ts, const int32_t* map) {
  const int ti = map[2 * blockIdx.x];
  const int64_t start = (int64_t)map[2 * blockIdx.x + 1] * OPT_CHUNK;
  const pkc_opt_tensor t = ts[ti];
  const bool vec = (t.n % 4 == 0) && ((uintptr_t)t.p % 16 == 0) && ((uintptr_t)t.g % 16 == 0) &&
                   ((uintptr_t)t.s1 % 16 == 0) && ((uintptr_t)t.s2 % 16 == 0) &&
                   ((uintptr_t)t.s3 % 16 == 0) && ((uintptr_t)t.mask % 16 == 0) &&
                   ((uintptr_t)t.qout % 16 == 0) && ((uintptr_t)t.bout % 8 == 0);
  if (vec) optim_chunk<true>(t, start);
  else optim_chunk<false>(t, start);
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
