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

// Elements per thread of one optimizer work item (256 threads).  The update also runs inside the
// grouped backward launches (PKC_OP_OPTIM), whose register allocation is the maximum over every
// operation they carry: at 16 elements per thread the update set it (193 VGPRs + 16 AGPRs: two
// waves per SIMD for the whole launch), at 8 the matmul body does (145 + 16: three waves).  C2 step,
// same box, two rounds (profiles/r03_opt_per_ab.txt): 16 -> 801-803k, 8 -> 846-848k, 4 -> 814-822k
// frames/s; B = 4096 5.15-5.16M -> 5.20-5.21M.  (Round 1, one-kernel updates: 4 / 16 0.200 ms,
// 8 0.203, 32 0.259.)  2048-element items.
#ifndef PKC_OPT_PER
#define PKC_OPT_PER 8
#endif
constexpr int OPT_T = 256, OPT_PER = PKC_OPT_PER, OPT_CHUNK = OPT_T * OPT_PER;

// Every operand of a thread's OPT_PER elements is requested before any is used (independent
// loads in flight instead of one round trip per element); states the optimizer does not keep are
// never touched.  VEC: the tensor's pointers are 16-byte aligned and n % 4 == 0.
// DIRECT: the streams to touch follow from the pointers alone (pkc_opt_seg: s1 NULL when the update
// keeps no first state, qout NULL unless quantised), so no load waits on the descriptor's fields.
template <bool VEC, bool DIRECT = false>
__device__ __forceinline__ void optim_chunk(const pkc_opt_tensor& t, int64_t start) {
  constexpr int V = 4, NV = OPT_PER / V;
  const bool st1 = DIRECT ? t.s1 != nullptr : (t.kind != PKC_OPT_SGD || t.momentum != 0.f);
  const bool st2 = t.s2 != nullptr, st3 = t.s3 != nullptr, msk = t.mask != nullptr;
  const bool qw = DIRECT ? t.qout != nullptr : t.qbits > 0;
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
        if (qw) qq[l] = quant_w(e.p, t.qbits);
      }
      const int64_t i = idx[j];
      *reinterpret_cast<float4*>(t.p + i) = P[j];
      if (st1) *reinterpret_cast<float4*>(t.s1 + i) = S1[j];
      if (st2) *reinterpret_cast<float4*>(t.s2 + i) = S2[j];
      if (st3) *reinterpret_cast<float4*>(t.s3 + i) = S3[j];
      if (qw) *reinterpret_cast<float4*>(t.qout + i) = Q;
      if (t.bout) {   // one 8-byte store (bout % 8 == 0 on this path)
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 h;
        h[0] = (__bf16)P[j].x; h[1] = (__bf16)P[j].y; h[2] = (__bf16)P[j].z; h[3] = (__bf16)P[j].w;
        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(t.bout) + i) = h;
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
      if (qw) t.qout[i] = quant_w(e[j].p, t.qbits);
      if (t.bout) reinterpret_cast<__bf16*>(t.bout)[i] = (__bf16)e[j].p;
    }
  }
}

// A direct work-item run (pkc_opt_seg) as the grouped launch's kernel arguments carry it: op-local
// work items [begin, end) are chunks chunk0 .. of tensor `tensor`.
struct OptSegK {
  float* p; const float* g; float* s1; float* s2; float* s3; const float* mask; float* qout; void* bout;
  int64_t n;
  int tensor, chunk0, begin, end;
};

__device__ __forceinline__ bool optim_vec(const pkc_opt_tensor& t) {
  return (t.n % 4 == 0) && ((uintptr_t)t.p % 16 == 0) && ((uintptr_t)t.g % 16 == 0) &&
         ((uintptr_t)t.s1 % 16 == 0) && ((uintptr_t)t.s2 % 16 == 0) &&
         ((uintptr_t)t.s3 % 16 == 0) && ((uintptr_t)t.mask % 16 == 0) &&
         ((uintptr_t)t.qout % 16 == 0) && ((uintptr_t)t.bout % 8 == 0);
}

// work item `chunk` of a direct run: pointers from the kernel arguments, hyper-parameters from the
// descriptor (its scalar loads are in flight with the first data loads)
__device__ __forceinline__ void optim_seg_wg(const pkc_opt_tensor* ts, const OptSegK& sg, int chunk) {
  pkc_opt_tensor t = ts[sg.tensor];
  t.p = sg.p; t.g = sg.g; t.s1 = sg.s1; t.s2 = sg.s2; t.s3 = sg.s3; t.mask = sg.mask;
  t.qout = sg.qout; t.bout = sg.bout; t.n = sg.n;
  const int64_t start = (int64_t)(sg.chunk0 + chunk) * OPT_CHUNK;
  if (optim_vec(t)) optim_chunk<true, true>(t, start);
  else optim_chunk<false, true>(t, start);
}

// work item `wg` of a chunk map (pairs tensor, chunk) over the descriptor array ts
__device__ __forceinline__ void optim_wg(const pkc_opt_tensor* ts, const int32_t* map, int wg) {
  const int ti = map[2 * wg];
  const int64_t start = (int64_t)map[2 * wg + 1] * OPT_CHUNK;
  const pkc_opt_tensor t = ts[ti];
  if (optim_vec(t)) optim_chunk<true>(t, start);
  else optim_chunk<false>(t, start);
}

}  // namespace pkc
