// pkc_quant.hip — fake quantisation and pattern masks of the CGS variants.
//
//   weight fake-quant  quantized_modules.py:77-97 (balanced=False): q = sign(w)*ceil(|w|*2^(b-1))/2^(b-1)
//                      on the clamped weight (the clamp itself is fused into pkc_optim_step)
//   input fake-quant   quantized_modules.py:99-119: var = max(|max x|, |min x|) over the whole
//                      tensor, q = sign(x)*ceil(|x/var|*2^(b-1))/2^(b-1)*var (skipped when var == 0),
//                      applied in place by every QuantizeLinear that reads the tensor, so an LSTM
//                      layer input is re-quantised once per gate (q1..q4) — reproduced exactly
//   pattern mask       sparsity.py:1112-1146: per 8x8 tile, score_p = sum |W| * pattern_p, every
//                      pattern whose score equals the maximum is selected (ties -> mask > 1)
#include "pkc_common.h"

namespace pkc {

__device__ __forceinline__ float qweight(float w, float scale) {
  // op order of Quantize: abs, *2^(b-1), ceil, /2^(b-1), *sign
  const float s = w > 0.f ? 1.f : (w < 0.f ? -1.f : 0.f);
  return ceilf(fabsf(w) * scale) / scale * s;
}

__device__ __forceinline__ float qinput(float x, float var, float scale) {
  // op order of Quantize_inp (if_forward=False): x/var, abs, *2^(B-1), ceil, /2^(B-1), *var, *sign
  const float s = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
  return ceilf(fabsf(x / var) * scale) / scale * var * s;
}

__global__ void fq_weight_kernel(const float* w, float* q, int64_t n, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    q[i] = qweight(w[i], scale);
}

// max(|max x|, |min x|) partials -> work[blockIdx] (then a 1-block finish)
__global__ __launch_bounds__(256) void absmax_partial_kernel(const float* x, int64_t n, float* part) {
  __shared__ float smx[256], smn[256];
  float mx = -INFINITY, mn = INFINITY;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
  }
  smx[threadIdx.x] = mx;
  smn[threadIdx.x] = mn;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      smx[threadIdx.x] = fmaxf(smx[threadIdx.x], smx[threadIdx.x + o]);
      smn[threadIdx.x] = fminf(smn[threadIdx.x], smn[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = smx[0];
    part[2 * blockIdx.x + 1] = smn[0];
  }
}

__global__ void absmax_finish_kernel(float* part, int nparts, float* var_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float mx = -INFINITY, mn = INFINITY;
  for (int i = 0; i < nparts; ++i) {
    mx = fmaxf(mx, part[2 * i]);
    mn = fminf(mn, part[2 * i + 1]);
  }
  const float a = fabsf(mx), b = fabsf(mn);
  *var_out = a > b ? a : b;
}

__global__ void fq_input_kernel(const float* x, float* q, int64_t n, const float* var, float scale) {
  const float v = *var;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    q[i] = v == 0.f ? x[i] : qinput(x[i], v, scale);
}

__global__ void pattern_mask_kernel(const float* W, int R, int Cc, const float* pat, int P, int ph,
                                    int pw, float* mask) {
  const int tiles_c = Cc / pw;
  const int ntiles = (R / ph) * tiles_c;
  for (int tix = blockIdx.x * blockDim.x + threadIdx.x; tix < ntiles; tix += gridDim.x * blockDim.x) {
    const int ti = tix / tiles_c, tj = tix % tiles_c;
    float best = -INFINITY;
    float score[32];
    for (int p = 0; p < P; ++p) {
      float s = 0.f;
      for (int a = 0; a < ph; ++a)
        for (int b = 0; b < pw; ++b)
          s += fabsf(W[(int64_t)(ti * ph + a) * Cc + tj * pw + b]) * pat[(p * ph + a) * pw + b];
      score[p] = s;
      best = fmaxf(best, s);
    }
    for (int a = 0; a < ph; ++a)
      for (int b = 0; b < pw; ++b) {
        float m = 0.f;
        for (int p = 0; p < P; ++p)
          if (score[p] >= best) m += pat[(p * ph + a) * pw + b];
        mask[(int64_t)(ti * ph + a) * Cc + tj * pw + b] = m;
      }
  }
}

// The 8 x 8 form (every pattern_shape the reference cfgs use): one thread per tile, its 64 |W| in
// registers (lane l reads tile tj0 + l: a row's 64 lanes read 2 KB contiguous), the P <= 32 scores
// in registers (the generic kernel's indexed score[] array lives in scratch), patterns read
// uniformly (scalar loads).  The scores sum in the generic kernel's order (a, then b) and the
// ties select the same patterns: bit-identical masks.
template <int PMAX>
__global__ __launch_bounds__(256) void pattern_mask8_kernel(const float* __restrict__ W, int R,
                                                            int Cc, const float* __restrict__ pat,
                                                            int P, float* __restrict__ mask) {
  const int tiles_c = Cc / 8;
  const int ntiles = (R / 8) * tiles_c;
  const int tix = blockIdx.x * blockDim.x + threadIdx.x;
  if (tix >= ntiles) return;
  const int ti = tix / tiles_c, tj = tix % tiles_c;
  const float* w0 = W + (int64_t)ti * 8 * Cc + tj * 8;
  float x[64];
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const float4 u = *reinterpret_cast<const float4*>(w0 + (int64_t)a * Cc);
    const float4 v = *reinterpret_cast<const float4*>(w0 + (int64_t)a * Cc + 4);
    x[8 * a + 0] = fabsf(u.x); x[8 * a + 1] = fabsf(u.y); x[8 * a + 2] = fabsf(u.z);
    x[8 * a + 3] = fabsf(u.w); x[8 * a + 4] = fabsf(v.x); x[8 * a + 5] = fabsf(v.y);
    x[8 * a + 6] = fabsf(v.z); x[8 * a + 7] = fabsf(v.w);
  }
  float score[PMAX];
  float best = -INFINITY;
#pragma unroll
  for (int p = 0; p < PMAX; ++p) {
    float s = 0.f;
    if (p < P) {
#pragma unroll
      for (int e = 0; e < 64; ++e) s += x[e] * pat[p * 64 + e];
      best = fmaxf(best, s);
    }
    score[p] = s;
  }
  float* m0 = mask + (int64_t)ti * 8 * Cc + tj * 8;
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < PMAX; ++p) {
      if (p < P && score[p] >= best) {
#pragma unroll
        for (int b = 0; b < 8; ++b) m[b] += pat[p * 64 + 8 * a + b];
      }
    }
    *reinterpret_cast<float4*>(m0 + (int64_t)a * Cc) = make_float4(m[0], m[1], m[2], m[3]);
    *reinterpret_cast<float4*>(m0 + (int64_t)a * Cc + 4) = make_float4(m[4], m[5], m[6], m[7]);
  }
}

}  // namespace pkc

extern "C" int pkc_fakequant_weight(const float* w, float* q, int64_t n, int bits, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(w && q && n >= 0 && bits > 0 && bits < 31, "pkc_fakequant_weight: bad arguments");
  if (n == 0) return PKC_OK;
  const float scale = ldexpf(1.f, bits - 1);
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(fq_weight_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), w, q, n, scale);
  PKC_LAUNCH_CHECK("pkc_fakequant_weight");
  return PKC_OK;
}

extern "C" int pkc_fakequant_input(const float* x, float* out, int64_t n, int bits, int reps,
                                   float* work, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(x && out && work && n > 0 && bits > 0 && bits < 31 && reps >= 1 && reps <= 8,
                "pkc_fakequant_input: bad arguments");
  // out holds reps consecutive tensors q1..q_reps; work >= 2*64 + 8 floats.  Only q1 needs the
  // max-abs reduction: Q maps the max-abs element x* to exactly +-var (x*/var = +-1) and every
  // other element to a magnitude <= var, so every later call's per-tensor var is the same.
  const float scale = ldexpf(1.f, bits - 1);
  const int nparts = 64;
  hipLaunchKernelGGL(absmax_partial_kernel, dim3(nparts), dim3(256), 0, S(stream), x, n, work);
  hipLaunchKernelGGL(absmax_finish_kernel, dim3(1), dim3(64), 0, S(stream), work, nparts,
                     work + 2 * nparts);
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  const float* src = x;
  for (int r = 0; r < reps; ++r) {
    float* dst = out + (int64_t)r * n;
    hipLaunchKernelGGL(fq_input_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), src, dst, n,
                       work + 2 * nparts, scale);
    src = dst;
  }
  PKC_LAUNCH_CHECK("pkc_fakequant_input");
  return PKC_OK;
}

extern "C" int pkc_pattern_mask(const float* W, int rows, int cols, const float* patterns, int P,
                                int ph, int pw, float* mask, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(W && patterns && mask && P > 0 && P <= 32 && ph > 0 && pw > 0 && rows % ph == 0 &&
                    cols % pw == 0,
                "pkc_pattern_mask: bad arguments (rows/cols must be multiples of the pattern)");
  const int ntiles = (rows / ph) * (cols / pw);
  if (ph == 8 && pw == 8 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)mask & 15) == 0) {
    const dim3 g((ntiles + 255) / 256);
    if (P <= 16)
      hipLaunchKernelGGL(pattern_mask8_kernel<16>, g, dim3(256), 0, S(stream), W, rows, cols, patterns,
                         P, mask);
    else
      hipLaunchKernelGGL(pattern_mask8_kernel<32>, g, dim3(256), 0, S(stream), W, rows, cols, patterns,
                         P, mask);
    PKC_LAUNCH_CHECK("pkc_pattern_mask");
    return PKC_OK;
  }
  hipLaunchKernelGGL(pattern_mask_kernel, dim3((ntiles + 127) / 128), dim3(128), 0, S(stream), W, rows,
                     cols, patterns, P, ph, pw, mask);
  PKC_LAUNCH_CHECK("pkc_pattern_mask");
  return PKC_OK;
}
