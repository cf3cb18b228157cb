// pkc_prune.hip — magnitude pruning of the reference (quantized_modules.py:15-28):
//   thr = np.percentile(|W|, perc)   (numpy 'linear' method)
//   W  *= (|W| > thr)                (strict; applied every forward, neural_networks.py:276-278,
//                                     887-896, 997-1005, and at chunk end, core.py:291-296)
// The percentile is two exact order statistics of |W| found on the GPU by radix select on the
// IEEE bits of |W| (monotone for non-negative floats): four 8-bit histogram passes for the lower
// rank, then one pass for the next larger key; the interpolation follows numpy's _lerp (float32
// difference, float64 weight, float32 result).  No host round trip: the whole op is graph-safe.
#include "pkc_common.h"

namespace pkc {

struct PruneState {
  uint32_t prefix, k, count_le, min_gt;
  uint32_t hist[256];
};

__global__ void prune_init_kernel(PruneState* st, uint32_t k) {
  const int t = threadIdx.x;
  st->hist[t] = 0;
  if (t == 0) {
    st->prefix = 0;
    st->k = k;
    st->count_le = 0;
    st->min_gt = 0xffffffffu;
  }
}

__device__ __forceinline__ uint32_t akey(const float* w, int64_t i) {
  return __float_as_uint(fabsf(w[i]));
}

__global__ __launch_bounds__(256) void prune_hist_kernel(const float* w, int64_t n, PruneState* st,
                                                         int pass) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int shift = 24 - 8 * pass;
  const uint32_t prefix = st->prefix;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t key = akey(w, i);
    if (pass == 0 || (key >> (shift + 8)) == prefix) atomicAdd(&h[(key >> shift) & 255u], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&st->hist[threadIdx.x], h[threadIdx.x]);
}

__global__ void prune_scan_kernel(PruneState* st) {
  if (threadIdx.x == 0) {
    uint32_t cum = 0, digit = 255;
    for (uint32_t d = 0; d < 256; ++d) {
      const uint32_t c = st->hist[d];
      if (cum + c > st->k) {
        digit = d;
        break;
      }
      cum += c;
    }
    st->k -= cum;
    st->prefix = (st->prefix << 8) | digit;
  }
  __syncthreads();
  st->hist[threadIdx.x] = 0;
}

__global__ __launch_bounds__(256) void prune_next_kernel(const float* w, int64_t n, PruneState* st) {
  __shared__ uint32_t cnt, mn;
  if (threadIdx.x == 0) {
    cnt = 0;
    mn = 0xffffffffu;
  }
  __syncthreads();
  const uint32_t lo = st->prefix;
  uint32_t c = 0, m = 0xffffffffu;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t key = akey(w, i);
    if (key <= lo) ++c;
    else m = min(m, key);
  }
  atomicAdd(&cnt, c);
  atomicMin(&mn, m);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&st->count_le, cnt);
    atomicMin(&st->min_gt, mn);
  }
}

// numpy _lerp: a + (b-a)*t for t < 0.5, b - (b-a)*(1-t) otherwise; b-a in float32
__device__ __forceinline__ float np_lerp(float a, float b, double t) {
  const float d = b - a;
  const double r = t < 0.5 ? (double)a + (double)d * t : (double)b - (double)d * (1.0 - t);
  return (float)r;
}

__global__ __launch_bounds__(256) void prune_apply_kernel(float* w, int64_t n, const PruneState* st,
                                                          uint32_t hi_rank, double frac,
                                                          float* mask) {
  const uint32_t lo = st->prefix;
  const uint32_t hi = (st->count_le > hi_rank) ? lo : st->min_gt;
  const float thr = np_lerp(__uint_as_float(lo), __uint_as_float(hi), frac);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = w[i];
    const bool keep = fabsf(v) > thr;
    if (mask) mask[i] = keep ? 1.f : 0.f;
    w[i] = keep ? v : 0.f;
  }
}

}  // namespace pkc

extern "C" int64_t pkc_prune_work_size(void) { return (int64_t)sizeof(pkc::PruneState); }

extern "C" int pkc_prune(float* w, int64_t n, double perc, float* mask, void* work, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(w && work && n > 0 && n < 0xffffffffLL && perc >= 0.0 && perc <= 100.0,
                "pkc_prune: bad arguments");
  PruneState* st = reinterpret_cast<PruneState*>(work);
  // numpy 'linear' (_compute_virtual_index with alpha = beta = 1, same float64 operation order):
  // index = n*q + (1 + q*(1 - 1 - 1)) - 1, lo = floor(index), gamma = index - lo
  const double q = perc / 100.0;
  const double idx = (double)n * q + (1.0 + q * (1.0 - 1.0 - 1.0)) - 1.0;
  double lo_d = floor(idx);
  if (lo_d > (double)(n - 1)) lo_d = (double)(n - 1);
  const uint32_t lo = (uint32_t)lo_d;
  const uint32_t hi = lo + 1 < (uint64_t)n ? lo + 1 : lo;
  const double frac = idx - lo_d;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipStream_t s = S(stream);
  hipLaunchKernelGGL(prune_init_kernel, dim3(1), dim3(256), 0, s, st, lo);
  for (int pass = 0; pass < 4; ++pass) {
    hipLaunchKernelGGL(prune_hist_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, n, st, pass);
    hipLaunchKernelGGL(prune_scan_kernel, dim3(1), dim3(256), 0, s, st);
  }
  hipLaunchKernelGGL(prune_next_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, n, st);
  hipLaunchKernelGGL(prune_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w, n, st, hi, frac,
                     mask);
  PKC_LAUNCH_CHECK("pkc_prune");
  return PKC_OK;
}
