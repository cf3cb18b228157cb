// pkc_norm.hip — the reference's LayerNorm (neural_networks.py:40-51) forward and backward.
//
//   y = gamma * (x - mean) / (std + eps) + beta,  per row over the N features, std UNBIASED
//   (torch.Tensor.std default), eps = 1e-6 added to std (not to the variance).
// Backward with xh = (x - mean) / d, d = std + eps, gh = dy * gamma:
//   dx_i = (gh_i - mean(gh)) / d - xh_i * sum_j(gh_j xh_j) / ((N - 1) std)
//   dgamma = sum_rows dy * xh,  dbeta = sum_rows dy,  (dbias of the Linear in front = sum_rows dx)
// Row kernels: one wave per row (4 rows per workgroup); column sums: 64 columns x 4 row-threads.
#include "pkc_common.h"

namespace pkc {

constexpr int NW = 4;   // rows (waves) per workgroup

__global__ __launch_bounds__(64 * NW) void ln_fwd_kernel(int M, int N, int nslab, const float* x,
                                                         int64_t ss, const float* bias,
                                                         const float* gamma, const float* beta,
                                                         float eps, float* y, float* xhat,
                                                         float* rowstat) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * NW + (threadIdx.x >> 6);
  if (r >= M) return;
  const float* xr = x + (int64_t)r * N;
  auto val = [&](int j) {
    float v = 0.f;
    for (int s = 0; s < nslab; ++s) v += xr[(int64_t)s * ss + j];
    return v + (bias ? bias[j] : 0.f);
  };
  float sum = 0.f;
  for (int j = lane; j < N; j += 64) sum += val(j);
  const float mean = warp_sum(sum) / (float)N;
  float sq = 0.f;
  for (int j = lane; j < N; j += 64) {
    const float d = val(j) - mean;
    sq += d * d;
  }
  const float sd = sqrtf(warp_sum(sq) / (float)(N - 1));
  const float den = sd + eps;
  for (int j = lane; j < N; j += 64) {
    const float xh = (val(j) - mean) / den;
    xhat[(int64_t)r * N + j] = xh;
    y[(int64_t)r * N + j] = gamma[j] * xh + beta[j];
  }
  if (lane == 0) {
    rowstat[2 * r] = den;
    rowstat[2 * r + 1] = sd;
  }
}

__device__ __forceinline__ float slabs(const float* p, int ns, int64_t ss) {
  float v = 0.f;
  for (int s = 0; s < ns; ++s) v += p[(int64_t)s * ss];
  return v;
}

__global__ __launch_bounds__(64 * NW) void ln_bwd_rows_kernel(int M, int N, int ns, const float* dy,
                                                              int64_t ss, const float* xhat,
                                                              const float* gamma,
                                                              const float* rowstat, float* dx) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * NW + (threadIdx.x >> 6);
  if (r >= M) return;
  const float* g = dy + (int64_t)r * N;
  const float* xh = xhat + (int64_t)r * N;
  float sg = 0.f, sgx = 0.f;
  for (int j = lane; j < N; j += 64) {
    const float gh = slabs(g + j, ns, ss) * gamma[j];
    sg += gh;
    sgx += gh * xh[j];
  }
  sg = warp_sum(sg);
  sgx = warp_sum(sgx);
  const float den = rowstat[2 * r], sd = rowstat[2 * r + 1];
  const float mg = sg / (float)N;
  const float k = sd > 0.f ? sgx / ((float)(N - 1) * sd) : 0.f;   // torch masks std == 0 to 0
  for (int j = lane; j < N; j += 64) {
    const float gh = slabs(g + j, ns, ss) * gamma[j];
    dx[(int64_t)r * N + j] = (gh - mg) / den - xh[j] * k;
  }
}

// column sums over rows: dgamma = sum dy*xh, dbeta = sum dy, dbias = sum dx
__global__ __launch_bounds__(256) void ln_bwd_cols_kernel(int M, int N, int ns, const float* dy,
                                                          int64_t ss, const float* xhat,
                                                          const float* dx,
                                                          float* dgamma, float* dbeta,
                                                          float* dbias) {
  __shared__ float red[3][256];
  const int c = blockIdx.x * 64 + threadIdx.x % 64;
  const int t = threadIdx.x / 64;
  float a = 0.f, b = 0.f, d = 0.f;
  if (c < N)
    for (int r = t; r < M; r += 4) {
      const int64_t i = (int64_t)r * N + c;
      const float g = slabs(dy + i, ns, ss);
      a += g * xhat[i];
      b += g;
      d += dx[i];
    }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  red[2][threadIdx.x] = d;
  __syncthreads();
  if (t == 0 && c < N) {
    const int cl = threadIdx.x;
    auto tot = [&](int k) { return (red[k][cl] + red[k][64 + cl]) + (red[k][128 + cl] + red[k][192 + cl]); };
    if (dgamma) dgamma[c] = tot(0);
    if (dbeta) dbeta[c] = tot(1);
    if (dbias) dbias[c] = tot(2);
  }
}

}  // namespace pkc

extern "C" int pkc_layernorm_fwd(int M, int N, int nslab, const float* xslab, int64_t slab_stride,
                                 const float* bias, const float* gamma, const float* beta, float eps,
                                 float* y, float* xhat, float* rowstat, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(M > 0 && N > 1 && nslab >= 1 && xslab && gamma && beta && y && xhat && rowstat,
                "pkc_layernorm_fwd: bad arguments");
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((M + NW - 1) / NW), dim3(64 * NW), 0, S(stream), M, N, nslab,
                     xslab, slab_stride, bias, gamma, beta, eps, y, xhat, rowstat);
  PKC_LAUNCH_CHECK("pkc_layernorm_fwd");
  return PKC_OK;
}

extern "C" int pkc_layernorm_bwd(int M, int N, int nslab, const float* dy, int64_t slab_stride,
                                 const float* xhat,
                                 const float* gamma, const float* rowstat, float* dx, float* dgamma,
                                 float* dbeta, float* dbias, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(M > 0 && N > 1 && nslab >= 1 && dy && xhat && gamma && rowstat && dx,
                "pkc_layernorm_bwd: bad arguments");
  hipLaunchKernelGGL(ln_bwd_rows_kernel, dim3((M + NW - 1) / NW), dim3(64 * NW), 0, S(stream), M, N,
                     nslab, dy, slab_stride, xhat, gamma, rowstat, dx);
  PKC_LAUNCH_CHECK("pkc_layernorm_bwd rows");
  if (dgamma || dbeta || dbias) {
    hipLaunchKernelGGL(ln_bwd_cols_kernel, dim3((N + 63) / 64), dim3(256), 0, S(stream), M, N, nslab,
                       dy, slab_stride, xhat, dx, dgamma, dbeta, dbias);
    PKC_LAUNCH_CHECK("pkc_layernorm_bwd cols");
  }
  return PKC_OK;
}
