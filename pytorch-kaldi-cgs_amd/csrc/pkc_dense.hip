// pkc_dense.hip — the elementwise/normalisation work of one dense layer, fused around the matmul.
//
// Forward  (neural_networks.py:306-317):   out = drop(act(BN(sum_s zslab[s] + bias)))
// Backward (autograd of the same ops):     dz, dgamma, dbeta, dbias from dL/d out
//
// Element-parallel, two launches per direction (BatchNorm1d needs per-column statistics over all M
// rows, i.e. a grid-wide reduction, cut at the launch boundary instead of a grid barrier):
//   stats : grid (ceil(N/64), ceil(M/16)), 64 columns x 4 row-threads x 4 rows per workgroup;
//           sums the split-K slabs (independent loads, fixed order), writes z, and per 16-row block
//           the column mean / M2 (forward, merged with Chan's formula) or sum(dy) / sum(dy*xhat).
//   apply : same grid; merges the partials of its columns, normalises / applies the BN backward.
#include "pkc_common.h"

namespace pkc {

constexpr int EC = 64, ER = 4, ERB = 16, ET = EC * ER;   // cols, row-threads, rows/block, threads
constexpr int RPT = ERB / ER;                            // rows per thread

__device__ __forceinline__ float slab_sum(const float* __restrict__ p, int64_t stride, int nslab) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 4 <= nslab; s += 4) {
    a0 += p[(int64_t)s * stride];
    a1 += p[(int64_t)(s + 1) * stride];
    a2 += p[(int64_t)(s + 2) * stride];
    a3 += p[(int64_t)(s + 3) * stride];
  }
  for (; s < nslab; ++s) a0 += p[(int64_t)s * stride];
  return (a0 + a1) + (a2 + a3);
}

// column reduction over the ER row-threads of a block; result valid in every thread
__device__ __forceinline__ float colsum4(float v, float* red) {
  const int c = threadIdx.x % EC, t = threadIdx.x / EC;
  __syncthreads();
  red[t * EC + c] = v;
  __syncthreads();
  return (red[c] + red[EC + c]) + (red[2 * EC + c] + red[3 * EC + c]);
}

// ---------------------------------------------------------------------------------- forward
__global__ __launch_bounds__(ET) void dense_stats_kernel(pkc_dense_fwd_args a, float* part) {
  __shared__ float red[ET];
  const int c = blockIdx.x * EC + threadIdx.x % EC;
  const int t = threadIdx.x / EC;
  const int r0 = blockIdx.y * ERB;
  const bool cok = c < a.N;
  const int64_t N = a.N;
  const float b = (cok && a.bias) ? a.bias[c] : 0.f;
  float z[RPT];
  float s = 0.f;
  int nb = 0;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = r0 + t + ER * i;
    z[i] = 0.f;
    if (cok && r < a.M) {
      z[i] = slab_sum(a.zslab + r * N + c, a.slab_stride, a.nslab) + b;
      a.xhat[r * N + c] = z[i];
      s += z[i];
      ++nb;
    }
  }
  const int nrows = min(ERB, a.M - r0);
  const float mean_b = colsum4(s, red) / (float)nrows;
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < RPT; ++i)
    if (i < nb) {  // rows are filled in order, so the first nb entries are valid
      const float d = z[i] - mean_b;
      m2 += d * d;
    }
  m2 = colsum4(m2, red);
  if (cok && t == 0) {
    part[(int64_t)blockIdx.y * 2 * N + c] = mean_b;
    part[(int64_t)blockIdx.y * 2 * N + N + c] = m2;
  }
}

__global__ __launch_bounds__(ET) void dense_apply_kernel(pkc_dense_fwd_args a, const float* part) {
  __shared__ float stat[2 * EC];
  const int c = blockIdx.x * EC + threadIdx.x % EC;
  const int t = threadIdx.x / EC;
  const int r0 = blockIdx.y * ERB;
  const bool cok = c < a.N;
  const int64_t N = a.N;
  float mean = 0.f, invstd = 1.f, gam = 1.f, bet = 0.f;
  if (a.norm == PKC_NORM_BN_TRAIN) {
    if (t == 0 && cok) {   // Chan merge of the per-16-row partials of this column
      const int nrb = (a.M + ERB - 1) / ERB;
      float n = 0.f, mu = 0.f, M2 = 0.f;
      for (int k = 0; k < nrb; ++k) {
        const float nk = (float)min(ERB, a.M - k * ERB);
        const float mk = part[(int64_t)k * 2 * N + c];
        const float M2k = part[(int64_t)k * 2 * N + N + c];
        const float nn = n + nk;
        const float d = mk - mu;
        mu += d * nk / nn;
        M2 += M2k + d * d * n * nk / nn;
        n = nn;
      }
      const float var = M2 / (float)a.M;
      stat[threadIdx.x] = mu;
      stat[EC + threadIdx.x] = var;
      if (blockIdx.y == 0) {
        const float is = 1.f / sqrtf(var + a.eps);
        a.save_mean[c] = mu;
        a.save_invstd[c] = is;
        const float cn = (float)(a.count_n > 0 ? a.count_n : a.M);
        const float unb = cn > 1.f ? var * cn / (cn - 1.f) : var;
        a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * mu;
        a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unb;
      }
    }
    __syncthreads();
    if (cok) {
      const int cl = threadIdx.x % EC;
      mean = stat[cl];
      invstd = 1.f / sqrtf(stat[EC + cl] + a.eps);
      gam = a.gamma[c];
      bet = a.beta[c];
    }
  } else if (a.norm == PKC_NORM_BN_EVAL && cok) {
    mean = a.running_mean[c];
    invstd = 1.f / sqrtf(a.running_var[c] + a.eps);
    gam = a.gamma[c];
    bet = a.beta[c];
  }
  if (!cok) return;
  const bool drop = a.drop_p > 0.f;
  const float scale = drop ? 1.f / (1.f - a.drop_p) : 1.f;
  const uint32_t thr = drop ? (uint32_t)((double)(1.f - a.drop_p) * 4294967296.0) : 0u;
  const int64_t step = a.step_ctr ? *a.step_ctr : 0;
  const float b = a.bias ? a.bias[c] : 0.f;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = r0 + t + ER * i;
    if (r >= a.M) break;
    const int64_t idx = r * N + c;
    // BN training: z was staged in xhat by the stats pass; otherwise sum the slabs here
    const float z = (a.norm == PKC_NORM_BN_TRAIN) ? a.xhat[idx]
                                                 : slab_sum(a.zslab + idx, a.slab_stride, a.nslab) + b;
    const float xh = (a.norm == PKC_NORM_NONE) ? z : (z - mean) * invstd;
    const float y = (a.norm == PKC_NORM_NONE) ? z : xh * gam + bet;
    float o = act_fwd(a.act, y);
    if (drop) {
      uint8_t k;
      if (a.keep_in) k = a.keep_in[idx];
      else k = hash3(a.seed, (uint64_t)a.stream_id, (uint64_t)step * (uint64_t)(a.M * N) + idx) < thr;
      if (a.keep_out) a.keep_out[idx] = k;
      o = k ? o * scale : 0.f;
    }
    if (a.xhat) a.xhat[idx] = xh;
    a.out[idx] = o;
  }
}

// ---------------------------------------------------------------------------------- backward
__global__ __launch_bounds__(ET) void dense_bwd_stats_kernel(pkc_dense_bwd_args a, float* part) {
  __shared__ float red[ET];
  const int c = blockIdx.x * EC + threadIdx.x % EC;
  const int t = threadIdx.x / EC;
  const int r0 = blockIdx.y * ERB;
  const bool cok = c < a.N;
  const int64_t N = a.N;
  const bool bn = a.norm == PKC_NORM_BN_TRAIN;
  const float gam = (cok && bn) ? a.gamma[c] : 1.f;
  const float bet = (cok && bn) ? a.beta[c] : 0.f;
  const bool drop = a.drop_p > 0.f;
  const float scale = drop ? 1.f / (1.f - a.drop_p) : 1.f;
  float sdy = 0.f, sdyx = 0.f;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = r0 + t + ER * i;
    if (cok && r < a.M) {
      const int64_t idx = r * N + c;
      float g = slab_sum(a.gslab + idx, a.slab_stride, a.nslab);
      if (drop) g = a.keep[idx] ? g * scale : 0.f;
      const float xh = a.xhat[idx];
      const float y = bn ? xh * gam + bet : xh;
      const float dy = g * act_bwd(a.act, y, act_fwd(a.act, y));
      a.dz[idx] = dy;
      sdy += dy;
      sdyx += dy * xh;
    }
  }
  sdy = colsum4(sdy, red);
  sdyx = colsum4(sdyx, red);
  if (cok && t == 0) {
    part[(int64_t)blockIdx.y * 2 * N + c] = sdy;
    part[(int64_t)blockIdx.y * 2 * N + N + c] = sdyx;
  }
}

__global__ __launch_bounds__(ET) void dense_bwd_apply_kernel(pkc_dense_bwd_args a, const float* part) {
  const int c = blockIdx.x * EC + threadIdx.x % EC;
  const int t = threadIdx.x / EC;
  const int r0 = blockIdx.y * ERB;
  if (c >= a.N) return;
  const int64_t N = a.N;
  const int nrb = (a.M + ERB - 1) / ERB;
  float tdy = 0.f, tdyx = 0.f;
  for (int k = 0; k < nrb; ++k) {      // fixed order -> deterministic
    tdy += part[(int64_t)k * 2 * N + c];
    tdyx += part[(int64_t)k * 2 * N + N + c];
  }
  const bool bn = a.norm == PKC_NORM_BN_TRAIN;
  if (blockIdx.y == 0 && t == 0) {
    if (bn) {
      if (a.dgamma) a.dgamma[c] = tdyx;
      if (a.dbeta) a.dbeta[c] = tdy;
      // a bias in front of BatchNorm cancels in (z - mean): its gradient is exactly zero
      if (a.dbias) a.dbias[c] = 0.f;
    } else if (a.dbias) {
      a.dbias[c] = tdy;
    }
  }
  if (!bn) return;
  const float invM = 1.f / (float)a.M;
  const float k = a.gamma[c] * a.save_invstd[c];
  const float mdy = tdy * invM, mdyx = tdyx * invM;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = r0 + t + ER * i;
    if (r >= a.M) break;
    const int64_t idx = r * N + c;
    a.dz[idx] = k * (a.dz[idx] - mdy - a.xhat[idx] * mdyx);
  }
}

__global__ __launch_bounds__(ET) void colsum_kernel(int M, int N, int nslab, const float* x,
                                                    int64_t slab, float* out, int accumulate) {
  // one workgroup per 64 columns, 4 row-threads striding over all rows (bias grad of a head)
  __shared__ float red[ET];
  const int c = blockIdx.x * EC + threadIdx.x % EC;
  const int t = threadIdx.x / EC;
  float s0 = 0.f, s1 = 0.f;
  if (c < N) {
    int r = t;
    for (; r + ER < M; r += 2 * ER) {
      s0 += slab_sum(x + (int64_t)r * N + c, slab, nslab);
      s1 += slab_sum(x + (int64_t)(r + ER) * N + c, slab, nslab);
    }
    if (r < M) s0 += slab_sum(x + (int64_t)r * N + c, slab, nslab);
  }
  const float s = colsum4(s0 + s1, red);
  if (c < N && t == 0) out[c] = accumulate ? out[c] + s : s;
}

}  // namespace pkc

extern "C" int64_t pkc_dense_work_size(int M, int N) {
  return 2 * (int64_t)((M + pkc::ERB - 1) / pkc::ERB) * N;
}

extern "C" int pkc_dense_fwd(const pkc_dense_fwd_args* a, float* work, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(a && a->M > 0 && a->N > 0 && a->nslab >= 1 && a->zslab && a->out,
                "pkc_dense_fwd: bad arguments");
  PKC_CHECK_ARG(a->norm != PKC_NORM_BN_TRAIN ||
                    (a->gamma && a->beta && a->running_mean && a->running_var && a->save_mean &&
                     a->save_invstd && a->xhat && work),
                "pkc_dense_fwd: BN training needs gamma/beta/running stats/save buffers/xhat/work");
  PKC_CHECK_ARG(a->norm != PKC_NORM_BN_EVAL || (a->gamma && a->beta && a->running_mean &&
                                                a->running_var),
                "pkc_dense_fwd: BN eval needs gamma/beta/running stats");
  PKC_CHECK_ARG(a->drop_p >= 0.f && a->drop_p < 1.f, "pkc_dense_fwd: drop_p out of range");
  PKC_CHECK_ARG(a->nslab == 1 || a->slab_stride >= (int64_t)a->M * a->N,
                "pkc_dense_fwd: slab_stride too small");
  dim3 grid((a->N + EC - 1) / EC, (a->M + ERB - 1) / ERB);
  if (a->norm == PKC_NORM_BN_TRAIN) {
    hipLaunchKernelGGL(dense_stats_kernel, grid, dim3(ET), 0, S(stream), *a, work);
    PKC_LAUNCH_CHECK("pkc_dense_fwd stats");
  }
  hipLaunchKernelGGL(dense_apply_kernel, grid, dim3(ET), 0, S(stream), *a, work);
  PKC_LAUNCH_CHECK("pkc_dense_fwd apply");
  return PKC_OK;
}

extern "C" int pkc_dense_bwd(const pkc_dense_bwd_args* a, float* work, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(a && a->M > 0 && a->N > 0 && a->nslab >= 1 && a->gslab && a->xhat && a->dz && work,
                "pkc_dense_bwd: bad arguments");
  PKC_CHECK_ARG(a->norm != PKC_NORM_BN_TRAIN || (a->gamma && a->beta && a->save_invstd),
                "pkc_dense_bwd: BN needs gamma/beta/save_invstd");
  PKC_CHECK_ARG(a->norm != PKC_NORM_BN_EVAL, "pkc_dense_bwd: backward through eval BN unsupported");
  PKC_CHECK_ARG(a->drop_p == 0.f || a->keep, "pkc_dense_bwd: dropout needs the keep mask");
  dim3 grid((a->N + EC - 1) / EC, (a->M + ERB - 1) / ERB);
  hipLaunchKernelGGL(dense_bwd_stats_kernel, grid, dim3(ET), 0, S(stream), *a, work);
  PKC_LAUNCH_CHECK("pkc_dense_bwd stats");
  hipLaunchKernelGGL(dense_bwd_apply_kernel, grid, dim3(ET), 0, S(stream), *a, work);
  PKC_LAUNCH_CHECK("pkc_dense_bwd apply");
  return PKC_OK;
}

extern "C" int pkc_colsum(int M, int N, int nslab, const float* x, int64_t slab_stride, float* out,
                          int accumulate, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(M > 0 && N > 0 && nslab >= 1 && x && out, "pkc_colsum: bad arguments");
  hipLaunchKernelGGL(colsum_kernel, dim3((N + EC - 1) / EC), dim3(ET), 0, S(stream), M, N, nslab, x,
                     slab_stride, out, accumulate);
  PKC_LAUNCH_CHECK("pkc_colsum");
  return PKC_OK;
}
