// pkc_loss.hip — fused LogSoftmax + NLLLoss + error rate + backward for one output head.
//
// Replaces, per head, the reference's LogSoftmax (neural_networks.py:73-74), nn.NLLLoss mean
// (utils.py:1811-1812, 1935-1952), cost_err argmax (utils.py:1993-2011) and their autograd backward
// (d logits = w/M * (softmax - onehot)) with one row-parallel pass: one wave per frame row, the
// split-K slabs of the head matmul summed in fixed order.
#include "pkc_common.h"

namespace pkc {

constexpr int LW = 4;  // waves per workgroup

__device__ __forceinline__ float slab_sum4(const float* __restrict__ p, int64_t stride, int nslab) {
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

// WPR waves cooperate on one row (WPR = 4 for wide heads such as 1928 senones, 1 for narrow ones)
template <int WPR>
__global__ __launch_bounds__(64 * LW) void nll_kernel(pkc_nll_args a) {
  constexpr int RPB = LW / WPR;             // rows per workgroup
  constexpr int T = 64 * WPR;               // threads per row
  __shared__ float sh_m[LW], sh_s[LW];
  __shared__ int sh_a[LW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rl = wave / WPR;                // row within the workgroup
  const int tr = threadIdx.x - rl * T;      // thread index within the row
  const int r = blockIdx.x * RPB + rl;
  const bool rok = r < a.M;
  const int64_t N = a.N;
  float* zrow = a.logp + (int64_t)(rok ? r : 0) * N;   // z staged in the logp row
  float mx = -INFINITY;
  int arg = 0x7fffffff;
  if (rok)
    for (int j = tr; j < a.N; j += T) {
      float z = slab_sum4(a.zslab + r * N + j, a.slab_stride, a.nslab);
      if (a.bias) z += a.bias[j];
      zrow[j] = z;
      if (z > mx) { mx = z; arg = j; }   // first max per thread (ascending j)
    }
  // argmax: max value, smallest index among equals
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  if (WPR > 1) {
    if (lane == 0) { sh_m[wave] = mx; sh_a[wave] = arg; }
    __syncthreads();
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) {
      const float om = sh_m[w];
      const int oa = sh_a[w];
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
  }
  float se = 0.f;
  if (rok)
    for (int j = tr; j < a.N; j += T) se += expf(zrow[j] - mx);
  se = warp_sum(se);
  if (WPR > 1) {
    if (lane == 0) sh_s[wave] = se;
    __syncthreads();
    se = 0.f;
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) se += sh_s[w];
  }
  if (!rok) return;
  const float lse = mx + logf(se);
  const int y = a.labels ? a.labels[(int64_t)r * a.label_stride] : -1;
  const float gscale = a.weight / (float)a.M;
  float lp_y = 0.f;
  for (int j = tr; j < a.N; j += T) {
    const float lp = zrow[j] - lse;
    if (j == y) lp_y = lp;
    if (a.dlogits) {
      const float p = expf(lp);
      a.dlogits[(int64_t)r * N + j] = gscale * (j == y ? p - 1.f : p);
    }
    zrow[j] = a.log_prior ? lp - a.log_prior[j] : lp;
  }
  // exactly one thread of the row saw j == y: it writes the row's loss / error
  if (y >= 0 && y < a.N && (y % T) == tr) {
    if (a.row_loss) a.row_loss[r] = -lp_y;
    if (a.row_err) a.row_err[r] = (arg != y) ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(256) void loss_finalize_kernel(int nheads, const float* const* rl,
                                                            const float* w, int M,
                                                            const float* rerr, float* out,
                                                            float* acc) {
  __shared__ float red[256];
  float total = 0.f;
  for (int h = 0; h <= nheads; ++h) {
    const float* src = h < nheads ? rl[h] : rerr;
    float s = 0.f;
    for (int i = threadIdx.x; i < M; i += 256) s += src[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    const float mean = red[0] / (float)M;
    __syncthreads();
    if (threadIdx.x == 0) {
      if (h < nheads) {
        out[2 + h] = mean;
        total += w[h] * mean;
      } else {
        out[0] = total;
        out[1] = mean;
        if (acc) {
          acc[0] += total;
          acc[1] += mean;
        }
      }
    }
  }
}

}  // namespace pkc

extern "C" int pkc_nll_fused(const pkc_nll_args* a, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(a && a->M > 0 && a->N > 0 && a->nslab >= 1 && a->zslab && a->logp,
                "pkc_nll_fused: bad arguments");
  PKC_CHECK_ARG(a->labels || !a->dlogits, "pkc_nll_fused: dlogits needs labels");
  if (a->N >= 512)
    hipLaunchKernelGGL(nll_kernel<4>, dim3(a->M), dim3(64 * LW), 0, S(stream), *a);
  else
    hipLaunchKernelGGL(nll_kernel<1>, dim3((a->M + LW - 1) / LW), dim3(64 * LW), 0, S(stream), *a);
  PKC_LAUNCH_CHECK("pkc_nll_fused");
  return PKC_OK;
}

extern "C" int pkc_loss_finalize(int nheads, const float* const* row_loss, const float* weights,
                                 int M, const float* row_err, float* out, float* acc, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(nheads >= 1 && nheads <= 8 && row_loss && weights && row_err && out && M > 0,
                "pkc_loss_finalize: bad arguments");
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, S(stream), nheads, row_loss,
                     weights, M, row_err, out, acc);
  PKC_LAUNCH_CHECK("pkc_loss_finalize");
  return PKC_OK;
}
