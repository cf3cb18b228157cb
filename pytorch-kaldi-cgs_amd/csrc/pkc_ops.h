// pkc_ops.h — small device-side operation bodies shared by their own launches and by the
// grouped launch of pkc_gemm_grouped (several independent operations per kernel boundary).
#pragma once
#include "pkc_common.h"

namespace pkc {

// Reduce per-row losses: see pkc_loss_finalize (include/pkc.h).  One 256-thread workgroup.
__device__ __forceinline__ void loss_finalize_body(int nheads, const float* const* rl,
                                                   const float* w, int M, const float* rerr,
                                                   float* out, float* acc, int64_t* advance) {
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
        // the step's batch counter advances here, after every gather of this step has read it
        if (advance) *advance = *advance + 1;
      }
    }
  }
}


// Column sums of an M x N row-major matrix for 64 columns starting at c0 (head bias gradient:
// autograd of + bias).  256 threads = 64 columns x 4 row-threads, 8 independent rows in flight.
__device__ __forceinline__ void colsum_body(int M, int N, const float* __restrict__ x,
                                            float* __restrict__ out, int c0) {
  __shared__ float red[256];
  const int c = c0 + threadIdx.x % 64;
  const int t = threadIdx.x / 64;
  const int cc = min(c, N - 1);
  float acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = 0.f;
  for (int r0 = 0; r0 < M; r0 += 32) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = x[(int64_t)min(r0 + t + 4 * u, M - 1) * N + cc];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += (r0 + t + 4 * u < M) ? v[u] : 0.f;
  }
  const float s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  red[threadIdx.x] = s;
  __syncthreads();
  if (t == 0 && c < N) {
    const int cl = threadIdx.x % 64;
    out[c] = (red[cl] + red[64 + cl]) + (red[128 + cl] + red[192 + cl]);
  }
}

// C[i] = sum_{s < ns} A[s * stride + i] for 1024 elements i = i0 .. i0 + 1023 (< n), slab order
// (deterministic); float4 when vec (16-byte aligned bases, stride and n multiples of 4).
__device__ __forceinline__ void slabsum_body(int ns, int n, const float* __restrict__ A,
                                             int64_t stride, float* __restrict__ C, int64_t i0,
                                             bool vec) {
  const int64_t i = i0 + 4 * threadIdx.x;
  if (vec) {
    if (i >= n) return;
    float4 acc = *reinterpret_cast<const float4*>(A + i);
    for (int s = 1; s < ns; ++s) {
      const float4 x = *reinterpret_cast<const float4*>(A + (int64_t)s * stride + i);
      acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w;
    }
    *reinterpret_cast<float4*>(C + i) = acc;
    return;
  }
  for (int64_t j = i; j < i + 4 && j < n; ++j) {
    float acc = A[j];
    for (int s = 1; s < ns; ++s) acc += A[(int64_t)s * stride + j];
    C[j] = acc;
  }
}

}  // namespace pkc
