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

// One row r of the batch gather (pkc_batch_gather, include/pkc.h): row i*B + r of the chunk's
// feature matrix (i = *ctr % n_batches, the device batch counter) into x_out (+ its bf16 copy) and
// its label columns into lab_out; 256 threads.  Shared by batch_gather_kernel and the grouped
// launch's PKC_OP_GATHER.
__device__ __forceinline__ void gather_row_body(const float* feats, int64_t ld, int F,
                                                const int32_t* labels, int nlab, int B,
                                                int64_t n_batches, const int64_t* ctr,
                                                float* x_out, int32_t* lab_out, __bf16* xb,
                                                bool vec, int r) {
  const int64_t i = *ctr % n_batches;
  const int64_t row0 = i * B;
  const float* src = feats + (row0 + r) * ld;
  if (vec) {   // 16-byte rows (F % 4 == 0, aligned): one load per thread for a 440-wide row
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    for (int c = 4 * threadIdx.x; c < F; c += 1024) {
      const float4 v = *reinterpret_cast<const float4*>(src + c);
      *reinterpret_cast<float4*>(x_out + (int64_t)r * F + c) = v;
      if (xb) {
        bf16x4 h;
        h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
        *reinterpret_cast<bf16x4*>(xb + (int64_t)r * F + c) = h;
      }
    }
  } else {
    for (int c = threadIdx.x; c < F; c += 256) {
      const float v = src[c];
      x_out[(int64_t)r * F + c] = v;
      if (xb) xb[(int64_t)r * F + c] = (__bf16)v;
    }
  }
  if (threadIdx.x < nlab) lab_out[r * nlab + threadIdx.x] = labels[(row0 + r) * nlab + threadIdx.x];
}

}  // namespace pkc
