// Diagnostic micro-benchmark of the recurrent matmul-step structure (C4 shape: B2 = 32 rows,
// H = 1024, 4 gates): which part of a step launch costs what.  Not part of the library.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/rnn_diag.hip -o /tmp/rnn_diag
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int RT = 256;

template <int S>
__device__ __forceinline__ void load_strip(const float* row, bool ok, int kb, int kmax, float* v) {
#pragma unroll
  for (int s = 0; s < S; s += 4) {
    const int k = kb + s;
    const bool in = ok && k < kmax;
    const float4 x = *reinterpret_cast<const float4*>(row + (in ? k : 0));
    v[s] = in ? x.x : 0.f; v[s + 1] = in ? x.y : 0.f; v[s + 2] = in ? x.z : 0.f; v[s + 3] = in ? x.w : 0.f;
  }
}

// MODE bits: 1 = load A (h rows), 2 = load B (U rows), 4 = MFMA, 8 = A from LDS-staged tile
template <int S, int MODE>
__global__ __launch_bounds__(RT) void step(const float* h, const float* U, float* out, int H, int B2,
                                           float* hout) {
  __shared__ float red[4 * 32 * 17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  const int u0 = blockIdx.x * 4;
  const int gi = c / 4, u = u0 + c % 4;
  const int kb = (w * 4 + q) * S;
  float va[S], vb[S], vu[S];
  if (MODE & 8) {
    // stage the 32 x H tile of h through LDS with coalesced 16-B loads, rows padded by 4 floats
    extern __shared__ float hl[];
    const int LD = H + 4;
    for (int e = threadIdx.x; e < 32 * H / 4; e += RT) {
      const int r = e / (H / 4), k4 = e % (H / 4);
      const float4 x = *reinterpret_cast<const float4*>(h + (int64_t)(r < B2 ? r : 0) * H + 4 * k4);
      *reinterpret_cast<float4*>(hl + r * LD + 4 * k4) = x;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < S; s += 4) {
      const float4 x = *reinterpret_cast<const float4*>(hl + c * LD + kb + s);
      const float4 y = *reinterpret_cast<const float4*>(hl + (16 + c) * LD + kb + s);
      va[s] = x.x; va[s + 1] = x.y; va[s + 2] = x.z; va[s + 3] = x.w;
      vb[s] = y.x; vb[s + 1] = y.y; vb[s + 2] = y.z; vb[s + 3] = y.w;
    }
  } else if (MODE & 1) {
    load_strip<S>(h + (int64_t)c * H, c < B2, kb, H, va);
    load_strip<S>(h + (int64_t)(16 + c) * H, 16 + c < B2, kb, H, vb);
  } else {
#pragma unroll
    for (int s = 0; s < S; ++s) { va[s] = 1.f + s; vb[s] = 2.f + s; }
  }
  if (MODE & 2) {
    load_strip<S>(U + ((int64_t)gi * H + u) * H, true, kb, H, vu);
  } else {
#pragma unroll
    for (int s = 0; s < S; ++s) vu[s] = 0.5f * s;
  }
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
  if (MODE & 4) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(va[s], vu[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(vb[s], vu[s], acc1, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < S; ++s) { acc0[s & 3] += va[s] * vu[s]; acc1[s & 3] += vb[s] * vu[s]; }
  }
  float* rw = red + w * 32 * 17;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rw[(4 * q + i) * 17 + c] = acc0[i];
    rw[(16 + 4 * q + i) * 17 + c] = acc1[i];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 16; e += RT) {
    const int r = e >> 4, cc = e & 15;
    const int o = r * 17 + cc;
    const float v = (red[o] + red[32 * 17 + o]) + (red[2 * 32 * 17 + o] + red[3 * 32 * 17 + o]);
    if (r < B2) hout[(int64_t)r * H + u0 + (cc & 3)] = tanhf(v * 1e-3f);
  }
}

template <int MODE>
float run(const float* h, const float* U, float* out, float* h2, int H, int B2, int T) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  dim3 grid(H / 4);
  const size_t lds = (MODE & 8) ? sizeof(float) * 32 * (H + 4) : 0;
  for (int t = 0; t < 5; ++t)
    hipLaunchKernelGGL((step<64, MODE>), grid, dim3(RT), lds, 0, (t & 1) ? h2 : h, U, out, H, B2,
                       (t & 1) ? (float*)h : h2);
  hipEventRecord(e0);
  for (int t = 0; t < T; ++t)
    hipLaunchKernelGGL((step<64, MODE>), grid, dim3(RT), lds, 0, (t & 1) ? h2 : h, U, out, H, B2,
                       (t & 1) ? (float*)h : h2);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / T;
}

int main() {
  const int H = 1024, B2 = 32, T = 200;
  float *h, *h2, *U, *out;
  hipMalloc(&h, sizeof(float) * B2 * H);
  hipMalloc(&h2, sizeof(float) * B2 * H);
  hipMalloc(&U, sizeof(float) * 4 * H * H);
  hipMalloc(&out, sizeof(float) * B2 * 4 * H);
  std::vector<float> hv(4 * H * H, 0.01f);
  hipMemcpy(U, hv.data(), sizeof(float) * 4 * H * H, hipMemcpyHostToDevice);
  hipMemcpy(h, hv.data(), sizeof(float) * B2 * H, hipMemcpyHostToDevice);
  hipMemcpy(h2, hv.data(), sizeof(float) * B2 * H, hipMemcpyHostToDevice);
  printf("full (A+B+mfma)    %.2f us\n", run<7>(h, U, out, h2, H, B2, T));
  printf("A only + mfma      %.2f us\n", run<5>(h, U, out, h2, H, B2, T));
  printf("B only + mfma      %.2f us\n", run<6>(h, U, out, h2, H, B2, T));
  printf("mfma only          %.2f us\n", run<4>(h, U, out, h2, H, B2, T));
  printf("A+B, no mfma       %.2f us\n", run<3>(h, U, out, h2, H, B2, T));
  printf("nothing            %.2f us\n", run<0>(h, U, out, h2, H, B2, T));
  printf("A via LDS + B + mfma %.2f us\n", run<14>(h, U, out, h2, H, B2, T));
  printf("A via LDS + mfma   %.2f us\n", run<12>(h, U, out, h2, H, B2, T));
  return 0;
}
