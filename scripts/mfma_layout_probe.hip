// Operand / result lane layout of the multi-block f32 MFMA v_mfma_f32_4x4x1f32 (16 blocks of
// 4x4x1) on gfx950: which A lane and which B lane feed each (lane, register) of the result.
// Diagnostic, not part of the library.  Build: hipcc -O2 --offload-arch=gfx950 <this> -o probe
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out) {
  const int l = threadIdx.x;
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  // (1) A = 1, B = lane + 1: each result is the B lane of its column
  f32x4 d1 = __builtin_amdgcn_mfma_f32_4x4x1f32(1.f, (float)(l + 1), z, 0, 0, 0);
  // (2) A = lane + 1, B = 1: each result is the A lane of its row
  f32x4 d2 = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.f, z, 0, 0, 0);
  for (int i = 0; i < 4; ++i) {
    out[l * 8 + i] = d1[i];
    out[l * 8 + 4 + i] = d2[i];
  }
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 8 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[64 * 8];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lane: B-lane per reg | A-lane per reg (1-based; 0 = no contribution)\n");
  for (int l = 0; l < 64; ++l)
    printf("%2d: %3.0f %3.0f %3.0f %3.0f | %3.0f %3.0f %3.0f %3.0f\n", l, h[l * 8], h[l * 8 + 1],
           h[l * 8 + 2], h[l * 8 + 3], h[l * 8 + 4], h[l * 8 + 5], h[l * 8 + 6], h[l * 8 + 7]);
  hipFree(d);
  return 0;
}
