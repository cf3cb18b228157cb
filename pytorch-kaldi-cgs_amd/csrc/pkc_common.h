// pkc — MI355X-native hot path of pytorch-kaldi-CGS run_nn(): shared device/host helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/pkc.h"

namespace pkc {

// Thread-local last-error string (pkc_last_error()).
void set_error(const char* fmt, ...);

#define PKC_CHECK_ARG(cond, ...)                                                   \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      ::pkc::set_error(__VA_ARGS__);                                               \
      return PKC_ERR_ARG;                                                          \
    }                                                                              \
  } while (0)

#define PKC_LAUNCH_CHECK(where)                                                    \
  do {                                                                             \
    hipError_t e_ = hipGetLastError();                                             \
    if (e_ != hipSuccess) {                                                        \
      ::pkc::set_error("%s: %s", where, hipGetErrorString(e_));                    \
      return PKC_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

// a HIP runtime call's status into the library error (returns PKC_ERR_HIP from the caller)
#define PKC_HIP_CHECK(call, where)                                                 \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess) {                                                        \
      ::pkc::set_error("%s: %s", where, hipGetErrorString(e_));                    \
      return PKC_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double warp_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based dropout RNG (splitmix64 finaliser over (seed, stream, index)).
__device__ __forceinline__ uint32_t hash3(uint64_t seed, uint64_t stream, uint64_t idx) {
  uint64_t z = seed ^ (stream * 0x9E3779B97F4A7C15ull) ^ (idx * 0xD1B54A32D192ED03ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

// Dropout mask bits: a 32-bit murmur3 finaliser of the element's flat index, keyed by a
// per-(seed, layer, step) 32-bit key (hash_seed: one 64-bit mix per thread, not per element).
// The reference draws torch.bernoulli; any independent uniform stream is equivalent.
__device__ __forceinline__ uint32_t hash_seed(uint64_t seed, uint64_t stream, uint64_t step) {
  return (uint32_t)(hash3(seed, stream, step * 0x2545F4914F6CDD1Dull + 0x5bd1e995ull) >> 0);
}
__device__ __forceinline__ uint32_t hash_drop(uint32_t key, uint32_t idx) {
  uint32_t h = idx * 0x9E3779B1u ^ key;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// Activations (reference neural_networks.py:54-78).  'linear' is LeakyReLU(1) == identity.
__device__ __forceinline__ float act_fwd(int act, float y) {
  switch (act) {
    case PKC_ACT_RELU: return y > 0.f ? y : 0.f;
    case PKC_ACT_TANH: return tanhf(y);
    case PKC_ACT_SIGMOID: return 1.f / (1.f + expf(-y));
    case PKC_ACT_HTANH: return fminf(fmaxf(y, -1.f), 1.f);
    case PKC_ACT_LEAKY: return y > 0.f ? y : 0.2f * y;
    case PKC_ACT_ELU: return y > 0.f ? y : expm1f(y);
    default: return y;
  }
}
// derivative given pre-activation y and post-activation a
__device__ __forceinline__ float act_bwd(int act, float y, float a) {
  switch (act) {
    case PKC_ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case PKC_ACT_TANH: return 1.f - a * a;
    case PKC_ACT_SIGMOID: return a * (1.f - a);
    case PKC_ACT_HTANH: return (y > -1.f && y < 1.f) ? 1.f : 0.f;
    case PKC_ACT_LEAKY: return y > 0.f ? 1.f : 0.2f;
    case PKC_ACT_ELU: return y > 0.f ? 1.f : a + 1.f;
    default: return 1.f;
  }
}

// derivative expressed through the post-activation value a = act(y) (all act_fun choices are
// monotone, so the branch is recoverable from a)
__device__ __forceinline__ float act_bwd_out(int act, float a) {
  switch (act) {
    case PKC_ACT_RELU: return a > 0.f ? 1.f : 0.f;
    case PKC_ACT_TANH: return 1.f - a * a;
    case PKC_ACT_SIGMOID: return a * (1.f - a);
    case PKC_ACT_HTANH: return (a > -1.f && a < 1.f) ? 1.f : 0.f;
    case PKC_ACT_LEAKY: return a > 0.f ? 1.f : 0.2f;
    case PKC_ACT_ELU: return a > 0.f ? 1.f : a + 1.f;
    default: return 1.f;
  }
}

}  // namespace pkc
