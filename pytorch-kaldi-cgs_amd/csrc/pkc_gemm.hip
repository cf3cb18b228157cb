// pkc_gemm.hip — LDS-tiled MFMA matmul for the acoustic-model layers (gfx950 / CDNA4).
//
// Replaces the cuBLAS GEMMs the reference issues through nn.Linear / F.linear and their autograd
// backward (neural_networks.py:306-317, 951-954, 1554-1555).  One kernel template covers the three
// orientations of a Linear layer's training step (Y = X W^T, dX = dY W, dW = dY^T X) by loading
// either operand k-contiguous or m-contiguous and always staging it in LDS as [row][k].
//
// Tile 64x64x32, 256 threads = 4 waves of 32x32 sub-tiles:
//   PREC_FP32: v_mfma_f32_32x32x2_f32 (exact fp32 fma chain -> parity mode), 16 MFMA per k-tile;
//              lane half h feeds k = 16h + kk (a permutation of k shared by A and B, so each
//              lane reads 16 contiguous floats of its row with ds_read_b128).
//   PREC_BF16: v_mfma_f32_32x32x16_bf16 with fp32 accumulation, 2 MFMA per k-tile; operands are
//              rounded to bf16 when staged into LDS.
// Split-K over blockIdx.z writes deterministic partial slabs (summed by the consumer kernels).
#include "pkc_common.h"

namespace pkc {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int BM = 64, BN = 64, BK = 32, NT = 256;

template <int PREC>
struct Lds;
template <>
struct Lds<PKC_PREC_FP32> {
  using T = float;
  static constexpr int LD = BK + 4;  // 144-byte rows
  float a[BM * LD];
  float b[BN * LD];
};
template <>
struct Lds<PKC_PREC_BF16> {
  using T = __bf16;
  static constexpr int LD = BK + 8;  // 80-byte rows
  __bf16 a[BM * LD];
  __bf16 b[BN * LD];
};

// Register staging of one 64x32 operand tile (8 floats per thread).
template <bool KC, bool VEC>
struct Stage {
  float v[8];
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t ld, int r0, int rmax,
                                       int k0, int kend) {
    const int t = threadIdx.x;
    if (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int idx = t + NT * i;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (KC) {
          const int r = idx >> 3, k = (idx & 7) * 4;
          if (r0 + r < rmax && k0 + k < kend)
            x = *reinterpret_cast<const float4*>(P + (int64_t)(r0 + r) * ld + k0 + k);
        } else {
          const int k = idx >> 4, r = (idx & 15) * 4;
          if (k0 + k < kend && r0 + r < rmax)
            x = *reinterpret_cast<const float4*>(P + (int64_t)(k0 + k) * ld + r0 + r);
        }
        v[4 * i + 0] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int idx = t + NT * i;
        float x = 0.f;
        if (KC) {
          const int r = idx >> 5, k = idx & 31;
          if (r0 + r < rmax && k0 + k < kend) x = P[(int64_t)(r0 + r) * ld + k0 + k];
        } else {
          const int k = idx >> 6, r = idx & 63;
          if (k0 + k < kend && r0 + r < rmax) x = P[(int64_t)(k0 + k) * ld + r0 + r];
        }
        v[i] = x;
      }
    }
  }
  template <typename T, int LD>
  __device__ __forceinline__ void store(T* __restrict__ s) const {
    const int t = threadIdx.x;
    if (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int idx = t + NT * i;
        if (KC) {
          const int r = idx >> 3, k = (idx & 7) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) s[r * LD + k + j] = (T)v[4 * i + j];
        } else {
          const int k = idx >> 4, r = (idx & 15) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) s[(r + j) * LD + k] = (T)v[4 * i + j];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int idx = t + NT * i;
        if (KC) {
          const int r = idx >> 5, k = idx & 31;
          s[r * LD + k] = (T)v[i];
        } else {
          const int k = idx >> 6, r = idx & 63;
          s[r * LD + k] = (T)v[i];
        }
      }
    }
  }
};

template <int PREC, bool AKC, bool BKC, bool VEC>
__global__ __launch_bounds__(NT) void gemm_kernel(int M, int N, int K, const float* __restrict__ A,
                                                  int64_t lda, const float* __restrict__ B,
                                                  int64_t ldb, float* __restrict__ C, int64_t ldc,
                                                  int kchunk, int64_t slab_stride) {
  __shared__ Lds<PREC> sm;
  constexpr int LD = Lds<PREC>::LD;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  Stage<AKC, VEC> sa;
  Stage<BKC, VEC> sb;
  if (kbeg < kend) {
    sa.load(A, lda, m0, M, kbeg, kend);
    sb.load(B, ldb, n0, N, kbeg, kend);
  }
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    sa.template store<typename Lds<PREC>::T, LD>(sm.a);
    sb.template store<typename Lds<PREC>::T, LD>(sm.b);
    __syncthreads();
    if (k0 + BK < kend) {  // prefetch the next k-tile into registers while computing this one
      sa.load(A, lda, m0, M, k0 + BK, kend);
      sb.load(B, ldb, n0, N, k0 + BK, kend);
    }
    if constexpr (PREC == PKC_PREC_FP32) {
      const float4* pa = reinterpret_cast<const float4*>(&sm.a[(wm * 32 + r) * LD + 16 * h]);
      const float4* pb = reinterpret_cast<const float4*>(&sm.b[(wn * 32 + r) * LD + 16 * h]);
      float av[16], bv[16];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 x = pa[q], y = pb[q];
        av[4 * q] = x.x; av[4 * q + 1] = x.y; av[4 * q + 2] = x.z; av[4 * q + 3] = x.w;
        bv[4 * q] = y.x; bv[4 * q + 1] = y.y; bv[4 * q + 2] = y.z; bv[4 * q + 3] = y.w;
      }
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk], bv[kk], acc, 0, 0, 0);
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        bf16x8 av = *reinterpret_cast<const bf16x8*>(&sm.a[(wm * 32 + r) * LD + 16 * t + 8 * h]);
        bf16x8 bv = *reinterpret_cast<const bf16x8*>(&sm.b[(wn * 32 + r) * LD + 16 * t + 8 * h]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
      }
    }
  }
  // C/D map of the 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  float* Cz = C + (int64_t)blockIdx.z * slab_stride;
  const int col = n0 + wn * 32 + r;
  if (col < N) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = m0 + wm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (row < M) Cz[(int64_t)row * ldc + col] = acc[reg];
    }
  }
}

template <int PREC, bool AKC, bool BKC, bool VEC>
static int launch(int M, int N, int K, const float* A, int64_t lda, const float* B, int64_t ldb,
                  float* C, int64_t ldc, int splits, int64_t slab, hipStream_t s) {
  int kchunk = (K + splits - 1) / splits;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, splits);
  hipLaunchKernelGGL((gemm_kernel<PREC, AKC, BKC, VEC>), grid, dim3(NT), 0, s, M, N, K, A, lda, B,
                     ldb, C, ldc, kchunk, slab);
  PKC_LAUNCH_CHECK("pkc_gemm");
  return PKC_OK;
}

template <int PREC>
static int dispatch(int akc, int bkc, bool vec, int M, int N, int K, const float* A, int64_t lda,
                    const float* B, int64_t ldb, float* C, int64_t ldc, int splits, int64_t slab,
                    hipStream_t s) {
#define PKC_G(AK, BK_, V) \
  return launch<PREC, AK, BK_, V>(M, N, K, A, lda, B, ldb, C, ldc, splits, slab, s)
  if (akc && bkc) { if (vec) PKC_G(true, true, true); PKC_G(true, true, false); }
  if (akc && !bkc) { if (vec) PKC_G(true, false, true); PKC_G(true, false, false); }
  if (!akc && !bkc) { if (vec) PKC_G(false, false, true); PKC_G(false, false, false); }
  if (vec) PKC_G(false, true, true);
  PKC_G(false, true, false);
#undef PKC_G
}

}  // namespace pkc

extern "C" int pkc_gemm_pick_splits(int M, int N, int K) {
  using namespace pkc;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int ktiles = (K + BK - 1) / BK;
  // aim at ~one workgroup per CU (256 CUs); every extra split costs its consumer one more
  // M x N partial slab to read, so stop at 8
  int s = (256 + tiles - 1) / tiles;
  s = s < 1 ? 1 : s;
  s = s > 8 ? 8 : s;
  if (s > ktiles / 2) s = ktiles / 2 > 0 ? ktiles / 2 : 1;   // >= 2 k-tiles per split
  // make every split non-empty
  int kchunk = (((K + s - 1) / s + BK - 1) / BK) * BK;
  return (K + kchunk - 1) / kchunk;
}

extern "C" int pkc_gemm(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                        const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                        int64_t ldc, int splits, int64_t slab_stride, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "pkc_gemm: negative shape");
  PKC_CHECK_ARG(prec == PKC_PREC_FP32 || prec == PKC_PREC_BF16, "pkc_gemm: bad precision %d", prec);
  if (M == 0 || N == 0) return PKC_OK;
  PKC_CHECK_ARG(A && B && C, "pkc_gemm: null operand");
  PKC_CHECK_ARG(ldc >= N, "pkc_gemm: ldc < N");
  if (splits <= 0) splits = pkc_gemm_pick_splits(M, N, K);
  PKC_CHECK_ARG(splits == 1 || slab_stride >= (int64_t)M * ldc, "pkc_gemm: slab_stride too small");
  // float4 path: 16-byte aligned bases, leading dims and contiguous extents multiple of 4
  const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % 4 == 0 &&
                   ldb % 4 == 0 && (a_kcontig ? K % 4 == 0 : M % 4 == 0) &&
                   (b_kcontig ? K % 4 == 0 : N % 4 == 0);
  if (prec == PKC_PREC_FP32)
    return dispatch<PKC_PREC_FP32>(a_kcontig, b_kcontig, vec, M, N, K, A, lda, B, ldb, C, ldc,
                                   splits, slab_stride, S(stream));
  return dispatch<PKC_PREC_BF16>(a_kcontig, b_kcontig, vec, M, N, K, A, lda, B, ldb, C, ldc,
                                 splits, slab_stride, S(stream));
}
