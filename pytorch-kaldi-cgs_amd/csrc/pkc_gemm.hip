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
//   PREC_BF16IN: the same MFMA with operands already stored as bf16 in HBM (the bf16 copies of
//              weights / activations / gradients the step keeps): half the bytes per workgroup,
//              one 16-byte load per thread per operand per k-tile.
//   PREC_BF16X3: compensated bf16 — fp32 operands split at staging into bf16 head + tail tiles
//              (hi = bf16(v), lo = bf16(v - hi)), 6 MFMA per k-tile (hi*hi + hi*lo + lo*hi): fp32-
//              class products (~2^-16 relative) on the bf16 MFMA, 3/16 of the exact-fp32 chain.
// Split-K over blockIdx.z writes deterministic partial slabs (summed by the consumer kernels).
#include "pkc_gemm_big.h"
#include "pkc_ops.h"
#include "pkc_optim.h"

namespace pkc {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int BM = 64, BN = 64, BK = 32, NT = 256;

template <int PREC>
struct Lds;
// LO: element offset of the bf16 tail tiles from the head tiles (PREC_BF16X3; 0: none)
template <>
struct Lds<PKC_PREC_FP32> {
  using T = float;
  static constexpr int LD = BK + 4;  // 144-byte rows
  static constexpr int LO = 0;
  float a[BM * LD];
  float b[BN * LD];
};
template <>
struct Lds<PKC_PREC_BF16> {
  using T = __bf16;
  static constexpr int LD = BK + 8;  // 80-byte rows
  static constexpr int LO = 0;
  __bf16 a[BM * LD];
  __bf16 b[BN * LD];
};
template <>
struct Lds<PKC_PREC_BF16X3> {
  using T = __bf16;
  static constexpr int LD = BK + 8;
  static constexpr int LO = (BM + BN) * LD;   // al = a + LO, bl = b + LO
  __bf16 a[BM * LD];
  __bf16 b[BN * LD];
  __bf16 al[BM * LD];
  __bf16 bl[BN * LD];
};

// one staged element: its bf16 head, and (LO > 0) its bf16 tail LO elements further
template <typename T, int LO>
__device__ __forceinline__ void put(T* __restrict__ s, int i, float v) {
  const T hv = (T)v;
  s[i] = hv;
  if constexpr (LO > 0) s[i + LO] = (T)(v - (float)hv);
}

// LDS swizzle of an m-contiguous (not k-contiguous) fp32 operand.  Its register stage holds 4
// consecutive ROWS of one k, so the store into the [row][k] tile is a column write: with the plain
// layout the rows of a wave's 64 lanes fall into two banks (8-way conflicts on every such store,
// the cost that dominated the sequence models' dW / dU matmuls).  Rotating each row's 16-byte
// k-chunks by row / 4 spreads them (2-way).  k-contiguous operands keep the plain layout, which
// their conflict-free 16-byte stores and fragment reads prefer; measured on the box, the same
// rotation of the bf16 tiles made the C2 step slower (0.204 vs 0.197 ms), so bf16 keeps it too.
__device__ __forceinline__ int swz4(int row, int c4) { return (c4 + (row >> 2)) & 7; }

// Register staging of one 64x32 operand tile (8 floats per thread).  Loads are issued
// unconditionally from clamped (always valid) addresses and out-of-range values are zeroed by a
// select afterwards: a load guarded by a runtime condition makes hipcc branch around it and drain
// the whole vmcnt queue, which would serialise the prefetch ring.
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
        int r, k;
        if (KC) { r = idx >> 3; k = (idx & 7) * 4; }
        else { k = idx >> 4; r = (idx & 15) * 4; }
        const bool ok = (r0 + r < rmax) && (k0 + k < kend);
        const int rr = min(r0 + r, rmax - (KC ? 1 : 4));
        const int kk = min(k0 + k, kend - (KC ? 4 : 1));
        const float4 x = KC ? *reinterpret_cast<const float4*>(P + (int64_t)rr * ld + kk)
                            : *reinterpret_cast<const float4*>(P + (int64_t)kk * ld + rr);
        v[4 * i + 0] = ok ? x.x : 0.f;
        v[4 * i + 1] = ok ? x.y : 0.f;
        v[4 * i + 2] = ok ? x.z : 0.f;
        v[4 * i + 3] = ok ? x.w : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int idx = t + NT * i;
        int r, k;
        if (KC) { r = idx >> 5; k = idx & 31; }
        else { k = idx >> 6; r = idx & 63; }
        const bool ok = (r0 + r < rmax) && (k0 + k < kend);
        const int rr = min(r0 + r, rmax - 1);
        const int kk = min(k0 + k, kend - 1);
        const float x = KC ? P[(int64_t)rr * ld + kk] : P[(int64_t)kk * ld + rr];
        v[i] = ok ? x : 0.f;
      }
    }
  }
  // VEC form with the row part of the addresses hoisted (StageH::lane_base / load_at): chunk i of
  // this thread is row (t >> 3) + 32 i, k (t & 7) * 4 (KC) or row (t & 15) * 4, k (t >> 4) + 16 i
  struct Base {
    const float* p[2];
    bool ok[2];
  };
  __device__ __forceinline__ static Base lane_base(const void* __restrict__ Pv, int64_t ld, int r0,
                                                   int rmax) {
    const float* P = reinterpret_cast<const float*>(Pv);
    const int t = threadIdx.x;
    Base b;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = KC ? (t >> 3) + 32 * i : (t & 15) * 4;
      const int rr = min(r0 + r, rmax - (KC ? 1 : 4));
      b.p[i] = KC ? P + (int64_t)rr * ld : P + rr;
      b.ok[i] = r0 + r < rmax;
    }
    return b;
  }
  __device__ __forceinline__ void load_at(const Base& b, int ld, int k0, int kend) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = KC ? (t & 7) * 4 : (t >> 4) + 16 * i;
      const bool ok = b.ok[i] && (k0 + k < kend);
      const int kk = min(k0 + k, kend - (KC ? 4 : 1));
      const float4 x = KC ? *reinterpret_cast<const float4*>(b.p[i] + kk)
                          : *reinterpret_cast<const float4*>(b.p[i] + (int64_t)kk * ld);
      v[4 * i + 0] = ok ? x.x : 0.f;
      v[4 * i + 1] = ok ? x.y : 0.f;
      v[4 * i + 2] = ok ? x.z : 0.f;
      v[4 * i + 3] = ok ? x.w : 0.f;
    }
  }
  template <typename T, int LD, int LO = 0>
  __device__ __forceinline__ void store(T* __restrict__ s) const {
    const int t = threadIdx.x;
    if (VEC) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int idx = t + NT * i;
        if (KC) {
          const int r = idx >> 3, k = (idx & 7) * 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) put<T, LO>(s, r * LD + k + j, v[4 * i + j]);
        } else {
          const int k = idx >> 4, r = (idx & 15) * 4;
          if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              s[(r + j) * LD + 4 * swz4(r + j, k >> 2) + (k & 3)] = (T)v[4 * i + j];
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) put<T, LO>(s, (r + j) * LD + k, v[4 * i + j]);
          }
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int idx = t + NT * i;
        if (KC) {
          const int r = idx >> 5, k = idx & 31;
          put<T, LO>(s, r * LD + k, v[i]);
        } else {
          const int k = idx >> 6, r = idx & 63;
          if constexpr (sizeof(T) == 4) s[r * LD + 4 * swz4(r, k >> 2) + (k & 3)] = (T)v[i];
          else put<T, LO>(s, r * LD + k, v[i]);
        }
      }
    }
  }
};

// [k][row] image of an m-contiguous bf16 64x32 operand tile: 32 k-rows of 64 elements (128 B),
// 16-byte chunk c of k-row k at chunk c ^ (((k >> 1) & 1) << 2).  A transposed fragment read of one
// 32-lane half touches 4 consecutive k-rows x 64 contiguous bytes: the XOR moves k-rows k + 2, k + 3
// to the other 64-byte half, so the four land on 64 distinct banks (conflict-free).
__device__ __forceinline__ int tr_off_s(int k, int c) { return 128 * k + 16 * (c ^ (((k >> 1) & 1) << 2)); }

// 32x32x16 operand fragment (lane l: row rb + (l & 31), k = kb + 8 (l >> 5) + j) from that image:
// two ds_read_b64_tr_b16 (lane 4q + p of a 16-lane group addresses k-row k0 + q, rows 4p .. 4p + 3
// of the group's 16; lane i receives row i of the 4 k-rows).
__device__ __forceinline__ bf16x8 tr_frag_s(const char* __restrict__ s, int rb, int kb, int lane) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef short v8s __attribute__((ext_vector_type(8)));
  typedef __attribute__((address_space(3))) v4s lv4s;
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int row = rb + 16 * ((lane >> 4) & 1) + 4 * p;
  const int k0 = kb + 8 * (lane >> 5) + q;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lv4s*)(s + tr_off_s(k0, row >> 3) + 8 * (p & 1)));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lv4s*)(s + tr_off_s(k0 + 4, row >> 3) + 8 * (p & 1)));
  const v8s w = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, w);
}

__device__ __forceinline__ bf16x8 ld8h(const __bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x8 zero8h() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

// Register staging of one 64x32 bf16 operand tile: one 16-byte load per thread (VEC) or eight
// 2-byte loads; clamped addresses + zeroing selects as in Stage.
template <bool KC, bool VEC>
struct StageH {
  bf16x8 v;
  __device__ __forceinline__ void load(const __bf16* __restrict__ P, int64_t ld, int r0, int rmax,
                                       int k0, int kend) {
    const int t = threadIdx.x;
    int r, k;
    if (KC) { r = t >> 2; k = (t & 3) * 8; }
    else { k = t >> 3; r = (t & 7) * 8; }
    if (VEC) {
      const bool ok = (r0 + r < rmax) && (k0 + k < kend);
      const int rr = min(r0 + r, rmax - (KC ? 1 : 8));
      const int kk = min(k0 + k, kend - (KC ? 8 : 1));
      const bf16x8 x = KC ? ld8h(P + (int64_t)rr * ld + kk) : ld8h(P + (int64_t)kk * ld + rr);
      v = ok ? x : zero8h();
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int rj = KC ? r : r + j, kj = KC ? k + j : k;
        const bool ok = (r0 + rj < rmax) && (k0 + kj < kend);
        const int rr = min(r0 + rj, rmax - 1), kk = min(k0 + kj, kend - 1);
        const __bf16 x = KC ? P[(int64_t)rr * ld + kk] : P[(int64_t)kk * ld + rr];
        v[j] = ok ? x : (__bf16)0.f;
      }
    }
  }
  // VEC form with the row part of the address hoisted: lane_base() once per launch (the row clamp
  // and, for KC, the 64-bit row product), load_at() per k-tile (a 32-bit k offset, or one
  // 32x32->64 product for m-contiguous operands).  Same clamps and zeroing as load().
  struct Base {
    const __bf16* p;
    bool ok;
  };
  __device__ __forceinline__ static Base lane_base(const void* __restrict__ Pv, int64_t ld, int r0,
                                                   int rmax) {
    const __bf16* P = reinterpret_cast<const __bf16*>(Pv);
    const int t = threadIdx.x;
    const int r = KC ? t >> 2 : (t & 7) * 8;
    const int rr = min(r0 + r, rmax - (KC ? 1 : 8));
    return Base{KC ? P + (int64_t)rr * ld : P + rr, r0 + r < rmax};
  }
  __device__ __forceinline__ void load_at(const Base& b, int ld, int k0, int kend) {
    const int t = threadIdx.x;
    const int k = KC ? (t & 3) * 8 : t >> 3;
    const bool ok = b.ok && (k0 + k < kend);
    const int kk = min(k0 + k, kend - (KC ? 8 : 1));
    const bf16x8 x = KC ? ld8h(b.p + kk) : ld8h(b.p + (int64_t)kk * ld);
    v = ok ? x : zero8h();
  }
  template <typename T, int LD, int LO = 0>
  __device__ __forceinline__ void store(T* __restrict__ s) const {
    static_assert(LO == 0, "bf16-stored operands have no tail");
    const int t = threadIdx.x;
    if (KC) {
      const int r = t >> 2, k = (t & 3) * 8;
      *reinterpret_cast<bf16x8*>(&s[r * LD + k]) = v;
    } else {
      // m-contiguous: the 8 rows of one k as they lie, into the [k][row] image (tr_off_s), read
      // back by the transposing fragment read (tr_frag_s) instead of 8 two-byte column writes
      const int k = t >> 3, r = (t & 7) * 8;
      *reinterpret_cast<bf16x8*>(reinterpret_cast<char*>(s) + tr_off_s(k, r >> 3)) = v;
    }
  }
};

template <bool BIN, bool KC, bool VEC>
struct StageSel {
  using T = Stage<KC, VEC>;
  using E = float;
};
template <bool KC, bool VEC>
struct StageSel<true, KC, VEC> {
  using T = StageH<KC, VEC>;
  using E = __bf16;
};

// ATR / BTR: the operand sits in LDS as a [k][row] image (bf16 m-contiguous operands stored as
// bf16: StageH) and is read with tr_frag_s
template <int PREC, bool AKC, bool BKC, bool ATR = false, bool BTR = false>
__device__ __forceinline__ void mfma_tile(const Lds<PREC>& sm, int wm, int wn, int r, int h,
                                          f32x16& acc) {
  constexpr int LD = Lds<PREC>::LD;
  const int ra = wm * 32 + r, rb = wn * 32 + r;
  if constexpr (PREC == PKC_PREC_FP32) {
    const float4* pa = reinterpret_cast<const float4*>(&sm.a[ra * LD + 16 * h]);
    const float4* pb = reinterpret_cast<const float4*>(&sm.b[rb * LD + 16 * h]);
    float av[16], bv[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 x, y;
      if constexpr (AKC) x = pa[q];
      else x = *reinterpret_cast<const float4*>(&sm.a[ra * LD + 4 * swz4(ra, 4 * h + q)]);
      if constexpr (BKC) y = pb[q];
      else y = *reinterpret_cast<const float4*>(&sm.b[rb * LD + 4 * swz4(rb, 4 * h + q)]);
      av[4 * q] = x.x; av[4 * q + 1] = x.y; av[4 * q + 2] = x.z; av[4 * q + 3] = x.w;
      bv[4 * q] = y.x; bv[4 * q + 1] = y.y; bv[4 * q + 2] = y.z; bv[4 * q + 3] = y.w;
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk], bv[kk], acc, 0, 0, 0);
  } else if constexpr (PREC == PKC_PREC_BF16X3) {
    // tails first (the small terms), then the heads, into the same fp32 accumulator
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ia = (wm * 32 + r) * LD + 16 * t + 8 * h, ib = (wn * 32 + r) * LD + 16 * t + 8 * h;
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(&sm.a[ia]);
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(&sm.b[ib]);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(&sm.al[ia]);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&sm.bl[ib]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bv, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    }
  } else {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      bf16x8 av, bv;
      if constexpr (ATR) av = tr_frag_s(reinterpret_cast<const char*>(sm.a), wm * 32, 16 * t, lane);
      else av = *reinterpret_cast<const bf16x8*>(&sm.a[(wm * 32 + r) * LD + 16 * t + 8 * h]);
      if constexpr (BTR) bv = tr_frag_s(reinterpret_cast<const char*>(sm.b), wn * 32, 16 * t, lane);
      else bv = *reinterpret_cast<const bf16x8*>(&sm.b[(wn * 32 + r) * LD + 16 * t + 8 * h]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    }
  }
}

// DEPTH k-tiles are in flight in registers at any time: with M = 128-row batches a workgroup's
// k-range is only a few tiles long, so the whole range is requested up front instead of one
// HBM/L2 round trip per tile.
// Column statistics of a finished 64x64 tile (pkc_gemm_colstats on the 64x64 body): per column,
// the mean of its rows < M plus bias[c] and M2 = sum (z - mean)^2 over the tile's 64 rows — two
// passes over the accumulators, the two 32-lane halves combined by a shuffle and the two row waves
// through LDS in a fixed order (big::tile_colstats at 64 rows).  part[by*2N + c], part[by*2N+N+c].
template <int PREC>
__device__ __forceinline__ void tile_colstats64(const f32x16& acc, Lds<PREC>& sm, int m0, int n0,
                                                int by, int M, int N, int wm, int wn, int r, int h,
                                                const float* __restrict__ bias,
                                                float* __restrict__ part) {
  float* red = reinterpret_cast<float*>(&sm);      // [2 passes][2 row waves][64 columns]
  const int nv = min(BM, M - m0);
  const int cl = wn * 32 + r;
  __syncthreads();                                 // the last k-tile's fragment reads are done
  float sum = 0.f;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int rl = wm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
    sum += rl < nv ? acc[reg] : 0.f;
  }
  sum += __shfl_xor(sum, 32);
  if (h == 0) red[wm * BN + cl] = sum;
  __syncthreads();
  const float mean = (red[cl] + red[BN + cl]) / (float)nv;
  float q = 0.f;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int rl = wm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
    const float d = acc[reg] - mean;
    q += rl < nv ? d * d : 0.f;
  }
  q += __shfl_xor(q, 32);
  if (h == 0) red[2 * BN + wm * BN + cl] = q;
  __syncthreads();
  const int col = n0 + cl;
  if (wm != 0 || h != 0 || col >= N) return;
  part[(int64_t)by * 2 * N + col] = mean + (bias ? bias[col] : 0.f);
  part[(int64_t)by * 2 * N + N + col] = red[2 * BN + cl] + red[3 * BN + cl];
}

template <int PREC, bool AKC, bool BKC, bool VEC, int DEPTH, bool BIN, bool STATS = false>
__device__ __forceinline__ void gemm_body(Lds<PREC>& sm, int bx, int by, int bz, int M, int N, int K,
                                          const void* __restrict__ Av, int64_t lda,
                                          const void* __restrict__ Bv, int64_t ldb,
                                          float* __restrict__ C, int64_t ldc, int kchunk,
                                          int64_t slab_stride, const float* __restrict__ bias = nullptr,
                                          float* __restrict__ part = nullptr) {
  using SA = typename StageSel<BIN, AKC, VEC>::T;
  using SB = typename StageSel<BIN, BKC, VEC>::T;
  const auto* A = reinterpret_cast<const typename StageSel<BIN, AKC, VEC>::E*>(Av);
  const auto* B = reinterpret_cast<const typename StageSel<BIN, BKC, VEC>::E*>(Bv);
  constexpr int LD = Lds<PREC>::LD;
  const int n0 = bx * BN, m0 = by * BM;
  const int kbeg = bz * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  SA sa[DEPTH];
  SB sb[DEPTH];
  bool done = false;
  if constexpr (VEC) {
    // 16-byte operands whose whole k-range fits one round of DEPTH tiles (every forward / dX / dW
    // matmul of the B = 128 step): the row part of each address computed once (lane_base), no
    // refill loads for tiles past the range and no zero tiles.  Longer ranges take the general
    // loop below.  (Leading dimensions are below 2^31 elements: pkc_gemm checks.)
    const int nk = (kend - kbeg + BK - 1) / BK;             // uniform
    if (kbeg < kend && nk <= DEPTH) {
      const typename SA::Base ab = SA::lane_base(A, lda, m0, M);
      const typename SB::Base bb = SB::lane_base(B, ldb, n0, N);
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        if (d >= nk) break;                                  // uniform
        sa[d].load_at(ab, (int)lda, kbeg + d * BK, kend);
        sb[d].load_at(bb, (int)ldb, kbeg + d * BK, kend);
      }
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        if (d >= nk) break;                                  // uniform
        __syncthreads();
        sa[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.a);
        sb[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.b);
        __syncthreads();
        mfma_tile<PREC, AKC, BKC, BIN && !AKC, BIN && !BKC>(sm, wm, wn, r, h, acc);
      }
      done = true;
    }
  }
  if constexpr (VEC) {
    if (!done && kbeg < kend) {   // uniform; the same rounds as below, row addresses hoisted
      const typename SA::Base ab = SA::lane_base(A, lda, m0, M);
      const typename SB::Base bb = SB::lane_base(B, ldb, n0, N);
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        sa[d].load_at(ab, (int)lda, kbeg + d * BK, kend);
        sb[d].load_at(bb, (int)ldb, kbeg + d * BK, kend);
      }
      for (int kt = kbeg; kt < kend; kt += DEPTH * BK) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
          __syncthreads();
          sa[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.a);
          sb[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.b);
          __syncthreads();
          const int kn = kt + (d + DEPTH) * BK;
          sa[d].load_at(ab, (int)lda, kn, kend);
          sb[d].load_at(bb, (int)ldb, kn, kend);
          mfma_tile<PREC, AKC, BKC, BIN && !AKC, BIN && !BKC>(sm, wm, wn, r, h, acc);
        }
      }
      done = true;
    }
  }
  if (!done && kbeg < kend) {   // uniform: an empty trailing split writes zeros
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      sa[d].load(A, lda, m0, M, kbeg + d * BK, kend);
      sb[d].load(B, ldb, n0, N, kbeg + d * BK, kend);
    }
    // whole rounds of DEPTH k-tiles; tiles past kend load clamped addresses and contribute zeros
    for (int kt = kbeg; kt < kend; kt += DEPTH * BK) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        __syncthreads();
        sa[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.a);
        sb[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.b);
        __syncthreads();
        const int kn = kt + (d + DEPTH) * BK;
        sa[d].load(A, lda, m0, M, kn, kend);
        sb[d].load(B, ldb, n0, N, kn, kend);
        mfma_tile<PREC, AKC, BKC, BIN && !AKC, BIN && !BKC>(sm, wm, wn, r, h, acc);
      }
    }
  }
  // C/D map of the 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  const int col = n0 + wn * 32 + r;
  const int row0 = m0 + wm * 32 + 4 * h;
  if (col < N) {
    float* Cr = C + (int64_t)bz * slab_stride + (int64_t)row0 * ldc + col;
    const int ldci = (int)ldc;          // < 2^26 (pkc_gemm checks): dr * ldci fits 32 bits
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int dr = (reg & 3) + 8 * (reg >> 2);
      if (row0 + dr < M) Cr[dr * ldci] = acc[reg];
    }
  }
  if constexpr (STATS) tile_colstats64<PREC>(acc, sm, m0, n0, by, M, N, wm, wn, r, h, bias, part);
}

// Block-sparse W (klist): the tile's k-tiles are klist[1..klist[0]] instead of a contiguous
// range; k-tiles past the list load clamped addresses as zeros.  A body of its own, so the dense
// body (the latency-bound B = 128 launches) keeps its exact instruction stream.
template <int PREC, bool AKC, bool BKC, bool VEC, int DEPTH, bool BIN, bool SPARSE = true>
__device__ __forceinline__ void gemm_body_sparse(Lds<PREC>& sm, int bx, int by, int bz, int M, int N, int K,
                                          const void* __restrict__ Av, int64_t lda,
                                          const void* __restrict__ Bv, int64_t ldb,
                                          float* __restrict__ C, int64_t ldc, int kchunk,
                                          int64_t slab_stride,
                                          const int32_t* __restrict__ klist = nullptr) {
  using SA = typename StageSel<BIN, AKC, VEC>::T;
  using SB = typename StageSel<BIN, BKC, VEC>::T;
  const auto* A = reinterpret_cast<const typename StageSel<BIN, AKC, VEC>::E*>(Av);
  const auto* B = reinterpret_cast<const typename StageSel<BIN, BKC, VEC>::E*>(Bv);
  constexpr int LD = Lds<PREC>::LD;
  const int n0 = bx * BN, m0 = by * BM;
  // (the list logic is compiled only into the SPARSE instances: the dense ones stay as lean as
  // they were, which the latency-bound B = 128 launches notice)
  const int kbeg = SPARSE ? 0 : bz * kchunk;
  const int kend = SPARSE ? K : min(K, kbeg + kchunk);
  const int nkt = SPARSE ? klist[0] : (kend - kbeg + BK - 1) / BK;     // uniform
  // first k of the i-th k-tile of this tile (dense: past kend loads zeros; sparse: kend)
  auto k0_of = [&](int i) {
    if constexpr (SPARSE) return i < nkt ? klist[1 + i] * BK : kend;
    else return kbeg + i * BK;
  };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r = lane & 31, h = lane >> 5;

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  SA sa[DEPTH];
  SB sb[DEPTH];
  if (nkt > 0) {   // uniform: an empty trailing split (or an all-zero sparse tile) writes zeros
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const int k0 = k0_of(d);
      sa[d].load(A, lda, m0, M, k0, kend);
      sb[d].load(B, ldb, n0, N, k0, kend);
    }
    // whole rounds of DEPTH k-tiles; tiles past the last one contribute zeros
    for (int i0 = 0; i0 < nkt; i0 += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        __syncthreads();
        sa[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.a);
        sb[d].template store<typename Lds<PREC>::T, LD, Lds<PREC>::LO>(sm.b);
        __syncthreads();
        const int kn = k0_of(i0 + d + DEPTH);
        sa[d].load(A, lda, m0, M, kn, kend);
        sb[d].load(B, ldb, n0, N, kn, kend);
        mfma_tile<PREC, AKC, BKC, BIN && !AKC, BIN && !BKC>(sm, wm, wn, r, h, acc);
      }
    }
  }
  // C/D map of the 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
  const int col = n0 + wn * 32 + r;
  float* Cz = C + (int64_t)bz * slab_stride;
  if (col < N) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = m0 + wm * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (row < M) Cz[(int64_t)row * ldc + col] = acc[reg];
    }
  }
}

// one-slab product + 64-row column statistics (pkc_gemm_colstats on the 64x64 body)
template <int PREC, bool AKC, bool BKC, int DEPTH, bool BIN>
__global__ __launch_bounds__(NT) void gemm_stats_kernel(int M, int N, int K,
                                                        const void* __restrict__ A, int64_t lda,
                                                        const void* __restrict__ B, int64_t ldb,
                                                        float* __restrict__ C, int64_t ldc,
                                                        const float* __restrict__ bias,
                                                        float* __restrict__ part) {
  __shared__ Lds<PREC> sm;
  gemm_body<PREC, AKC, BKC, true, DEPTH, BIN, true>(sm, blockIdx.x, blockIdx.y, 0, M, N, K, A, lda,
                                                    B, ldb, C, ldc, ((K + BK - 1) / BK) * BK, 0,
                                                    bias, part);
}

template <int PREC, bool AKC, bool BKC, bool VEC, int DEPTH, bool BIN>
__global__ __launch_bounds__(NT) void gemm_kernel(int M, int N, int K, const void* __restrict__ A,
                                                  int64_t lda, const void* __restrict__ B,
                                                  int64_t ldb, float* __restrict__ C, int64_t ldc,
                                                  int kchunk, int64_t slab_stride) {
  __shared__ Lds<PREC> sm;
  gemm_body<PREC, AKC, BKC, VEC, DEPTH, BIN>(sm, blockIdx.x, blockIdx.y, blockIdx.z, M, N, K, A, lda,
                                             B, ldb, C, ldc, kchunk, slab_stride);
}

// XCD-aware tile order for the standalone 128x128 launches of at most 256 workgroups (PKC_GEMM_XCD,
// default on; B = 4096 step 3.94-3.96 M -> 4.05-4.06 M frames/s, same run): workgroup
// w runs on XCD w % 8 (round-robin dispatch), so the linear id is remapped (bijectively, for any
// grid size) to give each XCD a contiguous run of tiles in (N-tile fastest, M-tile, split) order:
// the N-tiles of one A row-block share an XCD and its L2, and an XCD reads 1/8 of A instead of
// all of it.  Speed only: any placement computes the same tiles.
__device__ __forceinline__ void xcd_tile(int remap, int& bx, int& by, int& bz) {
  const int nx = gridDim.x, ny = gridDim.y;
  const int nwg = nx * ny * gridDim.z;
  int id = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  if (remap && nwg >= 16 && nwg <= 256) {     // one workgroup per CU at most (several tiles per
                                              // CU measured slower: 8192^3 750 -> 685 TF/s)
    const int xcd = id % 8, q = nwg / 8, r = nwg % 8;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
  }
  bx = id % nx;
  by = (id / nx) % ny;
  bz = id / (nx * ny);
}

// STATS: the tile's BatchNorm column statistics in the epilogue (pkc_gemm_colstats)
template <int NB, bool AKC, bool BKC, bool STATS>
__global__ __launch_bounds__(big::NT) void gemm_glds_kernel(int M, int N, int K,
                                                           const void* __restrict__ A, int64_t lda,
                                                           const void* __restrict__ B, int64_t ldb,
                                                           float* __restrict__ C, int64_t ldc,
                                                           int kchunk, int64_t slab_stride,
                                                           int remap, const float* __restrict__ bias,
                                                           float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char lds[big::gl_lds_bytes<NB>()];
  int bx, by, bz;
  xcd_tile(remap, bx, by, bz);
  big::body_glds<NB, AKC, BKC, STATS>(lds, bx, by, bz, M, N, K, A, lda, B, ldb, C, ldc, kchunk,
                                      slab_stride, bias, part);
}

template <int PREC, bool BIN, bool AKC, bool BKC, bool STATS>
__global__ __launch_bounds__(big::NT) void gemm_big_kernel(int M, int N, int K,
                                                          const void* __restrict__ A, int64_t lda,
                                                          const void* __restrict__ B, int64_t ldb,
                                                          float* __restrict__ C, int64_t ldc,
                                                          int kchunk, int64_t slab_stride,
                                                          int remap, const float* __restrict__ bias,
                                                          float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char lds[big::lds_bytes<PREC>()];
  int bx, by, bz;
  xcd_tile(remap, bx, by, bz);
  big::body<PREC, BIN, AKC, BKC, STATS>(lds, bx, by, bz, M, N, K, A, lda, B, ldb, C, ldc, kchunk,
                                        slab_stride, bias, part);
}

// Several independent matmuls in ONE launch (e.g. a layer's dW and dX, both heads' logits):
// workgroup ranges are assigned to problems in order; each workgroup dispatches on its problem's
// operand orientation.  One launch boundary instead of one per matmul.
constexpr int GMAX = 8;
struct GroupProb {
  int kind;              // PKC_OP_GEMM / COLSUM / LOSS / OPTIM / SLABSUM / GATHER
  int code;              // a_kcontig*4 + b_kcontig*2 + vec (+8: 128x128 tile body)
  int M, N, K, kchunk, tn, tmn, wg0;
  const void* A; int64_t lda; const void* B; int64_t ldb; float* C; int64_t ldc; int64_t slab;
  const void* X1; void* X2; void* X3;
  const int32_t* ktiles; int kmax;
  int bnb;               // >= 0: the BatchNorm-backward epilogue bnb[this] (dX problems)
};
constexpr int GBNB = 2;  // BatchNorm-backward epilogues per grouped launch
struct GroupArgs {
  GroupProb p[GMAX];
  int n;
  OptSegK seg[PKC_OPT_SEGS_MAX];   // direct PKC_OP_OPTIM runs (GroupProb: code 1, segments K .. K+N)
  big::BnEpi bnb[GBNB];
};

// SUM: the launch carries slab-sum operations (large-batch split-K dW); a separate instance,
// because that body alone raises the kernel's VGPRs from 152 to 191 (occupancy 3 -> 2), which the
// B = 128 step's lean launches cannot afford
// VO: every matmul of the launch takes the 16-byte operand path (the B = 128 step's): the 2-byte
// element-wise forms are not compiled in, so they do not set the launch's register allocation
template <int PREC, bool BIN, bool BIG, bool SP, bool SUM, int GD, bool VO>
__device__ __forceinline__ void grouped_body(const GroupArgs& g) {
  // BIG: at least one problem takes the 128x128 body; its LDS also holds the 64x64 tiles
  union alignas(16) Shm {
    Lds<PREC> t;
    char big[BIG ? big::lds_bytes<PREC>() : 16];
  };
  __shared__ Shm shm;
  Lds<PREC>& sm = shm.t;
  char* lds = shm.big;
  int i = 0;
#pragma unroll
  for (int j = 1; j < GMAX; ++j)
    if (j < g.n && (int)blockIdx.x >= g.p[j].wg0) i = j;
  const GroupProb& p = g.p[i];
  const int local = blockIdx.x - p.wg0;
  if (p.kind == PKC_OP_COLSUM) {
    colsum_body(p.M, p.N, reinterpret_cast<const float*>(p.A), p.C, local * 64);
    return;
  }
  if constexpr (SUM) {
    if (p.kind == PKC_OP_SLABSUM) {
      slabsum_body(p.M, p.N, reinterpret_cast<const float*>(p.A), p.slab, p.C,
                   (int64_t)local * 1024, p.code != 0);
      return;
    }
  }
  if (p.kind == PKC_OP_OPTIM) {
    if (p.code) {                    // direct runs: pointers in the kernel arguments
      int j = p.K;
#pragma unroll
      for (int u = 1; u < PKC_OPT_SEGS_MAX; ++u) {
        const int jj = min(p.K + u, PKC_OPT_SEGS_MAX - 1);   // in bounds even when speculated
        if (u < p.N && local >= g.seg[jj].begin) j = jj;
      }
      const OptSegK& sg = g.seg[j];
      optim_seg_wg(reinterpret_cast<const pkc_opt_tensor*>(p.A), sg, local - sg.begin);
      return;
    }
    optim_wg(reinterpret_cast<const pkc_opt_tensor*>(p.A), reinterpret_cast<const int32_t*>(p.B),
             local);
    return;
  }
  if (p.kind == PKC_OP_GATHER) {
    gather_row_body(reinterpret_cast<const float*>(p.A), p.lda, p.N,
                    reinterpret_cast<const int32_t*>(p.B), (int)p.ldb, p.M, p.slab,
                    reinterpret_cast<const int64_t*>(p.X1), p.C, reinterpret_cast<int32_t*>(p.X2),
                    reinterpret_cast<__bf16*>(p.X3), p.code != 0, local);
    return;
  }
  if (p.kind == PKC_OP_LOSS) {
    loss_finalize_body(p.M, reinterpret_cast<const float* const*>(p.A),
                       reinterpret_cast<const float*>(p.B), p.N, reinterpret_cast<const float*>(p.X1),
                       p.C, reinterpret_cast<float*>(p.X2), reinterpret_cast<int64_t*>(p.X3));
    return;
  }
  const int bz = local / p.tmn, rem = local % p.tmn;
  const int by = rem / p.tn, bx = rem % p.tn;
  if constexpr (BIG) {
    if (p.code >= 8 && p.bnb >= 0) {       // dX with the BatchNorm-backward epilogue
      big::body<PREC, BIN, true, false, false, true>(lds, bx, by, bz, p.M, p.N, p.K, p.A, p.lda, p.B,
                                                     p.ldb, p.C, p.ldc, p.kchunk, p.slab, nullptr,
                                                     nullptr, &g.bnb[p.bnb < GBNB ? p.bnb : 0]);
      return;
    }
    if (p.code >= 8) {
#define PKC_BB(AK, BK_)                                                                          \
  big::body<PREC, BIN, AK, BK_>(lds, bx, by, bz, p.M, p.N, p.K, p.A, p.lda, p.B, p.ldb, p.C, p.ldc, \
                                p.kchunk, p.slab)
      switch (p.code & 6) {
        case 6: PKC_BB(true, true); break;
        case 4: PKC_BB(true, false); break;
        case 2: PKC_BB(false, true); break;
        default: PKC_BB(false, false); break;
      }
#undef PKC_BB
      return;
    }
  }
  if (SP && p.ktiles) {              // block-sparse W: forward (B = W) and dX (B = W^T) forms
    const int32_t* kl = p.ktiles + (int64_t)bx * (p.kmax + 1);
#define PKC_GS(AK, BK_, V)                                                                      \
  gemm_body_sparse<PREC, AK, BK_, V, 4, BIN>(sm, bx, by, bz, p.M, p.N, p.K, p.A, p.lda, p.B,     \
                                            p.ldb, p.C, p.ldc, p.kchunk, p.slab, kl)
    switch (p.code & 7) {
      case 7: PKC_GS(true, true, true); break;
      case 6: PKC_GS(true, true, false); break;
      case 5: PKC_GS(true, false, true); break;
      default: PKC_GS(true, false, false); break;
    }
#undef PKC_GS
    return;
  }
#define PKC_GB(AK, BK_, V)                                                                      \
  gemm_body<PREC, AK, BK_, V, GD, BIN>(sm, bx, by, bz, p.M, p.N, p.K, p.A, p.lda, p.B, p.ldb, p.C, \
                                      p.ldc, p.kchunk, p.slab)
  if constexpr (VO) {
    switch (p.code) {
      case 7: PKC_GB(true, true, true); break;
      case 5: PKC_GB(true, false, true); break;
      case 1: PKC_GB(false, false, true); break;
      default: PKC_GB(false, true, true); break;
    }
    return;
  }
  switch (p.code) {
    case 7: PKC_GB(true, true, true); break;
    case 6: PKC_GB(true, true, false); break;
    case 5: PKC_GB(true, false, true); break;
    case 4: PKC_GB(true, false, false); break;
    case 1: PKC_GB(false, false, true); break;
    case 0: PKC_GB(false, false, false); break;
    case 3: PKC_GB(false, true, true); break;
    default: PKC_GB(false, true, false); break;
  }
#undef PKC_GB
}

template <int PREC, bool BIN, bool BIG, bool SP = false, bool SUM = false, int GD = 4,
          bool VO = false>
__global__ __launch_bounds__(NT) void gemm_grouped_kernel(GroupArgs g) {
  grouped_body<PREC, BIN, BIG, SP, SUM, GD, VO>(g);
}

// The vec-only instance held to 4 waves per SIMD (128 registers): at 113 VGPRs + 16 AGPRs the
// bf16 form sits one register above that step (PKC_GROUPED_VO=2)
template <int PREC, bool BIN>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4, 4)))
void gemm_grouped_vo4_kernel(GroupArgs g) {
  grouped_body<PREC, BIN, false, false, false, 4, true>(g);
}

// k-tiles in flight per workgroup for bf16-stored operands: a stage is one 16-byte register per
// operand, so depth 8 costs 32 VGPRs more and puts a B = 128 split's whole k-range in flight at
// once.  Standalone launches (PKC_GEMM_DEPTH, default 8): C2 706k -> 720k, B = 1024 1.97M ->
// 2.06M frames/s; grouped launches (PKC_GEMM_DEPTH_G, default 4): 8 measured 664-669k, the
// extra VGPRs cost their optimizer / dW work items residency (same runs)
// Launches whose matmuls are all 16-byte: PKC_GROUPED_VO=2 (default) the vec-only instance held to
// 4 waves per SIMD, 1 the vec-only instance, 0 the general instance.  Same box, two rounds
// (profiles/r03_grouped_vo_ab.txt): C2 bf16 847-851k / 852-854k / 856-859k frames/s for 0 / 1 / 2,
// the fp32 entry 622k (0) -> 634k (2)
static int grouped_vo() {
  static const int m = [] {
    const char* v = getenv("PKC_GROUPED_VO");
    return v ? atoi(v) : 2;
  }();
  return m;
}

static int bin_depth(bool grouped = false) {
  static const int d[2] = {[] {
    const char* v = getenv("PKC_GEMM_DEPTH");
    return v && atoi(v) == 4 ? 4 : 8;
  }(), [] {
    const char* v = getenv("PKC_GEMM_DEPTH_G");
    return v && atoi(v) == 8 ? 8 : 4;
  }()};
  return d[grouped ? 1 : 0];
}

template <int PREC, bool AKC, bool BKC, bool VEC, bool BIN>
static int launch(int M, int N, int K, const void* A, int64_t lda, const void* B, int64_t ldb,
                  float* C, int64_t ldc, int splits, int64_t slab, hipStream_t s) {
  int kchunk = (K + splits - 1) / splits;
  kchunk = ((kchunk + BK - 1) / BK) * BK;
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, splits);
  if (BIN && bin_depth() == 8)
    hipLaunchKernelGGL((gemm_kernel<PREC, AKC, BKC, VEC, 8, BIN>), grid, dim3(NT), 0, s, M, N, K, A,
                       lda, B, ldb, C, ldc, kchunk, slab);
  else
    hipLaunchKernelGGL((gemm_kernel<PREC, AKC, BKC, VEC, 4, BIN>), grid, dim3(NT), 0, s, M, N, K, A,
                       lda, B, ldb, C, ldc, kchunk, slab);
  PKC_LAUNCH_CHECK("pkc_gemm");
  return PKC_OK;
}

static int xcd_remap() {                      // PKC_GEMM_XCD=0: launch order (A/B)
  static const int on = [] {
    const char* v = getenv("PKC_GEMM_XCD");
    return v ? atoi(v) : 1;
  }();
  return on;
}

// PKC_GEMM_COLSTATS64=0: column statistics in the 128x128 body only (A/B)
static bool colstats64_enabled() {
  static const int on = [] {
    const char* v = getenv("PKC_GEMM_COLSTATS64");
    return v ? atoi(v) : 1;
  }();
  return on != 0;
}

static bool glds_enabled() {                   // PKC_GEMM_GLDS=0: register-staged body (A/B)
  static const int on = [] {
    const char* v = getenv("PKC_GEMM_GLDS");
    return v ? atoi(v) : 1;
  }();
  return on != 0;
}

static int glds_bufs() {                      // PKC_GLDS_BUFS: LDS-DMA ring depth (3, 4, 5)
  static const int nb = [] {
    const char* v = getenv("PKC_GLDS_BUFS");
    const int n = v ? atoi(v) : 3;
    return n < 3 ? 3 : n > 5 ? 5 : n;
  }();
  return nb;
}

template <int PREC, bool BIN, bool STATS = false>
static int launch_big(int akc, int bkc, int M, int N, int K, const void* A, int64_t lda,
                      const void* B, int64_t ldb, float* C, int64_t ldc, int splits, int64_t slab,
                      hipStream_t s, const float* bias = nullptr, float* part = nullptr) {
  constexpr int BKB = big::Cfg<PREC, BIN>::BK;
  int kchunk = (K + splits - 1) / splits;
  kchunk = ((kchunk + BKB - 1) / BKB) * BKB;
  dim3 grid((N + big::TN - 1) / big::TN, (M + big::TM - 1) / big::TM, splits);
  // LDS-DMA ring (bf16 operands, whole k-tiles) when the grid is one workgroup per CU at most:
  // 4096x1024x1024 27.8 -> 21.8 us (forward) / 27.7 -> 20.3 (dX); with several tiles per CU its
  // 96 KB of LDS (one workgroup per CU) loses to the register body (4096x1928x1024 31.6 -> 35.3,
  // 8192^3 755 -> 656 TF/s), same run
  if (BIN && K % 64 == 0 && (int64_t)grid.x * grid.y * grid.z <= 256 && glds_enabled()) {
#define PKC_L(NB, AK, BK_)                                                                      \
  hipLaunchKernelGGL((gemm_glds_kernel<NB, AK, BK_, STATS>), grid, dim3(big::NT), 0, s, M, N, K, A, \
                     lda, B, ldb, C, ldc, kchunk, slab, xcd_remap(), bias, part)
#define PKC_LN(NB)                                                                              \
  if (akc && bkc) PKC_L(NB, true, true);                                                        \
  else if (akc) PKC_L(NB, true, false);                                                         \
  else if (bkc) PKC_L(NB, false, true);                                                         \
  else PKC_L(NB, false, false)
    const int nb = glds_bufs();
    if (nb == 5) { PKC_LN(5); }
    else if (nb == 4) { PKC_LN(4); }
    else { PKC_LN(3); }
#undef PKC_LN
#undef PKC_L
    PKC_LAUNCH_CHECK("pkc_gemm (128x128 LDS-DMA)");
    return PKC_OK;
  }
#define PKC_L(AK, BK_)                                                                          \
  hipLaunchKernelGGL((gemm_big_kernel<PREC, BIN, AK, BK_, STATS>), grid, dim3(big::NT), 0, s, M, N, \
                     K, A, lda, B, ldb, C, ldc, kchunk, slab, xcd_remap(), bias, part)
  if (akc && bkc) PKC_L(true, true);
  else if (akc) PKC_L(true, false);
  else if (bkc) PKC_L(false, true);
  else PKC_L(false, false);
#undef PKC_L
  PKC_LAUNCH_CHECK("pkc_gemm (128x128)");
  return PKC_OK;
}

template <int PREC, bool BIN>
static int dispatch(int akc, int bkc, bool vec, int M, int N, int K, const void* A, int64_t lda,
                    const void* B, int64_t ldb, float* C, int64_t ldc, int splits, int64_t slab,
                    hipStream_t s) {
#define PKC_G(AK, BK_, V) \
  return launch<PREC, AK, BK_, V, BIN>(M, N, K, A, lda, B, ldb, C, ldc, splits, slab, s)
  if (akc && bkc) { if (vec) PKC_G(true, true, true); PKC_G(true, true, false); }
  if (akc && !bkc) { if (vec) PKC_G(true, false, true); PKC_G(true, false, false); }
  if (!akc && !bkc) { if (vec) PKC_G(false, false, true); PKC_G(false, false, false); }
  if (vec) PKC_G(false, true, true);
  PKC_G(false, true, false);
#undef PKC_G
}

// The 128x128 body takes a matmul with at least this many output tiles (alone: enough to fill the
// chip; in a grouped launch the other problems fill it).  In a grouped launch it also needs a long
// contraction: its 64 KB of LDS cuts the residency of every other workgroup of the launch, which
// the B = 128 step's short dW (K = 128) launches cannot afford (681k -> 627k frames/s when they
// took it).  PKC_GEMM_BIG=0 disables it (A/B runs).
constexpr int BIG_MIN_TILES = 160, BIG_MIN_TILES_GROUPED = 32, BIG_MIN_K_GROUPED = 1024;
static bool big_enabled() {
  static const int on = [] {
    const char* v = getenv("PKC_GEMM_BIG");
    return v ? atoi(v) : 1;
  }();
  return on != 0;
}
// compensated-bf16 problems of grouped launches on the 128x128 body (PKC_X3_GROUPED_BIG=0: the
// 64x64 body, whose grouped instances keep several workgroups per CU)
static bool x3_grouped_big() {
  static const int on = [] {
    const char* v = getenv("PKC_X3_GROUPED_BIG");
    return v ? atoi(v) : 1;
  }();
  return on != 0;
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
                        const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                        int64_t ldc, int splits, int64_t slab_stride, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "pkc_gemm: negative shape");
  PKC_CHECK_ARG(prec == PKC_PREC_FP32 || prec == PKC_PREC_BF16 || prec == PKC_PREC_BF16IN ||
                    prec == PKC_PREC_BF16X3,
                "pkc_gemm: bad precision %d", prec);
  if (M == 0 || N == 0) return PKC_OK;
  PKC_CHECK_ARG(A && B && C, "pkc_gemm: null operand");
  PKC_CHECK_ARG(lda > 0 && ldb > 0 && lda < (1ll << 31) && ldb < (1ll << 31),
                "pkc_gemm: leading dimensions must be in [1, 2^31)");
  PKC_CHECK_ARG(ldc >= N && ldc < (1ll << 26), "pkc_gemm: ldc must be in [N, 2^26)");
  if (splits <= 0) splits = pkc_gemm_pick_splits(M, N, K);
  PKC_CHECK_ARG(splits == 1 || slab_stride >= (int64_t)M * ldc, "pkc_gemm: slab_stride too small");
  // 16-byte path: aligned bases, leading dims and contiguous extents multiple of 16 bytes
  const int e = prec == PKC_PREC_BF16IN ? 8 : 4;
  const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % e == 0 &&
                   ldb % e == 0 && (a_kcontig ? K % e == 0 : M % e == 0) &&
                   (b_kcontig ? K % e == 0 : N % e == 0);
  if (big_enabled() && big::eligible(prec, a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, BIG_MIN_TILES)) {
    if (prec == PKC_PREC_FP32)
      return launch_big<PKC_PREC_FP32, false>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C, ldc,
                                              splits, slab_stride, S(stream));
    if (prec == PKC_PREC_BF16IN)
      return launch_big<PKC_PREC_BF16, true>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C, ldc,
                                             splits, slab_stride, S(stream));
    if (prec == PKC_PREC_BF16X3)
      return launch_big<PKC_PREC_BF16X3, false>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C,
                                                ldc, splits, slab_stride, S(stream));
    return launch_big<PKC_PREC_BF16, false>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C, ldc,
                                            splits, slab_stride, S(stream));
  }
  if (prec == PKC_PREC_FP32)
    return dispatch<PKC_PREC_FP32, false>(a_kcontig, b_kcontig, vec, M, N, K, A, lda, B, ldb, C,
                                          ldc, splits, slab_stride, S(stream));
  if (prec == PKC_PREC_BF16X3)
    return dispatch<PKC_PREC_BF16X3, false>(a_kcontig, b_kcontig, vec, M, N, K, A, lda, B, ldb, C,
                                            ldc, splits, slab_stride, S(stream));
  if (prec == PKC_PREC_BF16IN)
    return dispatch<PKC_PREC_BF16, true>(a_kcontig, b_kcontig, vec, M, N, K, A, lda, B, ldb, C,
                                         ldc, splits, slab_stride, S(stream));
  return dispatch<PKC_PREC_BF16, false>(a_kcontig, b_kcontig, vec, M, N, K, A, lda, B, ldb, C, ldc,
                                        splits, slab_stride, S(stream));
}

// 128 when a grouped dX problem of this shape takes the 128x128 body (the BatchNorm-backward
// epilogue's precondition, pkc_bn_bwd_epi), else 0
extern "C" int pkc_gemm_bnbwd_ok(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                                 const void* A, int64_t lda, const void* B, int64_t ldb) {
  using namespace pkc;
  if (!(prec == PKC_PREC_FP32 || prec == PKC_PREC_BF16 || prec == PKC_PREC_BF16IN) || M <= 0 ||
      N <= 0 || K <= 0 || lda <= 0 || ldb <= 0 || lda >= (1ll << 31) || ldb >= (1ll << 31) ||
      !a_kcontig || b_kcontig)
    return 0;
  return big_enabled() && big::eligible(prec, a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb,
                                        BIG_MIN_TILES_GROUPED, BIG_MIN_K_GROUPED) ? 128 : 0;
}

// Tile edge a GEMM problem of pkc_gemm_grouped runs on: 128 (the 128x128 body) or 64
extern "C" int pkc_gemm_grouped_tile(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                                     const void* A, int64_t lda, const void* B, int64_t ldb) {
  using namespace pkc;
  if (M <= 0 || N <= 0 || K <= 0 || lda <= 0 || ldb <= 0) return 64;
  return big_enabled() && (prec != PKC_PREC_BF16X3 || x3_grouped_big()) &&
                 big::eligible(prec, a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb,
                               BIG_MIN_TILES_GROUPED, BIG_MIN_K_GROUPED) ? 128 : 64;
}

// rows per partial block pkc_gemm_colstats writes for this shape: 128 (the 128x128 tile body),
// 64 (the 64x64 body, 16-byte operand paths), 0 (not taken)
extern "C" int pkc_gemm_colstats_ok(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                                    const void* A, int64_t lda, const void* B, int64_t ldb) {
  using namespace pkc;
  if (!(prec == PKC_PREC_FP32 || prec == PKC_PREC_BF16 || prec == PKC_PREC_BF16IN ||
        prec == PKC_PREC_BF16X3) || M <= 0 ||
      N <= 0 || K <= 0 || lda <= 0 || ldb <= 0 || lda >= (1ll << 31) || ldb >= (1ll << 31))
    return 0;
  if (big_enabled() &&
      big::eligible(prec, a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, BIG_MIN_TILES))
    return 128;
  const int e = prec == PKC_PREC_BF16IN ? 8 : 4;
  const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % e == 0 &&
                   ldb % e == 0 && (a_kcontig ? K % e == 0 : M % e == 0) &&
                   (b_kcontig ? K % e == 0 : N % e == 0);
  return vec && colstats64_enabled() ? 64 : 0;
}

extern "C" int pkc_gemm_colstats(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                                 const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                                 int64_t ldc, const float* bias, float* part, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(A && B && C && part && ldc >= N, "pkc_gemm_colstats: bad arguments");
  const int rows = pkc_gemm_colstats_ok(prec, a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb);
  PKC_CHECK_ARG(rows > 0, "pkc_gemm_colstats: %dx%dx%d (prec %d): no column-statistics body", M, N,
                K, prec);
  PKC_CHECK_ARG(ldc < (1ll << 26), "pkc_gemm_colstats: ldc must be below 2^26");
  if (rows == 64) {
    dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, 1);
#define PKC_CS(P, BIN, AK, BK_)                                                                  \
  hipLaunchKernelGGL((gemm_stats_kernel<P, AK, BK_, BIN ? 8 : 4, BIN>), grid, dim3(NT), 0, S(stream), \
                     M, N, K, A, lda, B, ldb, C, ldc, bias, part)
#define PKC_CSO(P, BIN)                                                                          \
  do {                                                                                         \
    if (a_kcontig && b_kcontig) PKC_CS(P, BIN, true, true);                                    \
    else if (a_kcontig) PKC_CS(P, BIN, true, false);                                           \
    else if (b_kcontig) PKC_CS(P, BIN, false, true);                                           \
    else PKC_CS(P, BIN, false, false);                                                         \
  } while (0)
    if (prec == PKC_PREC_FP32) PKC_CSO(PKC_PREC_FP32, false);
    else if (prec == PKC_PREC_BF16X3) PKC_CSO(PKC_PREC_BF16X3, false);
    else if (prec == PKC_PREC_BF16IN) PKC_CSO(PKC_PREC_BF16, true);
    else PKC_CSO(PKC_PREC_BF16, false);
#undef PKC_CSO
#undef PKC_CS
    PKC_LAUNCH_CHECK("pkc_gemm_colstats (64x64)");
    return PKC_OK;
  }
  if (prec == PKC_PREC_FP32)
    return launch_big<PKC_PREC_FP32, false, true>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C,
                                                  ldc, 1, 0, S(stream), bias, part);
  if (prec == PKC_PREC_BF16IN)
    return launch_big<PKC_PREC_BF16, true, true>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C,
                                                 ldc, 1, 0, S(stream), bias, part);
  if (prec == PKC_PREC_BF16X3)
    return launch_big<PKC_PREC_BF16X3, false, true>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb,
                                                    C, ldc, 1, 0, S(stream), bias, part);
  return launch_big<PKC_PREC_BF16, false, true>(a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C,
                                                ldc, 1, 0, S(stream), bias, part);
}

extern "C" int pkc_gemm_grouped(int prec, const pkc_gemm_problem* probs, int n, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(probs && n >= 1 && n <= GMAX, "pkc_gemm_grouped: 1..%d problems", GMAX);
  PKC_CHECK_ARG(prec == PKC_PREC_FP32 || prec == PKC_PREC_BF16 || prec == PKC_PREC_BF16IN ||
                    prec == PKC_PREC_BF16X3,
                "pkc_gemm_grouped: bad precision %d", prec);
  GroupArgs g;
  memset(&g, 0, sizeof(g));
  int wg = 0, k = 0, nseg = 0, nbnb = 0;
  bool any_big = false, any_sparse = false, any_sum = false, all_vec = true;
  const int e = prec == PKC_PREC_BF16IN ? 8 : 4;
  // a launch with block-sparse problems runs the sparse instance, which has no 128x128 body
  for (int i = 0; i < n; ++i) any_sparse |= probs[i].kind == PKC_OP_GEMM && probs[i].ktiles != nullptr;
  for (int i = 0; i < n; ++i) {
    const pkc_gemm_problem& q = probs[i];
    if (q.kind == PKC_OP_OPTIM) {
      const pkc_opt_seg* sg = reinterpret_cast<const pkc_opt_seg*>(q.X1);
      const bool direct = sg && q.N >= 1 && nseg + q.N <= PKC_OPT_SEGS_MAX;
      PKC_CHECK_ARG(q.M > 0 && q.A && (q.B || direct), "pkc_gemm_grouped: optimizer op %d arguments",
                    i);
      GroupProb& p = g.p[k++];
      memset(&p, 0, sizeof(p));
      p.kind = q.kind;
      p.A = q.A; p.B = q.B;
      p.wg0 = wg;
      if (direct) {
        int c = 0;
        for (int j = 0; j < q.N; ++j) {
          PKC_CHECK_ARG(sg[j].nchunks > 0 && sg[j].chunk0 >= 0 && sg[j].tensor >= 0 && sg[j].p &&
                            sg[j].g && sg[j].n > (int64_t)(sg[j].chunk0 + sg[j].nchunks - 1) * OPT_CHUNK,
                        "pkc_gemm_grouped: optimizer op %d segment %d", i, j);
          OptSegK& d = g.seg[nseg + j];
          d.p = sg[j].p; d.g = sg[j].g; d.s1 = sg[j].s1; d.s2 = sg[j].s2; d.s3 = sg[j].s3;
          d.mask = sg[j].mask; d.qout = sg[j].qout; d.bout = sg[j].bout; d.n = sg[j].n;
          d.tensor = sg[j].tensor; d.chunk0 = sg[j].chunk0; d.begin = c;
          c += sg[j].nchunks;
          d.end = c;
        }
        PKC_CHECK_ARG(c == q.M, "pkc_gemm_grouped: optimizer op %d: segments hold %d chunks, M = %d",
                      i, c, q.M);
        p.code = 1; p.K = nseg; p.N = q.N;
        nseg += q.N;
      }
      wg += q.M;
      continue;
    }
    if (q.kind == PKC_OP_SLABSUM) {
      PKC_CHECK_ARG(q.M >= 1 && q.N >= 0 && q.A && q.C && (q.M == 1 || q.slab_stride >= q.N),
                    "pkc_gemm_grouped: slab-sum op %d arguments", i);
      if (q.N == 0) continue;
      GroupProb& p = g.p[k++];
      memset(&p, 0, sizeof(p));
      p.kind = q.kind;
      p.M = q.M; p.N = q.N; p.A = q.A; p.C = q.C; p.slab = q.slab_stride;
      p.code = ((uintptr_t)q.A % 16 == 0 && (uintptr_t)q.C % 16 == 0 && q.slab_stride % 4 == 0 &&
                q.N % 4 == 0) ? 1 : 0;
      p.wg0 = wg;
      wg += (q.N + 1023) / 1024;
      any_sum = true;
      continue;
    }
    if (q.kind == PKC_OP_GATHER) {
      PKC_CHECK_ARG(q.M > 0 && q.N > 0 && q.A && q.B && q.C && q.X1 && q.X2 && q.slab_stride > 0 &&
                        q.ldb >= 0 && q.ldb <= 256 && q.lda >= q.N,
                    "pkc_gemm_grouped: gather op %d arguments", i);
      GroupProb& p = g.p[k++];
      memset(&p, 0, sizeof(p));
      p.kind = q.kind;
      p.M = q.M; p.N = q.N; p.A = q.A; p.lda = q.lda; p.B = q.B; p.ldb = q.ldb; p.C = q.C;
      p.slab = q.slab_stride; p.X1 = q.X1; p.X2 = q.X2; p.X3 = q.X3;
      p.code = (q.N % 4 == 0 && q.lda % 4 == 0 && (uintptr_t)q.A % 16 == 0 &&
                (uintptr_t)q.C % 16 == 0 && (uintptr_t)q.X3 % 8 == 0) ? 1 : 0;
      p.wg0 = wg;
      wg += q.M;
      continue;
    }
    if (q.kind == PKC_OP_COLSUM || q.kind == PKC_OP_LOSS) {
      PKC_CHECK_ARG(q.M > 0 && q.N > 0 && q.A && q.C, "pkc_gemm_grouped: op %d arguments", i);
      PKC_CHECK_ARG(q.kind != PKC_OP_LOSS || (q.M <= 8 && q.B && q.X1),
                    "pkc_gemm_grouped: loss op %d arguments", i);
      GroupProb& p = g.p[k++];
      memset(&p, 0, sizeof(p));
      p.kind = q.kind;
      p.M = q.M; p.N = q.N; p.A = q.A; p.B = q.B; p.C = q.C; p.X1 = q.X1; p.X2 = q.X2; p.X3 = q.X3;
      p.wg0 = wg;
      wg += q.kind == PKC_OP_COLSUM ? (q.N + 63) / 64 : 1;
      continue;
    }
    PKC_CHECK_ARG(q.kind == PKC_OP_GEMM, "pkc_gemm_grouped: problem %d kind %d", i, q.kind);
    PKC_CHECK_ARG(q.M >= 0 && q.N >= 0 && q.K >= 0 && q.ldc >= q.N && q.ldc < (1ll << 26),
                  "pkc_gemm_grouped: problem %d shape", i);
    if (q.M == 0 || q.N == 0) continue;
    PKC_CHECK_ARG(q.A && q.B && q.C, "pkc_gemm_grouped: problem %d null operand", i);
    PKC_CHECK_ARG(q.lda > 0 && q.ldb > 0 && q.lda < (1ll << 31) && q.ldb < (1ll << 31),
                  "pkc_gemm_grouped: problem %d leading dimensions must be in [1, 2^31)", i);
    int splits = q.splits <= 0 ? pkc_gemm_pick_splits(q.M, q.N, q.K) : q.splits;
    PKC_CHECK_ARG(!q.ktiles || (splits == 1 && q.kmax >= 0 && q.a_kcontig),
                  "pkc_gemm_grouped: problem %d: k-tile lists need splits == 1 and a k-contiguous A",
                  i);
    PKC_CHECK_ARG(splits == 1 || q.slab_stride >= (int64_t)q.M * q.ldc,
                  "pkc_gemm_grouped: problem %d slab_stride too small", i);
    const bool vec = ((uintptr_t)q.A % 16 == 0) && ((uintptr_t)q.B % 16 == 0) && q.lda % e == 0 &&
                     q.ldb % e == 0 && (q.a_kcontig ? q.K % e == 0 : q.M % e == 0) &&
                     (q.b_kcontig ? q.K % e == 0 : q.N % e == 0);
    const bool bigp = !any_sparse && big_enabled() && (prec != PKC_PREC_BF16X3 || x3_grouped_big()) &&
                      big::eligible(prec, q.a_kcontig, q.b_kcontig, q.M, q.N, q.K,
                                                     q.A, q.lda, q.B, q.ldb, BIG_MIN_TILES_GROUPED,
                                                     BIG_MIN_K_GROUPED);
    any_big |= bigp;
    all_vec &= vec;
    const int bk = bigp ? (prec == PKC_PREC_FP32 ? 32 : 64) : BK;
    int kchunk = (q.K + splits - 1) / splits;
    kchunk = ((kchunk + bk - 1) / bk) * bk;
    const int tm = bigp ? big::TM : BM, tnn = bigp ? big::TN : BN;
    GroupProb& p = g.p[k++];
    p.kind = PKC_OP_GEMM;
    p.bnb = -1;
    if (q.X1) {            // pkc_bn_bwd_epi (host): the BatchNorm-backward epilogue
      const pkc_bn_bwd_epi* e = reinterpret_cast<const pkc_bn_bwd_epi*>(q.X1);
      PKC_CHECK_ARG(bigp && splits == 1 && q.a_kcontig && !q.b_kcontig && q.ldc == q.N && nbnb < GBNB &&
                        e->xhat && e->gamma && e->beta && e->part && (e->drop_p == 0.f || e->keep),
                    "pkc_gemm_grouped: problem %d: the BatchNorm-backward epilogue needs a one-slab dX "
                    "problem on the 128x128 body with ldc = N (pkc_gemm_bnbwd_ok), at most %d per "
                    "launch, and xhat / gamma / beta / part (+ keep with dropout)", i, GBNB);
      big::BnEpi& d = g.bnb[nbnb];
      d.xhat = e->xhat; d.keep = e->keep; d.gamma = e->gamma; d.beta = e->beta; d.part = e->part;
      d.act = e->act; d.drop_p = e->drop_p;
      p.bnb = nbnb++;
    }
    p.code = (q.a_kcontig ? 4 : 0) + (q.b_kcontig ? 2 : 0) + (vec ? 1 : 0) + (bigp ? 8 : 0);
    p.M = q.M; p.N = q.N; p.K = q.K; p.kchunk = kchunk;
    p.tn = (q.N + tnn - 1) / tnn;
    p.tmn = p.tn * ((q.M + tm - 1) / tm);
    p.wg0 = wg;
    p.A = q.A; p.lda = q.lda; p.B = q.B; p.ldb = q.ldb; p.C = q.C; p.ldc = q.ldc; p.slab = q.slab_stride;
    p.ktiles = q.ktiles; p.kmax = q.kmax;
    wg += p.tmn * splits;
  }
  g.n = k;
  if (k == 0) return PKC_OK;
  // separate instances for launches with 128x128 problems (64 KB of LDS) and with block-sparse
  // k-tile lists, so the plain launches of the B = 128 step keep their lean code and residency
#define PKC_GL(P, BIN)                                                                          \
  do {                                                                                          \
    if (any_sparse && any_sum)                                                                  \
      hipLaunchKernelGGL((gemm_grouped_kernel<P, BIN, false, true, true>), dim3(wg), dim3(NT), 0, \
                         S(stream), g);                                                         \
    else if (any_sparse)                                                                        \
      hipLaunchKernelGGL((gemm_grouped_kernel<P, BIN, false, true>), dim3(wg), dim3(NT), 0,      \
                         S(stream), g);                                                         \
    else if (any_sum)                                                                           \
      hipLaunchKernelGGL((gemm_grouped_kernel<P, BIN, true, false, true>), dim3(wg), dim3(NT), 0,  \
                         S(stream), g);                                                         \
    else if (any_big)                                                                           \
      hipLaunchKernelGGL((gemm_grouped_kernel<P, BIN, true>), dim3(wg), dim3(NT), 0, S(stream), g);  \
    else if (BIN && bin_depth(true) == 8)                                                       \
      hipLaunchKernelGGL((gemm_grouped_kernel<P, BIN, false, false, false, 8>), dim3(wg), dim3(NT), \
                         0, S(stream), g);                                                      \
    else if (all_vec && grouped_vo() == 2)                                                      \
      hipLaunchKernelGGL((gemm_grouped_vo4_kernel<P, BIN>), dim3(wg), dim3(NT), 0, S(stream), g); \
    else if (all_vec && grouped_vo() == 1)                                                      \
      hipLaunchKernelGGL((gemm_grouped_kernel<P, BIN, false, false, false, 4, true>), dim3(wg),  \
                         dim3(NT), 0, S(stream), g);                                            \
    else                                                                                        \
      hipLaunchKernelGGL((gemm_grouped_kernel<P, BIN, false>), dim3(wg), dim3(NT), 0, S(stream), g); \
  } while (0)
  if (prec == PKC_PREC_FP32) PKC_GL(PKC_PREC_FP32, false);
  else if (prec == PKC_PREC_BF16IN) PKC_GL(PKC_PREC_BF16, true);
  else if (prec == PKC_PREC_BF16X3) {
    // the 128x128 instances (128 KB of LDS for the head and tail images) only where a problem
    // takes that body; its slab sums ride the 64x64 instance otherwise
    constexpr int P = PKC_PREC_BF16X3;
    if (any_sparse && any_sum)
      hipLaunchKernelGGL((gemm_grouped_kernel<P, false, false, true, true>), dim3(wg), dim3(NT), 0,
                         S(stream), g);
    else if (any_sparse)
      hipLaunchKernelGGL((gemm_grouped_kernel<P, false, false, true>), dim3(wg), dim3(NT), 0,
                         S(stream), g);
    else if (any_big && any_sum)
      hipLaunchKernelGGL((gemm_grouped_kernel<P, false, true, false, true>), dim3(wg), dim3(NT), 0,
                         S(stream), g);
    else if (any_big)
      hipLaunchKernelGGL((gemm_grouped_kernel<P, false, true>), dim3(wg), dim3(NT), 0, S(stream), g);
    else if (any_sum)
      hipLaunchKernelGGL((gemm_grouped_kernel<P, false, false, false, true>), dim3(wg), dim3(NT), 0,
                         S(stream), g);
    else if (all_vec && grouped_vo() == 2)
      hipLaunchKernelGGL((gemm_grouped_vo4_kernel<P, false>), dim3(wg), dim3(NT), 0, S(stream), g);
    else
      hipLaunchKernelGGL((gemm_grouped_kernel<P, false, false>), dim3(wg), dim3(NT), 0, S(stream), g);
  } else PKC_GL(PKC_PREC_BF16, false);
#undef PKC_GL
  PKC_LAUNCH_CHECK("pkc_gemm_grouped");
  return PKC_OK;
}

namespace pkc {
__global__ void cast_bf16_kernel(const float* src, __bf16* dst, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (__bf16)src[i];
}
}  // namespace pkc

extern "C" int pkc_cast_bf16(const float* src, void* dst, int64_t n, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(src && dst && n >= 0, "pkc_cast_bf16: bad arguments");
  if (n == 0) return PKC_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cast_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, S(stream), src,
                     reinterpret_cast<__bf16*>(dst), n);
  PKC_LAUNCH_CHECK("pkc_cast_bf16");
  return PKC_OK;
}
