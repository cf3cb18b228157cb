// pkc_gemm_big.h — 128x128 MFMA tile body for the large-M matmuls (gfx950 / CDNA4).
//
// The 64x64 tile of pkc_gemm.hip is sized for the M = 128-row frame batches of the MLP step,
// where every matmul is short and latency-bound.  The sequence models' input projections
// (M = T*B = 2-16 k rows: neural_networks.py:951-954, 1554-1555), their backward, and the MLP at
// large batches are long contractions: there the 64x64 tile's 2 MFMAs per wave per barrier and
// 16 flop per staged byte leave the matrix pipe idle.  This body:
//   * 128x128 output tile per 256-thread workgroup, 4 waves in 2x2, each wave 64x64 = 2x2 blocks
//     of 32x32 accumulators (64 accumulator registers);
//   * one LDS row = 128 bytes of k: BK = 64 for bf16 operands (v_mfma_f32_32x32x16_bf16, 16 MFMA
//     per wave per k-tile), BK = 32 for exact fp32 (v_mfma_f32_32x32x2_f32, 64 MFMA per wave per
//     k-tile, the parity mode);
//   * double-buffered LDS (2 x 32 KB) with ONE barrier per k-tile: tile t+1 is written to the
//     other buffer after the MFMAs of tile t, from registers loaded one (16-byte staging: two)
//     k-tiles earlier;
//   * LDS image [row][128 B] with 16-byte chunk c of row r stored at c ^ ((r>>1 ^ r>>4) & 7): the
//     ds_read_b128 fragment reads of any 16 rows of a 32-row block hit 16 distinct bank groups
//     (conflict-free), for both operand orientations;
//   * k-contiguous operands are staged with 16-byte loads and stores; m-contiguous ones (the
//     transposed operands of dX / dW) with 16-byte loads along m and a transposing store (bf16:
//     two k-adjacent chunks packed into dwords).
// Split-K (blockIdx.z-style slice index) writes deterministic partial slabs like pkc_gemm.
#pragma once
#include "pkc_common.h"

namespace pkc {
namespace big {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int TM = 128, TN = 128, NT = 256;
constexpr int ROWB = 128;                       // bytes of k per LDS row
constexpr int TILE_BYTES = TM * ROWB;           // one operand tile in LDS (16 KB)
constexpr int LDS_BYTES = 2 * 2 * TILE_BYTES;   // A and B, double-buffered (64 KB)
// PKC_PREC_BF16X3 (compensated bf16) stages every fp32 operand tile as TWO bf16 images, the head
// hi = bf16(v) and the tail lo = bf16(v - hi): a buffer is [A hi][B hi][A lo][B lo] (64 KB), two
// buffers 128 KB (one workgroup per CU)
template <int PREC>
constexpr int buf_bytes() { return (PREC == PKC_PREC_BF16X3 ? 4 : 2) * TILE_BYTES; }
template <int PREC>
constexpr int lds_bytes() { return 2 * buf_bytes<PREC>(); }
constexpr int LO_OFF = 2 * TILE_BYTES;          // the tail image of an operand, after both heads

__device__ __forceinline__ int swz(int r) { return ((r >> 1) ^ (r >> 4)) & 7; }

// [k][row] image of a bf16 m-contiguous operand tile: 64 k-rows of 128 elements (256 B), 16-byte
// chunk c of k-row k at chunk c ^ xr(k).  The transposed fragment read (tr_frag) of one 32-lane
// half touches 4 consecutive k-rows x 4 consecutive chunks (c0 % 4 == 0): the XOR puts them on 16
// distinct chunks = all 64 banks (conflict-free); the 16-byte staging stores fill whole k-rows.
__device__ __forceinline__ int xr(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
__device__ __forceinline__ int tr_off(int k, int c) { return 256 * k + 16 * (c ^ xr(k)); }

typedef short v4s __attribute__((ext_vector_type(4)));

// 32x32x16 bf16 operand fragment (lane l: row rb + (l & 31), k = kb + 8 (l >> 5) + j, j = 0..7) from
// a [k][row] image: two ds_read_b64_tr_b16, each giving a lane 4 consecutive k of its row.  Lane
// 4q + p of a 16-lane group addresses k-row (k0 + q), rows 4p .. 4p + 3 of the group's 16.
__device__ __forceinline__ bf16x8 tr_frag(const char* __restrict__ s, int rb, int kb, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int row = rb + 16 * ((lane >> 4) & 1) + 4 * p;
  const int k0 = kb + 8 * (lane >> 5) + q;
  typedef __attribute__((address_space(3))) v4s lv4s;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lv4s*)(s + tr_off(k0, row >> 3) + 8 * (p & 1)));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lv4s*)(s + tr_off(k0 + 4, row >> 3) + 8 * (p & 1)));
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s w = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, w);
}

// Element type in HBM (HE) and in LDS (LE); BK = k per LDS row.
template <int PREC, bool BIN>
struct Cfg {
  using HE = float;
  using LE = float;
  static constexpr int BK = 32;
};
template <>
struct Cfg<PKC_PREC_BF16, false> {
  using HE = float;
  using LE = __bf16;
  static constexpr int BK = 64;
};
template <>
struct Cfg<PKC_PREC_BF16X3, false> {
  using HE = float;
  using LE = __bf16;
  static constexpr int BK = 64;
};
template <>
struct Cfg<PKC_PREC_BF16, true> {
  using HE = __bf16;
  using LE = __bf16;
  static constexpr int BK = 64;
};

// One operand tile (128 rows x BK) staged through registers.  HBM chunks are 16 bytes:
// EPC elements.  KC: row-major [row][k] in HBM; otherwise [k][row].
template <int PREC, bool BIN, bool KC>
struct Stage {
  using C = Cfg<PREC, BIN>;
  using HE = typename C::HE;
  using LE = typename C::LE;
  static constexpr int BK = C::BK;
  static constexpr int EPC = 16 / sizeof(HE);                  // elements per 16-byte chunk
  static constexpr int NCH = TM * BK / EPC / NT;               // chunks per thread (4 or 8)
  // bf16 m-contiguous operands stored as bf16 (BIN): staged as they lie, a [k][row] image read
  // back with the transposing ds_read_b64_tr_b16 (tr_frag); fp32 ones converted to bf16 on the way
  // (PAIR): two k-adjacent chunks packed into dwords and stored transposed
  static constexpr bool TR = !KC && sizeof(HE) == 2 && sizeof(LE) == 2;
  static constexpr bool PAIR = !KC && sizeof(LE) == 2 && !TR;
  static constexpr bool X3 = PREC == PKC_PREC_BF16X3;   // also the tail image at + LO_OFF
  float4 v[NCH];

  // chunk i of this thread -> (row, k) of its first element
  __device__ __forceinline__ void coord(int i, int& r, int& k) const {
    const int t = threadIdx.x;
    if (KC) {
      constexpr int CPR = BK / EPC;                            // chunks per row
      const int idx = t + NT * i;
      r = idx / CPR;
      k = (idx % CPR) * EPC;
    } else if (PAIR) {
      // chunk pairs (k, k+1) of the same rows: i even/odd = k even/odd
      constexpr int CPK = TM / EPC;                            // chunks per k
      const int idx = t + NT * (i >> 1);
      r = (idx % CPK) * EPC;
      k = (idx / CPK) * 2 + (i & 1);
    } else {
      constexpr int CPK = TM / EPC;
      const int idx = t + NT * i;
      r = (idx % CPK) * EPC;
      k = idx / CPK;
    }
  }

  // Clamped (always valid) addresses, out-of-range elements zeroed by selects afterwards: a load
  // under a runtime branch makes hipcc drain vmcnt around it (pkc_gemm.hip Stage).
  __device__ __forceinline__ void load(const HE* __restrict__ P, int64_t ld, int r0, int rmax,
                                       int k0, int kend) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int r, k;
      coord(i, r, k);
      const bool ok = (r0 + r < rmax) && (k0 + k < kend);
      const int rr = min(r0 + r, rmax - (KC ? 1 : EPC));
      const int kk = min(k0 + k, kend - (KC ? EPC : 1));
      const float4 x = KC ? *reinterpret_cast<const float4*>(P + (int64_t)rr * ld + kk)
                          : *reinterpret_cast<const float4*>(P + (int64_t)kk * ld + rr);
      v[i] = ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  // The row part of each chunk's address, computed once per tile loop (load_at adds the k-tile's
  // offset): recomputing the clamps and 64-bit row products for every chunk of every k-tile put
  // the staging instructions on par with the tile's MFMAs (cf. GldsOperand).
  struct Base {
    const HE* p[NCH];
    bool ok[NCH];
  };
  __device__ __forceinline__ static Base base(const HE* __restrict__ P, int64_t ld, int r0,
                                              int rmax) {
    Base b;
    Stage tmp;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int r, k;
      tmp.coord(i, r, k);
      const int rr = min(r0 + r, rmax - (KC ? 1 : EPC));
      b.p[i] = KC ? P + (int64_t)rr * ld : P + rr;
      b.ok[i] = r0 + r < rmax;
    }
    return b;
  }
  __device__ __forceinline__ void load_at(const Base& b, int ld, int k0, int kend) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int r, k;
      coord(i, r, k);
      const bool ok = b.ok[i] && (k0 + k < kend);
      const int kk = min(k0 + k, kend - (KC ? EPC : 1));
      const float4 x = KC ? *reinterpret_cast<const float4*>(b.p[i] + kk)
                          : *reinterpret_cast<const float4*>(b.p[i] + (int64_t)kk * ld);
      v[i] = ok ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  // Element access by value only: taking the address of v[] makes the compiler promote the
  // staging array into extra LDS (16 KB per workgroup), with a round trip per element.
  __device__ __forceinline__ static uint32_t word(const float4& x, int w) {
    return __float_as_uint(w == 0 ? x.x : w == 1 ? x.y : w == 2 ? x.z : x.w);
  }
  __device__ __forceinline__ static float fl(const float4& x, int w) {
    return w == 0 ? x.x : w == 1 ? x.y : w == 2 ? x.z : x.w;
  }
  __device__ __forceinline__ static uint32_t bf16bits(float f) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)f);
  }
  // the tail of the compensated split: v - hi is exact in fp32, rounded once to bf16
  __device__ __forceinline__ static uint32_t lobits(float f) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)(f - (float)(__bf16)f));
  }

  __device__ __forceinline__ void store(char* __restrict__ s) const {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      int r, k;
      coord(i, r, k);
      if (KC) {
        const int kb = k * (int)sizeof(LE);                    // byte offset of k in the row
        char* dst = s + r * ROWB + 16 * ((kb >> 4) ^ swz(r)) + (kb & 15);
        if constexpr (sizeof(HE) == sizeof(LE)) {
          *reinterpret_cast<float4*>(dst) = v[i];
        } else {                                               // fp32 -> bf16: 8 bytes
          uint2 h;
          h.x = bf16bits(v[i].x) | (bf16bits(v[i].y) << 16);
          h.y = bf16bits(v[i].z) | (bf16bits(v[i].w) << 16);
          *reinterpret_cast<uint2*>(dst) = h;
          if constexpr (X3) {
            uint2 l;
            l.x = lobits(v[i].x) | (lobits(v[i].y) << 16);
            l.y = lobits(v[i].z) | (lobits(v[i].w) << 16);
            *reinterpret_cast<uint2*>(dst + LO_OFF) = l;
          }
        }
      } else if (TR) {
        *reinterpret_cast<float4*>(s + tr_off(k, r >> 3)) = v[i];
      } else if (PAIR) {
        if (i & 1) continue;                                   // handled with its even partner
        const int kb = k * 2;
        const int co = kb & 15;                                // dword-aligned: k even
#pragma unroll
        for (int j = 0; j < EPC; ++j) {
          uint32_t p;
          if constexpr (sizeof(HE) == 2) {                     // bf16 element j of each chunk
            const uint32_t a = word(v[i], j >> 1), b = word(v[i + 1], j >> 1);
            p = (j & 1) ? ((a >> 16) | (b & 0xFFFF0000u)) : ((a & 0xFFFFu) | (b << 16));
          } else {
            p = bf16bits(fl(v[i], j)) | (bf16bits(fl(v[i + 1], j)) << 16);
          }
          const int rj = r + j;
          char* dst = s + rj * ROWB + 16 * ((kb >> 4) ^ swz(rj)) + co;
          *reinterpret_cast<uint32_t*>(dst) = p;
          if constexpr (X3)
            *reinterpret_cast<uint32_t*>(dst + LO_OFF) =
                lobits(fl(v[i], j)) | (lobits(fl(v[i + 1], j)) << 16);
        }
      } else {                                                 // fp32 m-contiguous
        const int kb = k * 4;
#pragma unroll
        for (int j = 0; j < EPC; ++j) {
          const int rj = r + j;
          *reinterpret_cast<float*>(s + rj * ROWB + 16 * ((kb >> 4) ^ swz(rj)) + (kb & 15)) =
              fl(v[i], j);
        }
      }
    }
  }
};

__device__ __forceinline__ float4 lds16(const char* s, int r, int c) {
  return *reinterpret_cast<const float4*>(s + r * ROWB + 16 * (c ^ swz(r)));
}

// MFMAs of one k-tile for this wave's 64x64 sub-tile (rows wm*64 + 32a, cols wn*64 + 32b).
template <int PREC, bool ATR = false, bool BTR = false>
__device__ __forceinline__ void tile_mfma(const char* __restrict__ sa, const char* __restrict__ sb,
                                          int wm, int wn, int lane, f32x16 (&acc)[2][2]) {
  const int r = lane & 31, h = lane >> 5;
  if constexpr (PREC == PKC_PREC_FP32) {
    // lane half h takes k = 16h + kk (kk = 0..15), the same permutation of k for A and B
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      float av[16];
      const int ra = wm * 64 + 32 * a + r;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = lds16(sa, ra, 4 * h + q);
        av[4 * q] = x.x; av[4 * q + 1] = x.y; av[4 * q + 2] = x.z; av[4 * q + 3] = x.w;
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float bv[16];
        const int rb = wn * 64 + 32 * b + r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 y = lds16(sb, rb, 4 * h + q);
          bv[4 * q] = y.x; bv[4 * q + 1] = y.y; bv[4 * q + 2] = y.z; bv[4 * q + 3] = y.w;
        }
#pragma unroll
        for (int kk = 0; kk < 16; ++kk)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk], bv[kk], acc[a][b], 0, 0, 0);
      }
    }
  } else if constexpr (PREC == PKC_PREC_BF16X3) {
    // compensated products: the tails' cross terms first, then the heads' product (lo*lo, 2^-16
    // relative, dropped); the images are row-major ([row][128 B] swizzled), A/B tails at + LO_OFF
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bf16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const float4 x = lds16(sa, wm * 64 + 32 * a + r, 2 * t + h);
        const float4 xl = lds16(sa + LO_OFF, wm * 64 + 32 * a + r, 2 * t + h);
        ah[a] = *reinterpret_cast<const bf16x8*>(&x);
        al[a] = *reinterpret_cast<const bf16x8*>(&xl);
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const float4 y = lds16(sb, wn * 64 + 32 * b + r, 2 * t + h);
        const float4 yl = lds16(sb + LO_OFF, wn * 64 + 32 * b + r, 2 * t + h);
        bh[b] = *reinterpret_cast<const bf16x8*>(&y);
        bl[b] = *reinterpret_cast<const bf16x8*>(&yl);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bl[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[a], bh[b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[a], bh[b], acc[a][b], 0, 0, 0);
        }
    }
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t) {                     // k = 16t + 8h + j
      bf16x8 av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        if constexpr (ATR) {
          av[a] = tr_frag(sa, wm * 64 + 32 * a, 16 * t, lane);
        } else {
          const float4 x = lds16(sa, wm * 64 + 32 * a + r, 2 * t + h);
          av[a] = *reinterpret_cast<const bf16x8*>(&x);
        }
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if constexpr (BTR) {
          bv[b] = tr_frag(sb, wn * 64 + 32 * b, 16 * t, lane);
        } else {
          const float4 y = lds16(sb, wn * 64 + 32 * b + r, 2 * t + h);
          bv[b] = *reinterpret_cast<const bf16x8*>(&y);
        }
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
  }
}

// Column statistics of a finished 128x128 tile for the BatchNorm that consumes it (the large-batch
// MLP forward, pkc_gemm_colstats): per column, the mean of its rows < M in this tile plus bias[c],
// and M2 = sum (z - mean)^2 — two passes over the accumulators (sums, then squared deviations from
// the tile mean), combined over the two 32-lane halves (shuffle) and the two row waves (LDS) in a
// fixed order.  -> part[by * 2N + c] = mean, part[by * 2N + N + c] = M2 (by = 128-row block), the
// per-block partials pkc_dense_fwd_pre merges with Chan's formula.  Every wave calls it (barriers).
__device__ __forceinline__ void tile_colstats(const f32x16 (&acc)[2][2], char* __restrict__ lds,
                                              int m0, int n0, int by, int M, int N, int wm, int wn,
                                              int lane, const float* __restrict__ bias,
                                              float* __restrict__ part) {
  float* red = reinterpret_cast<float*>(lds);     // [2 passes][2 row waves][128 columns]
  const int r = lane & 31, h = lane >> 5;
  const int nv = min(TM, M - m0);                 // valid rows of the tile (>= 1)
  float mean[2];
  __syncthreads();                                // every wave is done with the operand buffers
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    float s = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int rl = wm * 64 + 32 * a + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        s += rl < nv ? acc[a][b][reg] : 0.f;
      }
    s += __shfl_xor(s, 32);
    if (h == 0) red[wm * TN + wn * 64 + 32 * b + r] = s;
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int cl = wn * 64 + 32 * b + r;
    mean[b] = (red[cl] + red[TN + cl]) / (float)nv;
    float q = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int rl = wm * 64 + 32 * a + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const float d = acc[a][b][reg] - mean[b];
        q += rl < nv ? d * d : 0.f;
      }
    q += __shfl_xor(q, 32);
    if (h == 0) red[2 * TN + wm * TN + cl] = q;
  }
  __syncthreads();
  if (wm != 0 || h != 0) return;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int cl = wn * 64 + 32 * b + r, col = n0 + cl;
    if (col >= N) continue;
    part[(int64_t)by * 2 * N + col] = mean[b] + (bias ? bias[col] : 0.f);
    part[(int64_t)by * 2 * N + N + col] = red[2 * TN + cl] + red[3 * TN + cl];
  }
}

// BatchNorm-backward epilogue of a dX tile (pkc_bn_bwd_epi): the product g becomes
// dy = g * keep / (1 - p) * act'(gamma xhat + beta), stored in place of g, and the tile's column
// sums of dy and dy * xhat over its rows < M go to part[by*2N + c], part[by*2N + N + c] — one pass
// over the accumulators, the two 32-lane halves combined by a shuffle and the two row waves
// through LDS in a fixed order (as tile_colstats).  ldc == N (the layout of xhat and keep).
struct BnEpi {
  const float* xhat; const uint8_t* keep; const float* gamma; const float* beta;
  float* part; int act; float drop_p;
};
__device__ __forceinline__ void tile_bnbwd(f32x16 (&acc)[2][2], char* __restrict__ lds, int m0,
                                           int n0, int by, int M, int N, int wm, int wn, int lane,
                                           const BnEpi& e) {
  float* red = reinterpret_cast<float*>(lds);     // [2 sums][2 row waves][128 columns]
  const int r = lane & 31, h = lane >> 5;
  const bool drop = e.drop_p > 0.f;
  const float scale = drop ? 1.f / (1.f - e.drop_p) : 1.f;
  __syncthreads();                                // every wave is done with the operand buffers
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int col = n0 + wn * 64 + 32 * b + r;
    const bool cok = col < N;
    const int cc = cok ? col : N - 1;
    const float gam = e.gamma[cc], bet = e.beta[cc];
    float sdy = 0.f, sdyx = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = m0 + wm * 64 + 32 * a + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        const bool ok = cok && row < M;
        const int64_t idx = (int64_t)(ok ? row : 0) * N + cc;
        const float xh = e.xhat[idx];
        float g = acc[a][b][reg];
        if (drop) g = e.keep[idx] ? g * scale : 0.f;
        const float y = xh * gam + bet;
        const float dy = ok ? g * act_bwd(e.act, y, act_fwd(e.act, y)) : 0.f;
        acc[a][b][reg] = dy;
        sdy += dy;
        sdyx += dy * xh;
      }
    }
    sdy += __shfl_xor(sdy, 32);
    sdyx += __shfl_xor(sdyx, 32);
    if (h == 0) {
      red[wm * TN + wn * 64 + 32 * b + r] = sdy;
      red[2 * TN + wm * TN + wn * 64 + 32 * b + r] = sdyx;
    }
  }
  __syncthreads();
  if (wm != 0 || h != 0) return;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int cl = wn * 64 + 32 * b + r, col = n0 + cl;
    if (col >= N) continue;
    e.part[(int64_t)by * 2 * N + col] = red[cl] + red[TN + cl];
    e.part[(int64_t)by * 2 * N + N + col] = red[2 * TN + cl] + red[3 * TN + cl];
  }
}

// C/D map of the 32x32 MFMA: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
__device__ __forceinline__ void tile_store(const f32x16 (&acc)[2][2], int m0, int n0, int M, int N,
                                           int wm, int wn, int lane, float* __restrict__ Cz,
                                           int64_t ldc) {
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int col = n0 + wn * 64 + 32 * b + r;
    if (col >= N) continue;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = m0 + wm * 64 + 32 * a + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (row < M) Cz[(int64_t)row * ldc + col] = acc[a][b][reg];
      }
    }
  }
}

// C[bz slab][m0.., n0..] = A[m0.., kbeg..kend) . B[n0.., kbeg..kend)^T for one 128x128 tile.
// `lds` is lds_bytes<PREC>() of workgroup memory.  STATS: also the tile's column statistics
// (tile_colstats; one slab, kchunk >= K).
// BNB: the BatchNorm-backward epilogue (tile_bnbwd with *bnb) before the store
template <int PREC, bool BIN, bool AKC, bool BKC, bool STATS = false, bool BNB = false>
__device__ __forceinline__ void body(char* __restrict__ lds, int bx, int by, int bz, int M, int N,
                                     int K, const void* __restrict__ Av, int64_t lda,
                                     const void* __restrict__ Bv, int64_t ldb,
                                     float* __restrict__ Cp, int64_t ldc, int kchunk,
                                     int64_t slab_stride, const float* __restrict__ bias = nullptr,
                                     float* __restrict__ part = nullptr,
                                     const BnEpi* bnb = nullptr) {
  using Cf = Cfg<PREC, BIN>;
  using HE = typename Cf::HE;
  constexpr int BK = Cf::BK;
  const HE* A = reinterpret_cast<const HE*>(Av);
  const HE* B = reinterpret_cast<const HE*>(Bv);
  const int m0 = by * TM, n0 = bx * TN;
  const int kbeg = bz * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  // Tile t lives in LDS buffer t&1 (A at lds + (t&1)*2*TILE_BYTES, B right after it; computed,
  // not indexed from a pointer array, which would be promoted into extra LDS).
  // DEPTH 2 (bf16 and fp32 operands staged as they are stored): two register stages, so a k-tile's
  // loads are issued two k-tiles before its LDS store; a workgroup alone on its CU (one 128x128
  // tile per CU) otherwise waits a full HBM/L2 latency every k-tile.  DEPTH 1 for the fp32->bf16
  // staging, whose stages take twice the registers.
  constexpr int DEPTH = (sizeof(HE) == sizeof(typename Cf::LE)) ? 2 : 1;
  Stage<PREC, BIN, AKC> na, nna;      // tile t+1, tile t+2 (DEPTH 2)
  Stage<PREC, BIN, BKC> nb, nnb;
  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;   // uniform
  if (nk > 0) {
    // leading dimensions < 2^31 elements (pkc_gemm / pkc_gemm_grouped check)
    const typename Stage<PREC, BIN, AKC>::Base ab = Stage<PREC, BIN, AKC>::base(A, lda, m0, M);
    const typename Stage<PREC, BIN, BKC>::Base bb = Stage<PREC, BIN, BKC>::base(B, ldb, n0, N);
    const int la = (int)lda, lb = (int)ldb;
    na.load_at(ab, la, kbeg, kend);
    nb.load_at(bb, lb, kbeg, kend);
    na.store(lds);
    nb.store(lds + TILE_BYTES);
    na.load_at(ab, la, kbeg + BK, kend);               // past kend: clamped, zeroed, never stored
    nb.load_at(bb, lb, kbeg + BK, kend);
    if constexpr (DEPTH == 2) {
      nna.load_at(ab, la, kbeg + 2 * BK, kend);
      nnb.load_at(bb, lb, kbeg + 2 * BK, kend);
    }
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      char* cur = lds + (t & 1) * buf_bytes<PREC>();
      char* nxt = lds + ((t + 1) & 1) * buf_bytes<PREC>();
      tile_mfma<PREC, Stage<PREC, BIN, AKC>::TR, Stage<PREC, BIN, BKC>::TR>(cur, cur + TILE_BYTES,
                                                                         wm, wn, lane, acc);
      if (t + 1 < nk) {                               // uniform
        na.store(nxt);
        nb.store(nxt + TILE_BYTES);
        if constexpr (DEPTH == 2) {
          na = nna;
          nb = nnb;
          nna.load_at(ab, la, kbeg + (t + 3) * BK, kend);
          nnb.load_at(bb, lb, kbeg + (t + 3) * BK, kend);
        } else {
          na.load_at(ab, la, kbeg + (t + 2) * BK, kend);
          nb.load_at(bb, lb, kbeg + (t + 2) * BK, kend);
        }
      }
      __syncthreads();
    }
  }
  if constexpr (BNB) tile_bnbwd(acc, lds, m0, n0, by, M, N, wm, wn, lane, *bnb);
  tile_store(acc, m0, n0, M, N, wm, wn, lane, Cp + (int64_t)bz * slab_stride, ldc);
  if constexpr (STATS) tile_colstats(acc, lds, m0, n0, by, M, N, wm, wn, lane, bias, part);
}

// ------------------------------------------------------------------------------------------
// LDS-DMA form of the bf16 body (operands stored as bf16, k-range a multiple of 64): one workgroup
// per CU holds a 128x128 tile, so a k-tile whose loads are issued only two k-tiles ahead through
// registers waits most of a memory round trip (the 4096x1024x1024 forward: 27 us = 12 % of the
// CUs' MFMA rate).  Here global_load_lds writes the operand images straight into a ring of NB LDS
// buffers (32 KB each): NB - 1 k-tiles stay in flight across each barrier (counted vmcnt, raw s_barrier:
// __syncthreads() would drain the DMA), no staging registers, no ds_write pass.  The DMA writes
// each wave-instruction's 64 x 16 bytes linearly, so the swizzles of the register path's images
// (swz for row images, xr for the [k][row] images) go on the per-lane SOURCE addresses instead.
// NB buffers in the ring, NB - 1 k-tiles in flight: a lone workgroup per CU keeps only
// (NB - 1) x 32 KB of operand requests outstanding, so its k-tile rate is that over the load
// latency under full-chip traffic (PKC_GLDS_BUFS selects NB = 3, 4 or 5; 5 = all 160 KB of LDS).
template <int NB>
constexpr int gl_lds_bytes() { return NB * 2 * TILE_BYTES; }

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glb_void;

// One 16 KB operand image of k-tile [k0, k0 + 64) is 16 wave-instructions of 1 KB, 4 per wave:
// KC: piece j = rows 8j .. 8j+7 of 128 B, lane slot (lane & 7); otherwise k-rows 4j .. 4j+3 of
// 256 B, slot (lane & 15), swizzled on the source address.  The 4 pieces this wave issues are kept
// as per-lane source pointers computed ONCE and advanced by a uniform byte step per k-tile:
// recomputed per tile, that piece / swizzle / clamp arithmetic with its 64-bit row products was
// ~130 vector instructions ahead of each tile's 16 MFMAs (PMC: 47 % of the wave cycles issuing
// instructions against 20 % in MFMAs).
template <bool KC>
struct GldsOperand {
  const char* p[4];
  int64_t step;                               // bytes per 64-deep k-tile

  __device__ __forceinline__ void init(const __bf16* __restrict__ P, int64_t ld, int r0, int rmax,
                                       int k0) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * i + w;
      const __bf16* src;
      if constexpr (KC) {
        const int r = 8 * j + (lane >> 3);
        const int c = (lane & 7) ^ swz(r);
        src = P + (int64_t)min(r0 + r, rmax - 1) * ld + k0 + 8 * c;
      } else {
        const int k = 4 * j + (lane >> 4);
        const int c = (lane & 15) ^ xr(k);
        src = P + (int64_t)(k0 + k) * ld + min(r0 + 8 * c, rmax - 8);
      }
      p[i] = reinterpret_cast<const char*>(src);
    }
    step = KC ? 128 : 128 * ld;
  }

  // the image of k-tile t (k0 + 64 t) into dst
  __device__ __forceinline__ void issue(int t, char* dst) const {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t off = (int64_t)t * step;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((glb_void*)(p[i] + off), (lds_void*)(dst + 1024 * (4 * i + w)),
                                       16, 0, 0);
  }
};

// s_waitcnt vmcnt(8 n): 8 glds per thread per k-tile, n later k-tiles left in flight
__device__ __forceinline__ void wait_tiles(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
  }
}

template <int NB, bool AKC, bool BKC, bool STATS = false>
__device__ __forceinline__ void body_glds(char* __restrict__ lds, int bx, int by, int bz, int M,
                                          int N, int K, const void* __restrict__ Av, int64_t lda,
                                          const void* __restrict__ Bv, int64_t ldb,
                                          float* __restrict__ Cp, int64_t ldc, int kchunk,
                                          int64_t slab_stride, const float* __restrict__ bias = nullptr,
                                          float* __restrict__ part = nullptr) {
  const __bf16* A = reinterpret_cast<const __bf16*>(Av);
  const __bf16* B = reinterpret_cast<const __bf16*>(Bv);
  const int m0 = by * TM, n0 = bx * TN;
  const int kbeg = bz * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;
  const int nk = kbeg < kend ? (kend - kbeg) / 64 : 0;      // uniform; k-range % 64 == 0
  static_assert(NB >= 3 && NB <= 5, "body_glds: 3..5 ring buffers");
  auto buf = [&](int t) { return lds + (t % NB) * 2 * TILE_BYTES; };
  GldsOperand<AKC> ga;
  GldsOperand<BKC> gb;
  ga.init(A, lda, m0, M, kbeg);
  gb.init(B, ldb, n0, N, kbeg);
  auto issue = [&](int t) {
    ga.issue(t, buf(t));
    gb.issue(t, buf(t) + TILE_BYTES);
  };
#pragma unroll
  for (int t = 0; t < NB - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    // tile t + NB - 1 refills the buffer of tile t - 1, released by the barrier ending iteration
    // t - 1
    if (t + NB - 1 < nk) issue(t + NB - 1);
    // this thread's DMAs of tile t are done once at most the later tiles' 8 each are in flight
    wait_tiles(min(NB - 1, nk - 1 - t));
    __builtin_amdgcn_s_barrier();             // ... and every thread's
    asm volatile("" ::: "memory");
    const char* cur = buf(t);
    tile_mfma<PKC_PREC_BF16, !AKC, !BKC>(cur, cur + TILE_BYTES, wm, wn, lane, acc);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();             // every wave has read buffer t % NB
    asm volatile("" ::: "memory");
  }
  tile_store(acc, m0, n0, M, N, wm, wn, lane, Cp + (int64_t)bz * slab_stride, ldc);
  if constexpr (STATS) tile_colstats(acc, lds, m0, n0, by, M, N, wm, wn, lane, bias, part);
}

// Which problems take this body: 16-byte operand paths (aligned bases and leading dimensions,
// contiguous extents multiples of a chunk) and enough 128x128 tiles to fill the chip.
__host__ inline bool eligible(int prec, int akc, int bkc, int M, int N, int K, const void* A,
                              int64_t lda, const void* B, int64_t ldb, int min_tiles,
                              int min_k = 128) {
  const int e = prec == PKC_PREC_BF16IN ? 8 : 4;
  const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % e == 0 &&
                   ldb % e == 0 && (akc ? K % e == 0 : M % e == 0) && (bkc ? K % e == 0 : N % e == 0);
  const int64_t tiles = (int64_t)((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  // exact fp32 runs at the vector rate: the 64x64 tile already streams fast enough for it and
  // balances better over the CUs (C4's projections: 83 vs 73 TF/s, same run); the 128x128 tile
  // wins only once there are several tiles per CU (4096^3: 118 vs 109 TF/s)
  if (prec == PKC_PREC_FP32) min_tiles = min_tiles > 1024 ? min_tiles : 1024;
  return vec && tiles >= min_tiles && K >= min_k;
}

}  // namespace big
}  // namespace pkc
