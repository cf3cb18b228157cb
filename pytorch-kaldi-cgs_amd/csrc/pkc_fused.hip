// pkc_fused.hip — a BatchNorm'd MLP layer's forward in ONE launch at the reference's frame batch
// (batch_size_train = 128, cfg/TIMIT_baselines/TIMIT_MLP_fmllr.cfg; neural_networks.py:306-317:
// drop(act(BN(W x + b)))).
//
// The B = 128 step was a chain of latency-bound launches: a split-K matmul writing fp32 partial
// slabs (128 workgroups, ~5 us), then pkc_dense_fwd's small kernel summing them and applying
// BatchNorm / activation / dropout (~5 us), per layer.  BatchNorm's statistics are per COLUMN over
// the batch rows, so a workgroup that owns every row of a column strip has them locally: here each
// workgroup computes a 128-row x 16-column strip of z = X W^T over the FULL contraction and applies
// the whole epilogue to it — no slabs, no second launch.
//
// Strip product: 8 waves split the contraction into contiguous k-ranges; each wave holds the 8
// row tiles (16 x 16, v_mfma_f32_16x16x32_bf16, fp32 accumulation) of its range, its operands
// staged k-step by k-step through its own LDS images (strip_product).  The 8 partial strips are
// summed through LDS in wave order, then the column statistics (two passes, as pkc_dense_fwd) and
// the element-wise epilogue run on the finished strip.
//
// Operands: PKC_PREC_BF16IN (bf16 copies in HBM, the step's bf16-store mode) or PKC_PREC_BF16
// (fp32 in HBM, rounded to bf16 on load — the same RNE rounding, so both forms give identical
// results).  Exact fp32 keeps the split-K path (its 16x slower MFMA needs the 128-workgroup grid).
#include "pkc_common.h"

namespace pkc {
namespace fused {

constexpr int NW = 8, NT = 64 * NW;     // waves / threads per workgroup
constexpr int MR = 128;                 // rows (the whole batch)
constexpr int NC = 16;                  // columns per workgroup
constexpr int MT = MR / 16;             // row tiles

typedef __attribute__((ext_vector_type(8))) __bf16 bf8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// Phase trace (PKC_TRACE measurement builds only; scripts/trace_fused.py): per workgroup, after
// draining its memory counters, thread 0 stores the shader clock at each phase boundary (stamps 0
// and 7: the 100 MHz real-time clock), read back with pkc_trace_read_fused.
#ifdef PKC_TRACE
constexpr int FTRACE_WG = 4096;
__device__ unsigned long long ftrace_buf[FTRACE_WG * 8];
__device__ __forceinline__ void ftrace(int i) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const unsigned long long v = (i == 0 || i == 7) ? __builtin_amdgcn_s_memrealtime()
                                                  : __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x < FTRACE_WG)
    reinterpret_cast<volatile unsigned long long*>(ftrace_buf)[blockIdx.x * 8 + i] = v;
}
#define PKC_FTR(i) ::pkc::fused::ftrace(i)
#else
#define PKC_FTR(i) do { } while (0)
#endif

__device__ __forceinline__ bf8 zero8() {
  bf8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
  return v;
}

// 8 consecutive k of an operand row as bf16: stored bf16 (BIN) or fp32 rounded to nearest even
template <bool BIN>
__device__ __forceinline__ bf8 ld8(const void* base, int64_t off) {
  if constexpr (BIN) {
    return *reinterpret_cast<const bf8*>(reinterpret_cast<const __bf16*>(base) + off);
  } else {
    const float* p = reinterpret_cast<const float*>(base) + off;
    const float4 x = *reinterpret_cast<const float4*>(p);
    const float4 y = *reinterpret_cast<const float4*>(p + 4);
    bf8 v;
    v[0] = (__bf16)x.x; v[1] = (__bf16)x.y; v[2] = (__bf16)x.z; v[3] = (__bf16)x.w;
    v[4] = (__bf16)y.x; v[5] = (__bf16)y.y; v[6] = (__bf16)y.z; v[7] = (__bf16)y.w;
    return v;
  }
}

// This wave's partial of the workgroup's 128 x 16 strip z[m][n0 + j] = sum_k A[m][k] B[n0 + j][k]
// over its k-range, both operands k-contiguous.
//
// Operand staging.  An MFMA fragment gives lane (c = lane % 16, q = lane / 16) row c at k-chunk q,
// so loading fragments straight from memory makes every 4-lane quad of a load touch 4 rows: the
// address unit then moves one lane per cycle (measured: 63 cycles per 1 KB wave-load, the whole
// kernel 12.8 us at K = 1024 against 8.1 for the split-K matmul + BatchNorm pair).  Each wave
// instead stages its k-steps through its own LDS region: one k-step image is the 128 A rows and
// 16 B rows x 64 bytes (32 bf16), row r's four 16-byte chunks at slots 4 r + (kq ^ h(r)),
// h(r) = -(r / 4) mod 4 — quads of lanes load the 64 contiguous bytes of one row (coalesced), and
// the fragment reads (ds_read_b128, lane groups {0-3,12-15,20-27}, ...) hit 16 distinct bank
// quads.  Bf16-stored full k-steps come by LDS-DMA (global_load_lds: no staging registers, no
// ds_write); fp32 operands (rounded to bf16 here) and the partial last k-step (k >= K zeroed)
// through registers and ds_write_b128 into the same slots, so every form feeds the MFMAs the same
// values in the same order.  Two images per wave: the next k-step's loads are in flight during
// this one's MFMAs; only wave-local ordering (vmcnt / lgkmcnt), no workgroup barrier.
constexpr int ROWS = MR + NC;                 // image rows: A rows, then B rows
constexpr int IMG_BYTES = ROWS * 64;          // one k-step image (9 KB)
constexpr int WAVE_BYTES = 2 * IMG_BYTES;
constexpr int STAGE_BYTES = NW * WAVE_BYTES;  // 144 KB
constexpr int DMA_PER_STEP = ROWS * 4 / 64;   // 16-byte slots / 64 lanes = 9 wave-instructions

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glb_void;

__device__ __forceinline__ int img_h(int r) { return (-(r >> 2)) & 3; }

// the source element of image slot s = 64 i + lane of k-step ks (row clamped to the valid rows:
// rows >= M are never read back as results; k past K handled by the callers)
struct SlotSrc {
  int64_t off;     // element offset
  bool isb;        // a B row
  int k0;          // first k of the chunk
};
__device__ __forceinline__ SlotSrc slot_src(int i, int lane, int ks, int M, int64_t lda, int64_t ldb,
                                            int n0) {
  const int r = 16 * i + (lane >> 2);
  const int kq = (lane & 3) ^ img_h(r);
  SlotSrc o;
  o.k0 = 32 * ks + 8 * kq;
  o.isb = r >= MR;
  o.off = o.isb ? (int64_t)(n0 + r - MR) * ldb + o.k0 : (int64_t)min(r, M - 1) * lda + o.k0;
  return o;
}

// register-staged k-step (fp32 operands, or the partial last step): load, round, zero k >= K,
// ds_write_b128 into the image
template <bool BIN>
__device__ __forceinline__ void stage_regs(char* img, const void* __restrict__ A, int64_t lda,
                                           const void* __restrict__ B, int64_t ldb, int M, int K,
                                           int n0, int ks) {
  const int lane = threadIdx.x & 63;
  const bf8 z8 = zero8();
  bf8 v[DMA_PER_STEP];
#pragma unroll
  for (int i = 0; i < DMA_PER_STEP; ++i) {
    const SlotSrc o = slot_src(i, lane, ks, M, lda, ldb, n0);
    const bool ok = o.k0 < K;                    // K % 8 == 0: a chunk is all in or all out
    const int64_t off = ok ? o.off : 0;
    const bf8 x = ld8<BIN>(o.isb ? B : A, off);
    v[i] = ok ? x : z8;
  }
#pragma unroll
  for (int i = 0; i < DMA_PER_STEP; ++i)
    *reinterpret_cast<bf8*>(img + 1024 * i + 16 * lane) = v[i];
}

// LDS-DMA k-step (bf16 operands, k-step inside [0, K))
__device__ __forceinline__ void stage_dma(char* img, const __bf16* __restrict__ A, int64_t lda,
                                          const __bf16* __restrict__ B, int64_t ldb, int M, int n0,
                                          int ks) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < DMA_PER_STEP; ++i) {
    const SlotSrc o = slot_src(i, lane, ks, M, lda, ldb, n0);
    __builtin_amdgcn_global_load_lds((glb_void*)((o.isb ? B : A) + o.off),
                                     (lds_void*)(img + 1024 * i), 16, 0, 0);
  }
}

template <bool BIN>
__device__ __forceinline__ void strip_product(char* stage, const void* __restrict__ A, int64_t lda,
                                              const void* __restrict__ B, int64_t ldb, int M,
                                              int K, int n0, f32x4 (&acc)[MT]) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int nks = (K + 31) / 32;
  const int ks0 = w * nks / NW, ks1 = (w + 1) * nks / NW;
  const int nst = ks1 - ks0;                   // uniform
  char* mine = stage + w * WAVE_BYTES;
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per-lane fragment offsets in an image: A tile t row 16 t + c, B row MR + c, chunk q
  const int hq = (q ^ img_h(c)) * 16;
  const int afr = 64 * c + hq, bfr = 64 * (MR + c) + hq;
  const __bf16* Ab = reinterpret_cast<const __bf16*>(A);
  const __bf16* Bb = reinterpret_cast<const __bf16*>(B);
  // a k-step by DMA only when the operands are bf16 and the step lies inside [0, K)
  auto issue = [&](int i) {
    char* img = mine + (i & 1) * IMG_BYTES;
    const int ks = ks0 + i;
    if (BIN && 32 * (ks + 1) <= K) stage_dma(img, Ab, lda, Bb, ldb, M, n0, ks);
    else stage_regs<BIN>(img, A, lda, B, ldb, M, K, n0, ks);
  };
  if (nst > 0) issue(0);
  if (nst > 1) issue(1);
  for (int i = 0; i < nst; ++i) {
    // step i's image: its DMAs complete once at most step i + 1's are still in flight (register
    // steps are complete here: their values were written by this wave's own ds_writes)
    if (i + 1 < nst) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const char* img = mine + (i & 1) * IMG_BYTES;
    bf8 a[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) a[t] = *reinterpret_cast<const bf8*>(img + 1024 * t + afr);
    const bf8 b = *reinterpret_cast<const bf8*>(img + bfr);
    // every read of this image done before step i + 2 overwrites it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i + 2 < nst) issue(i + 2);
#pragma unroll
    for (int t = 0; t < MT; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t], b, acc[t], 0, 0, 0);
  }
}

// The 8 waves' partial strips summed in wave order: thread (row = tid / 4, column group
// cg = tid % 4) gets z[row][n0 + 4 cg .. + 3].  red: NW x 128 x 16 floats of LDS.
__device__ __forceinline__ float4 strip_reduce(const f32x4 (&acc)[MT], float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  float* mine = red + w * MR * NC;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) mine[(16 * t + 4 * q + i) * NC + c] = acc[t][i];
  __syncthreads();
  const int row = threadIdx.x >> 2, cg = threadIdx.x & 3;
  float4 z = *reinterpret_cast<const float4*>(red + row * NC + 4 * cg);
#pragma unroll
  for (int v = 1; v < NW; ++v) {
    const float4 p = *reinterpret_cast<const float4*>(red + v * MR * NC + row * NC + 4 * cg);
    z.x += p.x; z.y += p.y; z.z += p.z; z.w += p.w;
  }
  return z;
}

// column sums over the workgroup's rows (one float4 of 4 columns per thread, column group
// tid % 4): within the wave by shuffles over the row bits of the lane, then the 8 waves in order
// through LDS (xr: NW x 4 float4 no earlier exchange reads)
__device__ __forceinline__ float4 col_sum(float4 v, float4* xr) {
#pragma unroll
  for (int o = 4; o < 64; o <<= 1) {
    v.x += __shfl_xor(v.x, o, 64);
    v.y += __shfl_xor(v.y, o, 64);
    v.z += __shfl_xor(v.z, o, 64);
    v.w += __shfl_xor(v.w, o, 64);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, cg = threadIdx.x & 3;
  if (lane < 4) xr[w * 4 + lane] = v;
  __syncthreads();
  float4 s = xr[cg];
#pragma unroll
  for (int u = 1; u < NW; ++u) {
    const float4 p = xr[u * 4 + cg];
    s.x += p.x; s.y += p.y; s.z += p.z; s.w += p.w;
  }
  return s;
}

__device__ __forceinline__ float f4g(const float4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}
__device__ __forceinline__ void f4s(float4& v, int j, float x) {
  if (j == 0) v.x = x; else if (j == 1) v.y = x; else if (j == 2) v.z = x; else v.w = x;
}
__device__ __forceinline__ void st_h4(void* p, int64_t i, float4 v) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  bf16x4 h;
  h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
  *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(p) + i) = h;
}

// Forward: z = X W^T (+ bias) over the strip, then pkc_dense_fwd's epilogue (BatchNorm with batch
// statistics — biased variance for the normalisation, unbiased for running_var — or running
// statistics in eval, activation, inverted dropout from the counter RNG or an injected mask) with
// every output of that kernel: out, out_bf16, xhat, keep_out, save_mean / save_invstd, running
// statistics.
template <bool BIN>
__global__ __launch_bounds__(NT) void dense_gemm_fwd_kernel(const void* __restrict__ A, int64_t lda,
                                                           const void* __restrict__ W, int64_t ldw,
                                                           int K, pkc_dense_fwd_args a) {
  // the k-step images of the 8 waves; after the products, the partial strips (strip_reduce)
  __shared__ __attribute__((aligned(16))) char stage[STAGE_BYTES];
  __shared__ float4 xr[2][NW * 4];
  float* red = reinterpret_cast<float*>(stage);
  static_assert(NW * MR * NC * 4 <= STAGE_BYTES, "partial strips must fit the staging LDS");
  PKC_FTR(0);
  const int n0 = blockIdx.x * NC;
  const int M = a.M;
  const int64_t N = a.N;
  const int row = threadIdx.x >> 2, cg = threadIdx.x & 3;
  const int c = n0 + 4 * cg;
  // per-column parameters requested up front (valid addresses; selected away when absent)
  const float* dummy = a.gamma ? a.gamma : a.bias;
  const bool hb = a.bias != nullptr, bnp = a.norm != PKC_NORM_NONE && dummy != nullptr;
  const float* pd = dummy ? dummy : reinterpret_cast<const float*>(a.save_mean);
  const float4 b0 = *reinterpret_cast<const float4*>(hb ? a.bias + c : pd);
  const float4 g0 = *reinterpret_cast<const float4*>(bnp ? a.gamma + c : pd);
  const float4 be0 = *reinterpret_cast<const float4*>(bnp ? a.beta + c : pd);
  const float4 rm0 = *reinterpret_cast<const float4*>(bnp ? a.running_mean + c : pd);
  const float4 rv0 = *reinterpret_cast<const float4*>(bnp ? a.running_var + c : pd);
  const int64_t step = a.step_ctr ? *a.step_ctr : 0;
  PKC_FTR(1);
  f32x4 acc[MT];
  strip_product<BIN>(stage, A, lda, W, ldw, M, K, n0, acc);
  __syncthreads();                                // every wave is done with its images
  PKC_FTR(2);
  float4 z = strip_reduce(acc, red);
  PKC_FTR(3);
  const bool rok = row < M;
  if (hb) z = make_float4(z.x + b0.x, z.y + b0.y, z.z + b0.z, z.w + b0.w);
  if (!rok) z = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 mean = make_float4(0.f, 0.f, 0.f, 0.f), invstd = make_float4(1.f, 1.f, 1.f, 1.f);
  float4 gam = make_float4(1.f, 1.f, 1.f, 1.f), bet = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.norm == PKC_NORM_BN_TRAIN) {
    const float4 sum = col_sum(z, xr[0]);
    const float inv = 1.f / (float)M;
    mean = make_float4(sum.x * inv, sum.y * inv, sum.z * inv, sum.w * inv);
    float4 d2 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rok) {
      const float dx = z.x - mean.x, dy = z.y - mean.y, dz = z.z - mean.z, dw = z.w - mean.w;
      d2 = make_float4(dx * dx, dy * dy, dz * dz, dw * dw);
    }
    const float4 m2 = col_sum(d2, xr[1]);
    const float4 var = make_float4(m2.x * inv, m2.y * inv, m2.z * inv, m2.w * inv);
    invstd = make_float4(1.f / sqrtf(var.x + a.eps), 1.f / sqrtf(var.y + a.eps),
                         1.f / sqrtf(var.z + a.eps), 1.f / sqrtf(var.w + a.eps));
    gam = g0;
    bet = be0;
    if (row == 0) {
      *reinterpret_cast<float4*>(a.save_mean + c) = mean;
      *reinterpret_cast<float4*>(a.save_invstd + c) = invstd;
      const float cn = (float)(a.count_n > 0 ? a.count_n : M);
      float4 rm = rm0, rv = rv0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float vj = f4g(var, j);
        const float unb = cn > 1.f ? vj * cn / (cn - 1.f) : vj;
        f4s(rm, j, (1.f - a.momentum) * f4g(rm, j) + a.momentum * f4g(mean, j));
        f4s(rv, j, (1.f - a.momentum) * f4g(rv, j) + a.momentum * unb);
      }
      *reinterpret_cast<float4*>(a.running_mean + c) = rm;
      *reinterpret_cast<float4*>(a.running_var + c) = rv;
    }
    PKC_FTR(4);
  } else if (a.norm == PKC_NORM_BN_EVAL) {
    mean = rm0;
    invstd = make_float4(1.f / sqrtf(rv0.x + a.eps), 1.f / sqrtf(rv0.y + a.eps),
                         1.f / sqrtf(rv0.z + a.eps), 1.f / sqrtf(rv0.w + a.eps));
    gam = g0;
    bet = be0;
  }
  if (!rok) return;
  const bool drop = a.drop_p > 0.f;
  const float scale = drop ? 1.f / (1.f - a.drop_p) : 1.f;
  const uint32_t thr = drop ? (uint32_t)((double)(1.f - a.drop_p) * 4294967296.0) : 0u;
  const uint32_t seed32 = hash_seed(a.seed, (uint64_t)a.stream_id, (uint64_t)step);
  const int64_t idx = (int64_t)row * N + c;
  float4 xh, o;
  uint32_t kw = 0;
  uchar4 kin = make_uchar4(1, 1, 1, 1);
  if (drop && a.keep_in) kin = *reinterpret_cast<const uchar4*>(a.keep_in + idx);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float zj = f4g(z, j);
    const float x = (a.norm == PKC_NORM_NONE) ? zj : (zj - f4g(mean, j)) * f4g(invstd, j);
    const float y = (a.norm == PKC_NORM_NONE) ? zj : x * f4g(gam, j) + f4g(bet, j);
    float v = act_fwd(a.act, y);
    if (drop) {
      uint32_t k;
      if (a.keep_in) k = j == 0 ? kin.x : (j == 1 ? kin.y : (j == 2 ? kin.z : kin.w));
      else k = hash_drop(seed32, (uint32_t)(idx + j)) < thr;
      kw |= (k ? 1u : 0u) << (8 * j);
      v = k ? v * scale : 0.f;
    }
    f4s(xh, j, x);
    f4s(o, j, v);
  }
  if (drop && a.keep_out) *reinterpret_cast<uint32_t*>(a.keep_out + idx) = kw;
  if (a.xhat) *reinterpret_cast<float4*>(a.xhat + idx) = xh;
  if (a.out) *reinterpret_cast<float4*>(a.out + idx) = o;
  if (a.out_bf16) st_h4(a.out_bf16, idx, o);
  PKC_FTR(5);
  PKC_FTR(7);
}

}  // namespace fused
}  // namespace pkc

#ifdef PKC_TRACE
extern "C" int pkc_trace_read_fused(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pkc::fused::ftrace_buf), sizeof(unsigned long long) * n,
                             0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

static bool al16(const void* p) { return (uintptr_t)p % 16 == 0; }

extern "C" int pkc_dense_gemm_fwd_ok(int prec, int M, int N, int K, const void* A, int64_t lda,
                                     const void* W, int64_t ldw) {
  using namespace pkc::fused;
  return (prec == PKC_PREC_BF16 || prec == PKC_PREC_BF16IN) && M > 0 && M <= MR && N > 0 &&
         N % NC == 0 && K > 0 && K % 8 == 0 && lda >= K && ldw >= K && lda % 8 == 0 &&
         ldw % 8 == 0 && al16(A) && al16(W) && lda < (1ll << 30) && ldw < (1ll << 30);
}

extern "C" int pkc_dense_gemm_fwd(int prec, const void* A, int64_t lda, const void* W, int64_t ldw,
                                  int K, const pkc_dense_fwd_args* a, void* stream) {
  using namespace pkc;
  using namespace pkc::fused;
  PKC_CHECK_ARG(a && A && W, "pkc_dense_gemm_fwd: null argument");
  PKC_CHECK_ARG(pkc_dense_gemm_fwd_ok(prec, a->M, a->N, K, A, lda, W, ldw),
                "pkc_dense_gemm_fwd: unsupported shape / precision / alignment (prec %d, M %d, "
                "N %d, K %d, lda %lld, ldw %lld)", prec, a->M, a->N, K, (long long)lda,
                (long long)ldw);
  PKC_CHECK_ARG(a->norm == PKC_NORM_NONE || a->norm == PKC_NORM_BN_TRAIN ||
                    a->norm == PKC_NORM_BN_EVAL,
                "pkc_dense_gemm_fwd: norm %d", a->norm);
  PKC_CHECK_ARG(a->norm == PKC_NORM_NONE || (a->gamma && a->beta && a->running_mean &&
                                             a->running_var),
                "pkc_dense_gemm_fwd: BatchNorm parameters missing");
  PKC_CHECK_ARG(a->norm != PKC_NORM_BN_TRAIN || (a->save_mean && a->save_invstd),
                "pkc_dense_gemm_fwd: BatchNorm training needs save_mean / save_invstd");
  PKC_CHECK_ARG(a->out || a->out_bf16, "pkc_dense_gemm_fwd: no output");
  PKC_CHECK_ARG((!a->out || al16(a->out)) && (!a->xhat || al16(a->xhat)) &&
                    (!a->out_bf16 || (uintptr_t)a->out_bf16 % 8 == 0) &&
                    (!a->bias || al16(a->bias)) && (!a->gamma || al16(a->gamma)) &&
                    (!a->beta || al16(a->beta)) && (!a->running_mean || al16(a->running_mean)) &&
                    (!a->running_var || al16(a->running_var)) &&
                    (!a->save_mean || al16(a->save_mean)) && (!a->save_invstd || al16(a->save_invstd)) &&
                    (!a->keep_out || (uintptr_t)a->keep_out % 4 == 0) &&
                    (!a->keep_in || (uintptr_t)a->keep_in % 4 == 0),
                "pkc_dense_gemm_fwd: outputs / parameters must be 16-byte aligned");
  PKC_CHECK_ARG(a->drop_p <= 0.f || a->keep_out || a->keep_in,
                "pkc_dense_gemm_fwd: dropout needs keep_out (or keep_in)");
  const dim3 grid(a->N / NC);
  if (prec == PKC_PREC_BF16IN)
    hipLaunchKernelGGL(dense_gemm_fwd_kernel<true>, grid, dim3(NT), 0, S(stream), A, lda, W, ldw, K,
                       *a);
  else
    hipLaunchKernelGGL(dense_gemm_fwd_kernel<false>, grid, dim3(NT), 0, S(stream), A, lda, W, ldw,
                       K, *a);
  PKC_LAUNCH_CHECK("pkc_dense_gemm_fwd");
  return PKC_OK;
}
