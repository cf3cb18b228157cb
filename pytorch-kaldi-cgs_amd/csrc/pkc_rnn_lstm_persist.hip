// pkc_rnn_lstm_persist.hip — grid-synchronised persistent time loops of a dense LSTM layer with
// quantised recurrent input (the C5 family: quantized_modules LSTM, qbits <= 16, U on a weight grid
// of <= 8 bits, uni-directional, B <= 16 rows; forward H in {512, 768, 1024}, BPTT H = 512).
// north_star: "recurrent time-step loops fused per wavefront"; the per-step form of the same
// arithmetic is pkc_rnn_impl.h rnn_fwd_mm (QX) and rnn_bwd_mm + rnn_bwd_epi.
//
// Reference: the LSTM step neural_networks.py:1077-1097; the four in-place QuantizeLinear calls on
// h_{t-1} per step quantized_modules.py:99-119.
//
// Unlike the liGRU loops (pkc_rnn_persist.hip: rows are independent, one workgroup owns a row for
// every step) an LSTM layer's U (4 x H x H) does not fit a workgroup: the units are dealt to
// H / 16 workgroups, each holding its 16 units' U rows of all four gates (forward; BPTT: its 16
// columns of U^T) as MFMA operands in registers for the whole loop, and every step hands h_t
// (BPTT: dgates_t) to every workgroup through memory — the measured alternative to a launch
// boundary per step (MI355X_MICROARCH.md, persistent-kernel price list):
//   * payload: stored by its owner with agent-scope write-through (sc1) stores, loaded by every
//     workgroup with sc1 loads (bypassing the reading CU's L1; nothing else reads it in the launch);
//   * step barrier: after every storing wave's s_waitcnt vmcnt(0) and a workgroup barrier, one
//     lane adds 1 to a monotone counter (agent-scope atomic); the next step's readers wait — one
//     lane polls with relaxed sc1 loads and s_sleep, the other waves at the workgroup barrier — for
//     NWG x (steps done).  Every spin is bounded: a launch whose peers never arrive sets the
//     timeout word (counter + 1) and ends;
//   * the step's inputs that do not depend on the recurrence (W x, dL/dy, saved gates) are
//     requested before the wait, so they arrive during it.
// Numerics: bit-identical to the per-step kernels (tests/test_gpu_lstm_persist.py):
//   forward: the per-step QX kernel's per-wave k-ranges (wave w: [w H / 8, (w + 1) H / 8)), whose
//     kh / kl x U_h sums are exact integers in any order, the same fmaf(256, hi, lo) x var_s per
//     wave, the same ((w0 + w1) + (w2 + w3)) + ((w4 + w5) + (w6 + w7)) across waves, then fwd_epi;
//   BPTT: per gate the per-step kernel's fp32 16x16x4 MFMA chains over the same lane-group strips
//     of j, the same sum over the 8 strips, rnn_bwd_epi's (((0 + s0) + s1) + s2) + s3 over the
//     gates and the shared lstm_grads.
#define PKC_RNN_PERSIST
#include "pkc_rnn_impl.h"

namespace pkc {
namespace lstmp {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr int UPW = 16;                   // units (BPTT: columns k) per workgroup
constexpr int ROWS = 16;                  // batch rows of the MFMA tiles (B <= 16)
constexpr int FNW = 8, FNT = 64 * FNW;    // forward: waves / threads per workgroup
constexpr int BNW = 16, BNT = 64 * BNW;   // BPTT: 8 strips x 2 gate pairs
constexpr int BS = 16;                    // BPTT strip per lane group (H = 512: 8 x 4 x 16)
constexpr unsigned SPIN_MAX = 1u << 25;   // polls (s_sleep 1 each) before a wait gives up

// Phase trace (PKC_TRACE measurement builds only; scripts/trace_steps.py --lstm-persist): lane 0
// of every wave of workgroup 0 accumulates the shader-clock cycles of each step phase over the
// loop ([fwd, bwd][wave][8]: five phase sums, then T), read back with
// pkc_trace_read_lstm_persist.  Forward phases: wait, h loads + var, quantise + MFMA + partials,
// cell update + stores, arrive; BPTT: wait, dgates loads + MFMA + partials, gate gradients +
// stores, arrive.
#ifdef PKC_TRACE
__device__ unsigned long long ltrace_buf[2 * BNW * 8];
#define LTR_DECL unsigned long long lt_acc[5] = {0, 0, 0, 0, 0}, lt_last = 0
#define LTR_MARK(i)                                                     \
  do {                                                                  \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();       \
    if ((i) > 0) lt_acc[(i) - 1] += now_ - lt_last;                     \
    lt_last = now_;                                                     \
  } while (0)
#define LTR_STORE(k)                                                    \
  do {                                                                  \
    if (blockIdx.x == 0 && blockIdx.y == 0 && (threadIdx.x & 63) == 0) { \
      volatile unsigned long long* b_ = ltrace_buf + ((k) * BNW + (threadIdx.x >> 6)) * 8; \
      for (int i_ = 0; i_ < 5; ++i_) b_[i_] = lt_acc[i_];               \
      b_[5] = (unsigned long long)T;                                    \
    }                                                                   \
  } while (0)
#else
#define LTR_DECL do { } while (0)
#define LTR_MARK(i) do { } while (0)
#define LTR_STORE(k) do { } while (0)
#endif

// Loads of a handed-off tensor: 16-byte sc1 buffer loads (bypassing this CU's L1; MI355X_MICROARCH
// visibility table, first row) through a raw descriptor over the tensor; an offset past its range
// (OOB, the padding rows >= B) reads zeros without a memory access.
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
constexpr unsigned OOB = 0x80000000u;   // >= the descriptors' num_records
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pub_rsrc(const void* base, int bytes = 0x7fffffff) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
// 8 bf16 of a handed-off bf16 tensor (one 16-byte sc1 load; OOB: zeros)
__device__ __forceinline__ rbf16x8 ld_pub_h8(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(rbf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16));
}
// two adjacent bf16 of a handed-off tensor as ONE 4-byte sc1 store (the visibility table's store
// sizes are 4, 8 and 16 bytes)
__device__ __forceinline__ void st_pub_h2(void* p, float x0, float x1) {
  const unsigned b = (unsigned)__builtin_bit_cast(unsigned short, (__bf16)x0) |
                     ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)x1) << 16);
  __hip_atomic_store((gu32*)p, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ld_pub4(__amdgpu_buffer_rsrc_t r, unsigned off, float* v) {
  const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);   // aux 16: sc1
  v[0] = __uint_as_float(x[0]);
  v[1] = __uint_as_float(x[1]);
  v[2] = __uint_as_float(x[2]);
  v[3] = __uint_as_float(x[3]);
}
__device__ __forceinline__ void st_pub(float* p, float v) {
  __hip_atomic_store((gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup barrier for LDS hand-offs only (no vmcnt drain: loads in flight stay in flight)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The step counter is sharded: NSH counters on 128-byte lines of their own after the launch's
// [counter, timeout] words (ctr + SHW (1 + s)); workgroup b adds its arrivals to shard b % NSH
// (blocks b and b + 8 share an XCD), so no line takes more than 1 / NSH of the grid's atomics
// (one counter serialises them: ≈ 12 ns each, MI355X_MICROARCH.md fanin row), and the poller sums
// every shard (the visibility table's first row: a poll of every shard of a sharded counter).
constexpr int NSH = 8, SHW = 32;
constexpr int CTR_FLOATS = (1 + NSH) * SHW;    // the launch's counter block in work (floats)

// This workgroup's payload of the step is stored: every storing wave drains its stores, then one
// lane (behind the workgroup barrier) adds the workgroup's arrival to its shard
__device__ __forceinline__ void arrive(unsigned* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned b = blockIdx.x + gridDim.x * blockIdx.y;
    __hip_atomic_fetch_add((gu32*)(ctr + SHW * (1 + b % NSH)), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Wait until the shards sum to >= target: wave 0 polls (lane s < NSH loads shard s, the wave sums
// them), the other waves wait at the barrier it then joins.  false on every thread of the
// workgroup when the wait timed out (the timeout word ctr[1] is then set).
__device__ __forceinline__ bool wait_ctr(unsigned* ctr, unsigned target, int* abort_lds) {
  if (threadIdx.x < 64) {
    const int l = threadIdx.x;
    unsigned spins = 0;
    int ab = 0;
    for (;;) {
      unsigned v = l < NSH ? __hip_atomic_load((gu32*)(ctr + SHW * (1 + l)), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0u;
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      const unsigned tot = (unsigned)__builtin_amdgcn_readfirstlane((int)v);   // lanes 0-7's sum
      if (tot >= target) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > SPIN_MAX) {
        if (l == 0) __hip_atomic_store((gu32*)(ctr + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ab = 1;
        break;
      }
    }
    if (l == 0) *abort_lds = ab;
  }
  lds_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // (no instruction: loads stay below)
  return *abort_lds == 0;
}

// The four gates' partial products of this wave's k-range: gate g reads q_{g+1} = Q(q_g), the
// strip re-quantised in place before each gate.  Q is idempotent on most grid values, so once
// Q(q) == q on every element of this wave's strips the later gates read the same q (the per-step
// kernel's `fixed` shortcut, taken one gate earlier here): their integer operands need no second
// quantisation.  Same values either way.  FAST: qin's form (one instance per launch of the step).
template <bool FAST, int KS>
__device__ __forceinline__ void gate_products(float* va, const QParams& qp,
                                              const rbf16x8 (&ub)[4][KS], f32x4 (&part)[4]) {
  rbf16x8 kh[KS], kl[KS];
  bool fixed = false;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    if (!fixed) {
      qsplit_strip<FAST, 8 * KS>(va, qp, kh, kl);
      if (g < 3) {
        bool eq = true;
#pragma unroll
        for (int s = 0; s < 8 * KS; ++s) eq &= qin<FAST>(va[s], qp) == va[s];
        fixed = __all(eq);
      }
    }
    f32x4 h0 = {0.f, 0.f, 0.f, 0.f}, l0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      h0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kh[s], ub[g][s], h0, 0, 0, 0);
      l0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kl[s], ub[g][s], l0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) part[g][i] = __builtin_fmaf(256.f, h0[i], l0[i]) * qp.var_s;
  }
}

// ----------------------------------------------------------------------------------- forward
// KS: 32-wide k-steps per wave (H = 256 KS).  Workgroup wg owns units [16 wg, 16 wg + 16).
template <int KS>
__global__ __launch_bounds__(FNT) void qx_fwd_loop(pkc_rnn_args a) {
  __shared__ float red[FNW][4][ROWS][UPW];     // each wave's four gate tiles of the step
  __shared__ float xm[FNW];                    // per-wave max|h_{t-1}|
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B = a.B, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int u0 = blockIdx.x * UPW;
  const unsigned nwg = gridDim.x;
  const int64_t n = (int64_t)B * H, TBH = (int64_t)T * B * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  // the wave's U fragments for the whole loop: gate g's tile column c = unit u0 + c, k = kw +
  // 32 s + 8 q .. + 7 (the per-step kernel's wave w covers the same k-range)
  const int kw = w * 32 * KS;
  rbf16x8 ub[4][KS];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      ub[g][s] = *reinterpret_cast<const rbf16x8*>(reinterpret_cast<const __bf16*>(a.U_h[g]) +
                                                   (int64_t)(u0 + c) * H + kw + 32 * s + 8 * q);
  // this thread's cell-update element (row r, unit j): its h, c and dropout value in registers
  const bool ep = tid < B * UPW;
  const int r = ep ? tid >> 4 : 0, j = u0 + (tid & 15);
  float hreg = 0.f, creg = 0.f;                // h_init = c_init = 0
  const float mreg = drop_val(a, r, j, B);
  const float qscale = ldexpf(1.f, a.qbits - 1);
  const __amdgpu_buffer_rsrc_t hsr = pub_rsrc(a.hs);
  const unsigned hoff = c < B ? 4u * (c * H + kw + 8 * q) : OOB;    // byte offset in hs[t]
  LTR_DECL;
  for (int t = 0; t < T; ++t) {
    LTR_MARK(0);
    // this step's gate pre-activations (independent of the recurrence: in flight during the wait)
    float wv[4];
    const int64_t pi = ix.pre(t, r, j);
#pragma unroll
    for (int g = 0; g < 4; ++g) wv[g] = a.wpre[g * TBH + pi];
    if (t > 0 && !wait_ctr(ctr, nwg * (unsigned)t, &abort_flag)) return;
    LTR_MARK(1);
    // h_{t-1} = hs[t]: this lane's MFMA A strips (row c; rows >= B are zeros)
    float va[8 * KS];
    const unsigned toff = c < B ? 4u * (unsigned)(t * n) : 0u;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      ld_pub4(hsr, hoff + toff + 128 * s, va + 8 * s);
      ld_pub4(hsr, hoff + toff + 128 * s + 16, va + 8 * s + 4);
    }
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < 8 * KS; ++s) mx = fmaxf(mx, fabsf(va[s]));
    mx = warp_max(mx);
    if (lane == 0) xm[w] = mx;
    lds_barrier();
    // var = max|h_{t-1}| over the whole tensor (the per-step kernel's max over the partials)
    float var = xm[0];
#pragma unroll
    for (int i = 1; i < FNW; ++i) var = fmaxf(var, xm[i]);
    var = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(var)));   // (uniform)
    const QParams qp = qparams(var, qscale);
    const bool qon = var != 0.f;
    LTR_MARK(2);
    f32x4 part[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) part[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (qon) {                                  // (var is wave-uniform: a scalar branch)
      if (qp.fast) gate_products<true, KS>(va, qp, ub, part);
      else gate_products<false, KS>(va, qp, ub, part);
    }
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w][g][4 * q + i][c] = part[g][i];
    lds_barrier();
    LTR_MARK(3);
    if (ep) {
      const int ul = tid & 15;
      float acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        auto p = [&](int v) { return red[v][g][r][ul]; };
        acc[g] = ((p(0) + p(1)) + (p(2) + p(3))) + ((p(4) + p(5)) + (p(6) + p(7)));
      }
      EpiIn e;
#pragma unroll
      for (int g = 0; g < 4; ++g) e.w[g] = wv[g];
      e.hp = hreg;
      e.cp = creg;
      e.m = mreg;
      const float vars[4] = {var, var, var, var};
      float cn = 0.f;
      hreg = fwd_epi<PKC_CELL_LSTM, true, false, true>(a, ix, t, r, j, acc, vars, qscale, e, &cn);
      creg = cn;
      st_pub(a.hs + (int64_t)(t + 1) * n + (int64_t)r * H + j, hreg);   // h_t to every workgroup
    }
    LTR_MARK(4);
    if (t + 1 < T) arrive(ctr);
    LTR_MARK(5);
  }
  LTR_STORE(0);
}

// ----------------------------------------------------------------------------------- BPTT
// dh_tt[r][k] = sum_g sum_j dgates_g[tt + 1][r][j] U_g[j][k] for the workgroup's 16 columns k;
// wave W: strip jr = W % 8 of j (the per-step kernel's wave), gates 2 (W / 8) and 2 (W / 8) + 1.
// SL: the strip per lane group (the per-step 8-wave kernel's S / 2: H / 32).  Bidirectional layers:
// B2 rows (RnnIdx maps the reversed direction's time).
// X3: the products in three bf16 parts per dgates element (d = hi + mid + lo exactly, RNE each;
// U^T on its <= 8-bit grid is exact in bf16) on v_mfma_f32_16x16x32_bf16 with fp32 accumulation —
// every product exact, the sums rounded in another order than the fp32 16x16x4 chains (not
// bit-identical to the per-step launches; tests/test_gpu_lstm_persist.py bounds the difference),
// at 12 instead of 32 MFMA issues per wave and step (the fp32 chains were half of a BPTT step:
// profiles/r06_lstm_persist_trace_c5.json).  !X3: the per-step kernel's fp32 chains, bit-identical.
// gridDim.y > 1: the B rows split over gridDim.y workgroups per column block (ceil(B / y) rows
// each, blockIdx.y = row block): each loads only its rows of dgates_t (C5: 48 of 96 KB per step;
// the payload bounds the step) — the elements' sums are unchanged (rows are independent).
template <bool X3, int SL = BS>
__global__ __launch_bounds__(BNT) void bwd_loop(pkc_rnn_args a) {
  static_assert(!X3 || SL == 16, "X3: two 8-wide bf16 k-steps per strip");
  __shared__ float red[4][8][ROWS][UPW];       // [gate][strip] partial tiles of the step
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B = ix.B2, T = a.T;   // (B: the rows, both directions of a bidirectional layer)
  const int tid = threadIdx.x, lane = tid & 63;
  const int W = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int jr = W & 7, gp = W >> 3;
  const int c = lane & 15, q = lane >> 4;
  const int k0 = blockIdx.x * UPW;
  const int rb = (B + (int)gridDim.y - 1) / (int)gridDim.y;   // rows per workgroup
  const int y0 = rb * (int)blockIdx.y;                          // its first row
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B * H, TB2H = (int64_t)T * B * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  const int kb = (jr * 4 + q) * SL;             // this lane group's strip of j
  // X3: lane group q's 8 j of k-step s at jx + 32 s (the strip's 64 j: 2 bf16 k-steps)
  const int jx = jr * 4 * SL + 8 * q;
  const int jl = X3 ? jx : kb;                  // the first of this lane's (two runs of) 8 / 16 j
  // U^T strips (B operand, column k0 + c) of the wave's two gates, for the whole loop
  float vu[2][SL];
  rbf16x8 uh[2][2];
#pragma unroll
  for (int gg = 0; gg < 2; ++gg) {
    const float* pu = a.ut + (int64_t)(2 * gp + gg) * H * H + (int64_t)(k0 + c) * H;
#pragma unroll
    for (int s = 0; s < SL; s += 4) {
      const int j = X3 ? jx + 32 * (s / 8) + (s % 8) : kb + s;
      const float4 v = *reinterpret_cast<const float4*>(pu + j);
      vu[gg][s] = v.x; vu[gg][s + 1] = v.y; vu[gg][s + 2] = v.z; vu[gg][s + 3] = v.w;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 8; ++i) uh[gg][s][i] = (__bf16)vu[gg][8 * s + i];
  }
  const bool ep = tid < rb * UPW && y0 + (tid >> 4) < B;
  const int r = ep ? y0 + (tid >> 4) : 0, k = k0 + (tid & 15);
  const int64_t e = (int64_t)r * H + k;
  const bool rc = c < rb && y0 + c < B;          // this lane's MFMA row y0 + c is one of ours
  // the carries of step T-1 (rnn_bwd_init, slot 0) and the dropout value
  float gcar = a.work[e], dccar = a.work[2 * n + e];
  const float mreg = drop_val(a, r, k, B);
  const __amdgpu_buffer_rsrc_t dgr = pub_rsrc(a.dgates);
  LTR_DECL;
  for (int tt = T - 2; tt >= 0; --tt) {
    LTR_MARK(0);
    const int t = tt + 1;
    // step tt's saved gates, c_tt, c_{tt-1} and dL/dy_tt: in flight during the wait
    const int64_t si = ix.st(tt, r, k);
    const float f = a.gates[si], ig = a.gates[TB2H + si], o = a.gates[2 * TB2H + si];
    const float cc = a.gates[3 * TB2H + si];
    const float cN = a.cs[(int64_t)(tt + 1) * n + e], cP = a.cs[(int64_t)tt * n + e];
    const float dyv = dy_at(a, ix.out(tt, r, k));
    if (tt < T - 2 && !wait_ctr(ctr, nwg * (unsigned)(T - 2 - tt), &abort_flag)) return;
    LTR_MARK(1);
    // dgates_t strips of the wave's two gates (row c; rows >= B read zeros), both requested
    // before the MFMA chains
    float va[2][SL];
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
      const unsigned off =
          rc ? 4u * (unsigned)((2 * gp + gg) * TB2H + t * n + (int64_t)(y0 + c) * H + jl) : OOB;
#pragma unroll
      for (int s = 0; s < SL; s += 4)
        ld_pub4(dgr, off + 4 * (X3 ? 32 * (s / 8) + (s % 8) : s), va[gg] + s);
    }
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (X3) {
        rbf16x8 ph[3][2];                       // hi, mid, lo parts of the two k-steps
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float x = va[gg][8 * s + i];
            const __bf16 h = (__bf16)x;
            const float r1 = x - (float)h;
            const __bf16 m = (__bf16)r1;
            ph[0][s][i] = h;
            ph[1][s][i] = m;
            ph[2][s][i] = (__bf16)(r1 - (float)m);
          }
#pragma unroll
        for (int p = 2; p >= 0; --p)            // small parts first
#pragma unroll
          for (int s = 0; s < 2; ++s)
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph[p][s], uh[gg][s], acc, 0, 0, 0);
      } else {
#pragma unroll
        for (int s = 0; s < SL; ++s)
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[gg][s], vu[gg][s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) red[2 * gp + gg][jr][4 * q + i][c] = acc[i];
    }
    lds_barrier();
    LTR_MARK(2);
    if (ep) {
      const int kl = tid & 15;
      float dh = 0.f;                           // rnn_bwd_epi: the gate slabs in order
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        auto p = [&](int v) { return red[g][v][r - y0][kl]; };
        dh += ((p(0) + p(1)) + (p(2) + p(3))) + ((p(4) + p(5)) + (p(6) + p(7)));
      }
      const float g = dyv + dh;                 // bwd_step_epi
      float dg[4];
      const float dco = lstm_grads(a.act, f, ig, o, cc, cN, cP, mreg, g, dccar, dg);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) st_pub(a.dgates + q4 * TB2H + si, dg[q4]);
      gcar = g;
      dccar = dco;
    }
    LTR_MARK(3);
    if (tt > 0) arrive(ctr);
    LTR_MARK(4);
    LTR_MARK(5);
  }
  LTR_STORE(1);
  // the carries of step 0 where the per-step form leaves them (slot (T-1) & 1)
  if (ep && T > 1) {
    const int p0 = (T - 1) & 1;
    a.work[p0 * n + e] = gcar;
    a.work[2 * n + p0 * n + e] = dccar;
  }
}

// ------------------------------------------------------------- bf16 step mode (C4's LSTM)
// Dense LSTM with bf16 step products (pkc_rnn_args.step_bf16, no quantised h), B2 <= 32 rows — a
// bidirectional layer's two directions share U (rows >= B run the reversed time, RnnIdx) —
// H = 256 KC, KC in {2, 3, 4}.  The per-step bf16 kernels' partition is kept element for element:
// wave w, lane group q own the contraction strip [(4 w + q) 8 KC, + 8 KC), MFMA i of a chain the 8
// k at + 8 i, two 16-row chains, the waves' partials summed ((0 + 1) + (2 + 3)) + ((4 + 5) +
// (6 + 7)); the handed-off operand is the bf16 copy the per-step kernels read (hs_h, dgates_h),
// stored as pairs of adjacent units.
// RS = 2 / 4 (B2 > 16, C4's 32 rows): the rows are split over RS workgroups per unit block
// (blockIdx.y = row block of 32 / RS rows, RS H / 16 workgroups): each reads and multiplies only
// its rows of the handed-off operand (a 16-row MFMA tile, rows past the block reading zeros
// without a memory access) — 1 / RS of the per-workgroup payload, which bounds the BPTT step
// (≈ 35 GB/s per CU) — and the elements' sums are unchanged (the row chains were independent).
constexpr int R32 = 32;

template <int KC, int RS>
__global__ __launch_bounds__(FNT) void bf_fwd_loop(pkc_rnn_args a, int co) {
  __shared__ float red[FNW][4][R32][UPW];       // each wave's four gate tiles (32 rows)
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int u0 = blockIdx.x * UPW;
  constexpr int RW = RS == 1 ? 32 : 32 / RS;          // rows of this workgroup
  const int y16 = RW * (int)blockIdx.y;                // its first row
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B2 * H, TBH = (int64_t)T * a.B * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  // lane group q's 8-wide chunk i: the per-step kernels' kb + 8 i with kb = (4 w + q) 8 KC
  // (co = 0), or 32 w KC + 8 (4 i + q) (co = 1: a row's four lane groups read 64 contiguous bytes
  // per load instead of four 16-byte pieces 16 KC bytes apart)
  const int kb = co ? 32 * w * KC + 8 * q : (4 * w + q) * 8 * KC;
  const int ks = co ? 32 : 8;                   // elements between chunks i and i + 1
  rbf16x8 ub[4][KC];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int i = 0; i < KC; ++i)
      ub[g][i] = *reinterpret_cast<const rbf16x8*>(reinterpret_cast<const __bf16*>(a.U_h[g]) +
                                                   (int64_t)(u0 + c) * H + kb + ks * i);
  const bool two = RS == 1 && B2 > 16;          // (uniform) the second 16-row chain
  const int r = y16 + (tid >> 4), j = u0 + (tid & 15);   // this thread's cell-update element
  const bool ep = (RS == 1 || tid < RW * UPW) && r < B2;
  const int rr = ep ? r : 0;
  float hreg = 0.f, creg = 0.f;
  const float mreg = drop_val(a, rr, j, B2);
  const __amdgpu_buffer_rsrc_t hr = pub_rsrc(a.hs_h);
  const unsigned oa = 2u * ((y16 + c) * H + kb), ob = 2u * ((16 + c) * H + kb);
  const bool ra = c < RW && y16 + c < B2, rb = 16 + c < B2;
  LTR_DECL;
  for (int t = 0; t < T; ++t) {
    LTR_MARK(0);
    float wv[4];
    const int64_t pi = ix.pre(t, rr, j);
#pragma unroll
    for (int g = 0; g < 4; ++g) wv[g] = a.wpre[g * TBH + pi];
    if (t > 0 && !wait_ctr(ctr, nwg * (unsigned)t, &abort_flag)) return;
    LTR_MARK(1);
    // h_{t-1} (bf16, hs_h[t]): the A operands of both row chains (rows >= B2 read zeros)
    const unsigned to = 2u * (unsigned)(t * n);
    rbf16x8 ha[KC], hb[KC];
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      ha[i] = ld_pub_h8(hr, ra ? oa + to + 2 * ks * i : OOB);
      if constexpr (RS == 1) hb[i] = ld_pub_h8(hr, two && rb ? ob + to + 2 * ks * i : OOB);
    }
    LTR_MARK(2);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha[i], ub[g][i], acc0, 0, 0, 0);
        if (two) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hb[i], ub[g][i], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[w][g][4 * q + i][c] = acc0[i];
        red[w][g][16 + 4 * q + i][c] = acc1[i];
      }
    }
    lds_barrier();
    LTR_MARK(3);
    float h = 0.f;
    if (ep) {
      const int ul = tid & 15;
      float acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        auto p = [&](int v) { return red[v][g][r - y16][ul]; };
        acc[g] = ((p(0) + p(1)) + (p(2) + p(3))) + ((p(4) + p(5)) + (p(6) + p(7)));
      }
      EpiIn e;
#pragma unroll
      for (int g = 0; g < 4; ++g) e.w[g] = wv[g];
      e.hp = hreg;
      e.cp = creg;
      e.m = mreg;
      const float vars[4] = {0.f, 0.f, 0.f, 0.f};
      float cn = 0.f;
      h = fwd_epi<PKC_CELL_LSTM, false, true, true>(a, ix, t, r, j, acc, vars, 1.f, e, &cn);
      hreg = h;
      creg = cn;
      a.hs[(int64_t)(t + 1) * n + (int64_t)r * H + j] = h;
    }
    // the bf16 h_t to every workgroup: units j, j + 1 (lanes l, l ^ 1) in one 4-byte store
    const float hn = __shfl_xor(h, 1, 64);
    if (ep && (tid & 1) == 0)
      st_pub_h2(reinterpret_cast<__bf16*>(a.hs_h) + (int64_t)(t + 1) * n + (int64_t)r * H + j, h, hn);
    LTR_MARK(4);
    if (t + 1 < T) arrive(ctr);
    LTR_MARK(5);
  }
  LTR_STORE(0);
}

// dh_tt[r][k] = sum_g sum_j dgates_g[tt + 1][r][j] U_g[j][k] for the workgroup's 16 columns k:
// wave w owns strip w of j for all four gates (the per-step kernel's wave w of each gate's launch)
template <int KC, int RS>
__global__ __launch_bounds__(FNT) void bf_bwd_loop(pkc_rnn_args a, int co) {
  __shared__ float red[4][FNW][R32][UPW];       // [gate][strip] partial tiles of the step
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int k0 = blockIdx.x * UPW;
  constexpr int RW = RS == 1 ? 32 : 32 / RS;          // rows of this workgroup
  const int y16 = RW * (int)blockIdx.y;                // its first row
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B2 * H, TB2H = (int64_t)T * B2 * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  // lane group q's 8-wide chunk i: the per-step kernels' kb + 8 i with kb = (4 w + q) 8 KC
  // (co = 0), or 32 w KC + 8 (4 i + q) (co = 1: a row's four lane groups read 64 contiguous bytes
  // per load instead of four 16-byte pieces 16 KC bytes apart)
  const int kb = co ? 32 * w * KC + 8 * q : (4 * w + q) * 8 * KC;
  const int ks = co ? 32 : 8;                   // elements between chunks i and i + 1
  // U^T fragments (ut_h[g][k][j], column k0 + c) of the four gates, for the whole loop
  rbf16x8 ub[4][KC];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int i = 0; i < KC; ++i)
      ub[g][i] = *reinterpret_cast<const rbf16x8*>(reinterpret_cast<const __bf16*>(a.ut_h) +
                                                   (int64_t)g * H * H + (int64_t)(k0 + c) * H +
                                                   kb + ks * i);
  const bool two = RS == 1 && B2 > 16;
  const int r = y16 + (tid >> 4), k = k0 + (tid & 15);
  const bool ep = (RS == 1 || tid < RW * UPW) && r < B2;
  const int rr = ep ? r : 0;
  const int64_t e = (int64_t)rr * H + k;
  float gcar = a.work[e], dccar = a.work[2 * n + e];   // step T-1's carries (rnn_bwd_init)
  const float mreg = drop_val(a, rr, k, B2);
  const __amdgpu_buffer_rsrc_t dr = pub_rsrc(a.dgates_h);
  const unsigned oa = 2u * ((y16 + c) * H + kb), ob = 2u * ((16 + c) * H + kb);
  const bool ra = c < RW && y16 + c < B2, rb = 16 + c < B2;
  LTR_DECL;
  for (int tt = T - 2; tt >= 0; --tt) {
    LTR_MARK(0);
    const int t = tt + 1;
    const int64_t si = ix.st(tt, rr, k);
    const float f = a.gates[si], ig = a.gates[TB2H + si], o = a.gates[2 * TB2H + si];
    const float cc = a.gates[3 * TB2H + si];
    const float cN = a.cs[(int64_t)(tt + 1) * n + e], cP = a.cs[(int64_t)tt * n + e];
    const float dyv = dy_at(a, ix.out(tt, rr, k));
    if (tt < T - 2 && !wait_ctr(ctr, nwg * (unsigned)(T - 2 - tt), &abort_flag)) return;
    LTR_MARK(1);
    // dgates_t (bf16) of all four gates requested at once: one memory round trip per step
    rbf16x8 ha[4][KC], hb[4][KC];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const unsigned go = 2u * (unsigned)(g * TB2H + t * n);
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        ha[g][i] = ld_pub_h8(dr, ra ? oa + go + 2 * ks * i : OOB);
        if constexpr (RS == 1) hb[g][i] = ld_pub_h8(dr, two && rb ? ob + go + 2 * ks * i : OOB);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < KC; ++i) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha[g][i], ub[g][i], acc0, 0, 0, 0);
        if (two) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hb[g][i], ub[g][i], acc1, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[g][w][4 * q + i][c] = acc0[i];
        red[g][w][16 + 4 * q + i][c] = acc1[i];
      }
    }
    lds_barrier();
    LTR_MARK(2);
    float dg[4] = {0.f, 0.f, 0.f, 0.f};
    if (ep) {
      const int kl = tid & 15;
      float dh = 0.f;                           // rnn_bwd_epi: the gate slabs in order
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        auto p = [&](int v) { return red[g][v][r - y16][kl]; };
        dh += ((p(0) + p(1)) + (p(2) + p(3))) + ((p(4) + p(5)) + (p(6) + p(7)));
      }
      const float g = dyv + dh;                 // bwd_step_epi
      const float dco = lstm_grads(a.act, f, ig, o, cc, cN, cP, mreg, g, dccar, dg);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) a.dgates[q4 * TB2H + si] = dg[q4];
      gcar = g;
      dccar = dco;
    }
    // the bf16 dgates_tt to every workgroup: columns k, k + 1 (lanes l, l ^ 1) per 4-byte store
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const float dn = __shfl_xor(dg[q4], 1, 64);
      if (ep && (tid & 1) == 0)
        st_pub_h2(reinterpret_cast<__bf16*>(a.dgates_h) + q4 * TB2H + si, dg[q4], dn);
    }
    LTR_MARK(3);
    if (tt > 0) arrive(ctr);
    LTR_MARK(4);
    LTR_MARK(5);
  }
  LTR_STORE(1);
  if (ep && T > 1) {
    const int p0 = (T - 1) & 1;
    a.work[p0 * n + e] = gcar;
    a.work[2 * n + p0 * n + e] = dccar;
  }
}

// ------------------------------------------------------------ fp32 step mode (C4 fp32's LSTM)
// The exact-fp32 step products (no quantised h, no bf16 copies) of a dense LSTM layer, H = 32 SL
// (512-1024), B2 <= 32 rows, in the per-step 8-wave kernel's tile form: workgroup wg owns units
// [16 wg, 16 wg + 16) as four 16-column tiles (column c of tile tl = gate c / 4 of unit
// 16 wg + 4 tl + c % 4, as rnn_fwd_mm lays its NG = 4 tile out) and a block of <= 16 rows
// (blockIdx.y): H / 16 x 2 workgroups for C4.  Lane group q of wave w holds U's fp32 strips
// [(4 w + q) SL, + SL) of its four columns in registers for the whole loop, each row's chain of
// v_mfma_f32_16x16x4_f32 runs the per-step order, the waves' partials are summed in red_sum4's
// order and fwd_epi updates the cell: bit-identical to the per-step launches.  (The first form —
// one tile per workgroup over H / 4 = 256 workgroups — ran 22 us per step: 256 arrivals on one
// counter and 256 readers of the whole 128 KB h_{t-1} per step.)
// h_t (fp32) is handed off as in the other loops.
template <int SL, int TL>
__global__ __launch_bounds__(FNT) void f32_fwd_loop(pkc_rnn_args a) {
  constexpr int NU = 4;                         // units per tile; TL tiles (4 TL units) per workgroup
  __shared__ float red[FNW][TL][ROWS][UPW];     // each wave's partial tiles (16 rows x 16 columns)
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int u0 = blockIdx.x * NU * TL;
  const int rb = (B2 + (int)gridDim.y - 1) / (int)gridDim.y;   // rows per workgroup (<= 16)
  const int y0 = rb * (int)blockIdx.y;
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B2 * H, TBH = (int64_t)T * a.B * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  const int kb = (4 * w + q) * SL;
  // tile tl's column c = gate c / 4 of unit u0 + 4 tl + c % 4 (rnn_fwd_mm's NG = 4 tile layout)
  float ub[TL][SL];
#pragma unroll
  for (int tl = 0; tl < TL; ++tl) {
    const float* pu = a.U[c / NU] + (int64_t)(u0 + NU * tl + c % NU) * H + kb;
#pragma unroll
    for (int s4 = 0; s4 < SL; s4 += 4) {
      const float4 v = *reinterpret_cast<const float4*>(pu + s4);
      ub[tl][s4] = v.x; ub[tl][s4 + 1] = v.y; ub[tl][s4 + 2] = v.z; ub[tl][s4 + 3] = v.w;
    }
  }
  // this thread's cell-update element: row y0 + tid / (4 TL), unit u0 + tid % (4 TL)
  const int r = y0 + tid / (NU * TL), j = u0 + tid % (NU * TL);
  const bool ep = tid < rb * NU * TL && r < B2;
  const int rr = ep ? r : 0;
  float hreg = 0.f, creg = 0.f;
  const float mreg = drop_val(a, rr, j, B2);
  const __amdgpu_buffer_rsrc_t hr = pub_rsrc(a.hs);
  const bool ra = c < rb && y0 + c < B2;
  const unsigned oa = 4u * ((y0 + c) * H + kb);
  LTR_DECL;
  for (int t = 0; t < T; ++t) {
    LTR_MARK(0);
    float wv[4];
    const int64_t pi = ix.pre(t, rr, j);
#pragma unroll
    for (int g = 0; g < 4; ++g) wv[g] = a.wpre[g * TBH + pi];
    if (t > 0 && !wait_ctr(ctr, nwg * (unsigned)t, &abort_flag)) return;
    LTR_MARK(1);
    // h_{t-1} (hs[t]): this lane's A strip (row y0 + c; rows outside the block read zeros)
    const unsigned to = 4u * (unsigned)(t * n);
    float va[SL];
#pragma unroll
    for (int m = 0; m < SL / 4; ++m) ld_pub4(hr, ra ? oa + to + 16 * m : OOB, va + 4 * m);
    LTR_MARK(2);
#pragma unroll
    for (int tl = 0; tl < TL; ++tl) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < SL; ++s2)             // mfma_chain's order
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[s2], ub[tl][s2], acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w][tl][4 * q + i][c] = acc[i];
    }
    lds_barrier();
    LTR_MARK(3);
    if (ep) {
      const int tl = (tid % (NU * TL)) / NU, ul = tid % NU;
      float acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        auto p = [&](int v) { return red[v][tl][r - y0][NU * g + ul]; };
        acc[g] = ((p(0) + p(1)) + (p(2) + p(3))) + ((p(4) + p(5)) + (p(6) + p(7)));
      }
      EpiIn e;
#pragma unroll
      for (int g = 0; g < 4; ++g) e.w[g] = wv[g];
      e.hp = hreg;
      e.cp = creg;
      e.m = mreg;
      const float vars[4] = {0.f, 0.f, 0.f, 0.f};
      float cn = 0.f;
      hreg = fwd_epi<PKC_CELL_LSTM, false, false, true>(a, ix, t, r, j, acc, vars, 1.f, e, &cn);
      creg = cn;
      st_pub(a.hs + (int64_t)(t + 1) * n + (int64_t)r * H + j, hreg);   // h_t to every workgroup
    }
    LTR_MARK(4);
    if (t + 1 < T) arrive(ctr);
    LTR_MARK(5);
  }
  LTR_STORE(0);
}

// BPTT of the same mode: dh_tt[r][k] = sum_g sum_j dgates_g[tt + 1][r][j] U_g[j][k] for the
// workgroup's 16 columns k and <= 16 rows (blockIdx.y: row block); wave w owns the per-step 8-wave
// kernel's strip w of j for ALL four gates (U^T strips: 4 SL registers; 16 waves of two gates each
// would leave 128 registers a wave for 4 SL + 2 SL), each gate's fp32 chain in the per-step order,
// the gates' dgates_t loaded two at a time (the next gate's strips in flight during a chain), the
// 8 strips summed as red_sum<8>, the gates as rnn_bwd_epi, then lstm_grads: bit-identical.
template <int SL>
__global__ __launch_bounds__(FNT) void f32_bwd_loop(pkc_rnn_args a) {
  __shared__ float red[4][FNW][ROWS][UPW];      // [gate][strip] partial tiles of the step
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B = ix.B2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int k0 = blockIdx.x * UPW;
  const int rb = (B + (int)gridDim.y - 1) / (int)gridDim.y;   // rows per workgroup (<= 16)
  const int y0 = rb * (int)blockIdx.y;
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B * H, TB2H = (int64_t)T * B * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  const int kb = (4 * w + q) * SL;
  float vu[4][SL];                              // U^T strips (ut[g][k0 + c][kb ..]) of the loop
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float* pu = a.ut + (int64_t)g * H * H + (int64_t)(k0 + c) * H + kb;
#pragma unroll
    for (int s4 = 0; s4 < SL; s4 += 4) {
      const float4 v = *reinterpret_cast<const float4*>(pu + s4);
      vu[g][s4] = v.x; vu[g][s4 + 1] = v.y; vu[g][s4 + 2] = v.z; vu[g][s4 + 3] = v.w;
    }
  }
  const bool ep = tid < rb * UPW && y0 + (tid >> 4) < B;
  const int r = ep ? y0 + (tid >> 4) : 0, k = k0 + (tid & 15);
  const int64_t e = (int64_t)r * H + k;
  const bool rc = c < rb && y0 + c < B;         // this lane's MFMA row y0 + c is one of ours
  float gcar = a.work[e], dccar = a.work[2 * n + e];   // step T-1's carries (rnn_bwd_init)
  const float mreg = drop_val(a, r, k, B);
  const __amdgpu_buffer_rsrc_t dgr = pub_rsrc(a.dgates);
  const unsigned lo = 4u * (unsigned)((int64_t)(y0 + c) * H + kb);   // this lane's strip in a slab
  LTR_DECL;
  for (int tt = T - 2; tt >= 0; --tt) {
    LTR_MARK(0);
    const int t = tt + 1;
    const int64_t si = ix.st(tt, r, k);
    const float f = a.gates[si], ig = a.gates[TB2H + si], o = a.gates[2 * TB2H + si];
    const float cc = a.gates[3 * TB2H + si];
    const float cN = a.cs[(int64_t)(tt + 1) * n + e], cP = a.cs[(int64_t)tt * n + e];
    const float dyv = dy_at(a, ix.out(tt, r, k));
    if (tt < T - 2 && !wait_ctr(ctr, nwg * (unsigned)(T - 2 - tt), &abort_flag)) return;
    LTR_MARK(1);
    float va[2][SL];
    auto ld_gate = [&](int g, float* v) {
      const unsigned off = 4u * (unsigned)(g * TB2H + t * n) + lo;
#pragma unroll
      for (int m = 0; m < SL / 4; ++m) ld_pub4(dgr, rc ? off + 16 * m : OOB, v + 4 * m);
    };
    ld_gate(0, va[0]);
    ld_gate(1, va[1]);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < SL; ++s2)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[g & 1][s2], vu[g][s2], acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) red[g][w][4 * q + i][c] = acc[i];
      if (g + 2 < 4) {
        // the chain has read its strips: reuse them for gate g + 2 (kept below the chain, so at
        // most two gates' strips are live)
        asm volatile("" ::"v"(acc) : "memory");
        ld_gate(g + 2, va[g & 1]);
      }
    }
    lds_barrier();
    LTR_MARK(2);
    if (ep) {
      const int kl = tid & 15;
      float dh = 0.f;                           // rnn_bwd_epi: the gate slabs in order
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        auto p = [&](int v) { return red[g][v][r - y0][kl]; };
        dh += ((p(0) + p(1)) + (p(2) + p(3))) + ((p(4) + p(5)) + (p(6) + p(7)));
      }
      const float g = dyv + dh;                 // bwd_step_epi
      float dg[4];
      const float dco = lstm_grads(a.act, f, ig, o, cc, cN, cP, mreg, g, dccar, dg);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) st_pub(a.dgates + q4 * TB2H + si, dg[q4]);
      gcar = g;
      dccar = dco;
    }
    LTR_MARK(3);
    if (tt > 0) arrive(ctr);
    LTR_MARK(4);
    LTR_MARK(5);
  }
  LTR_STORE(1);
  if (ep && T > 1) {
    const int p0 = (T - 1) & 1;
    a.work[p0 * n + e] = gcar;
    a.work[2 * n + p0 * n + e] = dccar;
  }
}

// The same BPTT with the step's dgates_t staged through LDS (f32_bwd_lds): 8-row blocks
// (blockIdx.y; 4 H / 16 workgroups for C4), the block's rows of all four gates (4 x 8 x H fp32,
// 128 KB at H = 1024) loaded in ONE round trip — 16-byte sc1 loads to registers, every lane 16 of
// them, then written to LDS — instead of f32_bwd_loop's two dependent round trips (its registers
// hold only two gates' strips beside the four gates' U^T).  The chains read their A strips from
// LDS: same operands, same order, bit-identical.  LDS rows padded by 4 floats.
constexpr int LRB = 8;                          // rows per workgroup
template <int SL>
__global__ __launch_bounds__(FNT) void f32_bwd_lds(pkc_rnn_args a) {
  constexpr int H_ = 32 * SL, LS = H_ + 4;       // (H is 32 SL by the dispatch)
  constexpr int NCH = 4 * LRB * H_ / 4;          // 16-byte chunks of the staged block
  static_assert(NCH % FNT == 0, "chunks per thread");
  constexpr int CPT = NCH / FNT;
  __shared__ __attribute__((aligned(16))) float stg[4 * LRB * LS];
  __shared__ float red[4][FNW][LRB][UPW];
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = H_, B = ix.B2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int k0 = blockIdx.x * UPW;
  const int y0 = LRB * (int)blockIdx.y;
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B * H, TB2H = (int64_t)T * B * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  const int kb = (4 * w + q) * SL;
  float vu[4][SL];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float* pu = a.ut + (int64_t)g * H * H + (int64_t)(k0 + c) * H + kb;
#pragma unroll
    for (int s4 = 0; s4 < SL; s4 += 4) {
      const float4 v = *reinterpret_cast<const float4*>(pu + s4);
      vu[g][s4] = v.x; vu[g][s4 + 1] = v.y; vu[g][s4 + 2] = v.z; vu[g][s4 + 3] = v.w;
    }
  }
  const bool ep = tid < LRB * UPW && y0 + (tid >> 4) < B;
  const int r = ep ? y0 + (tid >> 4) : 0, k = k0 + (tid & 15);
  const int64_t e = (int64_t)r * H + k;
  float gcar = a.work[e], dccar = a.work[2 * n + e];
  const float mreg = drop_val(a, r, k, B);
  const __amdgpu_buffer_rsrc_t dgr = pub_rsrc(a.dgates);
  // this thread's chunks: chunk i = tid + FNT m -> gate i / (LRB H / 4), row (i / (H / 4)) % LRB,
  // 4 floats at 4 (i % (H / 4)); rows past B read zeros
  unsigned goff[CPT];
  int soff[CPT];
#pragma unroll
  for (int m = 0; m < CPT; ++m) {
    const int i = tid + FNT * m;
    const int g = i / (LRB * H_ / 4), row = (i / (H_ / 4)) % LRB, k4 = i % (H_ / 4);
    goff[m] = y0 + row < B ? 4u * (unsigned)(g * TB2H + (int64_t)(y0 + row) * H + 4 * k4) : OOB;
    soff[m] = (g * LRB + row) * LS + 4 * k4;
  }
  const bool rc = c < LRB;                      // MFMA rows >= 8: zeros
  const float* arow = stg + (c & (LRB - 1)) * LS + kb;
  LTR_DECL;
  for (int tt = T - 2; tt >= 0; --tt) {
    LTR_MARK(0);
    const int t = tt + 1;
    const int64_t si = ix.st(tt, r, k);
    const float f = a.gates[si], ig = a.gates[TB2H + si], o = a.gates[2 * TB2H + si];
    const float cc = a.gates[3 * TB2H + si];
    const float cN = a.cs[(int64_t)(tt + 1) * n + e], cP = a.cs[(int64_t)tt * n + e];
    const float dyv = dy_at(a, ix.out(tt, r, k));
    if (tt < T - 2 && !wait_ctr(ctr, nwg * (unsigned)(T - 2 - tt), &abort_flag)) return;
    LTR_MARK(1);
    const unsigned to = 4u * (unsigned)(t * n);
    u32x4 st[CPT];
#pragma unroll
    for (int m = 0; m < CPT; ++m)
      st[m] = __builtin_amdgcn_raw_buffer_load_b128(dgr, (int)(goff[m] == OOB ? OOB : goff[m] + to), 0, 16);
#pragma unroll
    for (int m = 0; m < CPT; ++m) *reinterpret_cast<u32x4*>(stg + soff[m]) = st[m];
    lds_barrier();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float va[SL];
#pragma unroll
      for (int s4 = 0; s4 < SL; s4 += 4) {
        const float4 v = *reinterpret_cast<const float4*>(arow + g * LRB * LS + s4);
        va[s4] = rc ? v.x : 0.f; va[s4 + 1] = rc ? v.y : 0.f;
        va[s4 + 2] = rc ? v.z : 0.f; va[s4 + 3] = rc ? v.w : 0.f;
      }
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < SL; ++s2)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(va[s2], vu[g][s2], acc, 0, 0, 0);
      if (q < 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) red[g][w][4 * q + i][c] = acc[i];
      }
    }
    lds_barrier();
    LTR_MARK(2);
    if (ep) {
      const int kl = tid & 15;
      float dh = 0.f;                           // rnn_bwd_epi: the gate slabs in order
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        auto p = [&](int v) { return red[g][v][r - y0][kl]; };
        dh += ((p(0) + p(1)) + (p(2) + p(3))) + ((p(4) + p(5)) + (p(6) + p(7)));
      }
      const float g = dyv + dh;                 // bwd_step_epi
      float dg[4];
      const float dco = lstm_grads(a.act, f, ig, o, cc, cN, cP, mreg, g, dccar, dg);
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) st_pub(a.dgates + q4 * TB2H + si, dg[q4]);
      gcar = g;
      dccar = dco;
    }
    LTR_MARK(3);
    if (tt > 0) arrive(ctr);
    LTR_MARK(4);
    LTR_MARK(5);
  }
  LTR_STORE(1);
  if (ep && T > 1) {
    const int p0 = (T - 1) & 1;
    a.work[p0 * n + e] = gcar;
    a.work[2 * n + p0 * n + e] = dccar;
  }
}

// ----------------------------------------------------------- liGRU, exact-fp32 step mode (C3 fp32)
// The same grid-synchronised form for a liGRU layer whose step products stay fp32 (the parity
// mode; neural_networks.py:1573-1584): the units (BPTT: columns k) dealt to ceil(H / 16)
// workgroups of 16 waves, each holding its units' fp32 U rows of both gates (BPTT: Uᵀ columns)
// as v_mfma_f32_16x16x4_f32 B operands in registers; lane group q of wave w owns the contraction
// strip [(4 w + q) GK, + GK) (k >= H reads zeros), h_{t-1} / dgates_t handed off as in the LSTM
// loops (write-through stores, step counter).  B2 <= 16 rows (C3: both directions of B = 8).  The
// waves' partials are summed in the per-step kernels' red_sum order.  Two shapes: H <= 256 runs
// the per-step kernels' own 4-wave x 16-element strips (GW = 4, GK = 16), so for a dense U the
// loops are bit-identical to the per-step launches; 256 < H <= 768 runs 16 waves x 12 elements
// (C3's H = 550: 12 MFMAs per wave and step, not 16).  A block-sparse U multiplies as dense (its
// masked entries are exact zeros): the fp32 sums of the per-step block-sparse launches in another
// order.
constexpr int GKMAX = 768;             // largest H (16 x 4 x 12)

// GK consecutive floats of row `row` from k0 of a handed-off (rows x H) matrix at byte offset
// base: GK / 4 16-byte sc1 loads (rows >= nrows: out of range, zeros), elements k >= H zeroed
template <int GK>
__device__ __forceinline__ void ld_strip(__amdgpu_buffer_rsrc_t r, unsigned base, int row,
                                           int nrows, int H, int k0, float* v) {
  const bool ok = row < nrows;
  const unsigned off = ok ? base + 4u * (unsigned)(row * H + k0) : OOB;
#pragma unroll
  for (int m = 0; m < GK / 4; ++m) ld_pub4(r, off + 16 * m, v + 4 * m);
#pragma unroll
  for (int s = 0; s < GK; ++s) v[s] = k0 + s < H ? v[s] : 0.f;
}

// Forward: workgroup wg owns units [8 wg, 8 wg + 8): ONE 16-column MFMA tile holds both gates
// (column c: gate c / 8, unit 8 wg + c % 8), so a wave runs 12 MFMAs per step, not 24.
// Both loops: gridDim.y > 1 splits the B2 rows over that many workgroups per unit (column) block
// (ceil(B2 / y) rows each, blockIdx.y = row block): each loads only its rows of the handed-off
// h_{t-1} / dgates_t (MFMA rows past the block read zeros without a memory access); the elements'
// sums are unchanged (rows are independent).
constexpr int LUPW = 8;                // forward units per workgroup
template <int GW, int GK>
__global__ __launch_bounds__(64 * GW) void lg_fwd_loop(pkc_rnn_args a) {
  __shared__ float red[GW][ROWS][UPW];         // each wave's tile of the step
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int u0 = blockIdx.x * LUPW;
  const int rb = (B2 + (int)gridDim.y - 1) / (int)gridDim.y, y0 = rb * (int)blockIdx.y;
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B2 * H, TBH = (int64_t)T * a.B * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  const int kl = (4 * w + q) * GK;
  // B[k][column c] = U_{c / 8}[unit u0 + c % 8][k] over this lane's strip
  float ub[GK];
  const int uu = u0 + (c & 7);
  const float* Ug = a.U[c >> 3];
#pragma unroll
  for (int s = 0; s < GK; ++s) ub[s] = uu < H && kl + s < H ? Ug[(int64_t)uu * H + kl + s] : 0.f;
  const int r = y0 + (tid >> 3), j = u0 + (tid & 7);    // this thread's cell-update element
  const bool ep = tid < rb * LUPW && r < B2 && j < H;
  const int rr = ep ? r : 0, jj = ep ? j : 0;
  float hreg = 0.f;
  const float mreg = drop_val(a, rr, jj, B2);
  // (the descriptor spans hs exactly: a strip's tail past the last row reads zeros, not past it)
  const __amdgpu_buffer_rsrc_t hr = pub_rsrc(a.hs, (int)(4 * (T + 1) * n));
  LTR_DECL;
  for (int t = 0; t < T; ++t) {
    LTR_MARK(0);
    float wv[2];
    const int64_t pi = ix.pre(t, rr, jj);
#pragma unroll
    for (int g = 0; g < 2; ++g) wv[g] = a.wpre[g * TBH + pi];
    if (t > 0 && !wait_ctr(ctr, nwg * (unsigned)t, &abort_flag)) return;
    LTR_MARK(1);
    float hv[GK];
    ld_strip<GK>(hr, 4u * (unsigned)(t * n), c < rb ? y0 + c : B2, B2, H, kl, hv);
    LTR_MARK(2);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < GK; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s], ub[s], acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][4 * q + i][c] = acc[i];
    lds_barrier();
    LTR_MARK(3);
    if (ep) {
      const int ul = tid & 7;
      float acc2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        auto p = [&](int v) { return red[v][r - y0][8 * g + ul]; };
        float v = (p(0) + p(1)) + (p(2) + p(3));          // red_sum's order
#pragma unroll
        for (int w4 = 4; w4 < GW; w4 += 4) v += (p(w4) + p(w4 + 1)) + (p(w4 + 2) + p(w4 + 3));
        acc2[g] = v;
      }
      EpiIn e;
      e.w[0] = wv[0];
      e.w[1] = wv[1];
      e.w[2] = e.w[3] = 0.f;
      e.hp = hreg;
      e.cp = 0.f;
      e.m = mreg;
      const float vars[4] = {0.f, 0.f, 0.f, 0.f};
      hreg = fwd_epi<PKC_CELL_LIGRU, false, false, true>(a, ix, t, r, j, acc2, vars, 1.f, e);
      st_pub(a.hs + (int64_t)(t + 1) * n + (int64_t)r * H + j, hreg);   // h_t to every workgroup
    }
    LTR_MARK(4);
    if (t + 1 < T) arrive(ctr);
    LTR_MARK(5);
  }
  LTR_STORE(0);
}

// dh_tt[r][k] = sum_g sum_j dgates_g[tt + 1][r][j] U_g[j][k] for the workgroup's 16 columns k, then
// the liGRU gate gradients of step tt (bwd_step_epi + gate_grads, CELL_LIGRU)
template <int GW, int GK>
__global__ __launch_bounds__(64 * GW) void lg_bwd_loop(pkc_rnn_args a) {
  __shared__ float red[GW][2][ROWS][UPW];
  __shared__ int abort_flag;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2, T = a.T;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, q = lane >> 4;
  const int k0 = blockIdx.x * UPW;
  const int rb = (B2 + (int)gridDim.y - 1) / (int)gridDim.y, y0 = rb * (int)blockIdx.y;
  const unsigned nwg = gridDim.x * gridDim.y;
  const int64_t n = (int64_t)B2 * H, TB2H = (int64_t)T * B2 * H;
  unsigned* ctr = reinterpret_cast<unsigned*>(a.work + 4 * n);
  const int jl = (4 * w + q) * GK;
  // Uᵀ columns (B[j][k] = U_g[j][k] = ut[g][k][j]) over this lane's strip of j
  float ub[2][GK];
  const int kk = k0 + c;
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int s = 0; s < GK; ++s)
      ub[g][s] = kk < H && jl + s < H ? a.ut[(int64_t)g * H * H + (int64_t)kk * H + jl + s] : 0.f;
  const int r = y0 + (tid >> 4), k = k0 + (tid & 15);
  const bool ep = tid < rb * UPW && r < B2 && k < H;
  const int rr = ep ? r : 0, ke = ep ? k : 0;
  const int64_t e = (int64_t)rr * H + ke;
  float gcar = a.work[e];                       // g_{T-1} (rnn_bwd_init, slot 0)
  const float mreg = drop_val(a, rr, ke, B2);
  const __amdgpu_buffer_rsrc_t dgr = pub_rsrc(a.dgates, (int)(4 * 2 * TB2H));
  LTR_DECL;
  for (int tt = T - 2; tt >= 0; --tt) {
    LTR_MARK(0);
    const int t = tt + 1;
    // step tt's saved state and dL/dy, z_t of the carry term: in flight during the wait
    const int64_t si = ix.st(tt, rr, ke);
    const float z = a.gates[si], hcr = a.gates[TB2H + si];
    const float hp = a.hs[(int64_t)tt * n + e];
    const float zt = a.gates[ix.st(t, rr, ke)];
    const float dyv = dy_at(a, ix.out(tt, rr, ke));
    if (tt < T - 2 && !wait_ctr(ctr, nwg * (unsigned)(T - 2 - tt), &abort_flag)) return;
    LTR_MARK(1);
    float dv[2][GK];
#pragma unroll
    for (int g = 0; g < 2; ++g)
      ld_strip<GK>(dgr, 4u * (unsigned)(g * TB2H + t * n), c < rb ? y0 + c : B2, B2, H, jl, dv[g]);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < GK; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dv[g][s], ub[g][s], acc, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w][g][4 * q + i][c] = acc[i];
    }
    lds_barrier();
    LTR_MARK(2);
    if (ep) {
      const int kl = tid & 15;
      float dh = 0.f;                           // rnn_bwd_epi: the gate slabs in order
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        auto p = [&](int v) { return red[v][g][r - y0][kl]; };
        float v = (p(0) + p(1)) + (p(2) + p(3));          // red_sum's order
#pragma unroll
        for (int w4 = 4; w4 < GW; w4 += 4) v += (p(w4) + p(w4 + 1)) + (p(w4 + 2) + p(w4 + 3));
        dh += v;
      }
      dh = ligru_carry(dh, gcar, zt);           // bwd_step_epi: + g_t * z_t
      const float g = dyv + dh;
      float dg[2];
      ligru_grads(a.act, g, z, hcr, hp, mreg, dg);
      st_pub(a.dgates + si, dg[0]);
      st_pub(a.dgates + TB2H + si, dg[1]);
      gcar = g;
    }
    LTR_MARK(3);
    if (tt > 0) arrive(ctr);
    LTR_MARK(4);
    LTR_MARK(5);
  }
  LTR_STORE(1);
  if (ep && T > 1) a.work[((T - 1) & 1) * n + e] = gcar;   // step 0's carry where the per-step form leaves it
}

}  // namespace lstmp

static int device_cus();

bool rnn_lstm_persist_ok(const pkc_rnn_args* a, bool bwd) {
  const char* env = getenv("PKC_RNN_LSTM_PERSIST");   // "0": the per-step launches (A/B, tests)
  if (env && env[0] == '0') return false;
  if (a->cell != PKC_CELL_LSTM || a->ln_gamma || a->kmap_fwd || a->kmap_bwd || !a->work) return false;
  if (a->H / lstmp::UPW > device_cus()) return false;   // (every workgroup resident: one per CU)
  if ((int64_t)4 * (a->bidir ? 2 * a->B : a->B) * a->H < lstmp::CTR_FLOATS) return false;
  const int64_t B2 = a->bidir ? 2 * a->B : a->B;
  // byte offsets of the 16-byte payload loads (dgates: G x T x B2 x H floats) below the
  // descriptors' 2^31 - 16 range
  if ((int64_t)a->T * B2 * a->H * 4 * 4 >= (1ll << 31) - 64) return false;
  if (a->qh_exact) {                            // QX: quantised h, fp32 BPTT products
    if (a->bidir || a->qbits <= 0 || a->step_bf16 || a->B > lstmp::ROWS) return false;
    if (bwd) return a->H == 512 && a->dgates && a->ut;
    return a->H % 256 == 0 && a->H >= 512 && a->H <= 1024 && a->U_h[0] && a->U_h[1] &&
           a->U_h[2] && a->U_h[3] && a->hq;
  }
  if (a->step_bf16 && a->qbits <= 0) {          // bf16 step products
    if (B2 > lstmp::R32 || a->H % 256 || a->H < 512 || a->H > 1024 || !a->hs_h) return false;
    if (bwd) return a->dgates && a->ut_h && a->dgates_h;
    return a->U_h[0] && a->U_h[1] && a->U_h[2] && a->U_h[3];
  }
  if (a->qbits <= 0) {                          // exact fp32 step products (C4 fp32)
    const char* f32 = getenv("PKC_RNN_LSTM_F32");   // "0": the per-step launches
    if (f32 && f32[0] == '0') return false;
    if (B2 > lstmp::R32 || a->H % 256 || a->H < 512 || a->H > 1024) return false;
    if (a->H / 16 * ((B2 + 15) / 16) > device_cus()) return false;   // (co-residency)
    if (bwd) return a->dgates && a->ut;
    return a->U[0] && a->U[1] && a->U[2] && a->U[3];
  }
  return false;
}

// bf16 loops' contraction chunking (bf_fwd_loop / bf_bwd_loop `co`): the coalesced chunking by
// default (C4 bf16 19.9-20.0 vs 20.9-21.0 us per step-layer, same box; the bf16 sums of an
// element in another grouping: tests/test_gpu_steps.py holds every time step to the oracle), the
// per-step kernels' chunking with PKC_RNN_LSTM_CO=0 (bit-identical to the per-step launches)
static int lstm_bf16_coalesced() {
  const char* v = getenv("PKC_RNN_LSTM_CO");
  return v && v[0] == '0' ? 0 : 1;
}

// Compute units of the current device: a grid-synchronised loop needs every workgroup resident at
// once, and these workgroups (512-1024 threads, large register files) are sized for one per CU, so
// a row split is only taken while the whole grid still fits one workgroup per CU.
static int device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    return 256;
  return n;
}
// the largest of rs, rs / 2, ..., 1 whose grid (base workgroups x split) fits the device
static int fit_split(int rs, int base) {
  const int cus = device_cus();
  while (rs > 1 && base * rs > cus) rs = rs > 2 ? rs - 1 : 1;
  return rs;
}

// bf16 loops with more than 16 rows (C4: 2 x 16): the workgroups per unit block the rows are
// split over (PKC_RNN_LSTM_RS = 1, 2 or 4 for the forward loop, default 2; 1 keeps both 16-row
// chains in one workgroup; PKC_RNN_LSTM_RS_BWD for the BPTT loop, default 4)
static int lstm_bf16_rows_split(const pkc_rnn_args* a, bool bwd = false) {
  auto knob = [](const char* name, int dflt) {
    const char* v = getenv(name);
    const int x = v ? atoi(v) : dflt;
    return x == 1 || x == 2 || x == 4 ? x : dflt;
  };
  static const int rs = knob("PKC_RNN_LSTM_RS", 2);
  // (the BPTT's default is 4 row blocks: with the sharded step counter the 256-workgroup BPTT
  // measured 13.56 vs 14.83-14.89 us per step-layer at C4, profiles/r06_c4_bf16_bwd_rows_split_ab.txt)
  static const int rsb = knob("PKC_RNN_LSTM_RS_BWD", 4);
  if ((a->bidir ? 2 * a->B : a->B) <= 16) return 1;
  const int r = fit_split(bwd ? rsb : rs, a->H / lstmp::UPW);
  return r == 3 ? 2 : r;                        // (the bf16 loops take 1, 2 or 4)
}

// QX BPTT loop: workgroups per column block the B rows are split over (PKC_RNN_LSTM_QX_RS, default
// 4 when B > 8 — with the sharded counter 13.61-13.66 against 14.00 us per step-layer for 2 at C5,
// profiles/r06_c5_qx_bwd_rows_split_sharded_ab.txt; 1: all rows in one workgroup)
static int lstm_qx_bwd_rows_split(const pkc_rnn_args* a) {
  static const int rs = [] {
    const char* v = getenv("PKC_RNN_LSTM_QX_RS");
    const int x = v ? atoi(v) : 4;
    return x >= 1 && x <= 4 ? x : 4;
  }();
  return a->B > 8 ? fit_split(rs, a->H / lstmp::UPW) : 1;
}

// liGRU exact-fp32 step mode in the grid-synchronised loops (lg_fwd_loop / lg_bwd_loop)
bool rnn_ligru_grid_ok(const pkc_rnn_args* a, bool bwd) {
  const char* env = getenv("PKC_RNN_LIGRU_GRID");     // "0": the per-step launches
  if (env && env[0] == '0') return false;
  const int64_t B2 = a->bidir ? 2 * a->B : a->B;
  if (a->cell != PKC_CELL_LIGRU || a->step_bf16 || a->qbits > 0 || a->ln_gamma || !a->work ||
      B2 > lstmp::ROWS || a->H > lstmp::GKMAX)
    return false;
  if ((int64_t)a->T * B2 * a->H * 2 * 4 >= (1ll << 31) - 64) return false;
  if ((a->H + lstmp::LUPW - 1) / lstmp::LUPW > device_cus()) return false;   // (co-residency)
  if (4 * B2 * a->H < lstmp::CTR_FLOATS) return false;   // (the sharded counters in work[4n, 8n))
  return bwd ? (a->dgates && a->ut) : true;
}

// fp32 LSTM BPTT loop: row blocks per column block (each <= 16 rows, the MFMA tile;
// PKC_RNN_LSTM_F32_RS raises the count, e.g. 4 for 8-row blocks), bounded by co-residency
static int lstm_f32_bwd_rows_split(const pkc_rnn_args* a, int B2) {
  static const int rs = [] {
    const char* v = getenv("PKC_RNN_LSTM_F32_RS");
    const int x = v ? atoi(v) : 0;
    return x >= 1 && x <= 4 ? x : 0;
  }();
  const int need = (B2 + lstmp::ROWS - 1) / lstmp::ROWS;
  const int want = rs > need ? rs : need;
  const int r = fit_split(want, a->H / lstmp::UPW);
  return r < need ? need : r;
}

// fp32 LSTM forward loop: 16-column tiles per workgroup (PKC_RNN_LSTM_F32_TL = 2 or 4), 2 only
// while the grid (H / 8 x row blocks) keeps one workgroup per CU
static int lstm_f32_fwd_tiles(const pkc_rnn_args* a, int row_blocks) {
  static const int tl = [] {
    const char* v = getenv("PKC_RNN_LSTM_F32_TL");
    return v && atoi(v) == 2 ? 2 : 4;
  }();
  return tl == 2 && a->H / 8 * row_blocks <= device_cus() ? 2 : 4;
}

// fp32 LSTM BPTT with the dgates block staged in LDS (f32_bwd_lds; PKC_RNN_LSTM_F32_LDS=0: the
// register form f32_bwd_loop), when its 8-row blocks keep the grid at one workgroup per CU
static bool lstm_f32_bwd_lds(const pkc_rnn_args* a) {
  static const bool on = [] {
    const char* v = getenv("PKC_RNN_LSTM_F32_LDS");
    return !(v && v[0] == '0');
  }();
  const int B2 = a->bidir ? 2 * a->B : a->B;
  return on && a->H / lstmp::UPW * ((B2 + lstmp::LRB - 1) / lstmp::LRB) <= device_cus();
}

// liGRU grid loops: workgroups per unit block the B2 rows are split over (PKC_RNN_LIGRU_GRID_RS,
// default 2 when B2 > 8; 1: all rows in one workgroup)
static int ligru_grid_rows_split(const pkc_rnn_args* a) {
  static const int rs = [] {
    const char* v = getenv("PKC_RNN_LIGRU_GRID_RS");
    const int x = v ? atoi(v) : 2;
    return x >= 1 && x <= 4 ? x : 2;
  }();
  // (the forward's unit blocks are the larger grid: ceil(H / 8))
  return (a->bidir ? 2 * a->B : a->B) > 8 ? fit_split(rs, (a->H + lstmp::LUPW - 1) / lstmp::LUPW) : 1;
}

static int lstm_ctr_reset(const pkc_rnn_args* a, hipStream_t s) {
  const int64_t B2 = a->bidir ? 2 * a->B : a->B;
  PKC_HIP_CHECK(hipMemsetAsync(a->work + 4 * B2 * a->H, 0, sizeof(float) * lstmp::CTR_FLOATS, s),
                "pkc_rnn persistent LSTM counters");
  return PKC_OK;
}

int rnn_lstm_persist_fwd(const pkc_rnn_args* a, hipStream_t s) {
  using namespace lstmp;
  int st = lstm_ctr_reset(a, s);
  if (st) return st;
  const dim3 grid(a->H / UPW);
  const int kc = a->H / 256;
  if (a->qh_exact) {
    if (kc == 2) hipLaunchKernelGGL(qx_fwd_loop<2>, grid, dim3(FNT), 0, s, *a);
    else if (kc == 3) hipLaunchKernelGGL(qx_fwd_loop<3>, grid, dim3(FNT), 0, s, *a);
    else hipLaunchKernelGGL(qx_fwd_loop<4>, grid, dim3(FNT), 0, s, *a);
  } else if (!a->step_bf16) {                   // exact fp32 step products: 4 units per workgroup
    const int B2 = a->bidir ? 2 * a->B : a->B;
    const int ry = lstm_f32_bwd_rows_split(a, B2);              // row blocks of <= 16
    if (lstm_f32_fwd_tiles(a, ry) == 2) {                        // 8 units per workgroup
      const dim3 g8(a->H / 8, ry);
      if (kc == 2) hipLaunchKernelGGL((f32_fwd_loop<16, 2>), g8, dim3(FNT), 0, s, *a);
      else if (kc == 3) hipLaunchKernelGGL((f32_fwd_loop<24, 2>), g8, dim3(FNT), 0, s, *a);
      else hipLaunchKernelGGL((f32_fwd_loop<32, 2>), g8, dim3(FNT), 0, s, *a);
    } else {
      const dim3 g16(a->H / 16, ry);
      if (kc == 2) hipLaunchKernelGGL((f32_fwd_loop<16, 4>), g16, dim3(FNT), 0, s, *a);
      else if (kc == 3) hipLaunchKernelGGL((f32_fwd_loop<24, 4>), g16, dim3(FNT), 0, s, *a);
      else hipLaunchKernelGGL((f32_fwd_loop<32, 4>), g16, dim3(FNT), 0, s, *a);
    }
  } else {
    const int co = lstm_bf16_coalesced();
    const int rs = lstm_bf16_rows_split(a);
    if (rs == 4) {
      const dim3 g4(grid.x, 4);
      if (kc == 2) hipLaunchKernelGGL((bf_fwd_loop<2, 4>), g4, dim3(FNT), 0, s, *a, co);
      else if (kc == 3) hipLaunchKernelGGL((bf_fwd_loop<3, 4>), g4, dim3(FNT), 0, s, *a, co);
      else hipLaunchKernelGGL((bf_fwd_loop<4, 4>), g4, dim3(FNT), 0, s, *a, co);
    } else if (rs == 2) {
      const dim3 g2(grid.x, 2);
      if (kc == 2) hipLaunchKernelGGL((bf_fwd_loop<2, 2>), g2, dim3(FNT), 0, s, *a, co);
      else if (kc == 3) hipLaunchKernelGGL((bf_fwd_loop<3, 2>), g2, dim3(FNT), 0, s, *a, co);
      else hipLaunchKernelGGL((bf_fwd_loop<4, 2>), g2, dim3(FNT), 0, s, *a, co);
    } else if (kc == 2) hipLaunchKernelGGL((bf_fwd_loop<2, 1>), grid, dim3(FNT), 0, s, *a, co);
    else if (kc == 3) hipLaunchKernelGGL((bf_fwd_loop<3, 1>), grid, dim3(FNT), 0, s, *a, co);
    else hipLaunchKernelGGL((bf_fwd_loop<4, 1>), grid, dim3(FNT), 0, s, *a, co);
  }
  PKC_LAUNCH_CHECK("pkc_rnn_fwd persistent LSTM loop");
  return PKC_OK;
}

int rnn_ligru_grid_fwd(const pkc_rnn_args* a, hipStream_t s) {
  using namespace lstmp;
  int st = lstm_ctr_reset(a, s);
  if (st) return st;
  const dim3 grid((a->H + LUPW - 1) / LUPW, ligru_grid_rows_split(a));
  if (a->H <= 256) hipLaunchKernelGGL((lg_fwd_loop<4, 16>), grid, dim3(256), 0, s, *a);
  else hipLaunchKernelGGL((lg_fwd_loop<16, 12>), grid, dim3(1024), 0, s, *a);
  PKC_LAUNCH_CHECK("pkc_rnn_fwd grid-synchronised liGRU loop");
  return PKC_OK;
}

int rnn_ligru_grid_bwd(const pkc_rnn_args* a, hipStream_t s) {
  using namespace lstmp;
  if (a->T < 2) return PKC_OK;
  int st = lstm_ctr_reset(a, s);
  if (st) return st;
  const dim3 grid((a->H + UPW - 1) / UPW, ligru_grid_rows_split(a));
  if (a->H <= 256) hipLaunchKernelGGL((lg_bwd_loop<4, 16>), grid, dim3(256), 0, s, *a);
  else hipLaunchKernelGGL((lg_bwd_loop<16, 12>), grid, dim3(1024), 0, s, *a);
  PKC_LAUNCH_CHECK("pkc_rnn_bwd grid-synchronised liGRU loop");
  return PKC_OK;
}

int rnn_lstm_persist_bwd(const pkc_rnn_args* a, hipStream_t s) {
  using namespace lstmp;
  if (a->T < 2) return PKC_OK;
  int st = lstm_ctr_reset(a, s);
  if (st) return st;
  const dim3 grid(a->H / UPW);
  const int kc = a->H / 256;
  if (a->qh_exact) {
    const char* x3 = getenv("PKC_RNN_LSTM_PERSIST_X3");   // "0": the fp32 chains (bit-identical)
    const dim3 gq(grid.x, lstm_qx_bwd_rows_split(a));
    if (x3 && x3[0] == '0') hipLaunchKernelGGL(bwd_loop<false>, gq, dim3(BNT), 0, s, *a);
    else hipLaunchKernelGGL(bwd_loop<true>, gq, dim3(BNT), 0, s, *a);
  }
  else if (!a->step_bf16 && lstm_f32_bwd_lds(a)) {   // exact fp32, dgates staged in LDS
    const int B2 = a->bidir ? 2 * a->B : a->B;
    const dim3 gl(grid.x, (B2 + LRB - 1) / LRB);
    if (kc == 2) hipLaunchKernelGGL(f32_bwd_lds<16>, gl, dim3(FNT), 0, s, *a);
    else if (kc == 3) hipLaunchKernelGGL(f32_bwd_lds<24>, gl, dim3(FNT), 0, s, *a);
    else hipLaunchKernelGGL(f32_bwd_lds<32>, gl, dim3(FNT), 0, s, *a);
  }
  else if (!a->step_bf16) {                     // exact fp32: rows in blocks of <= 16
    const int B2 = a->bidir ? 2 * a->B : a->B;
    const dim3 gf(grid.x, lstm_f32_bwd_rows_split(a, B2));
    if (kc == 2) hipLaunchKernelGGL(f32_bwd_loop<16>, gf, dim3(FNT), 0, s, *a);
    else if (kc == 3) hipLaunchKernelGGL(f32_bwd_loop<24>, gf, dim3(FNT), 0, s, *a);
    else hipLaunchKernelGGL(f32_bwd_loop<32>, gf, dim3(FNT), 0, s, *a);
  } else {
    const int co = lstm_bf16_coalesced();
    const int rs = lstm_bf16_rows_split(a, true);
    if (rs == 4) {
      const dim3 g4(grid.x, 4);
      if (kc == 2) hipLaunchKernelGGL((bf_bwd_loop<2, 4>), g4, dim3(FNT), 0, s, *a, co);
      else if (kc == 3) hipLaunchKernelGGL((bf_bwd_loop<3, 4>), g4, dim3(FNT), 0, s, *a, co);
      else hipLaunchKernelGGL((bf_bwd_loop<4, 4>), g4, dim3(FNT), 0, s, *a, co);
    } else if (rs == 2) {
      const dim3 g2(grid.x, 2);
      if (kc == 2) hipLaunchKernelGGL((bf_bwd_loop<2, 2>), g2, dim3(FNT), 0, s, *a, co);
      else if (kc == 3) hipLaunchKernelGGL((bf_bwd_loop<3, 2>), g2, dim3(FNT), 0, s, *a, co);
      else hipLaunchKernelGGL((bf_bwd_loop<4, 2>), g2, dim3(FNT), 0, s, *a, co);
    } else if (kc == 2) hipLaunchKernelGGL((bf_bwd_loop<2, 1>), grid, dim3(FNT), 0, s, *a, co);
    else if (kc == 3) hipLaunchKernelGGL((bf_bwd_loop<3, 1>), grid, dim3(FNT), 0, s, *a, co);
    else hipLaunchKernelGGL((bf_bwd_loop<4, 1>), grid, dim3(FNT), 0, s, *a, co);
  }
  PKC_LAUNCH_CHECK("pkc_rnn_bwd persistent LSTM loop");
  return PKC_OK;
}

}  // namespace pkc

#ifdef PKC_TRACE
// measurement builds only: the persistent LSTM loops' per-wave phase sums (n <= 2 * 16 * 8)
extern "C" int pkc_trace_read_lstm_persist(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pkc::lstmp::ltrace_buf),
                             sizeof(unsigned long long) * n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

// which time-loop form pkc_rnn_fwd / pkc_rnn_bwd takes for these arguments: 1 the persistent liGRU
// loops, 2 the persistent LSTM loops, 0 one launch per step
extern "C" int pkc_rnn_persist_form(const pkc_rnn_args* a, int bwd) {
  if (!a) return 0;
  if (a->cell == PKC_CELL_LIGRU && pkc::rnn_persist_ok(a, bwd != 0)) return 1;
  if (pkc::rnn_lstm_persist_ok(a, bwd != 0) || pkc::rnn_ligru_grid_ok(a, bwd != 0)) return 2;
  return 0;
}
