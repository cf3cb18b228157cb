// pkc_rnn_impl.h — the serial time loops of the recurrent layers (forward and BPTT).
// Compiled as six translation units that build in parallel: the direction (PKC_RNN_FWD /
// PKC_RNN_BWD) times the cell family (PKC_RNN_PART 0: LSTM + the extern "C" dispatch,
// pkc_rnn_{fwd,bwd}.hip; 1: liGRU, pkc_rnn_{fwd,bwd}_ligru.hip; 2: GRU / minimalGRU / RNN,
// pkc_rnn_{fwd,bwd}_gru.hip).  Each instantiates only its own step kernels; every kernel and helper
// has internal linkage (an unnamed namespace), so the translation units share nothing but the
// entry points declared below.
//
// Reference: liGRU  neural_networks.py:1573-1584 (z = sig(wz+Uz h); hc = act(wh+Uh h)*drop;
//                   h = z*h + (1-z)*hc), shared-weight bidirectional rows via cat/flip
//                   (:1536-1538, :1590-1594);
//            LSTM   neural_networks.py:1077-1097 (f,i,o = sig(w+U h); c = i*act(wc+Uc h)*drop + f*c;
//                   h = o*act(c));
//            GRU    :1390-1396 (z, r = sig(w + U h); h = z*h + (1-z)*act(wh + Uh (r*h))*drop);
//            minimalGRU :1751-1755 (GRU with r replaced by z); RNN :1905-1907 (h = act(wh+Uh h)*drop).
// The input projections W x (+BN) are one big MFMA matmul over all T*B rows outside the loop
// (pkc_gemm + pkc_dense_fwd).  Bidirectional layers run both directions as one 2B-row batch:
// row r < B reads time t, row r >= B reads time T-1-t of the same (T, B, H) pre-activations (the
// reference's flip) and writes its h into the second half of the (T, B, 2H) output at T-1-t.
//
// Per time step the recurrent products are skinny matmuls [B2 x H] x [H x G*H] — a few hundred
// MFLOP for the 4x1024 LSTM, i.e. ~2 us of the chip's whole fp32 MFMA rate.  Each step is one
// launch of 256-thread workgroups that each own a 32-row x 16-column output tile and run exact-fp32
// v_mfma_f32_16x16x4_f32 chains over the whole contraction: the 4 waves x 4 lane groups split the
// contraction into 16 contiguous k-blocks of S values, every lane streams its k-block of one A row
// pair and one B row straight from global memory into registers (no LDS staging: each operand
// byte is used by exactly one lane), the four waves' partial tiles are summed in LDS and the cell
// update runs in the epilogue on the finished tile.  The forward tile holds all G gates of 16/G
// units, so the update needs nothing from other workgroups.
//
// BPTT: dh_{t-1}[r][k] = sum_g sum_j dg_g[t][r][j] U_g[j][k] contracts over G*H, so the step is
// split by gate across workgroups (B operand from a per-layer transposed copy U^T, made once per
// backward pass); the G partial tiles go to slabs and a small elementwise launch sums them and
// applies the carries and the gate gradients of step t-1.  One-gate products (RNN, the minimalGRU
// step, the d(r*h) / d(z*h) phases of the two-phase cells) finish in the matmul's own epilogue.
//
// GRU / minimalGRU multiply Uh with r*h (z*h), which needs r (z) of every unit of the row first:
// their forward step is two launches (gates that read h, then the candidate), their BPTT step two
// as well (d(rh) = Uh^T da then dr / dz, and dh_{t-1}).  r*h is kept per step (rh, (T, B2, H)):
// it is the input of the Uh gradient matmul.
#pragma once
#include "pkc_common.h"

#ifndef PKC_RNN_PART
#define PKC_RNN_PART 0
#endif

namespace pkc {

// the per-cell-family time loops (one translation unit each, see above)
int rnn_fwd_lstm(const pkc_rnn_args* a, hipStream_t s);
int rnn_fwd_ligru(const pkc_rnn_args* a, hipStream_t s);
int rnn_fwd_gru(const pkc_rnn_args* a, hipStream_t s);
int rnn_fwd_mingru(const pkc_rnn_args* a, hipStream_t s);
int rnn_fwd_rnn(const pkc_rnn_args* a, hipStream_t s);
int rnn_bwd_lstm(const pkc_rnn_args* a, float* dpre, hipStream_t s);
int rnn_bwd_ligru(const pkc_rnn_args* a, float* dpre, hipStream_t s);
int rnn_bwd_gru(const pkc_rnn_args* a, float* dpre, hipStream_t s);
int rnn_bwd_mingru(const pkc_rnn_args* a, float* dpre, hipStream_t s);
int rnn_bwd_rnn(const pkc_rnn_args* a, float* dpre, hipStream_t s);

namespace {

constexpr int RT = 256;          // threads per workgroup (4 waves)

// Phase trace (measurement builds only: -DPKC_TRACE, pkc/_build.py build(trace=True)).  PKC_TR(i)
// drains the workgroup's outstanding memory operations, then wave 0 lane 0 stores the shader clock
// (s_memtime) as stamp i of its workgroup: per-phase durations of one launch, read back with
// pkc_trace_read (the last launch of the traced kernel).  Stamps 0 and 7: the constant 100 MHz
// clock (s_memrealtime) at entry and exit, comparable across workgroups and XCDs.
#ifdef PKC_TRACE
constexpr int TRACE_SLOTS = 8, TRACE_WG = 4096;
__device__ unsigned long long trace_buf[TRACE_WG * TRACE_SLOTS];
__device__ __forceinline__ void trace_stamp(int i, bool real) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const unsigned long long v = real ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime();
  const int wg = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if (threadIdx.x == 0 && wg < TRACE_WG) {
    volatile unsigned long long* b = trace_buf;        // a vector store, kept in program order
    b[wg * TRACE_SLOTS + i] = v;
  }
}
#define PKC_TR(i) ::pkc::trace_stamp((i), (i) == 0 || (i) == 7)
#else
#define PKC_TR(i) do { } while (0)
#endif

__host__ __device__ constexpr int cell_gates(int cell) {
  return cell == PKC_CELL_LSTM ? 4 : cell == PKC_CELL_GRU ? 3 : cell == PKC_CELL_RNN ? 1 : 2;
}
// index of the candidate ("h") gate whose U multiplies r*h / z*h (two-phase cells)
__host__ __device__ constexpr int cand_gate(int cell) { return cell == PKC_CELL_GRU ? 2 : 1; }
__host__ __device__ constexpr bool two_phase(int cell) {
  return cell == PKC_CELL_GRU || cell == PKC_CELL_MINGRU;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
// The gates of the bf16 step mode (step_bf16: bf16 operands, ~2^-9 each): the hardware exp and
// reciprocal (about 2 ulp) instead of expf's range reduction and an IEEE division.  Every step of
// that mode uses it — the per-step kernels and the persistent loops alike.
__device__ __forceinline__ float sigm_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
template <bool BF>
__device__ __forceinline__ float sigm_mode(float x) { return BF ? sigm_fast(x) : sigm(x); }

struct RnnIdx {
  int T, B, B2, H;
  bool bidir;
  // (T, B, H) index of the pre-activation / gradient row used by step t, batch-row r
  __device__ __forceinline__ int64_t pre(int t, int r, int j) const {
    const int tt = (bidir && r >= B) ? T - 1 - t : t;
    const int rr = (bidir && r >= B) ? r - B : r;
    return ((int64_t)tt * B + rr) * H + j;
  }
  // index into the layer output (T, B, (bidir ? 2 : 1) * H)
  __device__ __forceinline__ int64_t out(int t, int r, int j) const {
    const int D = bidir ? 2 * H : H;
    if (bidir && r >= B) return ((int64_t)(T - 1 - t) * B + (r - B)) * D + H + j;
    return ((int64_t)t * B + r) * D + j;
  }
  __device__ __forceinline__ int64_t st(int t, int r, int j) const {   // (T, B2, H) state index
    return ((int64_t)t * B2 + r) * H + j;
  }
};

__device__ __forceinline__ RnnIdx mkidx(const pkc_rnn_args& a) {
  RnnIdx x;
  x.T = a.T; x.B = a.B; x.B2 = a.bidir ? 2 * a.B : a.B; x.H = a.H; x.bidir = a.bidir != 0;
  return x;
}

__device__ __forceinline__ float drop_val(const pkc_rnn_args& a, int r, int j, int B2) {
  // neural_networks.py:843-847 / 1543-1547: bernoulli(1-p) mask, NOT rescaled; eval: (1-p)
  if (!a.train) return 1.f - a.drop_p;
  if (a.drop_p <= 0.f) return 1.f;
  return a.drop_mask[(int64_t)r * a.H + j];
}

// Dynamic input quantisation of h_{t-1} (quantized_modules.py:99-119), applied in place by each of
// the four recurrent QuantizeLinear calls of a step (neural_networks.py:1086-1091): gate g reads
// q_{g+1} = Q(q_g) with its own per-tensor max-abs var_{g+1}.
//   q = sign(x) * ceil(|x / var| * 2^(b-1)) / 2^(b-1) * var      (var = max|x|; identity if var == 0)
// Every element of a call divides by the same var, so the quotient is formed from the correctly
// rounded reciprocal y = RN(1/var) and one fma correction (Markstein: q0 = RN(x*y),
// e = x - q0*var exact, RN(q0 + e*y) == RN(x/var) whenever the remainder does not underflow,
// i.e. |x| >= 2^-100), and / 2^(b-1) is the exact * 2^-(b-1).  For 2^-80 <= var <= 1 (an LSTM's
// h = o * tanh(c) has |h| < 1) a smaller |x| has x/var < 2^-20, where both quotients give
// ceil(.) = 1 (x != 0) or 0: the FAST form is bit-identical to the IEEE one (the sign of a zero
// quotient is dropped by the fabsf either way); any other var takes the IEEE division.
struct QParams {
  float var, rcp, scale, iscale;
  float var_s, rcp_s;     // var * 2^-(b-1) and RN(1/var) * 2^(b-1) (exact power-of-two scalings)
  bool fast;
};
__device__ __forceinline__ QParams qparams(float var, float scale) {
  QParams p;
  p.var = var;
  p.rcp = var != 0.f ? 1.f / var : 0.f;
  p.scale = scale;
  p.iscale = 1.f / scale;
  p.var_s = var * p.iscale;
  p.rcp_s = p.rcp * scale;
  p.fast = var >= 0x1p-80f && var <= 1.f;
  return p;
}
// FAST (6 VALU): the quotient is formed against the scaled divisor var_s = var 2^-(b-1), so
// RN(x / var_s) = 2^(b-1) RN(x / var) (a power-of-two scaling commutes with RN: x / var <= 1, and
// for |x| >= 2^-149 with var <= 1 a subnormal RN(x / var) still has ceil = 1 either way), one
// Markstein fma pair against rcp_s = RN(1 / var_s), ceil, then k * var_s = RN(k 2^-(b-1) var), the
// reference's one rounding of (k / 2^(b-1)) * var, and the sign copied from x (sign(x) * m for
// x != 0; a zero stays a zero).  Bit-identical to the IEEE form below in the FAST range.
template <bool FAST>
__device__ __forceinline__ float qin(float x, const QParams& p) {
  if constexpr (FAST) {
    float q = x * p.rcp_s;
    const float e = __builtin_fmaf(-q, p.var_s, x);
    q = __builtin_fmaf(e, p.rcp_s, q);
    return copysignf(ceilf(fabsf(q)) * p.var_s, x);
  } else {
    const float q = x / p.var;
    const float s = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
    return ceilf(fabsf(q) * p.scale) * p.iscale * p.var * s;
  }
}

// R16: the tile's second row strip is all zeros (Q(0) = 0): only va is quantised
template <bool FAST, int S, bool R16 = false>
__device__ __forceinline__ void qin_strips(float* va, float* vb, const QParams& p) {
#pragma unroll
  for (int s = 0; s < S; ++s) {
    va[s] = qin<FAST>(va[s], p);
    if constexpr (!R16) vb[s] = qin<FAST>(vb[s], p);
  }
}



#ifdef PKC_RNN_FWD
__global__ void rnn_drop_mask_kernel(pkc_rnn_args a, int B2) {
  const int64_t n = (int64_t)B2 * a.H;
  const uint32_t thr = (uint32_t)((double)(1.f - a.drop_p) * 4294967296.0);
  const int64_t step = a.step_ctr ? *a.step_ctr : 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v;
    if (a.drop_mask_in) v = a.drop_mask_in[i];
    else v = hash3(a.seed, (uint64_t)a.stream_id, (uint64_t)step * (uint64_t)n + i) < thr ? 1.f : 0.f;
    a.drop_mask[i] = v;
  }
}

#endif  // PKC_RNN_FWD

// ------------------------------------------------------------------------------- backward
__device__ __forceinline__ float dy_at(const pkc_rnn_args& a, int64_t i) {
  const int ns = a.dy_nslab > 0 ? a.dy_nslab : 1;
  float s = 0.f;
  for (int q = 0; q < ns; ++q) s += a.dy[(int64_t)q * a.dy_slab_stride + i];
  return s;
}

// LSTM gate gradients of one element from its saved gates (f, i, o, cc), c_t, c_{t-1}, the dropout
// value m, dL/dh_t = g and the carried dc; returns dc * f, the carry into step t-1 (the per-step
// kernels and the persistent BPTT loop share this arithmetic)
__device__ __forceinline__ float lstm_grads(int act, float f, float i, float o, float cc, float c,
                                            float cp, float m, float g, float dc_carry, float* dgo) {
#pragma clang fp contract(off)     // (as fwd_epi's LSTM update: the same rounding wherever inlined)
  const float tc = act_fwd(act, c);
  const float dc = g * o * act_bwd_out(act, tc) + dc_carry;
  dgo[0] = dc * cp * f * (1.f - f);
  dgo[1] = dc * cc * m * i * (1.f - i);
  dgo[2] = g * tc * o * (1.f - o);
  dgo[3] = dc * i * m * act_bwd_out(act, cc);
  return dc * f;
}

// liGRU gate gradients of one element from dL/dh_t = g, the saved z and act(a) (hcr), h_{t-1} and
// the dropout value m (shared by the per-step kernels and the grid-synchronised loops; unfused
// like lstm_grads)
__device__ __forceinline__ void ligru_grads(int act, float g, float z, float hcr, float hp, float m,
                                            float* dgo) {
#pragma clang fp contract(off)
  const float hc = hcr * m;
  const float dz = g * (hp - hc);
  const float dhc = g * (1.f - z);
  dgo[0] = dz * z * (1.f - z);
  dgo[1] = dhc * m * act_bwd_out(act, hcr);   // act' from the post-activation value
}
// the liGRU BPTT's carry term: dh + g_t * z_t (unfused)
__device__ __forceinline__ float ligru_carry(float dh, float gt, float zt) {
#pragma clang fp contract(off)
  return dh + gt * zt;
}

// Gate gradients of step t at (r, k) given the total dL/dh_t = g (and, LSTM, the carried dc).
template <int CELL>
__device__ __forceinline__ void gate_grads(const pkc_rnn_args& a, const RnnIdx& ix, int t, int r,
                                           int k, float g, float dc_carry, float* dgo,
                                           float* g_out, float* dc_out) {
  const int H = a.H;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H;
  const int64_t si = ix.st(t, r, k);
  const float m = drop_val(a, r, k, ix.B2);
  const float hp = a.hs[(int64_t)t * ix.B2 * H + (int64_t)r * H + k];
  if constexpr (CELL == PKC_CELL_LIGRU) {
    ligru_grads(a.act, g, a.gates[si], a.gates[TB2H + si], hp, m, dgo);
    *g_out = g;
  } else if constexpr (CELL == PKC_CELL_GRU) {
    // dz and da now; dr needs Uh^T da over the whole row (gru_bwd_rh)
    const float z = a.gates[si], hcr = a.gates[2 * TB2H + si];
    const float hc = hcr * m;
    dgo[0] = g * (hp - hc) * z * (1.f - z);
    dgo[2] = g * (1.f - z) * m * act_bwd_out(a.act, hcr);
    *g_out = g;
  } else if constexpr (CELL == PKC_CELL_MINGRU) {
    // da now; dz also needs Uh^T da (gru_bwd_rh), g is kept for it
    const float z = a.gates[si], hcr = a.gates[TB2H + si];
    dgo[1] = g * (1.f - z) * m * act_bwd_out(a.act, hcr);
    *g_out = g;
  } else if constexpr (CELL == PKC_CELL_RNN) {
    dgo[0] = g * m * act_bwd_out(a.act, a.gates[si]);
    *g_out = g;
  } else {
    const float f = a.gates[si], i = a.gates[TB2H + si], o = a.gates[2 * TB2H + si];
    const float cc = a.gates[3 * TB2H + si];
    const float c = a.cs[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + k];
    const float cp = a.cs[(int64_t)t * ix.B2 * H + (int64_t)r * H + k];
    *dc_out = lstm_grads(a.act, f, i, o, cc, c, cp, m, g, dc_carry, dgo);
    *g_out = g;
  }
}

// The gate gradients of step tt from the total dL/dh_tt = g (LSTM: plus the carried dc), into
// dgates and the ping-pong slot of step tt ((T-1-tt) & 1) of the g / dc carries.  HC: the bf16
// copy of dgates for the next bf16 BPTT product — 0 none, 1 always (the BF instances), 2 when
// dgates_h is set (one-off launches)
template <int G, int CELL, int HC>
__device__ __forceinline__ void gate_part(const pkc_rnn_args& a, const RnnIdx& ix, int tt, int r,
                                          int k, float g, float dc_carry) {
  const int64_t TB2H = (int64_t)a.T * ix.B2 * a.H;
  const int64_t n = (int64_t)ix.B2 * a.H;
  const int64_t e = (int64_t)r * a.H + k;
  const int p = (a.T - 1 - tt) & 1;
  float dg[4] = {0.f, 0.f, 0.f, 0.f}, go = 0.f, dco = 0.f;
  gate_grads<CELL>(a, ix, tt, r, k, g, dc_carry, dg, &go, &dco);
  const int64_t si = ix.st(tt, r, k);
  if constexpr (CELL == PKC_CELL_GRU) {
    a.dgates[si] = dg[0];
    a.dgates[2 * TB2H + si] = dg[2];
  } else if constexpr (CELL == PKC_CELL_MINGRU) {
    a.dgates[TB2H + si] = dg[1];
  } else {
#pragma unroll
    for (int q = 0; q < G; ++q) a.dgates[q * TB2H + si] = dg[q];
    if (HC == 1 || (HC == 2 && a.dgates_h)) {     // the next BPTT product's bf16 operand
#pragma unroll
      for (int q = 0; q < G; ++q) reinterpret_cast<__bf16*>(a.dgates_h)[q * TB2H + si] = (__bf16)dg[q];
    }
  }
  a.work[p * n + e] = go;
  if constexpr (CELL == PKC_CELL_LSTM) a.work[2 * n + p * n + e] = dco;
}

// first backward launch: step T-1, no recurrent gradient yet (with LayerNorm on h: only the
// post-norm gradient, the norm's backward and the gate gradients follow in rnn_ln_bwd_gates)
template <int G, int CELL>
__global__ void rnn_bwd_init(pkc_rnn_args a) {
  const RnnIdx ix = mkidx(a);
  const int64_t n = (int64_t)ix.B2 * a.H;
  const int t = a.T - 1;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / a.H), k = (int)(e % a.H);
    const float g = dy_at(a, ix.out(t, r, k));
    if (a.ln_gamma) a.ln_g[ix.st(t, r, k)] = g;
    else gate_part<G, CELL, 2>(a, ix, t, r, k, g, 0.f);
  }
}

// LayerNorm of the new hidden state (neural_networks.py:1093-1094, 1399-1400, 1581-1582,
// 1758-1759, 1909-1910): h_t <- gamma (h_t - mean) / (std + eps) + beta per row, std unbiased.
// One wave per row; saves xhat and (std + eps, std) for the backward.
#ifdef PKC_RNN_FWD
__global__ __launch_bounds__(256) void rnn_ln_fwd(pkc_rnn_args a, int t) {
  const RnnIdx ix = mkidx(a);
  const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= ix.B2) return;
  const int H = a.H;
  float* h = a.hs + (int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H;
  float sum = 0.f;
  for (int j = lane; j < H; j += 64) sum += h[j];
  const float mean = warp_sum(sum) / (float)H;
  float sq = 0.f;
  for (int j = lane; j < H; j += 64) {
    const float d = h[j] - mean;
    sq += d * d;
  }
  const float sd = sqrtf(warp_sum(sq) / (float)(H - 1));
  const float den = sd + a.ln_eps;
  for (int j = lane; j < H; j += 64) {
    const float xh = (h[j] - mean) / den;
    const float v = a.ln_gamma[j] * xh + a.ln_beta[j];
    a.ln_xhat[ix.st(t, r, j)] = xh;
    h[j] = v;
    a.y[ix.out(t, r, j)] = v;
  }
  if (lane == 0) {
    a.ln_stat[2 * ((int64_t)t * ix.B2 + r)] = den;
    a.ln_stat[2 * ((int64_t)t * ix.B2 + r) + 1] = sd;
  }
}

#endif  // PKC_RNN_FWD
// Backward of that LayerNorm for step tt (row-wise), then the gate gradients of step tt:
//   gh = g gamma, dh_raw = (gh - mean(gh)) / (std + eps) - xhat sum(gh xhat) / ((H - 1) std)
template <int G, int CELL>
__global__ __launch_bounds__(256) void rnn_ln_bwd_gates(pkc_rnn_args a, int tt) {
  const RnnIdx ix = mkidx(a);
  const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= ix.B2) return;
  const int H = a.H;
  const int64_t n = (int64_t)ix.B2 * H;
  const int64_t s0 = ix.st(tt, r, 0);
  float sg = 0.f, sgx = 0.f;
  for (int j = lane; j < H; j += 64) {
    const float gh = a.ln_g[s0 + j] * a.ln_gamma[j];
    sg += gh;
    sgx += gh * a.ln_xhat[s0 + j];
  }
  sg = warp_sum(sg);
  sgx = warp_sum(sgx);
  const float den = a.ln_stat[2 * ((int64_t)tt * ix.B2 + r)];
  const float sd = a.ln_stat[2 * ((int64_t)tt * ix.B2 + r) + 1];
  const float mg = sg / (float)H;
  // torch's std backward masks the zero-std case to 0 (a zero row: e.g. leading padding)
  const float kk = sd > 0.f ? sgx / ((float)(H - 1) * sd) : 0.f;
  const int src = (a.T - 1 - (tt + 1)) & 1;          // carry slot of step tt + 1
  for (int j = lane; j < H; j += 64) {
    const float gh = a.ln_g[s0 + j] * a.ln_gamma[j];
    const float g = (gh - mg) / den - a.ln_xhat[s0 + j] * kk;
    float dc_carry = 0.f;
    if constexpr (CELL == PKC_CELL_LSTM)
      if (tt < a.T - 1) dc_carry = a.work[2 * n + src * n + (int64_t)r * H + j];
    gate_part<G, CELL, 0>(a, ix, tt, r, j, g, dc_carry);
  }
}

// dgamma = sum_{t,r} g_post * xhat, dbeta = sum_{t,r} g_post over the T * B2 rows of the layer
#ifdef PKC_RNN_BWD
__global__ __launch_bounds__(256) void rnn_ln_param_grads(pkc_rnn_args a) {
  __shared__ float red[2][256];
  const RnnIdx ix = mkidx(a);
  const int H = a.H;
  const int c = blockIdx.x * 64 + threadIdx.x % 64, q = threadIdx.x / 64;
  const int64_t rows = (int64_t)a.T * ix.B2;
  float dg = 0.f, db = 0.f;
  if (c < H)
    for (int64_t r = q; r < rows; r += 4) {
      const float g = a.ln_g[r * H + c];
      dg += g * a.ln_xhat[r * H + c];
      db += g;
    }
  red[0][threadIdx.x] = dg;
  red[1][threadIdx.x] = db;
  __syncthreads();
  if (q == 0 && c < H) {
    const int l = threadIdx.x;
    a.ln_dgamma[c] = (red[0][l] + red[0][64 + l]) + (red[0][128 + l] + red[0][192 + l]);
    a.ln_dbeta[c] = (red[1][l] + red[1][64 + l]) + (red[1][128 + l] + red[1][192 + l]);
  }
}

#endif  // PKC_RNN_BWD

// ------------------------------------------------------------------------------- MFMA strips
typedef float f32x4 __attribute__((ext_vector_type(4)));

// v[s] = (ok && kb + s < kmax) ? row[kb + s] : 0 for s < S, with clamped (unconditional) loads;
// vw: wave-uniform vector width (4 when kmax % 4 == 0 and rows are 16-B aligned, 2, or 1).
template <int S>
__device__ __forceinline__ void load_strip(const float* row, bool ok, int kb, int kmax, int vw,
                                           float* v) {
  if (vw == 4) {
#pragma unroll
    for (int s = 0; s < S; s += 4) {
      const int k = kb + s;
      const bool in = ok && k < kmax;
      const float4 x = *reinterpret_cast<const float4*>(row + (in ? k : 0));
      v[s] = in ? x.x : 0.f; v[s + 1] = in ? x.y : 0.f;
      v[s + 2] = in ? x.z : 0.f; v[s + 3] = in ? x.w : 0.f;
    }
  } else if (vw == 2) {
#pragma unroll
    for (int s = 0; s < S; s += 2) {
      const int k = kb + s;
      const bool in = ok && k < kmax;
      const float2 x = *reinterpret_cast<const float2*>(row + (in ? k : 0));
      v[s] = in ? x.x : 0.f; v[s + 1] = in ? x.y : 0.f;
    }
  } else {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int k = kb + s;
      const bool in = ok && k < kmax;
      const float x = row[in ? k : 0];
      v[s] = in ? x : 0.f;
    }
  }
}

// Block-sparse form of load_strip: S/16 blocks of 16 contiguous k at blk[i] * 16 (blk < 0: zeros).
template <int S>
__device__ __forceinline__ void load_blocks(const float* row, bool ok, const int* blk, int kmax,
                                            int vw, float* v) {
#pragma unroll
  for (int i = 0; i < S / 16; ++i)
    load_strip<16>(row, ok && blk[i] >= 0, blk[i] >= 0 ? blk[i] * 16 : 0, kmax, vw, v + 16 * i);
}

// This lane group's S/16 block indices of a kmap tile row (S slots: lane group w*4+q owns slots
// [(w*4+q)*S/16, +S/16)).  The wave index is made uniform so the table is read with scalar loads
// (constant cache) — the same tiles are re-read every time step.
template <int S>
__device__ __forceinline__ void tile_blocks(const int32_t* row, int* blk) {
  typedef const __attribute__((address_space(4))) int32_t cint;
  const int wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = (threadIdx.x & 63) >> 4;
  cint* sl = (cint*)(row + wu * 4 * (S / 16));
#pragma unroll
  for (int i = 0; i < S / 16; ++i) {
    const int b0 = sl[i], b1 = sl[S / 16 + i], b2 = sl[2 * (S / 16) + i], b3 = sl[3 * (S / 16) + i];
    blk[i] = q == 0 ? b0 : (q == 1 ? b1 : (q == 2 ? b2 : b3));
  }
}

// The NW waves' 32x16 partial tiles of a K-split step product (MFMA C layout: column lane & 15,
// row 4 (lane >> 4) + i) go to red[NW][32][RED_ROW], column c at slot `col`; one barrier.  Each
// consumer then sums the NW partials of its own element(s) (red_sum / red_sum4) straight into its
// epilogue: no reduced tile, no second LDS pass, no second barrier (same-box A/B: C3 fp32, C4,
// C5 1-2% per step·layer).  The sums keep one order, (w0 + w1) + (w2 + w3) [+ ((w4 + w5) +
// (w6 + w7))], so every element is the fp32 value the former two-pass reduction produced.  Rows
// of RED_ROW = 20 floats keep 4-slot groups 16-byte aligned.
// R16: 16-row tiles (acc1 unused): rows 0..15 only.
constexpr int RED_ROW = 20;
template <int NW, bool R16 = false>
__device__ __forceinline__ void stage_partials(const f32x4& acc0, const f32x4& acc1, float* red,
                                               int col) {
  static_assert(NW % 4 == 0, "partials are summed in fours");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4;
  float* rw = red + w * 32 * RED_ROW;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rw[(4 * q + i) * RED_ROW + col] = acc0[i];
    if constexpr (!R16) rw[(16 + 4 * q + i) * RED_ROW + col] = acc1[i];
  }
  __syncthreads();
}
template <int NW>
__device__ __forceinline__ float red_sum(const float* red, int o) {
  constexpr int P = 32 * RED_ROW;
  float v = (red[o] + red[P + o]) + (red[2 * P + o] + red[3 * P + o]);
#pragma unroll
  for (int w4 = 4; w4 < NW; w4 += 4)
    v += (red[w4 * P + o] + red[(w4 + 1) * P + o]) + (red[(w4 + 2) * P + o] + red[(w4 + 3) * P + o]);
  return v;
}
// four consecutive slots (o % 4 == 0): 16-byte LDS reads, the same order per slot as red_sum
template <int NW>
__device__ __forceinline__ float4 red_sum4(const float* red, int o) {
  constexpr int P = 32 * RED_ROW;
  auto ld = [&](int w4) { return *reinterpret_cast<const float4*>(red + w4 * P + o); };
  auto add = [](float4 x, float4 y) { return make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w); };
  float4 v = add(add(ld(0), ld(1)), add(ld(2), ld(3)));
#pragma unroll
  for (int w4 = 4; w4 < NW; w4 += 4) v = add(v, add(add(ld(w4), ld(w4 + 1)), add(ld(w4 + 2), ld(w4 + 3))));
  return v;
}

// R16: the tile has only its first 16 rows (2B <= 16: C3, C5), the second chain is skipped
template <int S, bool R16 = false>
__device__ __forceinline__ void mfma_chain(const float* va, const float* vb, const float* vu,
                                           f32x4& acc0, f32x4& acc1) {
#pragma unroll
  for (int s = 0; s < S; ++s) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(va[s], vu[s], acc0, 0, 0, 0);
    if constexpr (!R16) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(vb[s], vu[s], acc1, 0, 0, 0);
  }
}

// bf16 step products (pkc_rnn_args.step_bf16): v_mfma_f32_16x16x32_bf16 takes 8 consecutive k of
// one row per lane (A: row lane & 15, B: column lane & 15, k = 8 (lane >> 4) + 0..7), so a lane
// group's strip of S contiguous k feeds S / 8 MFMAs, 8 values each, in place of the fp32 chain's S
// one-value MFMAs.  A and B lanes of one lane group hold the same k, so the sums are the same
// contraction (in another order) with bf16-rounded operands and fp32 accumulation.
typedef __attribute__((ext_vector_type(8))) __bf16 rbf16x8;

// v[i] = 8 bf16 of row[kb + 8i ..] (zeros past kmax or when !ok); v8: rows 16-byte aligned and
// kmax % 8 == 0 (then an 8-chunk is wholly inside or outside); else kmax % 2 == 0 (C3's H = 550):
// four 4-byte pair loads per chunk; else element loads
typedef __attribute__((ext_vector_type(2))) __bf16 rbf16x2;
template <int S>
__device__ __forceinline__ void load_strip_h(const __bf16* row, bool ok, int kb, int kmax, bool v8,
                                             rbf16x8* v) {
  const bool v2 = !v8 && (kmax & 1) == 0;
#pragma unroll
  for (int i = 0; i < S / 8; ++i) {
    const int k = kb + 8 * i;
    if (v8) {
      const bool in = ok && k < kmax;
      const rbf16x8 x = *reinterpret_cast<const rbf16x8*>(row + (in ? k : 0));
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = in ? x[j] : (__bf16)0.f;
    } else if (v2) {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const bool in = ok && k + j < kmax;          // pairs never straddle kmax (both even)
        const rbf16x2 x = *reinterpret_cast<const rbf16x2*>(row + (in ? k + j : 0));
        v[i][j] = in ? x[0] : (__bf16)0.f;
        v[i][j + 1] = in ? x[1] : (__bf16)0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool in = ok && k + j < kmax;
        const __bf16 x = row[in ? k + j : 0];
        v[i][j] = in ? x : (__bf16)0.f;
      }
    }
  }
}

// block-sparse form (kmap tiles): S/16 blocks of 16 contiguous k, two 8-value chunks each
template <int S>
__device__ __forceinline__ void load_blocks_h(const __bf16* row, bool ok, const int* blk, int kmax,
                                              bool v8, rbf16x8* v) {
#pragma unroll
  for (int i = 0; i < S / 16; ++i)
    load_strip_h<16>(row, ok && blk[i] >= 0, blk[i] >= 0 ? blk[i] * 16 : 0, kmax, v8, v + 2 * i);
}

template <int S, bool R16 = false>
__device__ __forceinline__ void mfma_chain_h(const rbf16x8* va, const rbf16x8* vb,
                                             const rbf16x8* vu, f32x4& acc0, f32x4& acc1) {
#pragma unroll
  for (int i = 0; i < S / 8; ++i) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[i], vu[i], acc0, 0, 0, 0);
    if constexpr (!R16) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb[i], vu[i], acc1, 0, 0, 0);
  }
}

// The quantised strip in place (q = Q(x), as qin) and the grid integers k = sign(x) ceil(|x| / var
// 2^(b-1)) of it as bf16 pairs kh = trunc(k / 256), kl = k - 256 kh (both exact, |kh| <= 128,
// |kl| <= 255): the operands of the exact quantised-h products (rnn_fwd_mm QX)
template <bool FAST, int S>
__device__ __forceinline__ void qsplit_strip(float* v, const QParams& p, rbf16x8* kh, rbf16x8* kl) {
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const float x = v[s];
    float m;
    if constexpr (FAST) {
      float q = x * p.rcp_s;
      const float e = __builtin_fmaf(-q, p.var_s, x);
      q = __builtin_fmaf(e, p.rcp_s, q);
      m = ceilf(fabsf(q));
      v[s] = copysignf(m * p.var_s, x);
    } else {
      m = ceilf(fabsf(x / p.var) * p.scale);
      const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
      v[s] = m * p.iscale * p.var * sg;
    }
    const float k = copysignf(m, x);
    const float hi = truncf(k * (1.f / 256.f));
    kh[s / 8][s % 8] = (__bf16)hi;
    kl[s / 8][s % 8] = (__bf16)__builtin_fmaf(-256.f, hi, k);
  }
}

// ------------------------------------------------------------------------------- forward step
// The cell update's inputs at (r, j) that do not depend on this step's products: the gate
// pre-activations W x (+BN), h_{t-1}, c_{t-1} (LSTM) and the dropout mask.  rnn_fwd_mm requests
// them before its operand strips, so they arrive while the MFMA chain runs instead of after it.
struct EpiIn {
  float w[4];
  float hp, cp, m;
};
template <int CELL, int NG>
__device__ __forceinline__ EpiIn epi_load(const pkc_rnn_args& a, const RnnIdx& ix, int t, int r,
                                          int j) {
  EpiIn e;
  const int H = a.H;
  const int64_t TBH = (int64_t)a.T * a.B * H;   // gate stride of the (G, T, B, H) pre-activations
  const int64_t pi = ix.pre(t, r, j);
#pragma unroll
  for (int g = 0; g < 4; ++g) e.w[g] = g < NG ? a.wpre[g * TBH + pi] : 0.f;
  const int64_t hi = (int64_t)t * ix.B2 * H + (int64_t)r * H + j;
  e.hp = a.hs[hi];
  if constexpr (CELL == PKC_CELL_LSTM) e.cp = a.cs[hi];
  else e.cp = 0.f;
  e.m = drop_val(a, r, j, ix.B2);
  return e;
}

// Cell update of step t at (r, j) from the recurrent products acc[g] = (U_g h_{t-1})[r][j].
// PUB (the persistent LSTM loops, pkc_rnn_lstm_persist.hip): h_t is handed to the other
// workgroups of the launch, so the caller stores it (hs, and hs_h in bf16 mode) in the hand-off's
// form; the LSTM's c_t is returned through c_out (kept in a register for the next step).
template <int CELL, bool QH, bool BF, bool PUB = false>
__device__ __forceinline__ float fwd_epi(const pkc_rnn_args& a, const RnnIdx& ix, int t, int r,
                                        int j, const float* acc, const float* vars, float qscale,
                                        const EpiIn& e, float* c_out = nullptr) {
  const int H = a.H;
  if constexpr (QH) {
    // the hidden state the reference keeps for step t-1 (hiddens[t-1], and the saved input of the
    // U backward) is the 4x re-quantised tensor; the last step's h is never quantised
    float v = e.hp;
    if (vars[0] != 0.f) {           // every var_g equals var_1 (see rnn_fwd_mm)
      const QParams qp = qparams(vars[0], qscale);
      if (qp.fast) {
#pragma unroll
        for (int g = 0; g < 4; ++g) v = qin<true>(v, qp);
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) v = qin<false>(v, qp);
      }
    }
    a.hq[(int64_t)t * ix.B2 * H + (int64_t)r * H + j] = v;
    if (t > 0) a.y[ix.out(t - 1, r, j)] = v;
  }
  const int64_t TBH = (int64_t)a.T * a.B * H;   // gate stride of the (G, T, B, H) pre-activations
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H; // gate stride of the saved activations
  const int64_t pi = ix.pre(t, r, j), si = ix.st(t, r, j);
  const float m = e.m;
  const float hp = e.hp;
  float h = 0.f;
  if constexpr (CELL == PKC_CELL_GRU) {
    // phase 1 of a GRU step: update / reset gates and r*h (the input of Uh)
    const float z = sigm(e.w[0] + acc[0]);
    const float rg = sigm(e.w[1] + acc[1]);
    a.gates[si] = z;
    a.gates[TB2H + si] = rg;
    a.rh[si] = rg * hp;
    return 0.f;
  } else if constexpr (CELL == PKC_CELL_MINGRU) {
    // phase 1 of a minimalGRU step: update gate and z*h (the input of Uh)
    const float z = sigm(e.w[0] + acc[0]);
    a.gates[si] = z;
    a.rh[si] = z * hp;
    return 0.f;
  } else if constexpr (CELL == PKC_CELL_RNN) {
    const float hcr = act_fwd(a.act, e.w[0] + acc[0]);
    h = hcr * m;
    a.gates[si] = hcr;
  } else if constexpr (CELL == PKC_CELL_LIGRU) {
#pragma clang fp contract(off)     // (as the LSTM branch below: the same rounding wherever inlined)
    const float z = sigm_mode<BF>(e.w[0] + acc[0]);
    const float hcr = act_fwd(a.act, e.w[1] + acc[1]);
    h = z * hp + (1.f - z) * (hcr * m);
    a.gates[si] = z;
    a.gates[TB2H + si] = hcr;
  } else {
    // LSTM gates (f, i, o, c); cs[t] = c_{t-1}.  No fma contraction here: the per-step kernels and
    // the persistent loop inline this in different code, where the compiler's contraction choices
    // differed (i cc m + f c_{t-1}); unfused, both round like the reference's separate ops.
#pragma clang fp contract(off)
    const float f = sigm_mode<BF>(e.w[0] + acc[0]);
    const float i = sigm_mode<BF>(e.w[1] + acc[1]);
    const float o = sigm_mode<BF>(e.w[2] + acc[2]);
    const float cc = act_fwd(a.act, e.w[3] + acc[3]);
    const float cp = e.cp;
    const float c = i * cc * m + f * cp;
    h = o * act_fwd(a.act, c);
    a.cs[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + j] = c;
    a.gates[si] = f;
    a.gates[TB2H + si] = i;
    a.gates[2 * TB2H + si] = o;
    a.gates[3 * TB2H + si] = cc;
    if (c_out) *c_out = c;
  }
  if constexpr (!PUB) {
    a.hs[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + j] = h;
    if constexpr (BF)   // the next step's bf16 operand (step_bf16: every step runs a BF instance)
      reinterpret_cast<__bf16*>(a.hs_h)[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + j] = (__bf16)h;
  }
  a.y[ix.out(t, r, j)] = h;
  return h;
}

// phase 2 of a GRU / minimalGRU step: h = z*h_{t-1} + (1-z)*act(wh + Uh (r|z)*h_{t-1})*drop
template <int HG>
__device__ __forceinline__ void cand_epi(const pkc_rnn_args& a, const RnnIdx& ix, int t, int r,
                                         int j, float acc) {
  const int H = a.H;
  const int64_t TBH = (int64_t)a.T * a.B * H;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H;
  const int64_t pi = ix.pre(t, r, j), si = ix.st(t, r, j);
  const float m = drop_val(a, r, j, ix.B2);
  const float hp = a.hs[(int64_t)t * ix.B2 * H + (int64_t)r * H + j];
  const float z = a.gates[si];
  const float hcr = act_fwd(a.act, a.wpre[HG * TBH + pi] + acc);
  const float h = z * hp + (1.f - z) * (hcr * m);
  a.gates[HG * TB2H + si] = hcr;
  a.hs[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + j] = h;
  a.y[ix.out(t, r, j)] = h;
}

// One forward step (PH = 0: the gates that read h_{t-1}; PH = 1: the candidate of a two-phase
// cell, reading rh).  Tile: rows [32*blockIdx.y, +32) x NG gates of NU = 16/NG units.
// NW waves (4: 256 threads, or 8: the contraction in 32 strips of S — half the operand loads per
// lane and half the MFMA chain per wave, for the long-H layers whose step is load-latency-bound)
// BF: bf16 step product (step_bf16: hs_h / U_h operands, mfma_chain_h)
// QX (quantised h, pkc_rnn_args.qh_exact): U is on an 8-bit grid (m / 128, |m| <= 128: exact in
// bf16, U_h) and q_g = RN(k var_s) with integers |k| <= 2^15, so U q_g = var_s U k up to the one
// rounding of each q: k = 256 kh + kl (|kh| <= 128, |kl| <= 255, both exact in bf16) and the two
// bf16 MFMA chains over (kh, U_h) and (kl, U_h) sum integer multiples of 2^-7 in fp32 (exactly up
// to H = 512, fp32-rounded beyond) — the products of the fp32 chain to within its own rounding, at
// 1/16 of its MFMA issue per chain
template <int NG, int CELL, int PH, int S, bool QH, bool SP = false, int NW = 4, bool R16 = false,
          bool BF = false, bool QX = false>
__global__ __launch_bounds__(64 * NW) void rnn_fwd_mm(pkc_rnn_args a, int t, int vw) {
  static_assert(NW == 4 || !SP, "block-sparse tables are laid out for 16 strips");
  static_assert(!QX || (QH && !SP && !BF && S % 8 == 0), "exact quantised-h products: dense QH");
  static_assert(!BF || (!QH && PH == 0), "bf16 steps: one-phase cells, no quantised h");
  PKC_TR(0);
  PKC_TR(1);
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  constexpr int NTH = 64 * NW;
  __shared__ __attribute__((aligned(16))) float red[NW * 32 * RED_ROW];
  constexpr int NU = 16 / NG;
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  const int u0 = bx * NU, r0 = by * (R16 ? 16 : 32);
  const float* src = (PH == 0 ? a.hs : a.rh) + (int64_t)t * B2 * H;
  const int ra = r0 + c, rb = r0 + 16 + c;
  const int gi = c / NU, u = u0 + c % NU;
  const float* pu = a.U[PH == 0 ? gi : cand_gate(CELL)] + (int64_t)(u < H ? u : 0) * H;
  // one epilogue element per thread (LSTM, liGRU, GRU phase 1): its inputs are requested first
  constexpr bool PF = PH == 0 && 32 * NU <= NTH;
  EpiIn pre;
  if constexpr (PF) {
    const int rl = (int)threadIdx.x / NU, ul = (int)threadIdx.x % NU;
    const int rr = min(r0 + rl, B2 - 1), jj = min(u0 + ul, H - 1);
    if ((int)threadIdx.x < 32 * NU) pre = epi_load<CELL, NG>(a, ix, t, rr, jj);
  }
  float vars[4] = {0.f, 0.f, 0.f, 0.f};
  const float qscale = QH ? ldexpf(1.f, a.qbits - 1) : 1.f;
  // QX: var = max|h_{t-1}| from the previous step's per-wave partials (a.work, two slots by step
  // parity, EW per workgroup), read beside the operand strips — no block reduction
  constexpr int EW = ((R16 ? 16 : 32) * NU + 63) / 64;   // waves holding epilogue elements
  const int npart = (int)(gridDim.x * gridDim.y) * EW;
  float pmax = 0.f;
  if constexpr (QX) {
    if (t > 0) {
      const float* part = a.work + ((t - 1) & 1) * npart;
      for (int i = lane; i < npart; i += 64) pmax = fmaxf(pmax, part[i]);
    }
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (BF) {
    const __bf16* srch = reinterpret_cast<const __bf16*>(a.hs_h) + (int64_t)t * B2 * H;
    const __bf16* puh = reinterpret_cast<const __bf16*>(a.U_h[gi]) + (int64_t)(u < H ? u : 0) * H;
    const bool v8 = vw == 4 && H % 8 == 0;
    rbf16x8 ha[S / 8], hb[S / 8], hu[S / 8];
    if constexpr (SP) {
      int blk[S / 16];
      tile_blocks<S>(a.kmap_fwd + (int64_t)bx * S, blk);
      load_blocks_h<S>(srch + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, blk, H, v8, ha);
      if constexpr (!R16) load_blocks_h<S>(srch + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, blk, H, v8, hb);
      load_blocks_h<S>(puh, u < H, blk, H, v8, hu);
    } else {
      const int kb = (w * 4 + q) * S;
      load_strip_h<S>(srch + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, kb, H, v8, ha);
      if constexpr (!R16) load_strip_h<S>(srch + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, kb, H, v8, hb);
      load_strip_h<S>(puh, u < H, kb, H, v8, hu);
    }
    PKC_TR(2);                      // operands (and the epilogue inputs) in registers
    PKC_TR(3);
    mfma_chain_h<S, R16>(ha, hb, hu, acc0, acc1);
  } else {
  float va[S], vb[S], vu[QX ? 1 : S];
  rbf16x8 hu[QX ? S / 8 : 1];
  if constexpr (SP) {
    static_assert(!QH && PH == 0, "block-sparse U: no quantised h, one-phase cells");
    int blk[S / 16];
    tile_blocks<S>(a.kmap_fwd + (int64_t)bx * S, blk);
    load_blocks<S>(src + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, blk, H, vw, va);
    if constexpr (!R16) load_blocks<S>(src + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, blk, H, vw, vb);
    load_blocks<S>(pu, u < H, blk, H, vw, vu);
  } else {
    const int kb = (w * 4 + q) * S;
    load_strip<S>(src + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, kb, H, vw, va);
    if constexpr (!R16) load_strip<S>(src + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, kb, H, vw, vb);
    if constexpr (QX) {
      const __bf16* puh = reinterpret_cast<const __bf16*>(a.U_h[gi]) + (int64_t)(u < H ? u : 0) * H;
      load_strip_h<S>(puh, u < H, kb, H, vw == 4 && H % 8 == 0, hu);
    } else {
      load_strip<S>(pu, u < H, kb, H, vw, vu);
    }
  }
  if constexpr (R16) {
#pragma unroll
    for (int s = 0; s < S; ++s) vb[s] = 0.f;
  }
  PKC_TR(2);                        // operands (and the epilogue inputs) in registers
  if constexpr (QH) {
    // each gate's QuantizeLinear re-quantises h in place (q1..q4): gate g's product reads
    // q_{g+1} = Q(q_g) with var_g = max|q_g| over the whole tensor.  With all B2 <= 32 rows in this
    // tile, the four waves' strips hold every element of h_{t-1} exactly once (rows >= B2 and
    // k >= H are zeros, which change neither max nor min), so var_g is a block reduction of the
    // registers: no second pass over global memory, and each element is quantised once per gate.
    //
    // Only var_1 needs the reduction: Q maps the max-abs element x* (|x*| = var) to exactly
    // +-var (x*/var = +-1, ceil(2^(b-1)) / 2^(b-1) = 1) and every other element to a magnitude
    // <= var (monotone rounding of ceil(.) / 2^(b-1) <= 1), so var_{g+1} = max|q_{g+1}| = var_g.
    // (NW waves x 4 lane groups x S = H: with 8 waves each holds half a 4-wave strip)
    __shared__ float qred[2 * NW];
    if constexpr (QX) {
      const float v1 = warp_max(pmax);
#pragma unroll
      for (int g = 0; g < 4; ++g) vars[g] = v1;
    } else {
      float mx = -INFINITY, mn = INFINITY;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        mx = fmaxf(mx, fmaxf(va[s], vb[s]));
        mn = fminf(mn, fminf(va[s], vb[s]));
      }
      mx = warp_max(mx);
      mn = -warp_max(-mn);
      if (lane == 0) { qred[w] = mx; qred[NW + w] = mn; }
      __syncthreads();
      mx = qred[0];
      mn = qred[NW];
#pragma unroll
      for (int i = 1; i < NW; ++i) {
        mx = fmaxf(mx, qred[i]);
        mn = fminf(mn, qred[NW + i]);
      }
      const float v1 = fabsf(mx) > fabsf(mn) ? fabsf(mx) : fabsf(mn);
#pragma unroll
      for (int g = 0; g < 4; ++g) vars[g] = v1;
    }
    PKC_TR(3);                      // var reduced
    const QParams qp = qparams(vars[0], qscale);
    const bool qon = vars[0] != 0.f;
    // gate g's columns take the product of q_{g+1}: one chain per gate into its own accumulators
    // over the unmasked U strip, and each output column (lane & 15, gate gi) keeps its gate's
    // accumulator — the same sums as masking the other gates' U columns to zero, without the
    // per-gate mask pass (S selects per lane per gate)
    f32x4 ag0[NG], ag1[NG];
    bool fixed = false;           // QX, 4 gates: q3 == q2 on every element of this wave's strips
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      ag0[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      ag1[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (QX) {
        if (g >= 2 && fixed) {    // then q4 = Q(q3) = q3 = q2: gates 2 and 3 repeat gate 1's sums
          ag0[g] = ag0[NG > 1 ? 1 : 0];
          ag1[g] = ag1[NG > 1 ? 1 : 0];
        } else if (qon) {
          rbf16x8 ah[S / 8], al[S / 8], bh[R16 ? 1 : S / 8], bl[R16 ? 1 : S / 8];
          if (qp.fast) qsplit_strip<true, S>(va, qp, ah, al);
          else qsplit_strip<false, S>(va, qp, ah, al);
          if constexpr (!R16) {
            if (qp.fast) qsplit_strip<true, S>(vb, qp, bh, bl);
            else qsplit_strip<false, S>(vb, qp, bh, bl);
          }
          f32x4 h0 = ag0[g], h1 = ag1[g], l0 = ag0[g], l1 = ag1[g];
          mfma_chain_h<S, R16>(ah, bh, hu, h0, h1);
          mfma_chain_h<S, R16>(al, bl, hu, l0, l1);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            ag0[g][i] = __builtin_fmaf(256.f, h0[i], l0[i]) * qp.var_s;
            if constexpr (!R16) ag1[g][i] = __builtin_fmaf(256.f, h1[i], l1[i]) * qp.var_s;
          }
          if (NG == 4 && g == 1) {
            // Q is idempotent on most grid values (k var_s divides back to k), but the rounding
            // of k var_s can push one to k + 1 once: test the third call on this wave's strips
            bool eq = true;
#pragma unroll
            for (int s2 = 0; s2 < S; ++s2) {
              eq = eq && (qp.fast ? qin<true>(va[s2], qp) : qin<false>(va[s2], qp)) == va[s2];
              if constexpr (!R16)
                eq = eq && (qp.fast ? qin<true>(vb[s2], qp) : qin<false>(vb[s2], qp)) == vb[s2];
            }
            fixed = __all(eq);
          }
        }
      } else {
        if (qon) {
          if (qp.fast) qin_strips<true, S, R16>(va, vb, qp);
          else qin_strips<false, S, R16>(va, vb, qp);
        }
        mfma_chain<S, R16>(va, vb, vu, ag0[g], ag1[g]);
      }
    }
    acc0 = ag0[0];
    acc1 = ag1[0];
#pragma unroll
    for (int g = 1; g < NG; ++g) {
      if (gi == g) {
        acc0 = ag0[g];
        acc1 = ag1[g];
      }
    }
  } else {
    mfma_chain<S, R16>(va, vb, vu, acc0, acc1);
  }
  }   // !BF
#ifdef PKC_TRACE
  asm volatile("" ::"v"(acc0[0]), "v"(acc1[0]));   // the products complete before stamp 4
#endif
  PKC_TR(4);
  // column c holds gate gi of unit u: staged at slot NG * (c % NU) + gi, so a unit's gates are
  // adjacent (one 16-byte read per wave partial for the LSTM)
  stage_partials<NW, R16>(acc0, acc1, red, NG * (c % NU) + gi);
  PKC_TR(5);
  float hmax = 0.f;               // QX: max|h| over this thread's elements
  for (int p = threadIdx.x; p < 32 * NU; p += NTH) {
    const int rl = p / NU, ul = p % NU;
    const int r = r0 + rl, j = u0 + ul;
    if ((R16 && rl >= 16) || r >= B2 || j >= H) continue;
    const int o = rl * RED_ROW + NG * ul;
    if constexpr (PH == 1) {
      cand_epi<cand_gate(CELL)>(a, ix, t, r, j, red_sum<NW>(red, o));
    } else {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (NG == 4) {
        const float4 s = red_sum4<NW>(red, o);
        acc[0] = s.x; acc[1] = s.y; acc[2] = s.z; acc[3] = s.w;
      } else {
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = red_sum<NW>(red, o + g);
      }
      float h;
      if constexpr (PF) h = fwd_epi<CELL, QH, BF>(a, ix, t, r, j, acc, vars, qscale, pre);
      else h = fwd_epi<CELL, QH, BF>(a, ix, t, r, j, acc, vars, qscale, epi_load<CELL, NG>(a, ix, t, r, j));
      if constexpr (QX) hmax = fmaxf(hmax, fabsf(h));
    }
  }
  if constexpr (QX) {             // this step's max|h| partials, one per epilogue wave
    if (w < EW) {
      const float m = warp_max(hmax);
      if (lane == 0) a.work[(t & 1) * npart + (blockIdx.x + gridDim.x * blockIdx.y) * EW + w] = m;
    }
  }
  PKC_TR(6);
  PKC_TR(7);
}

// BPTT step for target tt (t = tt + 1 has its gate gradients): dh = acc + carries, g = dy + dh,
// then the gate gradients of step tt at (r, k).
template <int G, int CELL, int HC>
__device__ __forceinline__ void bwd_step_epi(const pkc_rnn_args& a, const RnnIdx& ix, int tt, int r,
                                             int k, float acc) {
  const int H = a.H;
  const int t = tt + 1;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H;
  const int64_t n = (int64_t)ix.B2 * H;
  const int64_t e = (int64_t)r * H + k;
  const int src = (a.T - 1 - t) & 1;                     // ping-pong slot of g / dc of step t
  float dh = acc;
  float dc_carry = 0.f;
  if constexpr (CELL == PKC_CELL_LIGRU) {
    dh = ligru_carry(dh, a.work[src * n + e], a.gates[ix.st(t, r, k)]);     // + g_t * z_t
  } else if constexpr (CELL == PKC_CELL_GRU) {
    // g_t * z_t + d(rh)_t * r_t  (acc = Uz^T dz_t + Ur^T dr_t)
    dh += a.work[src * n + e] * a.gates[ix.st(t, r, k)] +
          a.work[2 * n + e] * a.gates[TB2H + ix.st(t, r, k)];
  } else if constexpr (CELL == PKC_CELL_MINGRU) {
    // (g_t + d(zh)_t) * z_t  (acc = Uz^T dz_t)
    dh += (a.work[src * n + e] + a.work[2 * n + e]) * a.gates[ix.st(t, r, k)];
  } else if constexpr (CELL == PKC_CELL_LSTM) {
    dc_carry = a.work[2 * n + src * n + e];                  // dc_t * f_t
  }
  const float g = dy_at(a, ix.out(tt, r, k)) + dh;
  if (a.ln_gamma) {                  // gradient of the normalised h: rnn_ln_bwd_gates goes on
    a.ln_g[ix.st(tt, r, k)] = g;
    return;
  }
  gate_part<G, CELL, HC>(a, ix, tt, r, k, g, dc_carry);
}

// d(rh)_t = Uh^T da_t (acc) of a two-phase cell -> dr_t (GRU) or dz_t (minimalGRU); d(rh) is kept
// in work[2n..3n) for the carry term of the next (earlier) step.
template <int CELL>
__device__ __forceinline__ void rh_epi(const pkc_rnn_args& a, const RnnIdx& ix, int t, int r, int k,
                                       float acc) {
  const int H = a.H;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H;
  const int64_t n = (int64_t)ix.B2 * H;
  const int64_t e = (int64_t)r * H + k, si = ix.st(t, r, k);
  const float hp = a.hs[(int64_t)t * ix.B2 * H + e];
  if constexpr (CELL == PKC_CELL_GRU) {
    const float rg = a.gates[TB2H + si];
    a.dgates[TB2H + si] = acc * hp * rg * (1.f - rg);
  } else {
    // minimalGRU: dz = g (h_{t-1} - hc) + d(zh) h_{t-1}; g_t sits in the ping-pong slot of step t
    const float g = a.work[((a.T - 1 - t) & 1) * n + e];
    const float z = a.gates[si], hc = a.gates[TB2H + si] * drop_val(a, r, k, ix.B2);
    a.dgates[si] = (g * (hp - hc) + acc * hp) * z * (1.f - z);
  }
  a.work[2 * n + e] = acc;
}

// MODE 0: the product of gate g0 + blockIdx.z into slab blockIdx.z (a.work + (4 + z) n);
// MODE 1: one-gate product + bwd_step_epi (t = tt + 1); MODE 2: one-gate product + rh_epi.
// out[r][k] = sum_j dg_g[t][r][j] * U_g[j][k], B operand from U^T (a.ut, G x H x H).
template <int G, int CELL, int MODE, int S, bool SP = false, int NW = 4, bool R16 = false,
          bool BF = false>
__global__ __launch_bounds__(64 * NW) void rnn_bwd_mm(pkc_rnn_args a, int t, int g0, int vw) {
  static_assert(NW == 4 || !SP, "block-sparse tables are laid out for 16 strips");
  static_assert(!BF || MODE <= 1, "bf16 steps: one-phase cells");
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  constexpr int NTH = 64 * NW;
  __shared__ __attribute__((aligned(16))) float red[NW * 32 * RED_ROW];
  const RnnIdx ix = mkidx(a);
  const int H = a.H, B2 = ix.B2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, q = lane >> 4;
  const int k0 = bx * 16, r0 = by * (R16 ? 16 : 32);
  const int g = g0 + bz;
  const int64_t TB2H = (int64_t)a.T * B2 * H;
  const float* dg = a.dgates + g * TB2H + (int64_t)t * B2 * H;
  const int ra = r0 + c, rb = r0 + 16 + c, k = k0 + c;
  const float* pu = a.ut + (int64_t)g * H * H + (int64_t)(k < H ? k : 0) * H;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (BF) {
    const __bf16* dgh = reinterpret_cast<const __bf16*>(a.dgates_h) + g * TB2H + (int64_t)t * B2 * H;
    const __bf16* puh = reinterpret_cast<const __bf16*>(a.ut_h) + (int64_t)g * H * H +
                        (int64_t)(k < H ? k : 0) * H;
    const bool v8 = vw == 4 && H % 8 == 0;
    rbf16x8 ha[S / 8], hb[S / 8], hu[S / 8];
    if constexpr (SP) {
      int blk[S / 16];
      tile_blocks<S>(a.kmap_bwd + ((int64_t)g * gridDim.x + bx) * S, blk);
      load_blocks_h<S>(dgh + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, blk, H, v8, ha);
      if constexpr (!R16) load_blocks_h<S>(dgh + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, blk, H, v8, hb);
      load_blocks_h<S>(puh, k < H, blk, H, v8, hu);
    } else {
      const int kb = (w * 4 + q) * S;
      load_strip_h<S>(dgh + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, kb, H, v8, ha);
      if constexpr (!R16) load_strip_h<S>(dgh + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, kb, H, v8, hb);
      load_strip_h<S>(puh, k < H, kb, H, v8, hu);
    }
    mfma_chain_h<S, R16>(ha, hb, hu, acc0, acc1);
  } else {
  float va[S], vb[S], vu[S];
  if constexpr (SP) {
    static_assert(MODE == 0, "block-sparse U: gate-split BPTT products only");
    int blk[S / 16];
    tile_blocks<S>(a.kmap_bwd + ((int64_t)g * gridDim.x + bx) * S, blk);
    load_blocks<S>(dg + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, blk, H, vw, va);
    if constexpr (!R16) load_blocks<S>(dg + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, blk, H, vw, vb);
    load_blocks<S>(pu, k < H, blk, H, vw, vu);
  } else {
    const int kb = (w * 4 + q) * S;
    load_strip<S>(dg + (int64_t)(ra < B2 ? ra : 0) * H, ra < B2, kb, H, vw, va);
    if constexpr (!R16) load_strip<S>(dg + (int64_t)(rb < B2 ? rb : 0) * H, rb < B2, kb, H, vw, vb);
    load_strip<S>(pu, k < H, kb, H, vw, vu);
  }
  mfma_chain<S, R16>(va, vb, vu, acc0, acc1);
  }   // !BF
  stage_partials<NW, R16>(acc0, acc1, red, c);
  const int64_t n = (int64_t)B2 * H;
  for (int p = threadIdx.x; p < 32 * 16; p += NTH) {
    const int rl = p >> 4, kl = p & 15;
    const int r = r0 + rl, kk = k0 + kl;
    if ((R16 && rl >= 16) || r >= B2 || kk >= H) continue;
    const float v = red_sum<NW>(red, rl * RED_ROW + kl);
    if constexpr (MODE == 0) a.work[(4 + bz) * n + (int64_t)r * H + kk] = v;
    else if constexpr (MODE == 1) bwd_step_epi<G, CELL, BF ? 1 : 0>(a, ix, t - 1, r, kk, v);
    else rh_epi<CELL>(a, ix, t, r, kk, v);
  }
}

// Sum of the NS gate slabs + bwd_step_epi for target tt (elementwise over B2 x H).
template <int G, int CELL, int NS, bool BF = false>
__global__ __launch_bounds__(256) void rnn_bwd_epi(pkc_rnn_args a, int tt) {
  const int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  const RnnIdx ix = mkidx(a);
  const int64_t n = (int64_t)ix.B2 * a.H;
  for (int64_t e = bx * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s) acc += a.work[(4 + s) * n + e];
    bwd_step_epi<G, CELL, BF ? 1 : 0>(a, ix, tt, (int)(e / a.H), (int)(e % a.H), acc);
  }
}

// ut[g][k][j] = U[g][j][k] (the B operand of the backward products), 32 x 32 tiles through LDS
#ifdef PKC_RNN_BWD
__global__ __launch_bounds__(256) void rnn_transpose_u(pkc_rnn_args a) {
  __shared__ float tl[32][33];
  const int H = a.H, g = blockIdx.z;
  const float* U = a.U[g];
  float* ut = a.ut + (int64_t)g * H * H;
  const int j0 = blockIdx.y * 32, k0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int j = j0 + i, k = k0 + tx;
    tl[i][tx] = (j < H && k < H) ? U[(int64_t)j * H + k] : 0.f;
  }
  __syncthreads();
  __bf16* uth = a.ut_h ? reinterpret_cast<__bf16*>(a.ut_h) + (int64_t)g * H * H : nullptr;
  for (int i = ty; i < 32; i += 8) {
    const int k = k0 + i, j = j0 + tx;
    if (k < H && j < H) {
      ut[(int64_t)k * H + j] = tl[tx][i];
      if (uth) uth[(int64_t)k * H + j] = (__bf16)tl[tx][i];
    }
  }
}

#endif  // PKC_RNN_BWD
// fold the per-direction gate gradients (G, T, B2, H) onto the (G, T, B, H) pre-activation rows
#ifdef PKC_RNN_BWD
__global__ void rnn_fold_kernel(pkc_rnn_args a, float* dpre) {
  const RnnIdx ix = mkidx(a);
  const int G = cell_gates(a.cell);
  const int64_t TBH = (int64_t)a.T * a.B * a.H;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * a.H;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < (int64_t)G * TBH;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(e / TBH);
    const int64_t rem = e % TBH;
    const int j = (int)(rem % a.H);
    const int b = (int)((rem / a.H) % a.B);
    const int t = (int)(rem / ((int64_t)a.H * a.B));
    float v = a.dgates[g * TB2H + ix.st(t, b, j)];
    if (ix.bidir) v += a.dgates[g * TB2H + ix.st(a.T - 1 - t, b + a.B, j)];
    dpre[e] = v;
  }
}

#endif  // PKC_RNN_BWD

template <int S>
struct SCase {};

static int pick_vw(int H) { return H % 4 == 0 ? 4 : (H % 2 == 0 ? 2 : 1); }

// 16-row step tiles up to 2B <= PKC_RNN_ROWS16 rows (default 16; 0: always the 32-row tiles).
// Clamped to 16: a 16-row tile holds rows [16 y, 16 y + 16) only, so with more rows the grid would
// have two row tiles — and the quantised-h step takes var (max |h_{t-1}|) from ONE tile's registers.
static bool rows16(int B2) {
  static const int lim = [] {
    const char* v = getenv("PKC_RNN_ROWS16");
    const int l = v ? atoi(v) : 16;
    return l < 16 ? l : 16;
  }();
  return B2 <= lim;
}

// 8-wave step tiles for the dense one-phase cells at S >= 32 (H > 256): half the operand strip
// per lane and half the MFMA chain per wave.  Same-run A/B (PKC_RNN_WAVES=4 / 8): C4 89.2k / 90.8k,
// C5 (8-wave BPTT only; its quantised forward keeps 4) 117.6k / 120.3k frames/s — the step is
// bound by h_{t-1} arriving from the other XCDs, not by the per-lane load or MFMA work.
// PKC_RNN_QH_WAVES (8 / 4): the quantised-h forward step (C5) as 8-wave tiles — half the strip,
// quantisation passes and MFMA chains per wave, two waves per SIMD to overlap one's
// quantisation arithmetic with the other's MFMAs
// (16-wave tiles of the exact form measured 20.05 vs 19.95 us per step.layer: the quantisation
// arithmetic is per-CU work, more waves only split it)
static bool qh_eight_waves(int S) {
  static const int w = [] {
    const char* v = getenv("PKC_RNN_QH_WAVES");
    return v ? atoi(v) : 8;
  }();
  return w == 8 && S >= 32;
}

static bool eight_waves(int S) {
  static const int w = [] {
    const char* v = getenv("PKC_RNN_WAVES");
    return v ? atoi(v) : 8;
  }();
  return w == 8 && S >= 32;
}

#ifdef PKC_RNN_FWD
template <int G, int CELL, int S, bool SP = false>
static int fwd_impl_s(const pkc_rnn_args* a, hipStream_t s) {
  const int B2 = a->bidir ? 2 * a->B : a->B;
  const int vw = pick_vw(a->H);
  const unsigned rows = (unsigned)((B2 + 31) / 32), rows_16 = (unsigned)((B2 + 15) / 16);
  if constexpr (two_phase(CELL)) {
    constexpr int NG = G - 1;                        // gates that read h_{t-1}
    dim3 g1((a->H + 16 / NG - 1) / (16 / NG), rows), g2((a->H + 15) / 16, rows);
    const bool r16 = rows16(B2);
    const dim3 g1r(g1.x, rows_16), g2r(g2.x, rows_16);
    for (int t = 0; t < a->T; ++t) {
      if (r16) {
        hipLaunchKernelGGL((rnn_fwd_mm<NG, CELL, 0, S, false, false, 4, true>), g1r, dim3(RT), 0, s,
                           *a, t, vw);
        hipLaunchKernelGGL((rnn_fwd_mm<1, CELL, 1, S, false, false, 4, true>), g2r, dim3(RT), 0, s,
                           *a, t, vw);
      } else {
        hipLaunchKernelGGL((rnn_fwd_mm<NG, CELL, 0, S, false>), g1, dim3(RT), 0, s, *a, t, vw);
        hipLaunchKernelGGL((rnn_fwd_mm<1, CELL, 1, S, false>), g2, dim3(RT), 0, s, *a, t, vw);
      }
      if (a->ln_gamma) hipLaunchKernelGGL(rnn_ln_fwd, dim3((B2 + 3) / 4), dim3(256), 0, s, *a, t);
    }
  } else {
    dim3 g1((a->H + 16 / G - 1) / (16 / G), rows);
    // 2B <= 16 rows (C3, C5): 16-row tiles, no second MFMA chain or operand strip
    const bool r16 = rows16(B2);
    const dim3 g16(g1.x, rows_16);
    if constexpr (!SP) {
      if (a->step_bf16) {              // bf16 step products (check(): dense, no qbits / LN)
        const bool ew = eight_waves(S);
        for (int t = 0; t < a->T; ++t) {
          if (r16 && ew)
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S / 2, false, false, 8, true, true>),
                               g16, dim3(2 * RT), 0, s, *a, t, vw);
          else if (r16)
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false, false, 4, true, true>),
                               g16, dim3(RT), 0, s, *a, t, vw);
          else if (ew)
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S / 2, false, false, 8, false, true>),
                               g1, dim3(2 * RT), 0, s, *a, t, vw);
          else
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false, false, 4, false, true>),
                               g1, dim3(RT), 0, s, *a, t, vw);
        }
        PKC_LAUNCH_CHECK("pkc_rnn_fwd bf16 step");
        return PKC_OK;
      }
    }
    for (int t = 0; t < a->T; ++t) {
      if (r16) {
        if constexpr (SP) {
          if (a->step_bf16)
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false, true, 4, true, true>), g16,
                               dim3(RT), 0, s, *a, t, vw);
          else
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false, true, 4, true>), g16, dim3(RT), 0, s,
                               *a, t, vw);
        } else if (a->qbits > 0 && qh_eight_waves(S)) {
          bool done = false;
          if constexpr (CELL == PKC_CELL_LSTM && (S / 2) % 8 == 0)
            if ((done = a->qh_exact != 0))
              hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S / 2, true, false, 8, true, false, true>),
                                 g16, dim3(2 * RT), 0, s, *a, t, vw);
          if (!done)
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S / 2, true, false, 8, true>), g16,
                               dim3(2 * RT), 0, s, *a, t, vw);
        } else if (a->qbits > 0) {
          bool done = false;
          if constexpr (CELL == PKC_CELL_LSTM && S % 8 == 0)
            if ((done = a->qh_exact != 0))
              hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, true, false, 4, true, false, true>), g16,
                                 dim3(RT), 0, s, *a, t, vw);
          if (!done)
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, true, false, 4, true>), g16, dim3(RT), 0,
                               s, *a, t, vw);
        }
        else if (eight_waves(S))
          hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S / 2, false, false, 8, true>), g16,
                             dim3(2 * RT), 0, s, *a, t, vw);
        else
          hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false, false, 4, true>), g16, dim3(RT), 0,
                             s, *a, t, vw);
      } else if constexpr (SP) {
        if (a->step_bf16)
          hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false, true, 4, false, true>), g1,
                             dim3(RT), 0, s, *a, t, vw);
        else
          hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false, true>), g1, dim3(RT), 0, s, *a, t, vw);
      } else if (a->qbits > 0) {
        bool done = false;
        if constexpr (CELL == PKC_CELL_LSTM && S % 8 == 0)
          if ((done = a->qh_exact != 0))
            hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, true, false, 4, false, false, true>), g1,
                               dim3(RT), 0, s, *a, t, vw);
        if (!done)
          hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, true>), g1, dim3(RT), 0, s, *a, t, vw);
      }
      else if (eight_waves(S))
        hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S / 2, false, false, 8>), g1, dim3(2 * RT), 0, s,
                           *a, t, vw);
      else
        hipLaunchKernelGGL((rnn_fwd_mm<G, CELL, 0, S, false>), g1, dim3(RT), 0, s, *a, t, vw);
      if (a->ln_gamma) hipLaunchKernelGGL(rnn_ln_fwd, dim3((B2 + 3) / 4), dim3(256), 0, s, *a, t);
    }
  }
  PKC_LAUNCH_CHECK("pkc_rnn_fwd step");
  return PKC_OK;
}

#endif  // PKC_RNN_FWD
#ifdef PKC_RNN_BWD
template <int G, int CELL, int S, bool SP = false>
static int bwd_impl_s(const pkc_rnn_args* a, float* dpre, hipStream_t s) {
  const int B2 = a->bidir ? 2 * a->B : a->B;
  const int vw = pick_vw(a->H);
  const unsigned rows = (unsigned)((B2 + 31) / 32), rows_16 = (unsigned)((B2 + 15) / 16);
  const bool r16 = rows16(B2);
  const int64_t n = (int64_t)B2 * a->H;
  const unsigned eb = (unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
  const dim3 tg((a->H + 31) / 32, (a->H + 31) / 32, G);
  hipLaunchKernelGGL(rnn_transpose_u, tg, dim3(256), 0, s, *a);
  hipLaunchKernelGGL((rnn_bwd_init<G, CELL>), dim3(64), dim3(256), 0, s, *a);
  const bool ln = a->ln_gamma != nullptr;
  const dim3 lg((B2 + 3) / 4);
  if (ln) hipLaunchKernelGGL((rnn_ln_bwd_gates<G, CELL>), lg, dim3(256), 0, s, *a, a->T - 1);
  PKC_LAUNCH_CHECK("pkc_rnn_bwd init");
  const unsigned kt = (unsigned)((a->H + 15) / 16);
  if constexpr (two_phase(CELL)) {
    constexpr int HG = cand_gate(CELL);
    // the candidate gate's U^T product (MODE 2) and the gates' sum (MODE 0 / 1)
    auto mm2 = [&](int t) {
      if (r16)
        hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 2, S, false, 4, true>), dim3(kt, rows_16, 1),
                           dim3(RT), 0, s, *a, t, HG, vw);
      else
        hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 2, S>), dim3(kt, rows, 1), dim3(RT), 0, s, *a, t,
                           HG, vw);
    };
    mm2(a->T - 1);
    for (int tt = a->T - 2; tt >= 0; --tt) {
      if constexpr (CELL == PKC_CELL_GRU) {           // Uz^T dz + Ur^T dr: two gate slabs
        if (r16)
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S, false, 4, true>), dim3(kt, rows_16, 2),
                             dim3(RT), 0, s, *a, tt + 1, 0, vw);
        else
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S>), dim3(kt, rows, 2), dim3(RT), 0, s, *a,
                             tt + 1, 0, vw);
        hipLaunchKernelGGL((rnn_bwd_epi<G, CELL, 2>), dim3(eb), dim3(256), 0, s, *a, tt);
      } else {                                        // minimalGRU: Uz^T dz, one gate
        if (r16)
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 1, S, false, 4, true>), dim3(kt, rows_16, 1),
                             dim3(RT), 0, s, *a, tt + 1, 0, vw);
        else
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 1, S>), dim3(kt, rows, 1), dim3(RT), 0, s, *a,
                             tt + 1, 0, vw);
      }
      if (ln) hipLaunchKernelGGL((rnn_ln_bwd_gates<G, CELL>), lg, dim3(256), 0, s, *a, tt);
      mm2(tt);
    }
  } else {
    if constexpr (!SP) {
      if (a->step_bf16) {              // bf16 BPTT products (dgates_h x ut_h)
        const bool ew = eight_waves(S);
        for (int tt = a->T - 2; tt >= 0; --tt) {
          if constexpr (G == 1) {
            if (r16)
              hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 1, S, false, 4, true, true>),
                                 dim3(kt, rows_16, 1), dim3(RT), 0, s, *a, tt + 1,
                                 0, vw);
            else
              hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 1, S, false, 4, false, true>),
                                 dim3(kt, rows, 1), dim3(RT), 0, s, *a, tt + 1, 0,
                                 vw);
          } else {
            const dim3 gg(kt, r16 ? rows_16 : rows, G);
            if (r16 && ew)
              hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S / 2, false, 8, true, true>),
                                 gg, dim3(2 * RT), 0, s, *a, tt + 1, 0, vw);
            else if (r16)
              hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S, false, 4, true, true>),
                                 gg, dim3(RT), 0, s, *a, tt + 1, 0, vw);
            else if (ew)
              hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S / 2, false, 8, false, true>),
                                 gg, dim3(2 * RT), 0, s, *a, tt + 1, 0, vw);
            else
              hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S, false, 4, false, true>),
                                 gg, dim3(RT), 0, s, *a, tt + 1, 0, vw);
            hipLaunchKernelGGL((rnn_bwd_epi<G, CELL, G, true>), dim3(eb), dim3(256), 0, s,
                               *a, tt);
          }
        }
        PKC_LAUNCH_CHECK("pkc_rnn_bwd bf16 step");
        hipLaunchKernelGGL(rnn_fold_kernel, dim3(1024), dim3(256), 0, s, *a, dpre);
        PKC_LAUNCH_CHECK("pkc_rnn_bwd fold");
        return PKC_OK;
      }
    }
    for (int tt = a->T - 2; tt >= 0; --tt) {
      if constexpr (G == 1) {
        if (r16)
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 1, S, false, 4, true>), dim3(kt, rows_16, 1),
                             dim3(RT), 0, s, *a, tt + 1, 0, vw);
        else
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 1, S>), dim3(kt, rows, 1), dim3(RT), 0, s, *a,
                             tt + 1, 0, vw);
      } else if (r16) {                               // 16-row tiles (C3, C5)
        if (!SP && eight_waves(S))
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S / 2, false, 8, true>), dim3(kt, rows_16, G), dim3(2 * RT), 0, s, *a, tt + 1, 0, vw);
        else if (SP && a->step_bf16)
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S, SP, 4, true, true>), dim3(kt, rows_16, G),
                             dim3(RT), 0, s, *a, tt + 1, 0, vw);
        else
          hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S, SP, 4, true>), dim3(kt, rows_16, G),
                             dim3(RT), 0, s, *a, tt + 1, 0, vw);
        if (SP && a->step_bf16)
          hipLaunchKernelGGL((rnn_bwd_epi<G, CELL, G, true>), dim3(eb), dim3(256), 0, s, *a, tt);
        else
          hipLaunchKernelGGL((rnn_bwd_epi<G, CELL, G>), dim3(eb), dim3(256), 0, s, *a, tt);
      } else if (!SP && eight_waves(S)) {
        hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S / 2, false, 8>), dim3(kt, rows, G),
                           dim3(2 * RT), 0, s, *a, tt + 1, 0, vw);
        hipLaunchKernelGGL((rnn_bwd_epi<G, CELL, G>), dim3(eb), dim3(256), 0, s, *a, tt);
      } else if (SP && a->step_bf16) {
        hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S, SP, 4, false, true>), dim3(kt, rows, G),
                           dim3(RT), 0, s, *a, tt + 1, 0, vw);
        hipLaunchKernelGGL((rnn_bwd_epi<G, CELL, G, true>), dim3(eb), dim3(256), 0, s, *a, tt);
      } else {
        hipLaunchKernelGGL((rnn_bwd_mm<G, CELL, 0, S, SP>), dim3(kt, rows, G), dim3(RT), 0, s, *a,
                           tt + 1, 0, vw);
        hipLaunchKernelGGL((rnn_bwd_epi<G, CELL, G>), dim3(eb), dim3(256), 0, s, *a, tt);
      }
      if (ln) hipLaunchKernelGGL((rnn_ln_bwd_gates<G, CELL>), lg, dim3(256), 0, s, *a, tt);
    }
  }
  if (ln) hipLaunchKernelGGL(rnn_ln_param_grads, dim3((a->H + 63) / 64), dim3(256), 0, s, *a);
  PKC_LAUNCH_CHECK("pkc_rnn_bwd step");
  hipLaunchKernelGGL(rnn_fold_kernel, dim3(1024), dim3(256), 0, s, *a, dpre);
  PKC_LAUNCH_CHECK("pkc_rnn_bwd fold");
  return PKC_OK;
}

#endif  // PKC_RNN_BWD
// contraction strip per lane: 16 lane groups x S >= H
#define PKC_S_DISPATCH(FN, ...)                                      \
  (a->H <= 256 ? FN<G, CELL, 16>(__VA_ARGS__)                        \
   : a->H <= 512 ? FN<G, CELL, 32>(__VA_ARGS__)                      \
   : a->H <= 768 ? FN<G, CELL, 48>(__VA_ARGS__)                      \
   : a->H <= 1024 ? FN<G, CELL, 64>(__VA_ARGS__)                     \
   : FN<G, CELL, 128>(__VA_ARGS__))

}  // namespace

// Persistent liGRU time loops (pkc_rnn_persist.hip): one launch per layer and direction of the
// whole forward / BPTT loop, for block-sparse U in bf16 step mode (pkc_rnn_args.persist_*)
bool rnn_persist_ok(const pkc_rnn_args* a, bool bwd);
int rnn_persist_fwd(const pkc_rnn_args* a, hipStream_t s);
int rnn_persist_bwd(const pkc_rnn_args* a, hipStream_t s);
// Persistent, grid-synchronised LSTM loops with quantised h (pkc_rnn_lstm_persist.hip)
bool rnn_lstm_persist_ok(const pkc_rnn_args* a, bool bwd);
int rnn_lstm_persist_fwd(const pkc_rnn_args* a, hipStream_t s);
int rnn_lstm_persist_bwd(const pkc_rnn_args* a, hipStream_t s);
// the liGRU exact-fp32 step mode in the same grid-synchronised form (pkc_rnn_lstm_persist.hip)
bool rnn_ligru_grid_ok(const pkc_rnn_args* a, bool bwd);
int rnn_ligru_grid_fwd(const pkc_rnn_args* a, hipStream_t s);
int rnn_ligru_grid_bwd(const pkc_rnn_args* a, hipStream_t s);

namespace {

#ifdef PKC_RNN_FWD
template <int G, int CELL>
static int fwd_impl(const pkc_rnn_args* a, hipStream_t s) {
  const int B2 = a->bidir ? 2 * a->B : a->B;
  PKC_HIP_CHECK(hipMemsetAsync(a->hs, 0, sizeof(float) * (size_t)B2 * a->H, s),   // h_init = 0
                "pkc_rnn_fwd h_init");
  if (a->hs_h)
    PKC_HIP_CHECK(hipMemsetAsync(a->hs_h, 0, 2 * (size_t)B2 * a->H, s), "pkc_rnn_fwd h_init (bf16)");
  if constexpr (CELL == PKC_CELL_LSTM)
    PKC_HIP_CHECK(hipMemsetAsync(a->cs, 0, sizeof(float) * (size_t)B2 * a->H, s), "pkc_rnn_fwd c_init");
  if (a->train && a->drop_p > 0.f) {
    hipLaunchKernelGGL(rnn_drop_mask_kernel, dim3(64), dim3(256), 0, s, *a, B2);
    PKC_LAUNCH_CHECK("pkc_rnn_fwd drop mask");
  }
  if constexpr (CELL == PKC_CELL_LIGRU) {
    if (rnn_persist_ok(a, false)) return rnn_persist_fwd(a, s);
    if (rnn_ligru_grid_ok(a, false)) return rnn_ligru_grid_fwd(a, s);
  }
  if constexpr (CELL == PKC_CELL_LSTM) {
    if (rnn_lstm_persist_ok(a, false)) return rnn_lstm_persist_fwd(a, s);
  }
  if constexpr (!two_phase(CELL) && G > 1) {
    if (a->kmap_fwd) {
      if (a->kmap_s_fwd == 16) return fwd_impl_s<G, CELL, 16, true>(a, s);
      if (a->kmap_s_fwd == 32) return fwd_impl_s<G, CELL, 32, true>(a, s);
      return fwd_impl_s<G, CELL, 64, true>(a, s);
    }
  }
  return PKC_S_DISPATCH(fwd_impl_s, a, s);
}

#endif  // PKC_RNN_FWD
#ifdef PKC_RNN_BWD
template <int G, int CELL>
static int bwd_impl(const pkc_rnn_args* a, float* dpre, hipStream_t s) {
  if constexpr (CELL == PKC_CELL_LIGRU) {
    if (rnn_persist_ok(a, true)) {
      const int H = a->H;
      hipLaunchKernelGGL(rnn_transpose_u, dim3((H + 31) / 32, (H + 31) / 32, G), dim3(256), 0, s, *a);
      hipLaunchKernelGGL((rnn_bwd_init<G, CELL>), dim3(64), dim3(256), 0, s, *a);
      PKC_LAUNCH_CHECK("pkc_rnn_bwd init");
      int st = rnn_persist_bwd(a, s);
      if (st) return st;
      hipLaunchKernelGGL(rnn_fold_kernel, dim3(1024), dim3(256), 0, s, *a, dpre);
      PKC_LAUNCH_CHECK("pkc_rnn_bwd fold");
      return PKC_OK;
    }
  }
  if constexpr (CELL == PKC_CELL_LIGRU) {
    if (rnn_ligru_grid_ok(a, true)) {
      const int H = a->H;
      hipLaunchKernelGGL(rnn_transpose_u, dim3((H + 31) / 32, (H + 31) / 32, G), dim3(256), 0, s, *a);
      hipLaunchKernelGGL((rnn_bwd_init<G, CELL>), dim3(64), dim3(256), 0, s, *a);
      PKC_LAUNCH_CHECK("pkc_rnn_bwd init");
      int st = rnn_ligru_grid_bwd(a, s);
      if (st) return st;
      hipLaunchKernelGGL(rnn_fold_kernel, dim3(1024), dim3(256), 0, s, *a, dpre);
      PKC_LAUNCH_CHECK("pkc_rnn_bwd fold");
      return PKC_OK;
    }
  }
  if constexpr (CELL == PKC_CELL_LSTM) {
    if (rnn_lstm_persist_ok(a, true)) {
      const int H = a->H;
      hipLaunchKernelGGL(rnn_transpose_u, dim3((H + 31) / 32, (H + 31) / 32, G), dim3(256), 0, s, *a);
      hipLaunchKernelGGL((rnn_bwd_init<G, CELL>), dim3(64), dim3(256), 0, s, *a);
      PKC_LAUNCH_CHECK("pkc_rnn_bwd init");
      int st = rnn_lstm_persist_bwd(a, s);
      if (st) return st;
      hipLaunchKernelGGL(rnn_fold_kernel, dim3(1024), dim3(256), 0, s, *a, dpre);
      PKC_LAUNCH_CHECK("pkc_rnn_bwd fold");
      return PKC_OK;
    }
  }
  if constexpr (!two_phase(CELL) && G > 1) {
    if (a->kmap_bwd) {
      if (a->kmap_s_bwd == 16) return bwd_impl_s<G, CELL, 16, true>(a, dpre, s);
      if (a->kmap_s_bwd == 32) return bwd_impl_s<G, CELL, 32, true>(a, dpre, s);
      return bwd_impl_s<G, CELL, 64, true>(a, dpre, s);
    }
  }
  return PKC_S_DISPATCH(bwd_impl_s, a, dpre, s);
}

#endif  // PKC_RNN_BWD
[[maybe_unused]] int check(const pkc_rnn_args* a, bool bwd) {
  PKC_CHECK_ARG(a && a->T > 0 && a->B > 0 && a->H > 0 && a->H <= 2048, "pkc_rnn: bad shape (H <= 2048)");
  PKC_CHECK_ARG(a->cell >= PKC_CELL_LIGRU && a->cell <= PKC_CELL_RNN, "pkc_rnn: bad cell %d", a->cell);
  PKC_CHECK_ARG(!two_phase(a->cell) || (a->rh && a->qbits <= 0),
                "pkc_rnn: GRU / minimalGRU need rh and no qbits");
  PKC_CHECK_ARG(a->cell == PKC_CELL_LSTM || a->qbits <= 0, "pkc_rnn: input quantisation only for LSTM");
  PKC_CHECK_ARG(a->wpre && a->hs && a->gates && a->y, "pkc_rnn: null buffer");
  PKC_CHECK_ARG(a->cell != PKC_CELL_LSTM || a->cs, "pkc_rnn: LSTM needs cs");
  const int G = cell_gates(a->cell);
  for (int g = 0; g < G; ++g) PKC_CHECK_ARG(a->U[g], "pkc_rnn: null U[%d]", g);
  PKC_CHECK_ARG(!a->train || a->drop_p <= 0.f || a->drop_mask, "pkc_rnn: dropout needs drop_mask");
  if (bwd) PKC_CHECK_ARG(a->dy && a->dgates && a->work && a->ut, "pkc_rnn_bwd: null buffer");
  PKC_CHECK_ARG(!a->ln_gamma || (a->ln_beta && a->ln_xhat && a->ln_stat && a->H > 1 &&
                                 (!bwd || (a->ln_g && a->ln_dgamma && a->ln_dbeta))),
                "pkc_rnn: LayerNorm needs beta, xhat, stat (+ g, dgamma, dbeta for the backward)");
  PKC_CHECK_ARG(a->qbits <= 0 || (a->hq && !a->bidir && a->B <= 32), "pkc_rnn: quantised h needs "
                "hq, a uni-directional layer and B <= 32");
  if (a->step_bf16) {
    PKC_CHECK_ARG((a->cell == PKC_CELL_LIGRU || a->cell == PKC_CELL_LSTM || a->cell == PKC_CELL_RNN) &&
                      a->qbits <= 0 && !a->ln_gamma,
                  "pkc_rnn: bf16 steps only for liGRU / LSTM / RNN without quantised h or "
                  "LayerNorm");
    PKC_CHECK_ARG(a->hs_h, "pkc_rnn: bf16 steps need hs_h");
    for (int g = 0; g < G; ++g) PKC_CHECK_ARG(a->U_h[g], "pkc_rnn: bf16 steps need U_h[%d]", g);
    if (bwd) PKC_CHECK_ARG(a->ut_h && a->dgates_h, "pkc_rnn_bwd: bf16 steps need ut_h, dgates_h");
  }
  if (a->qh_exact) {
    // (no LayerNorm: the per-wave max|h| partials QX quantises the next step with are recorded
    // from the cell's h, which rnn_ln_fwd would then rewrite — the reference quantises the LN
    // output, neural_networks.py:1093-1094)
    PKC_CHECK_ARG(a->cell == PKC_CELL_LSTM && a->qbits > 0 && a->qbits <= 16 && !a->step_bf16 &&
                      a->work && !a->ln_gamma,
                  "pkc_rnn: qh_exact needs an LSTM with quantised h (qbits <= 16), no LayerNorm, "
                  "fp32 step products and work");
    for (int g = 0; g < G; ++g) PKC_CHECK_ARG(a->U_h[g], "pkc_rnn: qh_exact needs U_h[%d]", g);
  }
  if (a->kmap_fwd || a->kmap_bwd) {
    PKC_CHECK_ARG((a->cell == PKC_CELL_LIGRU || a->cell == PKC_CELL_LSTM) && a->qbits <= 0,
                  "pkc_rnn: block-sparse U only for liGRU / LSTM without quantised h");
    const int sf = a->kmap_s_fwd, sb = a->kmap_s_bwd;
    PKC_CHECK_ARG(!a->kmap_fwd || sf == 16 || sf == 32 || sf == 64, "pkc_rnn: kmap_s_fwd %d", sf);
    PKC_CHECK_ARG(!a->kmap_bwd || sb == 16 || sb == 32 || sb == 64, "pkc_rnn: kmap_s_bwd %d", sb);
  }
  return PKC_OK;
}

}  // namespace

// ---- this translation unit's cell family
#if defined(PKC_RNN_FWD) && PKC_RNN_PART == 0
int rnn_fwd_lstm(const pkc_rnn_args* a, hipStream_t s) { return fwd_impl<4, PKC_CELL_LSTM>(a, s); }
#elif defined(PKC_RNN_FWD) && PKC_RNN_PART == 1
int rnn_fwd_ligru(const pkc_rnn_args* a, hipStream_t s) { return fwd_impl<2, PKC_CELL_LIGRU>(a, s); }
#elif defined(PKC_RNN_FWD) && PKC_RNN_PART == 2
int rnn_fwd_gru(const pkc_rnn_args* a, hipStream_t s) { return fwd_impl<3, PKC_CELL_GRU>(a, s); }
int rnn_fwd_mingru(const pkc_rnn_args* a, hipStream_t s) { return fwd_impl<2, PKC_CELL_MINGRU>(a, s); }
int rnn_fwd_rnn(const pkc_rnn_args* a, hipStream_t s) { return fwd_impl<1, PKC_CELL_RNN>(a, s); }
#endif
#if defined(PKC_RNN_BWD) && PKC_RNN_PART == 0
int rnn_bwd_lstm(const pkc_rnn_args* a, float* d, hipStream_t s) { return bwd_impl<4, PKC_CELL_LSTM>(a, d, s); }
#elif defined(PKC_RNN_BWD) && PKC_RNN_PART == 1
int rnn_bwd_ligru(const pkc_rnn_args* a, float* d, hipStream_t s) { return bwd_impl<2, PKC_CELL_LIGRU>(a, d, s); }
#elif defined(PKC_RNN_BWD) && PKC_RNN_PART == 2
int rnn_bwd_gru(const pkc_rnn_args* a, float* d, hipStream_t s) { return bwd_impl<3, PKC_CELL_GRU>(a, d, s); }
int rnn_bwd_mingru(const pkc_rnn_args* a, float* d, hipStream_t s) { return bwd_impl<2, PKC_CELL_MINGRU>(a, d, s); }
int rnn_bwd_rnn(const pkc_rnn_args* a, float* d, hipStream_t s) { return bwd_impl<1, PKC_CELL_RNN>(a, d, s); }
#endif
}  // namespace pkc

#if defined(PKC_TRACE) && defined(PKC_RNN_FWD)
// measurement builds: this part's forward step-kernel stamps (pkc_trace_read merges the parts)
#define PKC_RNN_TRACE_NAME2(p) pkc_trace_read_fwd##p
#define PKC_RNN_TRACE_NAME(p) PKC_RNN_TRACE_NAME2(p)
extern "C" int PKC_RNN_TRACE_NAME(PKC_RNN_PART)(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(pkc::trace_buf), sizeof(unsigned long long) * n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

#if defined(PKC_RNN_FWD) && PKC_RNN_PART == 0
extern "C" int pkc_rnn_fwd(const pkc_rnn_args* a, void* stream) {
  using namespace pkc;
  int st = check(a, false);
  if (st) return st;
  switch (a->cell) {
    case PKC_CELL_LIGRU: return rnn_fwd_ligru(a, S(stream));
    case PKC_CELL_GRU: return rnn_fwd_gru(a, S(stream));
    case PKC_CELL_MINGRU: return rnn_fwd_mingru(a, S(stream));
    case PKC_CELL_RNN: return rnn_fwd_rnn(a, S(stream));
    default: return rnn_fwd_lstm(a, S(stream));
  }
}

#ifdef PKC_TRACE
extern "C" int pkc_trace_read_fwd0(unsigned long long* host, int n);
extern "C" int pkc_trace_read_fwd1(unsigned long long* host, int n);
extern "C" int pkc_trace_read_fwd2(unsigned long long* host, int n);
// measurement builds only: the forward step kernels' stamps (n <= TRACE_WG * TRACE_SLOTS) — the
// three parts' buffers merged (a part whose kernels did not run left zeros)
extern "C" int pkc_trace_read(unsigned long long* host, int n) {
  if (pkc_trace_read_fwd0(host, n)) return -1;
  unsigned long long* tmp = new unsigned long long[n];
  int st = 0;
  for (int p = 1; p <= 2 && !st; ++p) {
    st = p == 1 ? pkc_trace_read_fwd1(tmp, n) : pkc_trace_read_fwd2(tmp, n);
    for (int i = 0; i < n && !st; ++i) host[i] = host[i] > tmp[i] ? host[i] : tmp[i];
  }
  delete[] tmp;
  return st;
}
#endif

#endif
#if defined(PKC_RNN_BWD) && PKC_RNN_PART == 0
extern "C" int pkc_rnn_bwd(const pkc_rnn_args* a, float* dpre, void* stream) {
  using namespace pkc;
  int st = check(a, true);
  if (st) return st;
  PKC_CHECK_ARG(dpre, "pkc_rnn_bwd: null dpre");
  switch (a->cell) {
    case PKC_CELL_LIGRU: return rnn_bwd_ligru(a, dpre, S(stream));
    case PKC_CELL_GRU: return rnn_bwd_gru(a, dpre, S(stream));
    case PKC_CELL_MINGRU: return rnn_bwd_mingru(a, dpre, S(stream));
    case PKC_CELL_RNN: return rnn_bwd_rnn(a, dpre, S(stream));
    default: return rnn_bwd_lstm(a, dpre, S(stream));
  }
}
#endif
