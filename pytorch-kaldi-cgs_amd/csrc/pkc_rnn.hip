// pkc_rnn.hip — the serial time loops of liGRU and LSTM layers (forward and BPTT).
//
// Reference: liGRU  neural_networks.py:1573-1584 (z = sig(wz+Uz h); hc = act(wh+Uh h)*drop;
//                   h = z*h + (1-z)*hc), shared-weight bidirectional rows via cat/flip
//                   (:1536-1538, :1590-1594);
//            LSTM   neural_networks.py:1077-1097 (f,i,o = sig(w+U h); c = i*act(wc+Uc h)*drop + f*c;
//                   h = o*act(c)).
// The input projections W x (+BN) are one big MFMA matmul over all T*B rows outside the loop
// (pkc_gemm + pkc_dense_fwd); here each time step is ONE launch that computes every gate's
// recurrent product U h_{t-1} for a 16-unit x 16-row tile and applies the cell update in the
// epilogue.  Bidirectional layers run both directions as one 2B-row batch: row r < B reads time t,
// row r >= B reads time T-1-t of the same (T, B, H) pre-activations (the reference's flip), and
// writes its h into the second half of the (T, B, 2H) output at T-1-t.
//
// BPTT: one launch per step.  For its 16-unit column slice k the kernel forms
//   dh_{t-1}[r][k] = sum_g sum_j da_g[t][r][j] * U_g[j][k]   (+ elementwise carry terms)
// and immediately turns it into the gate gradients of step t-1 at (r, k), so the loop needs no
// second launch per step.  dU and dW are big matmuls after the loop.
//
// GRU (neural_networks.py:1390-1396: z, r = sig(w + U h); a = wh + Uh (r*h); hc = act(a)*drop;
// h = z*h + (1-z)*hc) multiplies Uh with r*h, which needs the r of every unit of the row first, so
// a step is two launches: (z, r, r*h) then (Uh (r*h), update).  Its BPTT step is two launches as
// well: d(rh) = Uh^T da (then dr), and dh_{t-1} = Uz^T dz + Ur^T dr + carries (then dz, da).
// r*h is kept for every step (rh, (T, B2, H)): it is the input of the Uh gradient matmul.
// minimalGRU (neural_networks.py:1751-1755) is the same two-phase step with r replaced by z
// (a = wh + Uh (z*h)); the plain RNN (:1905-1907, h = act(wh + Uh h)*drop) is one gate, one
// launch per step.
#include "pkc_common.h"

namespace pkc {

constexpr int RU = 16, RR = 16, RT = RU * RR, KC = 64;

__host__ __device__ constexpr int cell_gates(int cell) {
  return cell == PKC_CELL_LSTM ? 4 : cell == PKC_CELL_GRU ? 3 : cell == PKC_CELL_RNN ? 1 : 2;
}
// index of the candidate ("h") gate whose U multiplies r*h / z*h (two-phase cells)
__host__ __device__ constexpr int cand_gate(int cell) { return cell == PKC_CELL_GRU ? 2 : 1; }
__host__ __device__ constexpr bool two_phase(int cell) {
  return cell == PKC_CELL_GRU || cell == PKC_CELL_MINGRU;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

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
__device__ __forceinline__ float qin(float x, float var, float scale) {
  if (var == 0.f) return x;
  const float s = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
  return ceilf(fabsf(x / var) * scale) / scale * var * s;
}

template <int G>
__device__ void h_quant_vars(const float* hprev, int64_t n, float scale, float* vars) {
  // vars[g] = max(|max q_g|, |min q_g|) over all of h_{t-1}, q_0 = h (block-redundant reduction)
  __shared__ float rmx[RT], rmn[RT];
  for (int g = 0; g < G; ++g) {
    float mx = -INFINITY, mn = INFINITY;
    for (int64_t e = threadIdx.x; e < n; e += RT) {
      float v = hprev[e];
      for (int p = 0; p < g; ++p) v = qin(v, vars[p], scale);
      mx = fmaxf(mx, v);
      mn = fminf(mn, v);
    }
    rmx[threadIdx.x] = mx;
    rmn[threadIdx.x] = mn;
    __syncthreads();
    for (int o = RT / 2; o > 0; o >>= 1) {
      if (threadIdx.x < o) {
        rmx[threadIdx.x] = fmaxf(rmx[threadIdx.x], rmx[threadIdx.x + o]);
        rmn[threadIdx.x] = fminf(rmn[threadIdx.x], rmn[threadIdx.x + o]);
      }
      __syncthreads();
    }
    const float a = fabsf(rmx[0]), b = fabsf(rmn[0]);
    vars[g] = a > b ? a : b;
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------- forward step
template <int G, int CELL, bool QH>
__global__ __launch_bounds__(RT) void rnn_fwd_step(pkc_rnn_args a, int t) {
  __shared__ float hsm[QH ? G : 1][RR][KC + 1];
  __shared__ float usm[G][RU][KC + 1];
  const RnnIdx ix = mkidx(a);
  const int j = blockIdx.x * RU + threadIdx.x % RU;
  const int r = blockIdx.y * RR + threadIdx.x / RU;
  const int H = a.H;
  const float* hprev = a.hs + (int64_t)t * ix.B2 * H;     // hs[t] = h_{t-1}
  float vars[4] = {0.f, 0.f, 0.f, 0.f};
  const float qscale = QH ? ldexpf(1.f, a.qbits - 1) : 1.f;
  if (QH) h_quant_vars<G>(hprev, (int64_t)ix.B2 * H, qscale, vars);
  float acc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g] = 0.f;
  for (int k0 = 0; k0 < H; k0 += KC) {
    __syncthreads();
    for (int e = threadIdx.x; e < RR * KC; e += RT) {
      const int rr = e / KC, kk = e % KC;
      const int R = blockIdx.y * RR + rr, K = k0 + kk;
      float v = (R < ix.B2 && K < H) ? hprev[(int64_t)R * H + K] : 0.f;
      if (QH) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          v = qin(v, vars[g], qscale);
          hsm[g][rr][kk] = v;
        }
      } else {
        hsm[0][rr][kk] = v;
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
      for (int e = threadIdx.x; e < RU * KC; e += RT) {
        const int jj = e / KC, kk = e % KC;
        const int J = blockIdx.x * RU + jj, K = k0 + kk;
        usm[g][jj][kk] = (J < H && K < H) ? a.U[g][(int64_t)J * H + K] : 0.f;
      }
    __syncthreads();
    const int rl = threadIdx.x / RU, jl = threadIdx.x % RU;
#pragma unroll 8
    for (int kk = 0; kk < KC; ++kk) {
#pragma unroll
      for (int g = 0; g < G; ++g) acc[g] = fmaf(usm[g][jl][kk], hsm[QH ? g : 0][rl][kk], acc[g]);
    }
  }
  if (r >= ix.B2 || j >= H) return;
  if (QH) {
    // the hidden state the reference keeps for step t-1 (hiddens[t-1], and the saved input of the
    // U backward) is the 4x re-quantised tensor; the last step's h is never quantised
    float v = hprev[(int64_t)r * H + j];
#pragma unroll
    for (int g = 0; g < G; ++g) v = qin(v, vars[g], qscale);
    a.hq[(int64_t)t * ix.B2 * H + (int64_t)r * H + j] = v;
    if (t > 0) a.y[ix.out(t - 1, r, j)] = v;
  }
  const int64_t TBH = (int64_t)a.T * a.B * H;   // gate stride of the (G, T, B, H) pre-activations
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H; // gate stride of the saved activations
  const int64_t pi = ix.pre(t, r, j), si = ix.st(t, r, j);
  const float m = drop_val(a, r, j, ix.B2);
  const float hp = hprev[(int64_t)r * H + j];
  float h;
  if constexpr (CELL == PKC_CELL_GRU) {
    // phase 1 of a GRU step: update / reset gates and r*h (the input of Uh)
    const float z = sigm(a.wpre[pi] + acc[0]);
    const float rg = sigm(a.wpre[TBH + pi] + acc[1]);
    a.gates[si] = z;
    a.gates[TB2H + si] = rg;
    a.rh[si] = rg * hp;
    return;
  }
  if constexpr (CELL == PKC_CELL_MINGRU) {
    // phase 1 of a minimalGRU step: update gate and z*h (the input of Uh)
    const float z = sigm(a.wpre[pi] + acc[0]);
    a.gates[si] = z;
    a.rh[si] = z * hp;
    return;
  }
  if constexpr (CELL == PKC_CELL_RNN) {
    const float hcr = act_fwd(a.act, a.wpre[pi] + acc[0]);
    h = hcr * m;
    a.gates[si] = hcr;
    a.hs[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + j] = h;
    a.y[ix.out(t, r, j)] = h;
    return;
  }
  if constexpr (CELL == PKC_CELL_LIGRU) {
    // gates (z, h) -- liGRU
    const float z = sigm(a.wpre[pi] + acc[0]);
    const float hcr = act_fwd(a.act, a.wpre[TBH + pi] + acc[1]);
    const float hc = hcr * m;
    h = z * hp + (1.f - z) * hc;
    a.gates[si] = z;
    a.gates[TB2H + si] = hcr;
  } else if constexpr (CELL == PKC_CELL_LSTM) {
    // gates (f, i, o, c) -- LSTM; cs[t] = c_{t-1}
    const float f = sigm(a.wpre[pi] + acc[0]);
    const float i = sigm(a.wpre[TBH + pi] + acc[1]);
    const float o = sigm(a.wpre[2 * TBH + pi] + acc[2]);
    const float cc = act_fwd(a.act, a.wpre[3 * TBH + pi] + acc[3]);
    const float cp = a.cs[(int64_t)t * ix.B2 * H + (int64_t)r * H + j];
    const float c = i * cc * m + f * cp;
    h = o * act_fwd(a.act, c);
    a.cs[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + j] = c;
    a.gates[si] = f;
    a.gates[TB2H + si] = i;
    a.gates[2 * TB2H + si] = o;
    a.gates[3 * TB2H + si] = cc;
  }
  a.hs[(int64_t)(t + 1) * ix.B2 * H + (int64_t)r * H + j] = h;
  a.y[ix.out(t, r, j)] = h;
}

// phase 2 of a GRU / minimalGRU step: a = wh + Uh (r*h_{t-1} | z*h_{t-1});
// h = z*h_{t-1} + (1-z)*act(a)*drop.  HG: index of the candidate gate.
template <int HG>
__global__ __launch_bounds__(RT) void gru_fwd_h(pkc_rnn_args a, int t) {
  __shared__ float hsm[RR][KC + 1];
  __shared__ float usm[RU][KC + 1];
  const RnnIdx ix = mkidx(a);
  const int j = blockIdx.x * RU + threadIdx.x % RU;
  const int r = blockIdx.y * RR + threadIdx.x / RU;
  const int H = a.H;
  const float* src = a.rh + (int64_t)t * ix.B2 * H;
  const float* U = a.U[HG];
  float acc = 0.f;
  for (int k0 = 0; k0 < H; k0 += KC) {
    __syncthreads();
    for (int e = threadIdx.x; e < RR * KC; e += RT) {
      const int rr = e / KC, kk = e % KC;
      const int R = blockIdx.y * RR + rr, K = k0 + kk;
      hsm[rr][kk] = (R < ix.B2 && K < H) ? src[(int64_t)R * H + K] : 0.f;
    }
    for (int e = threadIdx.x; e < RU * KC; e += RT) {
      const int jj = e / KC, kk = e % KC;
      const int J = blockIdx.x * RU + jj, K = k0 + kk;
      usm[jj][kk] = (J < H && K < H) ? U[(int64_t)J * H + K] : 0.f;
    }
    __syncthreads();
    const int rl = threadIdx.x / RU, jl = threadIdx.x % RU;
#pragma unroll 8
    for (int kk = 0; kk < KC; ++kk) acc = fmaf(usm[jl][kk], hsm[rl][kk], acc);
  }
  if (r >= ix.B2 || j >= H) return;
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

// ------------------------------------------------------------------------------- backward
__device__ __forceinline__ float dy_at(const pkc_rnn_args& a, int64_t i) {
  const int ns = a.dy_nslab > 0 ? a.dy_nslab : 1;
  float s = 0.f;
  for (int q = 0; q < ns; ++q) s += a.dy[(int64_t)q * a.dy_slab_stride + i];
  return s;
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
    const float z = a.gates[si], hcr = a.gates[TB2H + si];
    const float hc = hcr * m;
    const float dz = g * (hp - hc);
    const float dhc = g * (1.f - z);
    dgo[0] = dz * z * (1.f - z);
    dgo[1] = dhc * m * act_bwd_out(a.act, hcr);   // act' from the post-activation value
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
    const float tc = act_fwd(a.act, c);
    const float dc = g * o * act_bwd_out(a.act, tc) + dc_carry;
    dgo[0] = dc * cp * f * (1.f - f);
    dgo[1] = dc * cc * m * i * (1.f - i);
    dgo[2] = g * tc * o * (1.f - o);
    dgo[3] = dc * i * m * act_bwd_out(a.act, cc);
    *dc_out = dc * f;            // carried into step t-1
    *g_out = g;
  }
}

// first backward launch: step T-1, no recurrent gradient yet
template <int G, int CELL>
__global__ void rnn_bwd_init(pkc_rnn_args a) {
  const RnnIdx ix = mkidx(a);
  const int64_t n = (int64_t)ix.B2 * a.H;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * a.H;
  const int t = a.T - 1;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(e / a.H), k = (int)(e % a.H);
    const float g = dy_at(a, ix.out(t, r, k));
    float dg[4], go, dco = 0.f;
    gate_grads<CELL>(a, ix, t, r, k, g, 0.f, dg, &go, &dco);
    if constexpr (CELL == PKC_CELL_GRU) {
      a.dgates[ix.st(t, r, k)] = dg[0];
      a.dgates[2 * TB2H + ix.st(t, r, k)] = dg[2];
    } else if constexpr (CELL == PKC_CELL_MINGRU) {
      a.dgates[TB2H + ix.st(t, r, k)] = dg[1];
    } else {
#pragma unroll
      for (int q = 0; q < G; ++q) a.dgates[q * TB2H + ix.st(t, r, k)] = dg[q];
    }
    a.work[e] = go;                 // g ping  (step parity 1)
    a.work[2 * n + e] = dco;        // dc ping
  }
}

// launch for target step tt = t-1 (t = tt+1 already has its gate gradients)
template <int G, int CELL>
__global__ __launch_bounds__(RT) void rnn_bwd_step(pkc_rnn_args a, int tt) {
  __shared__ float dsm[G][RR][KC + 1];
  __shared__ float usm[G][KC][RU + 1];
  const RnnIdx ix = mkidx(a);
  const int H = a.H;
  const int k = blockIdx.x * RU + threadIdx.x % RU;
  const int r = blockIdx.y * RR + threadIdx.x / RU;
  const int t = tt + 1;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H;
  const int64_t n = (int64_t)ix.B2 * H;
  const int src = (a.T - 1 - t) & 1, dst = src ^ 1;      // ping-pong slots of g / dc
  float acc = 0.f;
  for (int j0 = 0; j0 < H; j0 += KC) {
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; ++g) {
      for (int e = threadIdx.x; e < RR * KC; e += RT) {
        const int rr = e / KC, jj = e % KC;
        const int R = blockIdx.y * RR + rr, J = j0 + jj;
        dsm[g][rr][jj] = (R < ix.B2 && J < H) ? a.dgates[g * TB2H + ix.st(t, R, J)] : 0.f;
      }
      for (int e = threadIdx.x; e < KC * RU; e += RT) {
        const int jj = e / RU, kk = e % RU;
        const int J = j0 + jj, K = blockIdx.x * RU + kk;
        usm[g][jj][kk] = (J < H && K < H) ? a.U[g][(int64_t)J * H + K] : 0.f;
      }
    }
    __syncthreads();
    const int rl = threadIdx.x / RU, kl = threadIdx.x % RU;
#pragma unroll 4
    for (int jj = 0; jj < KC; ++jj) {
#pragma unroll
      for (int g = 0; g < G; ++g) acc = fmaf(dsm[g][rl][jj], usm[g][jj][kl], acc);
    }
  }
  if (r >= ix.B2 || k >= H) return;
  const int64_t e = (int64_t)r * H + k;
  float dh = acc;
  float dc_carry = 0.f;
  if constexpr (CELL == PKC_CELL_LIGRU) {
    dh += a.work[src * n + e] * a.gates[ix.st(t, r, k)];     // g_t * z_t
  } else if constexpr (CELL == PKC_CELL_GRU) {
    // g_t * z_t + d(rh)_t * r_t  (acc = Uz^T dz_t + Ur^T dr_t)
    dh += a.work[src * n + e] * a.gates[ix.st(t, r, k)] +
          a.work[2 * n + e] * a.gates[TB2H + ix.st(t, r, k)];
  } else if constexpr (CELL == PKC_CELL_MINGRU) {
    // (g_t + d(zh)_t) * z_t  (acc = Uz^T dz_t)
    dh += (a.work[src * n + e] + a.work[2 * n + e]) * a.gates[ix.st(t, r, k)];
  } else if constexpr (CELL == PKC_CELL_RNN) {
    // acc = Uh^T da_t is the whole recurrent gradient
  } else {
    dc_carry = a.work[2 * n + src * n + e];                  // dc_t * f_t
  }
  const float g = dy_at(a, ix.out(tt, r, k)) + dh;
  float dg[4], go, dco = 0.f;
  gate_grads<CELL>(a, ix, tt, r, k, g, dc_carry, dg, &go, &dco);
  if constexpr (CELL == PKC_CELL_GRU) {
    a.dgates[ix.st(tt, r, k)] = dg[0];
    a.dgates[2 * TB2H + ix.st(tt, r, k)] = dg[2];
    a.work[dst * n + e] = go;
    return;
  }
  if constexpr (CELL == PKC_CELL_MINGRU) {
    a.dgates[TB2H + ix.st(tt, r, k)] = dg[1];
    a.work[dst * n + e] = go;
    return;
  }
#pragma unroll
  for (int q = 0; q < G; ++q) a.dgates[q * TB2H + ix.st(tt, r, k)] = dg[q];
  a.work[dst * n + e] = go;
  a.work[2 * n + dst * n + e] = dco;
}

// GRU: d(rh)_t[r][k] = sum_j da_t[r][j] Uh[j][k]; dr_t = d(rh) * h_{t-1} * r (1 - r).
// d(rh)_t is kept in work[2n..3n) for the carry term of the next (earlier) step.
template <int CELL>
__global__ __launch_bounds__(RT) void gru_bwd_rh(pkc_rnn_args a, int t) {
  constexpr int HG = cand_gate(CELL);
  __shared__ float dsm[RR][KC + 1];
  __shared__ float usm[KC][RU + 1];
  const RnnIdx ix = mkidx(a);
  const int H = a.H;
  const int k = blockIdx.x * RU + threadIdx.x % RU;
  const int r = blockIdx.y * RR + threadIdx.x / RU;
  const int64_t TB2H = (int64_t)a.T * ix.B2 * H;
  const int64_t n = (int64_t)ix.B2 * H;
  const float* U = a.U[HG];
  float acc = 0.f;
  for (int j0 = 0; j0 < H; j0 += KC) {
    __syncthreads();
    for (int e = threadIdx.x; e < RR * KC; e += RT) {
      const int rr = e / KC, jj = e % KC;
      const int R = blockIdx.y * RR + rr, J = j0 + jj;
      dsm[rr][jj] = (R < ix.B2 && J < H) ? a.dgates[HG * TB2H + ix.st(t, R, J)] : 0.f;
    }
    for (int e = threadIdx.x; e < KC * RU; e += RT) {
      const int jj = e / RU, kk = e % RU;
      const int J = j0 + jj, K = blockIdx.x * RU + kk;
      usm[jj][kk] = (J < H && K < H) ? U[(int64_t)J * H + K] : 0.f;
    }
    __syncthreads();
    const int rl = threadIdx.x / RU, kl = threadIdx.x % RU;
#pragma unroll 8
    for (int jj = 0; jj < KC; ++jj) acc = fmaf(dsm[rl][jj], usm[jj][kl], acc);
  }
  if (r >= ix.B2 || k >= H) return;
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

// fold the per-direction gate gradients (G, T, B2, H) onto the (G, T, B, H) pre-activation rows
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

template <int G, int CELL>
static int fwd_impl(const pkc_rnn_args* a, hipStream_t s) {
  const int B2 = a->bidir ? 2 * a->B : a->B;
  hipMemsetAsync(a->hs, 0, sizeof(float) * (size_t)B2 * a->H, s);            // h_init = 0
  if constexpr (CELL == PKC_CELL_LSTM) hipMemsetAsync(a->cs, 0, sizeof(float) * (size_t)B2 * a->H, s);
  if (a->train && a->drop_p > 0.f) {
    hipLaunchKernelGGL(rnn_drop_mask_kernel, dim3(64), dim3(256), 0, s, *a, B2);
    PKC_LAUNCH_CHECK("pkc_rnn_fwd drop mask");
  }
  dim3 grid((a->H + RU - 1) / RU, (B2 + RR - 1) / RR);
  if constexpr (two_phase(CELL)) {
    // phase 1 multiplies the gates that read h (GRU: z, r; minimalGRU: z) = all but the candidate
    for (int t = 0; t < a->T; ++t) {
      hipLaunchKernelGGL((rnn_fwd_step<G - 1, CELL, false>), grid, dim3(RT), 0, s, *a, t);
      hipLaunchKernelGGL(gru_fwd_h<cand_gate(CELL)>, grid, dim3(RT), 0, s, *a, t);
    }
    PKC_LAUNCH_CHECK("pkc_rnn_fwd gru step");
    return PKC_OK;
  }
  for (int t = 0; t < a->T; ++t) {
    if (a->qbits > 0)
      hipLaunchKernelGGL((rnn_fwd_step<G, CELL, true>), grid, dim3(RT), 0, s, *a, t);
    else
      hipLaunchKernelGGL((rnn_fwd_step<G, CELL, false>), grid, dim3(RT), 0, s, *a, t);
  }
  PKC_LAUNCH_CHECK("pkc_rnn_fwd step");
  return PKC_OK;
}

template <int G, int CELL>
static int bwd_impl(const pkc_rnn_args* a, float* dpre, hipStream_t s) {
  const int B2 = a->bidir ? 2 * a->B : a->B;
  hipLaunchKernelGGL((rnn_bwd_init<G, CELL>), dim3(64), dim3(256), 0, s, *a);
  PKC_LAUNCH_CHECK("pkc_rnn_bwd init");
  dim3 grid((a->H + RU - 1) / RU, (B2 + RR - 1) / RR);
  if constexpr (two_phase(CELL)) {
    hipLaunchKernelGGL(gru_bwd_rh<CELL>, grid, dim3(RT), 0, s, *a, a->T - 1);
    for (int tt = a->T - 2; tt >= 0; --tt) {
      hipLaunchKernelGGL((rnn_bwd_step<G - 1, CELL>), grid, dim3(RT), 0, s, *a, tt);
      hipLaunchKernelGGL(gru_bwd_rh<CELL>, grid, dim3(RT), 0, s, *a, tt);
    }
  } else {
    for (int tt = a->T - 2; tt >= 0; --tt)
      hipLaunchKernelGGL((rnn_bwd_step<G, CELL>), grid, dim3(RT), 0, s, *a, tt);
  }
  PKC_LAUNCH_CHECK("pkc_rnn_bwd step");
  hipLaunchKernelGGL(rnn_fold_kernel, dim3(1024), dim3(256), 0, s, *a, dpre);
  PKC_LAUNCH_CHECK("pkc_rnn_bwd fold");
  return PKC_OK;
}

static int check(const pkc_rnn_args* a, bool bwd) {
  PKC_CHECK_ARG(a && a->T > 0 && a->B > 0 && a->H > 0, "pkc_rnn: bad shape");
  PKC_CHECK_ARG(a->cell >= PKC_CELL_LIGRU && a->cell <= PKC_CELL_RNN, "pkc_rnn: bad cell %d", a->cell);
  PKC_CHECK_ARG(!two_phase(a->cell) || (a->rh && a->qbits <= 0),
                "pkc_rnn: GRU / minimalGRU need rh and no qbits");
  PKC_CHECK_ARG(a->cell == PKC_CELL_LSTM || a->cell == PKC_CELL_LIGRU || a->qbits <= 0,
                "pkc_rnn: input quantisation only for LSTM / liGRU");
  PKC_CHECK_ARG(a->wpre && a->hs && a->gates && a->y, "pkc_rnn: null buffer");
  PKC_CHECK_ARG(a->cell != PKC_CELL_LSTM || a->cs, "pkc_rnn: LSTM needs cs");
  const int G = cell_gates(a->cell);
  for (int g = 0; g < G; ++g) PKC_CHECK_ARG(a->U[g], "pkc_rnn: null U[%d]", g);
  PKC_CHECK_ARG(!a->train || a->drop_p <= 0.f || a->drop_mask, "pkc_rnn: dropout needs drop_mask");
  if (bwd) PKC_CHECK_ARG(a->dy && a->dgates && a->work, "pkc_rnn_bwd: null buffer");
  PKC_CHECK_ARG(a->qbits <= 0 || (a->hq && !a->bidir && (a->bidir ? 2 * a->B : a->B) <= RR),
                "pkc_rnn: quantised h needs hq, a uni-directional layer and <= %d rows", RR);
  return PKC_OK;
}

}  // namespace pkc

extern "C" int pkc_rnn_fwd(const pkc_rnn_args* a, void* stream) {
  using namespace pkc;
  int st = check(a, false);
  if (st) return st;
  if (a->cell == PKC_CELL_LIGRU) return fwd_impl<2, PKC_CELL_LIGRU>(a, S(stream));
  if (a->cell == PKC_CELL_GRU) return fwd_impl<3, PKC_CELL_GRU>(a, S(stream));
  if (a->cell == PKC_CELL_MINGRU) return fwd_impl<2, PKC_CELL_MINGRU>(a, S(stream));
  if (a->cell == PKC_CELL_RNN) return fwd_impl<1, PKC_CELL_RNN>(a, S(stream));
  return fwd_impl<4, PKC_CELL_LSTM>(a, S(stream));
}

extern "C" int pkc_rnn_bwd(const pkc_rnn_args* a, float* dpre, void* stream) {
  using namespace pkc;
  int st = check(a, true);
  if (st) return st;
  PKC_CHECK_ARG(dpre, "pkc_rnn_bwd: null dpre");
  if (a->cell == PKC_CELL_LIGRU) return bwd_impl<2, PKC_CELL_LIGRU>(a, dpre, S(stream));
  if (a->cell == PKC_CELL_GRU) return bwd_impl<3, PKC_CELL_GRU>(a, dpre, S(stream));
  if (a->cell == PKC_CELL_MINGRU) return bwd_impl<2, PKC_CELL_MINGRU>(a, dpre, S(stream));
  if (a->cell == PKC_CELL_RNN) return bwd_impl<1, PKC_CELL_RNN>(a, dpre, S(stream));
  return bwd_impl<4, PKC_CELL_LSTM>(a, dpre, S(stream));
}
