// pkc_loss.hip — fused LogSoftmax + NLLLoss + error rate + backward for one output head.
//
// Replaces, per head, the reference's LogSoftmax (neural_networks.py:73-74), nn.NLLLoss mean
// (utils.py:1811-1812, 1935-1952), cost_err argmax (utils.py:1993-2011) and their autograd backward
// (d logits = w/M * (softmax - onehot)) with one row-parallel pass: one wave per frame row, the
// split-K slabs of the head matmul summed in fixed order.
#include "pkc_ops.h"

namespace pkc {

constexpr int LW = 4;  // waves per workgroup

__device__ __forceinline__ float slab_sum4(const float* __restrict__ p, int64_t stride, int nslab) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 4 <= nslab; s += 4) {
    a0 += p[(int64_t)s * stride];
    a1 += p[(int64_t)(s + 1) * stride];
    a2 += p[(int64_t)(s + 2) * stride];
    a3 += p[(int64_t)(s + 3) * stride];
  }
  for (; s < nslab; ++s) a0 += p[(int64_t)s * stride];
  return (a0 + a1) + (a2 + a3);
}

// WPR waves cooperate on one row (WPR = 4 for wide heads such as 1928 senones, 1 for narrow ones)
template <int WPR>
__global__ __launch_bounds__(64 * LW) void nll_kernel(pkc_nll_args a) {
  constexpr int RPB = LW / WPR;             // rows per workgroup
  constexpr int T = 64 * WPR;               // threads per row
  __shared__ float sh_m[LW], sh_s[LW];
  __shared__ int sh_a[LW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rl = wave / WPR;                // row within the workgroup
  const int tr = threadIdx.x - rl * T;      // thread index within the row
  const int r = blockIdx.x * RPB + rl;
  const bool rok = r < a.M;
  const int64_t N = a.N;
  float* zrow = a.logp + (int64_t)(rok ? r : 0) * N;   // z staged in the logp row
  float mx = -INFINITY;
  int arg = 0x7fffffff;
  if (rok)
    for (int j = tr; j < a.N; j += T) {
      float z = slab_sum4(a.zslab + r * N + j, a.slab_stride, a.nslab);
      if (a.bias) z += a.bias[j];
      zrow[j] = z;
      if (z > mx) { mx = z; arg = j; }   // first max per thread (ascending j)
    }
  // argmax: max value, smallest index among equals
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  if (WPR > 1) {
    if (lane == 0) { sh_m[wave] = mx; sh_a[wave] = arg; }
    __syncthreads();
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) {
      const float om = sh_m[w];
      const int oa = sh_a[w];
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
  }
  float se = 0.f;
  if (rok)
    for (int j = tr; j < a.N; j += T) se += expf(zrow[j] - mx);
  se = warp_sum(se);
  if (WPR > 1) {
    if (lane == 0) sh_s[wave] = se;
    __syncthreads();
    se = 0.f;
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) se += sh_s[w];
  }
  if (!rok) return;
  const float lse = mx + logf(se);
  const int y = a.labels ? a.labels[(int64_t)r * a.label_stride] : -1;
  const float gscale = a.weight / (float)a.M;
  float lp_y = 0.f;
  for (int j = tr; j < a.N; j += T) {
    const float lp = zrow[j] - lse;
    if (j == y) lp_y = lp;
    if (a.dlogits) {
      const float p = expf(lp);
      const float d = gscale * (j == y ? p - 1.f : p);
      a.dlogits[(int64_t)r * N + j] = d;
      if (a.dlogits_bf16) reinterpret_cast<__bf16*>(a.dlogits_bf16)[(int64_t)r * N + j] = (__bf16)d;
    }
    zrow[j] = a.log_prior ? lp - a.log_prior[j] : lp;
  }
  // exactly one thread of the row saw j == y: it writes the row's loss / error
  if (y >= 0 && y < a.N && (y % T) == tr) {
    if (a.row_loss) a.row_loss[r] = -lp_y;
    if (a.row_err) a.row_err[r] = (arg != y) ? 1.f : 0.f;
  }
}

// Register-resident form for heads up to 8 values per thread (N <= 2048 with 4 waves per row,
// N <= 512 with one): the row's logits are summed from the slabs ONCE, kept in registers through
// max / sum-exp / outputs, and every slab load is issued up front (clamped, not branched).
struct NllShared {
  float m[LW], s[LW];
  int a[LW];
};

template <int WPR, int NS>
__device__ __forceinline__ void nll_reg_body(const pkc_nll_args& a, int block, NllShared& sh) {
  constexpr int RPB = LW / WPR;
  constexpr int T = 64 * WPR;
  constexpr int NPT = 8;
  float* sh_m = sh.m;
  float* sh_s = sh.s;
  int* sh_a = sh.a;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rl = wave / WPR;
  const int tr = threadIdx.x - rl * T;
  const int r = block * RPB + rl;
  const bool rok = r < a.M;
  const int64_t N = a.N;
  const int rr = rok ? r : a.M - 1;
  const float* zb = a.zslab + (int64_t)rr * N;
  // the row's label is requested with the logits (never after the reductions)
  const int y_ = *(a.labels ? a.labels + (int64_t)rr * a.label_stride
                            : reinterpret_cast<const int32_t*>(a.zslab));
  float v[NPT][NS];
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    const int j = min(tr + T * q, a.N - 1);
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int st = t < a.nslab ? t : a.nslab - 1;
      v[q][t] = zb[(int64_t)st * a.slab_stride + j];
    }
  }
  float z[NPT];
  float mx = -INFINITY;
  int arg = 0x7fffffff;
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    const int j = tr + T * q;
    float acc = v[q][0];
#pragma unroll
    for (int t = 1; t < NS; ++t) acc += (t < a.nslab) ? v[q][t] : 0.f;
    if (a.bias) acc += a.bias[min(j, a.N - 1)];
    z[q] = acc;
    if (j < a.N && acc > mx) { mx = acc; arg = j; }   // ascending j: first max per thread
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  if (WPR > 1) {
    if (lane == 0) { sh_m[wave] = mx; sh_a[wave] = arg; }
    __syncthreads();
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) {
      const float om = sh_m[w];
      const int oa = sh_a[w];
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
  }
  float se = 0.f;
#pragma unroll
  for (int q = 0; q < NPT; ++q)
    if (tr + T * q < a.N) se += expf(z[q] - mx);
  se = warp_sum(se);
  if (WPR > 1) {
    if (lane == 0) sh_s[wave] = se;
    __syncthreads();
    se = 0.f;
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) se += sh_s[w];
  }
  if (!rok) return;
  const float lse = mx + logf(se);
  const int y = a.labels ? y_ : -1;
  const float gscale = a.weight / (float)a.M;
  float* lrow = a.logp + (int64_t)r * N;
#pragma unroll
  for (int q = 0; q < NPT; ++q) {
    const int j = tr + T * q;
    if (j >= a.N) break;
    const float lp = z[q] - lse;
    if (a.dlogits) {
      const float p = expf(lp);
      const float d = gscale * (j == y ? p - 1.f : p);
      a.dlogits[(int64_t)r * N + j] = d;
      if (a.dlogits_bf16) reinterpret_cast<__bf16*>(a.dlogits_bf16)[(int64_t)r * N + j] = (__bf16)d;
    }
    lrow[j] = a.log_prior ? lp - a.log_prior[j] : lp;
    if (j == y) {   // exactly one thread of the row owns the label column
      if (a.row_loss) a.row_loss[r] = -lp;
      if (a.row_err) a.row_err[r] = (arg != y) ? 1.f : 0.f;
    }
  }
}

// The same with 16-byte accesses (N % 4 == 0, aligned rows): each thread owns two float4 column
// chunks (j = 4 (tr + T q) + e), so a row takes 2 NS load instructions per thread instead of 8 NS
template <int WPR, int NS>
__device__ __forceinline__ void nll_vec_body(const pkc_nll_args& a, int block, NllShared& sh) {
  constexpr int RPB = LW / WPR;
  constexpr int T = 64 * WPR;
  constexpr int NQ = 2;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rl = wave / WPR;
  const int tr = threadIdx.x - rl * T;
  const int r = block * RPB + rl;
  const bool rok = r < a.M;
  const int64_t N = a.N;
  const int rr = rok ? r : a.M - 1;
  const float* zb = a.zslab + (int64_t)rr * N;
  const int y_ = *(a.labels ? a.labels + (int64_t)rr * a.label_stride
                            : reinterpret_cast<const int32_t*>(a.zslab));
  float4 v[NQ][NS];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int j0 = min(4 * (tr + T * q), a.N - 4);
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      const int st = t < a.nslab ? t : a.nslab - 1;
      v[q][t] = *reinterpret_cast<const float4*>(zb + (int64_t)st * a.slab_stride + j0);
    }
  }
  float z[NQ][4];
  float mx = -INFINITY;
  int arg = 0x7fffffff;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int j0 = 4 * (tr + T * q);
    float4 acc = v[q][0];
#pragma unroll
    for (int t = 1; t < NS; ++t) {
      if (t < a.nslab) {
        acc.x += v[q][t].x; acc.y += v[q][t].y; acc.z += v[q][t].z; acc.w += v[q][t].w;
      }
    }
    if (a.bias) {
      const float4 b = *reinterpret_cast<const float4*>(a.bias + min(j0, a.N - 4));
      acc.x += b.x; acc.y += b.y; acc.z += b.z; acc.w += b.w;
    }
    z[q][0] = acc.x; z[q][1] = acc.y; z[q][2] = acc.z; z[q][3] = acc.w;
#pragma unroll
    for (int e = 0; e < 4; ++e)      // ascending j: first max per thread
      if (j0 < a.N && z[q][e] > mx) { mx = z[q][e]; arg = j0 + e; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  if (WPR > 1) {
    if (lane == 0) { sh.m[wave] = mx; sh.a[wave] = arg; }
    __syncthreads();
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) {
      const float om = sh.m[w];
      const int oa = sh.a[w];
      if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
    }
  }
  float se = 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    if (4 * (tr + T * q) < a.N) {
#pragma unroll
      for (int e = 0; e < 4; ++e) se += expf(z[q][e] - mx);
    }
  se = warp_sum(se);
  if (WPR > 1) {
    if (lane == 0) sh.s[wave] = se;
    __syncthreads();
    se = 0.f;
    for (int w = rl * WPR; w < rl * WPR + WPR; ++w) se += sh.s[w];
  }
  if (!rok) return;
  const float lse = mx + logf(se);
  const int y = a.labels ? y_ : -1;
  const float gscale = a.weight / (float)a.M;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int j0 = 4 * (tr + T * q);
    if (j0 >= a.N) break;
    const int64_t o = (int64_t)r * N + j0;
    float lp[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) lp[e] = z[q][e] - lse;
    if (a.dlogits) {
      float d[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = expf(lp[e]);
        d[e] = gscale * (j0 + e == y ? p - 1.f : p);
      }
      *reinterpret_cast<float4*>(a.dlogits + o) = make_float4(d[0], d[1], d[2], d[3]);
      if (a.dlogits_bf16) {
        bf16x4 h;
        h[0] = (__bf16)d[0]; h[1] = (__bf16)d[1]; h[2] = (__bf16)d[2]; h[3] = (__bf16)d[3];
        *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(a.dlogits_bf16) + o) = h;
      }
    }
    float4 w = make_float4(lp[0], lp[1], lp[2], lp[3]);
    if (a.log_prior) {
      const float4 pr = *reinterpret_cast<const float4*>(a.log_prior + j0);
      w.x -= pr.x; w.y -= pr.y; w.z -= pr.z; w.w -= pr.w;
    }
    *reinterpret_cast<float4*>(a.logp + o) = w;
    if (y >= j0 && y < j0 + 4) {   // exactly one thread of the row owns the label column
      if (a.row_loss) a.row_loss[r] = -lp[y - j0];
      if (a.row_err) a.row_err[r] = (arg != y) ? 1.f : 0.f;
    }
  }
}

template <int WPR, int NS>
__global__ __launch_bounds__(64 * LW) void nll_reg_kernel(pkc_nll_args a) {
  __shared__ NllShared sh;
  nll_reg_body<WPR, NS>(a, blockIdx.x, sh);
}

template <int WPR, int NS>
__global__ __launch_bounds__(64 * LW) void nll_vec_kernel(pkc_nll_args a) {
  __shared__ NllShared sh;
  nll_vec_body<WPR, NS>(a, blockIdx.x, sh);
}

// several heads' LogSoftmax/NLL in one launch (workgroup ranges per head)
constexpr int NLL_MAX = 4;
struct NllMulti {
  pkc_nll_args a[NLL_MAX];
  int wg0[NLL_MAX];
  int code[NLL_MAX];   // 8 * (16-byte form) + 4 * (wide) + log2(NS)
  int n;
};

__global__ __launch_bounds__(64 * LW) void nll_multi_kernel(NllMulti g) {
  __shared__ NllShared sh;
  int i = 0;
#pragma unroll
  for (int j = 1; j < NLL_MAX; ++j)
    if (j < g.n && (int)blockIdx.x >= g.wg0[j]) i = j;
  const int b = blockIdx.x - g.wg0[i];
  switch (g.code[i]) {
    case 8: nll_vec_body<1, 1>(g.a[i], b, sh); break;
    case 9: nll_vec_body<1, 2>(g.a[i], b, sh); break;
    case 10: nll_vec_body<1, 4>(g.a[i], b, sh); break;
    case 11: nll_vec_body<1, 8>(g.a[i], b, sh); break;
    case 12: nll_vec_body<4, 1>(g.a[i], b, sh); break;
    case 13: nll_vec_body<4, 2>(g.a[i], b, sh); break;
    case 14: nll_vec_body<4, 4>(g.a[i], b, sh); break;
    case 15: nll_vec_body<4, 8>(g.a[i], b, sh); break;
    case 0: nll_reg_body<1, 1>(g.a[i], b, sh); break;
    case 1: nll_reg_body<1, 2>(g.a[i], b, sh); break;
    case 2: nll_reg_body<1, 4>(g.a[i], b, sh); break;
    case 3: nll_reg_body<1, 8>(g.a[i], b, sh); break;
    case 4: nll_reg_body<4, 1>(g.a[i], b, sh); break;
    case 5: nll_reg_body<4, 2>(g.a[i], b, sh); break;
    case 6: nll_reg_body<4, 4>(g.a[i], b, sh); break;
    default: nll_reg_body<4, 8>(g.a[i], b, sh); break;
  }
}

// autograd backward of LogSoftmax(dim=1) under an arbitrary upstream gradient (a head of the
// architecture plug-in's trainable forward, whose loss is computed outside the library):
// dz = dy - exp(logp) * sum_c dy, one wave per row (torch's log_softmax backward)
__global__ __launch_bounds__(64 * LW) void logsoftmax_bwd_kernel(int M, int N, const float* logp,
                                                                 const float* dy, float* dz) {
  const int r = blockIdx.x * LW + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= M) return;
  const float* g = dy + (int64_t)r * N;
  const float* lp = logp + (int64_t)r * N;
  float* d = dz + (int64_t)r * N;
  float s = 0.f;
  for (int c = lane; c < N; c += 64) s += g[c];
#pragma unroll
  for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
  for (int c = lane; c < N; c += 64) d[c] = g[c] - expf(lp[c]) * s;
}

__global__ __launch_bounds__(256) void loss_finalize_kernel(int nheads, const float* const* rl,
                                                            const float* w, int M,
                                                            const float* rerr, float* out,
                                                            float* acc, int64_t* advance) {
  loss_finalize_body(nheads, rl, w, M, rerr, out, acc, advance);
}

}  // namespace pkc

// the 16-byte form: whole float4 column chunks, aligned rows (PKC_NLL_VEC=0: scalar form, A/B)
static bool nll_vec_ok(const pkc_nll_args* a) {
  static const int on = [] {
    const char* v = getenv("PKC_NLL_VEC");
    return v ? atoi(v) : 1;
  }();
  auto al = [](const void* p, int b) { return ((uintptr_t)p % b) == 0; };
  return on && a->N % 4 == 0 && a->N >= 4 && (a->nslab == 1 || a->slab_stride % 4 == 0) &&
         al(a->zslab, 16) && al(a->logp, 16) && al(a->dlogits, 16) && al(a->bias, 16) &&
         al(a->log_prior, 16) && al(a->dlogits_bf16, 8);
}

extern "C" int pkc_nll_fused(const pkc_nll_args* a, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(a && a->M > 0 && a->N > 0 && a->nslab >= 1 && a->zslab && a->logp,
                "pkc_nll_fused: bad arguments");
  PKC_CHECK_ARG(a->labels || !a->dlogits, "pkc_nll_fused: dlogits needs labels");
  const int ns = a->nslab <= 1 ? 1 : (a->nslab <= 2 ? 2 : (a->nslab <= 4 ? 4 : 8));
  const bool wide = a->N >= 512;
  if (a->nslab <= 8 && a->N <= (wide ? 2048 : 512)) {
    const dim3 grid(wide ? a->M : (a->M + LW - 1) / LW), blk(64 * LW);
#define PKC_NLL(K, W)                                                                 \
    switch (ns) {                                                                     \
      case 1: hipLaunchKernelGGL((K<W, 1>), grid, blk, 0, S(stream), *a); break;     \
      case 2: hipLaunchKernelGGL((K<W, 2>), grid, blk, 0, S(stream), *a); break;     \
      case 4: hipLaunchKernelGGL((K<W, 4>), grid, blk, 0, S(stream), *a); break;     \
      default: hipLaunchKernelGGL((K<W, 8>), grid, blk, 0, S(stream), *a); break;    \
    }
    const bool v4 = nll_vec_ok(a);
    if (wide) {
      if (v4) { PKC_NLL(nll_vec_kernel, 4) } else { PKC_NLL(nll_reg_kernel, 4) }
    } else {
      if (v4) { PKC_NLL(nll_vec_kernel, 1) } else { PKC_NLL(nll_reg_kernel, 1) }
    }
#undef PKC_NLL
  } else if (wide) {
    hipLaunchKernelGGL(nll_kernel<4>, dim3(a->M), dim3(64 * LW), 0, S(stream), *a);
  } else {
    hipLaunchKernelGGL(nll_kernel<1>, dim3((a->M + LW - 1) / LW), dim3(64 * LW), 0, S(stream), *a);
  }
  PKC_LAUNCH_CHECK("pkc_nll_fused");
  return PKC_OK;
}

static bool nll_reg_code(const pkc_nll_args* a, int* code, int* nwg) {
  using namespace pkc;
  const int ns = a->nslab <= 1 ? 0 : (a->nslab <= 2 ? 1 : (a->nslab <= 4 ? 2 : 3));
  const bool wide = a->N >= 512;
  if (a->nslab > 8 || a->N > (wide ? 2048 : 512)) return false;
  *code = (nll_vec_ok(a) ? 8 : 0) + (wide ? 4 : 0) + ns;
  *nwg = wide ? a->M : (a->M + LW - 1) / LW;
  return true;
}

extern "C" int pkc_nll_fused_multi(const pkc_nll_args* args, int n, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(args && n >= 1 && n <= NLL_MAX, "pkc_nll_fused_multi: 1..%d heads", NLL_MAX);
  NllMulti g;
  memset(&g, 0, sizeof(g));
  int wg = 0;
  for (int i = 0; i < n; ++i) {
    const pkc_nll_args* a = &args[i];
    PKC_CHECK_ARG(a->M > 0 && a->N > 0 && a->nslab >= 1 && a->zslab && a->logp,
                  "pkc_nll_fused_multi: head %d bad arguments", i);
    PKC_CHECK_ARG(a->labels || !a->dlogits, "pkc_nll_fused_multi: dlogits needs labels");
    int code, nwg;
    if (!nll_reg_code(a, &code, &nwg)) {   // a head outside the register-resident form
      for (int j = 0; j < n; ++j) {
        const int rc = pkc_nll_fused(&args[j], stream);
        if (rc != PKC_OK) return rc;
      }
      return PKC_OK;
    }
    g.a[i] = *a;
    g.code[i] = code;
    g.wg0[i] = wg;
    wg += nwg;
  }
  g.n = n;
  hipLaunchKernelGGL(nll_multi_kernel, dim3(wg), dim3(64 * LW), 0, S(stream), g);
  PKC_LAUNCH_CHECK("pkc_nll_fused_multi");
  return PKC_OK;
}

extern "C" int pkc_loss_finalize(int nheads, const float* const* row_loss, const float* weights,
                                 int M, const float* row_err, float* out, float* acc,
                                 int64_t* advance_ctr, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(nheads >= 1 && nheads <= 8 && row_loss && weights && row_err && out && M > 0,
                "pkc_loss_finalize: bad arguments");
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, S(stream), nheads, row_loss,
                     weights, M, row_err, out, acc, advance_ctr);
  PKC_LAUNCH_CHECK("pkc_loss_finalize");
  return PKC_OK;
}

extern "C" int pkc_logsoftmax_bwd(int M, int N, const float* logp, const float* dy, float* dz,
                                  void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(M > 0 && N > 0 && logp && dy && dz, "pkc_logsoftmax_bwd: bad arguments");
  hipLaunchKernelGGL(logsoftmax_bwd_kernel, dim3((M + LW - 1) / LW), dim3(64 * LW), 0, S(stream), M,
                     N, logp, dy, dz);
  PKC_LAUNCH_CHECK("pkc_logsoftmax_bwd");
  return PKC_OK;
}
