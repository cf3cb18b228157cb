// pkc_loader.hip — chunk preparation and batch assembly on the GPU.
//
// The reference expands the context window, normalises and shuffles every chunk in numpy float64
// on the host (data_io.py:105-145, 269-270) and then uploads an 11x larger float matrix
// (core.py:93-94).  Here only the raw N x D frames go host->device; the expansion
// (np.roll order: block b of row r is raw[(r + 2L - b) mod N]), the column statistics (fp64,
// population std as np.std) and the row permutation of the shuffle are applied on the device.
#include "pkc_common.h"
#include "pkc_ops.h"

namespace pkc {

__device__ __forceinline__ int64_t cw_src(int64_t r, int b, int L, int64_t N) {
  int64_t s = (r + 2 * L - b) % N;
  return s < 0 ? s + N : s;
}

// partial column sums of the expanded matrix: grid (ceil(C/64), P) ; work = [2][P][C]
__global__ __launch_bounds__(256) void cw_partial_kernel(const float* raw, int64_t N, int D, int L,
                                                         int R, const double* mean, double* work,
                                                         int P, int pass) {
  const int C = D * (L + R + 1);
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;  // 4 row groups
  const int64_t Nout = N - L - R;
  const int64_t per = (Nout + P - 1) / P;
  const int64_t r0 = blockIdx.y * per, r1 = min(Nout, r0 + per);
  __shared__ double red[256];
  double s = 0.0;
  if (col < C) {
    const int b = col / D, d = col % D;
    const double mu = pass ? mean[col] : 0.0;
    for (int64_t r = r0 + rg; r < r1; r += 4) {
      const double v = (double)raw[cw_src(r, b, L, N) * D + d];
      s += pass ? (v - mu) * (v - mu) : v;
    }
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (rg == 0 && col < C) {
    const double t = red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] +
                     red[threadIdx.x + 192];
    work[(int64_t)pass * P * C + (int64_t)blockIdx.y * C + col] = t;
  }
}

__global__ void cw_finalize_kernel(const double* work, int P, int C, int64_t Nout, double* mean,
                                   double* stdv, int pass) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= C) return;
  double s = 0.0;
  for (int p = 0; p < P; ++p) s += work[(int64_t)pass * P * C + (int64_t)p * C + col];
  if (pass == 0) mean[col] = s / (double)Nout;
  else stdv[col] = sqrt(s / (double)Nout);
}

// output row j of nrows: the expanded row row0 + perm[j] (row0 + j without perm)
__global__ __launch_bounds__(256) void cw_apply_kernel(const float* raw, int64_t N, int D, int L,
                                                       int R, const double* mean, const double* stdv,
                                                       const int64_t* perm, int64_t row0,
                                                       int64_t nrows, float* out, int64_t ld_out) {
  const int C = D * (L + R + 1);
  const int64_t row = blockIdx.y;  // output row
  if (row >= nrows) return;
  const int64_t src_row = row0 + (perm ? perm[row] : row);
  for (int col = blockIdx.x * 256 + threadIdx.x; col < C; col += gridDim.x * 256) {
    const int b = col / D, d = col % D;
    const double v = (double)raw[cw_src(src_row, b, L, N) * D + d];
    out[row * ld_out + col] = (float)((v - mean[col]) / stdv[col]);
  }
}

__global__ __launch_bounds__(256) void batch_gather_kernel(const float* feats, int64_t ld, int F,
                                                           const int32_t* labels, int nlab, int B,
                                                           int64_t n_batches, int64_t* ctr,
                                                           float* x_out, int32_t* lab_out,
                                                           int advance, unsigned* done,
                                                           __bf16* xb, bool vec) {
  gather_row_body(feats, ld, F, labels, nlab, B, n_batches, ctr, x_out, lab_out, xb, vec,
                  blockIdx.x);
  if (advance) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const unsigned prev = atomicAdd(done, 1u);
      if (prev == (unsigned)B - 1) {  // last block: every block has read the counter
        *ctr = *ctr + 1;
        *done = 0u;
      }
    }
  }
}

}  // namespace pkc

extern "C" int64_t pkc_cw_stats_work_size(int64_t N, int D, int L, int R) {
  (void)N;
  return 2 * 64 * (int64_t)D * (L + R + 1);  // doubles: [2][P=64][C]
}

extern "C" int pkc_cw_stats(const float* raw, int64_t N, int D, int L, int R, double* mean,
                            double* stdv, double* work, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(raw && mean && stdv && work && D > 0 && L >= 0 && R >= 0 && N > L + R,
                "pkc_cw_stats: bad arguments");
  const int C = D * (L + R + 1);
  const int P = 64;
  const int64_t Nout = N - L - R;
  dim3 grid((C + 63) / 64, P);
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(cw_partial_kernel, grid, dim3(256), 0, S(stream), raw, N, D, L, R, mean, work,
                       P, pass);
    PKC_LAUNCH_CHECK("pkc_cw_stats partial");
    hipLaunchKernelGGL(cw_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, S(stream), work, P, C,
                       Nout, mean, stdv, pass);
    PKC_LAUNCH_CHECK("pkc_cw_stats finalize");
  }
  return PKC_OK;
}

extern "C" int pkc_cw_apply(const float* raw, int64_t N, int D, int L, int R, const double* mean,
                            const double* stdv, const int64_t* perm, float* out, int64_t ld_out,
                            void* stream) {
  using namespace pkc;
  const int C = D * (L + R + 1);
  PKC_CHECK_ARG(raw && mean && stdv && out && N > L + R && ld_out >= C, "pkc_cw_apply: bad arguments");
  const int64_t Nout = N - L - R;
  PKC_CHECK_ARG(Nout < 2147483647LL, "pkc_cw_apply: chunk too large");
  dim3 grid((C + 255) / 256, (unsigned)Nout);
  hipLaunchKernelGGL(cw_apply_kernel, grid, dim3(256), 0, S(stream), raw, N, D, L, R, mean, stdv,
                     perm, (int64_t)0, Nout, out, ld_out);
  PKC_LAUNCH_CHECK("pkc_cw_apply");
  return PKC_OK;
}

// One feature stream of a multi-stream chunk (data_io.py:184-263): rows row0 .. row0 + nrows - 1
// of the stream's own expansion (its context window, its chunk statistics — np.roll wrap-around
// over the stream's N rows included), i.e. the rows the reference keeps after trimming every stream
// to the widest window (row0 = cw_left_max - L), written into its column range of the chunk
// matrix (out = the range's first column, ld_out = the chunk's width), optionally permuted.
extern "C" int pkc_cw_apply_rows(const float* raw, int64_t N, int D, int L, int R,
                                 const double* mean, const double* stdv, const int64_t* perm,
                                 int64_t row0, int64_t nrows, float* out, int64_t ld_out,
                                 void* stream) {
  using namespace pkc;
  const int C = D * (L + R + 1);
  PKC_CHECK_ARG(raw && mean && stdv && out && N > L + R && ld_out >= C && row0 >= 0 && nrows > 0 &&
                    row0 + nrows <= N - L - R && nrows < 2147483647LL,
                "pkc_cw_apply_rows: bad arguments");
  dim3 grid((C + 255) / 256, (unsigned)nrows);
  hipLaunchKernelGGL(cw_apply_kernel, grid, dim3(256), 0, S(stream), raw, N, D, L, R, mean, stdv,
                     perm, row0, nrows, out, ld_out);
  PKC_LAUNCH_CHECK("pkc_cw_apply_rows");
  return PKC_OK;
}

extern "C" int pkc_batch_gather(const float* feats, int64_t ld_feats, int F, const int32_t* labels,
                                int nlab, int B, int64_t n_batches, int64_t* step_ctr, float* x_out,
                                int32_t* lab_out, int advance, void* x_bf16, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(feats && labels && step_ctr && x_out && lab_out && B > 0 && n_batches > 0 &&
                    nlab >= 0 && nlab <= 256,
                "pkc_batch_gather: bad arguments");
  // the completion counter lives right after the step counter (caller allocates 2 int64)
  unsigned* done = reinterpret_cast<unsigned*>(step_ctr + 1);
  const bool vec = F % 4 == 0 && ld_feats % 4 == 0 && (uintptr_t)feats % 16 == 0 &&
                   (uintptr_t)x_out % 16 == 0 && (uintptr_t)x_bf16 % 8 == 0;
  hipLaunchKernelGGL(batch_gather_kernel, dim3(B), dim3(256), 0, S(stream), feats, ld_feats, F, labels,
                     nlab, B, n_batches, step_ctr, x_out, lab_out, advance, done,
                     reinterpret_cast<__bf16*>(x_bf16), vec);
  PKC_LAUNCH_CHECK("pkc_batch_gather");
  return PKC_OK;
}

namespace pkc {
__global__ __launch_bounds__(256) void seq_gather_kernel(const float* feats, int64_t ld, int F,
                                                         const int32_t* labels, int nlab,
                                                         const int64_t* beg, const int32_t* len,
                                                         const int32_t* left, int B, int max_len,
                                                         float* x_out, int32_t* lab_out) {
  const int t = blockIdx.x, k = blockIdx.y;      // output row (t, k) of the (max_len, B, F) batch
  const int l0 = left[k], n = len[k];
  const bool in = t >= l0 && t < l0 + n;
  const int64_t src = beg[k] + (t - l0);
  float* dst = x_out + ((int64_t)t * B + k) * F;
  for (int c = threadIdx.x; c < F; c += 256) dst[c] = in ? feats[src * ld + c] : 0.f;
  if (threadIdx.x < nlab)
    lab_out[((int64_t)t * B + k) * nlab + threadIdx.x] = in ? labels[src * nlab + threadIdx.x] : 0;
}
}  // namespace pkc

extern "C" int pkc_seq_gather(const float* feats, int64_t ld_feats, int F, const int32_t* labels,
                              int nlab, const int64_t* beg, const int32_t* len, const int32_t* left,
                              int B, int max_len, float* x_out, int32_t* lab_out, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(feats && beg && len && left && x_out && B > 0 && max_len > 0 && nlab <= 256 &&
                    (nlab == 0 || (labels && lab_out)),
                "pkc_seq_gather: bad arguments");
  hipLaunchKernelGGL(seq_gather_kernel, dim3(max_len, B), dim3(256), 0, S(stream), feats, ld_feats, F,
                     labels, nlab, beg, len, left, B, max_len, x_out, lab_out);
  PKC_LAUNCH_CHECK("pkc_seq_gather");
  return PKC_OK;
}
