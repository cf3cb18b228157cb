/* pkc.h — C ABI of libpkc.so, the MI355X-native (gfx950) hot path of pytorch-kaldi-CGS run_nn().
 *
 * Every entry point replaces an implicit PyTorch-eager op sequence of the reference (file:line
 * cited per function, paths relative to the reference repo).  Conventions:
 *   - plain pointers + sizes, no torch types; all device pointers are caller-owned HBM buffers,
 *     the library never allocates device memory on a hot call;
 *   - `stream` is a hipStream_t passed as void*; every call is asynchronous on that stream;
 *   - return 0 (PKC_OK) or a negative status; pkc_last_error() gives a thread-local message;
 *   - thread-safe across streams (no global mutable state besides the error string).
 * Layouts: row-major matrices, fp32 in HBM ("parity" precision); PKC_PREC_BF16 computes the
 * matmuls on bf16 MFMA with fp32 accumulation ("performance" precision).
 */
#ifndef PKC_H_
#define PKC_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped whenever an entry point is added or a struct changes (tests/test_abi_layout.py asserts it):
 * 1: rounds 1-3; 2: pkc_logsoftmax_bwd, and the structs as they stand after round 3 (which appended
 * pkc_dense_bwd_args.dz_scratch without a bump); 3: pkc_opt_seg (direct PKC_OP_OPTIM);
 * 4: PKC_PREC_BF16X3; 5: pkc_rnn_args.step_bf16 and its bf16 operand copies;
 * 6: pkc_bn_bwd_epi, pkc_gemm_bnbwd_ok, pkc_dense_bwd_pre;
 * 7: pkc_src_digest, pkc_gemm_grouped_tile, pkc_rnn_args.persist_* (persistent liGRU time loops);
 * 8: pkc_rnn_args.qh_exact (exact quantised-h step products). */
#define PKC_ABI_VERSION 9

enum { PKC_OK = 0, PKC_ERR_ARG = -1, PKC_ERR_HIP = -2, PKC_ERR_IO = -3, PKC_ERR_UNSUPPORTED = -4 };
/* FP32: exact fp32 MFMA (parity); BF16: fp32 operands rounded to bf16 for the MFMA;
 * BF16IN: operands stored as bf16 in HBM (A and B point at bf16 arrays), fp32 accumulation;
 * BF16X3: compensated bf16 — fp32 operands split at staging into a bf16 head and a bf16 tail
 * (a = hi + lo, lo = bf16(a - hi)) and multiplied as hi*hi + hi*lo + lo*hi on the bf16 MFMA with
 * fp32 accumulation: products to ~2^-16 relative (the dropped lo*lo term), i.e. fp32-class
 * results at 3/16 of the exact-fp32 MFMA cost.  Every tile body takes it (64x64 and 128x128,
 * pkc_gemm, pkc_gemm_grouped, pkc_gemm_colstats). */
enum { PKC_PREC_FP32 = 0, PKC_PREC_BF16 = 1, PKC_PREC_BF16IN = 2, PKC_PREC_BF16X3 = 3 };
/* neural_networks.py:54-78 act_fun */
enum { PKC_ACT_LINEAR = 0, PKC_ACT_RELU = 1, PKC_ACT_TANH = 2, PKC_ACT_SIGMOID = 3,
       PKC_ACT_HTANH = 4, PKC_ACT_LEAKY = 5, PKC_ACT_ELU = 6 };
enum { PKC_NORM_NONE = 0, PKC_NORM_BN_TRAIN = 1, PKC_NORM_BN_EVAL = 2 };
enum { PKC_OPT_SGD = 0, PKC_OPT_RMSPROP = 1, PKC_OPT_ADAM = 2 };

int pkc_abi_version(void);
const char* pkc_last_error(void);
/* SHA-256 (hex) of the csrc/ + include/ sources this library was linked from (generated at build
 * time; pkc._lib refuses a library whose digest differs from its tree's). */
const char* pkc_src_digest(void);

/* ---------------------------------------------------------------------------------------------
 * Matmul (replaces the cuBLAS GEMMs behind nn.Linear / F.linear in the reference:
 * neural_networks.py:306-317 (MLP wx), 951-954 (LSTM W), 1554-1555 (liGRU W) and their autograd
 * backward).  Computes, for split z = 0..splits-1 over the K range [z*Kc, (z+1)*Kc):
 *     C[z*slab_stride + m*ldc + n] = sum_k A(m,k) * B(n,k)
 * with A(m,k) = a_kcontig ? A[m*lda+k] : A[k*lda+m] and B(n,k) = b_kcontig ? B[n*ldb+k] : B[k*ldb+n].
 * forward  Y = X W^T      : a_kcontig=1, b_kcontig=1
 * backward dX = dY W      : a_kcontig=1, b_kcontig=0
 * backward dW = dY^T X    : a_kcontig=0, b_kcontig=0
 * Split-K partial slabs are summed by the consumer kernels (dense_fwd/dense_bwd/nll) in a fixed
 * order, so results are deterministic.  splits<=0 picks a split count for the shape.
 * Leading dimensions (elements): lda, ldb in [1, 2^31), ldc in [N, 2^26) — the kernels keep row
 * offsets in 32 bits (PKC_ERR_ARG otherwise; pkc_gemm_grouped checks the same per problem).
 * ------------------------------------------------------------------------------------------- */
int pkc_gemm(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
             const void* A, int64_t lda, const void* B, int64_t ldb,
             float* C, int64_t ldc, int splits, int64_t slab_stride, void* stream);
int pkc_gemm_pick_splits(int M, int N, int K);
/* Up to 8 independent operations in one launch — the launch boundary (~1.5-1.9 us on MI355X)
 * dominates a 128-row batch's matmuls, so a layer's dW and dX, two heads' logits, or the heads'
 * dW/dX together with their bias gradients and the loss reduction share one kernel.
 *   PKC_OP_GEMM  : exactly pkc_gemm(prec, a_kcontig, b_kcontig, M, N, K, A, lda, B, ldb, C, ldc,
 *                  splits, slab_stride)
 *   PKC_OP_COLSUM: C[n] = sum_m A[m*N + n]  (M rows, N columns, fp32)
 *   PKC_OP_SLABSUM: C[i] = sum_{s<M} A[s*slab_stride + i], i < N, summed in slab order (fp32): the
 *                  partial slabs of a split-K matmul (e.g. a large-batch dW) into one result
 *   PKC_OP_LOSS  : pkc_loss_finalize(nheads = M, row_loss = A, weights = B, rows = N,
 *                  row_err = X1, out = C, acc = X2, advance_ctr = X3)
 *   PKC_OP_OPTIM : pkc_optim_step(tensors_dev = A, chunk_map_dev = B, nchunks = M) — the update of
 *                  a layer whose gradients are complete rides in a later launch of the backward.
 *                  Direct form (X1 != NULL): X1 is a HOST array of N pkc_opt_seg (read during the
 *                  call) listing the op's work items as runs of chunks of single tensors, M = the
 *                  sum of their nchunks.  Their pointers travel in the kernel arguments, so a work
 *                  item's loads start without the map -> descriptor round trips; the
 *                  hyper-parameters (lr, step, ...) are still read from tensors_dev[tensor], so a
 *                  captured graph sees set_lr / step updates.  When a launch's direct segments would
 *                  exceed PKC_OPT_SEGS_MAX the op falls back to the map (B then required).
 *   PKC_OP_GATHER: pkc_batch_gather(feats = A, ld_feats = lda, F = N, labels = B, nlab = ldb,
 *                  B = M rows, n_batches = slab_stride, step_ctr = X1, x_out = C, lab_out = X2,
 *                  advance = 0, x_bf16 = X3) — the next batch's gather sharing a launch with the
 *                  previous step's last weight update (neither reads what the other writes)
 * Block-sparse GEMM (static HCGS masks multiplied into W, HCGS.py:24-28 /
 * neural_networks.py:258, 858-861): with ktiles != NULL (and splits == 1) the 64-column output
 * tile j reads only the 32-deep k-tiles ktiles[j * (kmax + 1) + 1 .. + count], count =
 * ktiles[j * (kmax + 1)]: the k-tiles whose B rows (64 of them) hold a nonzero.  Exact: every
 * skipped product is a zero weight, so the sums are those of the dense matmul. */
enum { PKC_OP_GEMM = 0, PKC_OP_COLSUM = 1, PKC_OP_LOSS = 2, PKC_OP_OPTIM = 3, PKC_OP_SLABSUM = 4,
       PKC_OP_GATHER = 5 };
typedef struct {
  int a_kcontig, b_kcontig, M, N, K, splits;
  const void* A; int64_t lda; const void* B; int64_t ldb;
  float* C; int64_t ldc; int64_t slab_stride;
  int kind; const void* X1; void* X2; void* X3;
  const int32_t* ktiles; int kmax;              /* block-sparse k-tile lists (device), or NULL */
} pkc_gemm_problem;
int pkc_gemm_grouped(int prec, const pkc_gemm_problem* probs, int n, void* stream);
/* The first half of a large-batch BatchNorm'd layer's backward in the epilogue of the dX matmul
 * that produces its output gradient g (neural_networks.py:306-317 under autograd): a PKC_OP_GEMM
 * problem of pkc_gemm_grouped with X1 = a HOST pointer to a pkc_bn_bwd_epi (read during the call)
 * stores dy = g * keep / (1 - drop_p) * act'(gamma * xhat + beta) in C instead of g, and per
 * 128-row block b the column sums sum dy and sum dy * xhat in part[b*2N + n], part[b*2N + N + n]
 * — what pkc_dense_bwd's statistics pass computes, without re-reading g.  The problem must be
 * one slab (splits = 1) with ldc = N and take the 128x128 body: pkc_gemm_bnbwd_ok says whether it
 * does.  pkc_dense_bwd_pre (dz = that C, part in work, part_rows = 128) finishes the backward. */
typedef struct pkc_bn_bwd_epi_s {
  const float* xhat; const uint8_t* keep; const float* gamma; const float* beta;
  float* part; int act; float drop_p;
} pkc_bn_bwd_epi;
int pkc_gemm_bnbwd_ok(int prec, int a_kcontig, int b_kcontig, int M, int N, int K, const void* A,
                      int64_t lda, const void* B, int64_t ldb);
/* Tile edge (128: the 128x128 body, else 64) a GEMM problem of pkc_gemm_grouped takes, so a
 * host can size the launch's split-K over the tiles it will really have. */
int pkc_gemm_grouped_tile(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                          const void* A, int64_t lda, const void* B, int64_t ldb);

/* Large-batch forward matmul of a BatchNorm'd layer (neural_networks.py:306-311: BN(wx(x)) over
 * the batch) with the BatchNorm column statistics in the matmul's epilogue: one slab
 * C = A B^T (as pkc_gemm, splits = 1) and, per row block b of C, the block's column mean of
 * C + bias and M2 = sum (C - mean)^2 into part[b*2N + n], part[b*2N + N + n] — the partials
 * pkc_dense_fwd_pre merges, so no separate statistics pass reads C.  pkc_gemm_colstats_ok returns
 * the rows per partial block for the shape — 128 (128x128 tile body), 64 (64x64 body, 16-byte
 * operand paths), 0 (not available) — which is the part_rows to pass to pkc_dense_fwd_pre; bias
 * may be NULL; part holds 2 N ceil(M / rows) floats (a pkc_dense_work_size(M, N) buffer does). */
int pkc_gemm_colstats_ok(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                         const void* A, int64_t lda, const void* B, int64_t ldb);
int pkc_gemm_colstats(int prec, int a_kcontig, int b_kcontig, int M, int N, int K,
                      const void* A, int64_t lda, const void* B, int64_t ldb, float* C,
                      int64_t ldc, const float* bias, float* part, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Dense layer epilogue, forward (neural_networks.py:306-317: drop(act(BN(z)))) where
 * z = sum_{s<nslab} zslab[s] + bias.  BN in training mode uses batch statistics over the M rows
 * (biased variance for normalisation, unbiased for running_var, momentum as nn.BatchNorm1d).
 * Outputs: out (M x N) and, for the backward, xhat (normalised z; == z when norm NONE) and the
 * dropout keep mask (u8; NULL when p == 0).  Dropout is inverted (x*keep/(1-p)) as nn.Dropout.
 * When keep_in != NULL the mask is read instead of generated (parity tests).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int M, N, nslab;
  const float* zslab; int64_t slab_stride;   /* nslab partial slabs, each M x N (ldz = N) */
  const float* bias;                          /* N or NULL */
  int norm;                                   /* PKC_NORM_* */
  const float* gamma; const float* beta;      /* N */
  float* running_mean; float* running_var;    /* N (updated in BN_TRAIN) */
  float momentum, eps;
  float* save_mean; float* save_invstd;       /* N (written in BN_TRAIN, read in backward) */
  int act;                                    /* PKC_ACT_* */
  float drop_p; uint64_t seed; const int64_t* step_ctr; int64_t stream_id;
  const uint8_t* keep_in;                     /* optional injected dropout mask (M x N) */
  uint8_t* keep_out;                          /* M x N, may be NULL when drop_p == 0 */
  float* xhat;                                /* M x N (BN input normalised), may be NULL in eval */
  float* out;        /* M x N; may be NULL when out_bf16 is set (no reader of the fp32 copy) */
  int64_t count_n;   /* rows BatchNorm1d sees for the unbiased running_var (0 -> M); a shared-
                        weight bidirectional layer normalises 2x duplicated rows (2*M) */
  void* out_bf16;    /* optional bf16 copy of out (M x N): the next layer's PKC_PREC_BF16IN operand */
} pkc_dense_fwd_args;
int pkc_dense_fwd(const pkc_dense_fwd_args* a, float* work, void* stream);
/* pkc_dense_fwd in BatchNorm training mode (norm == PKC_NORM_BN_TRAIN, nslab == 1) whose column
 * partials the producing matmul already wrote into work at part_rows rows per block
 * (pkc_gemm_colstats: 128): merges them (Chan, fixed order) and applies — the same outputs with
 * the statistics summed in that blocking. */
int pkc_dense_fwd_pre(const pkc_dense_fwd_args* a, float* work, int part_rows, void* stream);
/* A BatchNorm'd layer's matmul AND epilogue in one launch at M <= 128 rows (the reference's
 * batch_size_train; ABI 9): z = A W^T (A: M x K, lda; W: N x K, ldw; both k-contiguous), then
 * exactly pkc_dense_fwd's epilogue on z + bias (a->zslab / nslab / slab_stride are not read).
 * Each workgroup owns a 128-row x 16-column strip over the full contraction, so the BatchNorm
 * column statistics need nothing from other workgroups.  prec: PKC_PREC_BF16IN (A, W bf16) or
 * PKC_PREC_BF16 (fp32, rounded to bf16 on load: identical results); fp32 accumulation.
 * pkc_dense_gemm_fwd_ok: 1 when the shape / precision / alignment is supported (N % 16 == 0,
 * K % 8 == 0, lda and ldw multiples of 8, A and W 16-byte aligned). */
int pkc_dense_gemm_fwd_ok(int prec, int M, int N, int K, const void* A, int64_t lda, const void* W,
                          int64_t ldw);
int pkc_dense_gemm_fwd(int prec, const void* A, int64_t lda, const void* W, int64_t ldw, int K,
                       const pkc_dense_fwd_args* a, void* stream);
/* floats of device workspace pkc_dense_fwd / pkc_dense_bwd need (per-16-row column partials) */
int64_t pkc_dense_work_size(int M, int N);

/* Dense layer backward through dropout, activation, BN and bias (autograd of the same ops).
 * g = sum_s gslab[s] (dL/d out).  Writes dz (M x N, dL/dz), dgamma, dbeta, dbias (N).  A bias in
 * front of BatchNorm cancels in z - mean(z): its gradient is written as exactly 0 (the reference's
 * autograd value is rounding noise of order 1e-9 with no effect on any output). */
typedef struct {
  int M, N, nslab;
  const float* gslab; int64_t slab_stride;
  int norm, act;
  const float* gamma; const float* beta; const float* save_invstd;
  const float* xhat; const uint8_t* keep; float drop_p;
  float* dz; float* dgamma; float* dbeta; float* dbias;
  void* dz_bf16;     /* optional bf16 copy of dz (M x N): the dW / dX PKC_PREC_BF16IN operand */
  int dz_scratch;    /* 1 (training BatchNorm with dz_bf16): the caller reads only dz_bf16; dz is
                        scratch between the passes and the final fp32 gradient is not stored */
} pkc_dense_bwd_args;
int pkc_dense_bwd(const pkc_dense_bwd_args* a, float* work, void* stream);
/* pkc_dense_bwd after a dX matmul with the pkc_bn_bwd_epi epilogue: a->dz holds dy, work the
 * per-part_rows-block column sums; finalize (dgamma, dbeta) and apply only (BN training). */
int pkc_dense_bwd_pre(const pkc_dense_bwd_args* a, float* work, int part_rows, void* stream);
/* SyncBN (cross-rank BatchNorm statistics): the training-mode BatchNorm of
 * pkc_dense_fwd / pkc_dense_bwd split around a collective the caller runs (sync_bn of the
 * reference recipe; the reference itself has no multi-GPU training).
 *   pkc_dense_fwd_stats: this rank's column state (n, mean, M2) -> state[3N] (floats: N counts,
 *     N means, N M2).  The caller gathers the R ranks' states into states[R][3N] (e.g. an
 *     all-reduce SUM of a zero-filled buffer that rank r writes at row r);
 *   pkc_dense_fwd_sync_apply: merges them in rank order (Chan), writes save_mean / save_invstd /
 *     running statistics (unbiased over the global count) and applies BN / act / dropout to this
 *     rank's rows.
 *   pkc_dense_bwd_stats: this rank's column sums (sum dy, sum dy * xhat) -> sums[2N] and the LOCAL
 *     dgamma / dbeta (the gradient all-reduce sums them); after an all-reduce SUM of sums[2N],
 *   pkc_dense_bwd_sync_apply applies the BatchNorm backward with the global sums over total_rows.
 * work: pkc_dense_work_size(M, N) floats, the same buffer for both halves of a direction. */
int pkc_dense_fwd_stats(const pkc_dense_fwd_args* a, float* work, float* state, void* stream);
int pkc_dense_fwd_sync_apply(const pkc_dense_fwd_args* a, float* work, const float* states,
                             int nranks, void* stream);
int pkc_dense_bwd_stats(const pkc_dense_bwd_args* a, float* work, float* sums, void* stream);
int pkc_dense_bwd_sync_apply(const pkc_dense_bwd_args* a, float* work, const float* sums,
                             int total_rows, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Fused LogSoftmax + NLLLoss(mean) + error rate + d(loss)/d(logits) for one output head
 * (neural_networks.py:73-74 LogSoftmax(dim=1); utils.py:1935-1952 NLLLoss; utils.py:1993-2011
 * cost_err; autograd backward softmax - onehot).  logits = sum_s zslab[s] + bias.
 * labels are read as float from a strided column (the reference stores them as float columns of
 * the chunk, core.py:94, cast with .long() at utils.py:1942).  Per-row loss/err go to row_loss /
 * row_err; dlogits = weight/M * (softmax - onehot) (NULL in forward-only mode); logp (M x N) is
 * the head output (NULL when not needed).  prior (N, log prior) is subtracted from logp when
 * non-NULL (core.py:242-245 posterior normalisation).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int M, N, nslab;
  const float* zslab; int64_t slab_stride; const float* bias;
  const int32_t* labels; int64_t label_stride;
  float weight;
  float* logp; const float* log_prior;
  float* dlogits; float* row_loss; float* row_err;
  void* dlogits_bf16;  /* optional bf16 copy of dlogits (operand of the fused row backward) */
} pkc_nll_args;
int pkc_nll_fused(const pkc_nll_args* a, void* stream);

/* LogSoftmax backward for an upstream gradient dy (M x N, row-major): dz = dy - exp(logp) *
 * rowsum(dy).  The architecture plug-in's trainable head forward (neural_networks.py:73-74 under
 * the reference's autograd, core.py:221-232); dz may alias dy. */
int pkc_logsoftmax_bwd(int M, int N, const float* logp, const float* dy, float* dz, void* stream);

/* Reduce per-row losses of up to 8 heads: loss_final = sum_h w_h * mean(row_loss_h),
 * err = mean(row_err_of_err_head); writes out[0]=loss_final, out[1]=err, out[2+h]=mean loss h and
 * accumulates acc[0]+=loss_final, acc[1]+=err (core.py:251-252 loss_sum/err_sum on device). */
int pkc_loss_finalize(int nheads, const float* const* row_loss, const float* weights, int M,
                      const float* row_err, float* out, float* acc, int64_t* advance_ctr,
                      void* stream);   /* advance_ctr (optional): += 1 after the reduction */
/* Several heads' pkc_nll_fused in one launch (n <= 4). */
int pkc_nll_fused_multi(const pkc_nll_args* args, int n, void* stream);

/* Column sums over rows of sum_s slabs (bias gradient of a head: autograd of + bias). */
int pkc_colsum(int M, int N, int nslab, const float* x, int64_t slab_stride, float* out,
               int accumulate, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Multi-tensor optimizer step (torch.optim SGD / RMSprop / Adam as built by utils.py:1833-1881,
 * stepped at core.py:230-232) fused with the reference's per-forward weight preparation:
 * p <- clamp(p_new * mask, -clampv, clampv) when mask / clampv>0 are given — the in-place HCGS /
 * pattern multiply (neural_networks.py:258, 858-861, 980-983) and the in-place QuantizeLinear
 * clamp (quantized_modules.py:79) that the next forward would otherwise apply.
 * ------------------------------------------------------------------------------------------- */
typedef struct pkc_opt_tensor_s {
  float* p; const float* g; float* s1; float* s2; float* s3; const float* mask;
  int64_t n;
  int kind;            /* PKC_OPT_* */
  float lr, wd, momentum, dampening, alpha, eps, beta1, beta2, clampv;
  int nesterov, centered, amsgrad, step;   /* step = 1-based count for this tensor */
  float* qout; int qbits;   /* QuantizeLinear: also write the fake-quantised weight (qbits > 0) */
  void* bout;               /* optional bf16 copy of the updated parameter (MFMA operand) */
} pkc_opt_tensor;
int pkc_optim_step(const pkc_opt_tensor* tensors_dev, int ntensors, const int32_t* chunk_map_dev,
                   int nchunks, void* stream);
/* One run of work items of a direct PKC_OP_OPTIM operation (pkc_gemm_grouped): chunks
 * [chunk0, chunk0 + nchunks) (pkc_optim_chunks' 2048-element items) of tensor `tensor` of the
 * descriptor array.  p .. bout and n repeat that descriptor's, except that s1 / s2 / s3 / qout are
 * NULL where the update keeps no such state (SGD without momentum: s1 NULL; qout NULL unless
 * qbits > 0): the kernel decides which streams to touch from these pointers alone. */
#define PKC_OPT_SEGS_MAX 8     /* direct segments per grouped launch */
typedef struct pkc_opt_seg_s {
  int tensor, chunk0, nchunks, reserved;
  float* p; const float* g; float* s1; float* s2; float* s3; const float* mask;
  float* qout; void* bout;
  int64_t n;
} pkc_opt_seg;
/* Host helper: size of the chunk map (pairs tensor,start) for pkc_optim_step. */
int pkc_optim_chunks(const int64_t* sizes, int ntensors, int32_t* map_out, int cap);

/* p <- clamp(p * mask) (mask may be NULL, clampv <= 0 disables the clamp). */
int pkc_apply_mask(float* p, const float* mask, int64_t n, float clampv, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Batch assembly for non-sequential models (core.py:203-205: inp = data_set[b:b+B]):
 * copy rows [i*B, (i+1)*B) of the chunk's feature matrix and label columns into static buffers,
 * with i read from a device counter (so the step can be replayed from a hipGraph); the counter
 * is incremented by the last block when `advance` is set (otherwise by the step's loss
 * reduction, pkc_loss_finalize's advance_ctr).
 * ------------------------------------------------------------------------------------------- */
int pkc_batch_gather(const float* feats, int64_t ld_feats, int F, const int32_t* labels, int nlab,
                     int B, int64_t n_batches, int64_t* step_ctr, float* x_out, int32_t* lab_out,
                     int advance, void* x_bf16, void* stream);   /* x_bf16: optional bf16 copy */

/* ---------------------------------------------------------------------------------------------
 * LayerNorm of the reference (neural_networks.py:40-51, used by MLP dnn_use_laynorm /
 * dnn_use_laynorm_inp): y = gamma * (x - mean) / (std + eps) + beta per row over N features,
 * std unbiased, x = sum_s xslab[s] + bias.  Saves xhat = (x - mean)/(std + eps) and
 * rowstat[2r] = std + eps, rowstat[2r+1] = std for the backward.
 * ------------------------------------------------------------------------------------------- */
int pkc_layernorm_fwd(int M, int N, int nslab, const float* xslab, int64_t slab_stride,
                      const float* bias, const float* gamma, const float* beta, float eps,
                      float* y, float* xhat, float* rowstat, void* stream);
/* dx from dy = sum_s dy[s] (split-K slabs of the consumers' dX); dgamma = sum_rows dy*xhat,
 * dbeta = sum_rows dy, dbias = sum_rows dx (each optional) */
int pkc_layernorm_bwd(int M, int N, int nslab, const float* dy, int64_t slab_stride,
                      const float* xhat, const float* gamma,
                      const float* rowstat, float* dx, float* dgamma, float* dbeta, float* dbias,
                      void* stream);

/* ---------------------------------------------------------------------------------------------
 * Magnitude pruning (quantized_modules.py:15-28): thr = np.percentile(|W|, perc) (numpy 'linear'),
 * W *= (|W| > thr) in place; mask (optional) receives the {0,1} mask.  Exact order statistics by
 * GPU radix select, no host round trip.  work: pkc_prune_work_size() bytes of device memory.
 * ------------------------------------------------------------------------------------------- */
int64_t pkc_prune_work_size(void);
int pkc_prune(float* w, int64_t n, double perc, float* mask, void* work, void* stream);

/* ---------------------------------------------------------------------------------------------
 * [model] regularisers cost_l1 / cost_l2 / cost_gl (utils.py:24-60, 1954-1991): the loss term
 * lam * sum of block norms (l1: |.|_1 per parameter; l2: |.|_2 per parameter; gl: |.|_2 per
 * torch.chunk block) and its gradient.  A block is cut into row-slice items; items of one block are
 * contiguous and block_start[b]..block_start[b+1] indexes them.
 *   pkc_reg_partial : partial[i] = sum |x| (L1) or sum x^2 (L2) over item i
 *   pkc_reg_finalize: coef[b] = lam (L1) or lam / ||block b|| (L2, 0 for a zero block);
 *                     loss_rows[0..nrows) = lam * sum_b ||block b||  (a pseudo loss head)
 *   pkc_reg_grad    : g += coef[block] * sign(x) (L1) or coef[block] * x (L2), items with g set
 *                     (g = ... for items with assign set)
 * ------------------------------------------------------------------------------------------- */
enum { PKC_REG_L1 = 1, PKC_REG_L2 = 2 };
typedef struct pkc_reg_item_s {
  const float* p;     /* parameter (row-major, leading dimension ld) */
  float* g;           /* its gradient buffer (NULL: loss term only) */
  int64_t ld;
  int r0, r1, c0, c1; /* the item's rectangle */
  int block;          /* block index */
  int assign;         /* 1: g = term gradient (a parameter only the term trains); 0: g += */
} pkc_reg_item;
int pkc_reg_partial(int kind, const pkc_reg_item* items_dev, int nitems, float* partial,
                    void* stream);
int pkc_reg_finalize(int kind, const int32_t* block_start_dev, int nblocks, const float* partial,
                     float lam, float* coef, float* loss_rows, int nrows, void* stream);
int pkc_reg_grad(int kind, const pkc_reg_item* items_dev, int nitems, const float* coef,
                 void* stream);

/* dst (bf16) = src (fp32), n elements (bf16 operand copies for the MFMA matmuls) */
int pkc_cast_bf16(const float* src, void* dst, int64_t n, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Chunk preparation on the GPU (data_io.py:105-145 context_window + load_chunk normalisation,
 * data_io.py:269-270 frame shuffle as a row permutation):
 *   cw_stats : column mean / population std (fp64) of the context-expanded chunk;
 *   cw_apply : out[r] = (expand(raw)[perm[r]] - mean) / std as fp32, labels shifted by -lab_min.
 * raw is N x D (length-sorted concatenated utterances); expanded row r (0 <= r < N-L-R), block b
 * (0..L+R) holds raw[(r + 2L - b) mod N] (np.roll order, future frame first).
 * ------------------------------------------------------------------------------------------- */
int pkc_cw_stats(const float* raw, int64_t N, int D, int L, int R, double* mean, double* std,
                 double* work, void* stream);
int64_t pkc_cw_stats_work_size(int64_t N, int D, int L, int R);
int pkc_cw_apply(const float* raw, int64_t N, int D, int L, int R, const double* mean,
                 const double* std, const int64_t* perm, float* out, int64_t ld_out, void* stream);
/* One feature stream of a multi-stream chunk (data_io.py:184-263, ABI 9): expanded rows
 * row0 + perm[j] (row0 + j without perm), j < nrows, of this stream's own expansion and statistics
 * — the rows the reference keeps after trimming every stream to the widest context window
 * (row0 = cw_left_max - L, nrows = N - cw_left_max - cw_right_max) — written to out (the stream's
 * first column in the chunk matrix) with row stride ld_out (the chunk's width). */
int pkc_cw_apply_rows(const float* raw, int64_t N, int D, int L, int R, const double* mean,
                      const double* std, const int64_t* perm, int64_t row0, int64_t nrows,
                      float* out, int64_t ld_out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Kaldi feature front-end (replaces the `apply-cmvn ... | add-deltas ...` stages of the fea_opts
 * pipe that data_io.py:18 runs through read_mat_ark, data_io.py:645-664; Kaldi's ApplyCmvn and
 * DeltaFeatures restated).  raw: Nsrc x D frames of whole utterances; output row r (of Nout, in
 * the sorted / split load_dataset order) is source frame src_row[r] of utterance u = utt_of_row[r],
 * whose frames are [utt_beg[u], utt_end[u]) of raw.  cmvn_mode 0 none, 1 means (x + offset),
 * 2 means+vars (x * scale + offset); norm[utt_norm[u]] = {offset[D], scale[D]} (fp32, computed by
 * the host as ApplyCmvn does in double).  scales: (order+1) x (2*maxoff+1) delta windows (zero
 * outside each order's own window); frames clamp to the utterance.  out: Nout x D*(order+1).
 * order <= 7.
 * ------------------------------------------------------------------------------------------- */
int pkc_feat_frontend(const float* raw, int D, int64_t Nout, const int32_t* src_row,
                      const int32_t* utt_of_row, const int32_t* utt_beg, const int32_t* utt_end,
                      const int32_t* utt_norm, const float* norm, int cmvn_mode,
                      const float* scales, int order, int maxoff, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Recurrent layers: the per-time-step loops of liGRU (neural_networks.py:1573-1584), LSTM
 * (neural_networks.py:1077-1097), GRU (:1390-1396, gates z, r, h), minimalGRU (:1751-1755, gates
 * z, h) and RNN (:1905-1907, gate h).  wpre holds the gate pre-activations W x (+BN) for the T*B input
 * rows, gate-major (G, T, B, H): liGRU gates (z, h), LSTM gates (f, i, o, c).  Bidirectional
 * layers (liGRU's shared-weight cat/flip convention, :1536-1538) run 2B rows per step; rows >= B
 * read time T-1-t and write the second half of the (T, B, 2H) output y.  Forward saves
 * hs (T+1, B2, H) [hs[0] = 0], cs (LSTM, T+1, B2, H) and gate activations (G, T, B2, H) for BPTT.
 * Dropout: bernoulli(1-p) mask per (row, unit), shared by all steps and NOT rescaled; (1-p) at eval.
 * pkc_rnn_bwd: dy = dL/dy (layer output layout); writes dgates (G, T, B2, H) = dL/d pre-activation
 * per direction and dpre (G, T, B, H) = the same folded over directions (input of the BN / W
 * backward); work = 8*B2*H floats (carries + per-gate partial products).
 * ------------------------------------------------------------------------------------------- */
enum { PKC_CELL_LIGRU = 0, PKC_CELL_LSTM = 1, PKC_CELL_GRU = 2, PKC_CELL_MINGRU = 3, PKC_CELL_RNN = 4 };
typedef struct {
  int cell, T, B, H, bidir, act, train;
  const float* wpre;
  const float* U[4];
  float drop_p; uint64_t seed; const int64_t* step_ctr; int64_t stream_id;
  const float* drop_mask_in;   /* optional injected (B2, H) mask */
  float* drop_mask;            /* (B2, H) mask in use */
  float* hs; float* cs; float* gates; float* y;
  const float* dy; int dy_nslab; int64_t dy_slab_stride;   /* dL/dy as split-K partial slabs */
  float* dgates; float* work;
  /* QuantizeLinear U layers with input quantisation (quantized_modules.py:99-119): h_{t-1} is
   * re-quantised once per gate (q1..q4, per-tensor max-abs) before each U product; U[] then points
   * at the fake-quantised weights.  hq (T+1, B2, H) receives q4(h_{t-1}) — the value the reference
   * keeps as hiddens[t-1] and as the saved input of the U backward. qbits = 0: off. */
  int qbits; float* hq;
  /* GRU / minimalGRU: r*h_{t-1} (z*h_{t-1}) per step, (T, B2, H) — the input of the Uh product
   * and of its gradient matmul.  NULL for the other cells. */
  float* rh;
  /* pkc_rnn_bwd: G x H x H scratch for the transposed U (the B operand of the BPTT products) */
  float* ut;
  /* LayerNorm of h after every step (use_laynorm; neural_networks.py:40-51 applied at :1093-1094,
   * :1581-1582 ...): gamma / beta (H), NULL = off; xhat (T, B2, H) and stat (T, B2, 2) saved by the
   * forward; g (T, B2, H) the post-norm gradients, dgamma / dbeta (H) written by the backward. */
  const float* ln_gamma; const float* ln_beta; float ln_eps;
  float* ln_xhat; float* ln_stat; float* ln_g; float* ln_dgamma; float* ln_dbeta;
  /* Block-sparse U (static HCGS masks, HCGS.py:24-28; liGRU / LSTM, no quantised h): per
   * workgroup tile, the indices of the 16-wide contraction blocks holding a nonzero of the mask
   * (-1 = empty slot), kmap_s* slots per tile (16, 32 or 64; 16 lane groups x kmap_s/16 blocks).
   *   kmap_fwd [ceil(H / (16/G))][kmap_s_fwd]: blocks of k (h_{t-1} / U columns) that the forward
   *     tile of 16/G units x G gates reads;
   *   kmap_bwd [G][ceil(H/16)][kmap_s_bwd]: blocks of j (U rows) that the BPTT tile of 16 columns k
   *     of gate g reads.
   * NULL: dense contraction over all H. */
  const int32_t* kmap_fwd; const int32_t* kmap_bwd; int kmap_s_fwd, kmap_s_bwd;
  /* bf16 step products (the performance mode of the sequence configs; liGRU / LSTM / RNN, dense U,
   * no quantised h, no LayerNorm): step_bf16 = 1 runs U h_{t-1} and the BPTT products dgates U^T on
   * v_mfma_f32_16x16x32_bf16 with fp32 accumulation, reading bf16 copies of their operands:
   *   hs_h (T+1, B2, H) bf16 copy of hs, written by the forward steps (hs_h[0] = 0);
   *   U_h[g] (H x H) bf16 copies of U[g] (the caller keeps them current);
   *   ut_h (G x H x H) bf16 U^T, written by pkc_rnn_bwd's transpose;
   *   dgates_h (G, T, B2, H) bf16 copy of dgates, written by the backward steps.
   * Cell state, gates, h and every other quantity stay fp32.  0: exact-fp32 products. */
  int step_bf16;
  void* hs_h; const void* U_h[4]; void* ut_h; void* dgates_h;
  /* Persistent time loops (liGRU with bf16 step products and a block-sparse U, H <= 576): the
   * whole forward (and BPTT) time loop of a layer in ONE launch of ceil(B2 / rows_per_wg)
   * workgroups, each owning its batch rows for all T steps with the layer's nonzero U (U^T)
   * blocks held in registers and LDS as MFMA operands and h_{t-1} (dgates_t) in LDS — no per-step
   * launch, no cross-workgroup hand-off (rows are independent).  persist_fwd / persist_bwd:
   * [nwaves][nslots] int32 fragment plans (pkc_rnn_persist_geometry): bits 0-7 the output tile
   * (16 units; BPTT: 16 columns k), 8-15 the 32-wide contraction block + 1 (0 = none), bit 16 the
   * last fragment of this wave's part of the tile, bit 17 valid, bit 18 set on that flush when
   * the part is the second of a tile cut between two waves, bits 19-21 its spill-over tile index
   * (distinct per cut tile, < nwaves - 1).  persist_kb = the forward plan's nslots.
   * NULL (or a layer outside these limits): the per-step launches. */
  const int32_t* persist_fwd; const int32_t* persist_bwd; int persist_kb;
  /* Exact quantised-h step products (qbits > 0, step_bf16 = 0): the caller guarantees U[g] lies on
   * a weight grid of <= 8 bits (m / 2^(b-1), |m| <= 2^(b-1): exact in bf16) and passes its bf16
   * copies in U_h[g].  The forward step then writes the grid integers k of q_g (|k| <= 2^(qbits-1))
   * as two exact bf16 parts and evaluates U q_g = var 2^-(qbits-1) U k on the bf16 MFMA with fp32
   * accumulation (exact integer sums up to H = 512): the fp32 products to within their own
   * rounding.  Each step leaves its per-wave max|h| partials in work (two slots by step parity,
   * at most 2 x H floats; work's 8 x B2 x H hold them) for the next step's var.
   * 0: the exact-fp32 chain. */
  int qh_exact;
} pkc_rnn_args;
int pkc_fakequant_weight(const float* w, float* q, int64_t n, int bits, void* stream);
/* out = q1..q_reps (reps consecutive n-float tensors) of the in-place input quantisation that
 * `reps` successive QuantizeLinear calls apply to one tensor; work >= 136 floats. */
int pkc_fakequant_input(const float* x, float* out, int64_t n, int bits, int reps, float* work,
                        void* stream);
/* Pattern mask (sparsity.py:1112-1146) of W (rows x cols, multiples of ph x pw) for P <= 32
 * patterns (P x ph x pw, {0,1}); ties select every maximal pattern (mask values can exceed 1). */
int pkc_pattern_mask(const float* W, int rows, int cols, const float* patterns, int P, int ph,
                     int pw, float* mask, void* stream);
/* Sequence batch assembly (core.py:183-214): sentence k of the batch starts at chunk row beg[k],
 * has len[k] frames and is placed at time offset left[k] (python random.randint(0, max_len-len),
 * drawn on the host in the reference's order); the rest of the (max_len, B, F) input is zero and
 * the labels of padded frames are 0 (they count in the loss, as in the reference). */
int pkc_seq_gather(const float* feats, int64_t ld_feats, int F, const int32_t* labels, int nlab,
                   const int64_t* beg, const int32_t* len, const int32_t* left, int B, int max_len,
                   float* x_out, int32_t* lab_out, void* stream);
/* Geometry of the persistent liGRU loops' plan tables (pkc_rnn_args.persist_*): waves per
 * workgroup, fragment slots per wave of the forward plan (= persist_kb) and of the BPTT plan,
 * batch rows per workgroup, largest H. */
int pkc_rnn_persist_geometry(int* nwaves, int* nslots_fwd, int* nslots_bwd, int* rows_per_wg,
                             int* hmax);
/* Which time-loop form pkc_rnn_fwd (bwd = 0) / pkc_rnn_bwd (bwd = 1) takes for these arguments:
 * 1 the persistent liGRU loops (persist_* plans above); 2 the persistent grid-synchronised loops —
 * qh_exact LSTM (uni-directional, B <= 16; forward H in {512, 768, 1024}, BPTT H = 512), dense LSTM
 * in bf16 step mode (B2 <= 32, H in {512, 768, 1024}) and liGRU in exact-fp32 step mode
 * (B2 <= 16, H <= 768): the layer's units dealt to H / 16 (liGRU forward: H / 8) workgroups that
 * hand h_t / dgates_t to each other every step; work's floats [4 B2 H, 4 B2 H + 4) hold their step
 * counter and timeout word; 0 one launch per time step.  Environment: PKC_RNN_LSTM_PERSIST=0 and
 * PKC_RNN_LIGRU_GRID=0 disable form 2 for LSTM / liGRU. */
int pkc_rnn_persist_form(const pkc_rnn_args* a, int bwd);
int pkc_rnn_fwd(const pkc_rnn_args* a, void* stream);
int pkc_rnn_bwd(const pkc_rnn_args* a, float* dpre, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Host-side Kaldi ark I/O (data_io.py:770-806 write_mat; 645-711 read_mat_ark binary FM/DM).
 * ------------------------------------------------------------------------------------------- */
int pkc_ark_write_mat(const char* path, int append, const char* key, int64_t rows, int64_t cols,
                      const float* data);
/* Index a binary ark of FM matrices: fills up to cap entries of (data byte offset, rows, cols)
 * and key offsets into keys_buf; returns the number of matrices or <0. */
int64_t pkc_ark_index(const char* path, int64_t* offsets, int64_t* rows, int64_t* cols, int64_t cap,
                      char* keys_buf, int64_t keys_cap);
int pkc_ark_read_rows(const char* path, int64_t offset, int64_t rows, int64_t cols, float* dst);
/* Kaldi "CM " compressed matrix (data_io.py:729-766): blob = the bytes after "\0BCM ";
 * pkc_ark_cm_size -> its byte length; pkc_ark_decode_cm -> rows x cols float32, row-major. */
int64_t pkc_ark_cm_size(const unsigned char* blob, int64_t nbytes);
int pkc_ark_decode_cm(const unsigned char* blob, int64_t nbytes, float* out);

/* ---------------------------------------------------------------------------------------------
 * Chunk-level data parallelism (the reference trains on one GPU, core.py:216-232):
 * one RCCL all-reduce (SUM) of the flat fp32 gradient buffer per step over xGMI, for hosts that
 * do not use torch.distributed.  Rank 0: pkc_dp_unique_id (pkc_dp_unique_id_bytes() bytes),
 * shipped to the other ranks by the host; every rank: pkc_dp_comm_init on its GPU (device < 0:
 * the current one), then pkc_dp_allreduce(comm, grads, n, stream) between the backward and the
 * optimizer launches of each step, with the loss gradient pre-scaled by 1/world (or by the
 * rank's share of the frames) so the sum is the gradient of the global mean loss.
 * ------------------------------------------------------------------------------------------- */
int pkc_dp_unique_id_bytes(void);
int pkc_dp_unique_id(void* id_out);
int pkc_dp_comm_init(void** comm_out, int world, const void* id, int rank, int device);
int pkc_dp_allreduce(void* comm, float* buf, int64_t n, void* stream);
int pkc_dp_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* PKC_H_ */
