// pkc_frontend.hip — the Kaldi feature front-end of the reference's loader pipeline, on the GPU.
//
// Every shipped cfg reads features through
//   copy-feats scp:<scp> ark:- | apply-cmvn --utt2spk=ark:<u2s> ark:<cmvn> ark:- ark:- |
//   add-deltas --delta-order=<0|2> ark:- ark:- |
// (data_io.py:18 builds the pipe; cfg/*/*.cfg fea_opts).  The build image has no Kaldi, so the
// two stages run here, on the raw chunk after it lands in HBM and BEFORE the sort / split of
// load_dataset (data_io.py:34-79) — deltas of a split piece read across the cut, as they do when
// Kaldi computed them on the whole utterance.
//
// Kaldi semantics restated (Kaldi is a third-party dependency absent from /root/reference; its
// algorithm is restated from transform/cmvn.cc ApplyCmvn and feat/feature-functions.cc
// DeltaFeatures — parity UNPINNED against Kaldi itself, pinned against oracle/kaldi_feat.c):
//   cmvn (host precomputes, per speaker, float offset[d] and scale[d] exactly as ApplyCmvn):
//     means only : x' = x + offset                  (AddVecToRows, float add)
//     means+vars : x' = (x * scale) + offset        (MulColsVec then AddVecToRows, no fusion)
//   deltas: out[o*D + d] = sum_{j=-m..m, scale_o[j] != 0} scale_o[j] * x'[clamp(t+j)][d], summed
//     in ascending j as Kaldi's per-j AddVec (BLAS saxpy: one fused multiply-add per term), with
//     t+j clamped to the ORIGINAL utterance's frames.
// One thread per (output row, feature dim): HBM-bound, 4*D*(2m+1) B read (L2-served after the first
// touch) + 4*D*(O+1) B written per row.
#include "pkc_common.h"

#pragma clang fp contract(off)

namespace pkc {

constexpr int FE_MAX_ORDER = 7;

__global__ __launch_bounds__(256) void feat_frontend_kernel(
    const float* __restrict__ raw, int D, int64_t Nout, const int32_t* __restrict__ srow,
    const int32_t* __restrict__ urow, const int32_t* __restrict__ ubeg,
    const int32_t* __restrict__ uend, const int32_t* __restrict__ unorm,
    const float* __restrict__ norm, int cmvn_mode, const float* __restrict__ scales, int order,
    int maxoff, float* __restrict__ out) {
  const int64_t total = Nout * D;
  const int W = 2 * maxoff + 1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / D;
    const int d = (int)(i - r * D);
    const int u = urow[r];
    const int64_t s = srow[r], b = ubeg[u], e = uend[u] - 1;
    float off = 0.f, sc = 1.f;
    if (cmvn_mode) {
      const float* nt = norm + (int64_t)unorm[u] * 2 * D;
      off = nt[d];
      sc = nt[D + d];
    }
    float acc[FE_MAX_ORDER + 1];
#pragma unroll
    for (int o = 0; o <= FE_MAX_ORDER; ++o) acc[o] = 0.f;
    for (int j = -maxoff; j <= maxoff; ++j) {
      int64_t f = s + j;
      f = f < b ? b : (f > e ? e : f);
      float x = raw[f * D + d];
      if (cmvn_mode == 2) x = __fmul_rn(x, sc);
      if (cmvn_mode) x = __fadd_rn(x, off);
#pragma unroll
      for (int o = 0; o <= FE_MAX_ORDER; ++o) {
        if (o > order) break;
        const float w = scales[o * W + j + maxoff];
        if (w != 0.f) acc[o] = __builtin_fmaf(w, x, acc[o]);
      }
    }
    float* dst = out + r * (int64_t)D * (order + 1) + d;
#pragma unroll
    for (int o = 0; o <= FE_MAX_ORDER; ++o) {
      if (o > order) break;
      dst[(int64_t)o * D] = acc[o];
    }
  }
}

}  // namespace pkc

extern "C" int pkc_feat_frontend(const float* raw, int D, int64_t Nout, const int32_t* src_row,
                                 const int32_t* utt_of_row, const int32_t* utt_beg,
                                 const int32_t* utt_end, const int32_t* utt_norm, const float* norm,
                                 int cmvn_mode, const float* scales, int order, int maxoff,
                                 float* out, void* stream) {
  using namespace pkc;
  PKC_CHECK_ARG(raw && src_row && utt_of_row && utt_beg && utt_end && scales && out && D > 0 &&
                    Nout >= 0 && order >= 0 && order <= FE_MAX_ORDER && maxoff >= 0 &&
                    cmvn_mode >= 0 && cmvn_mode <= 2 && (cmvn_mode == 0 || (norm && utt_norm)),
                "pkc_feat_frontend: bad arguments");
  if (Nout == 0) return PKC_OK;
  const int64_t total = Nout * D;
  const int64_t want = (total + 255) / 256;
  const unsigned grid = (unsigned)(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(feat_frontend_kernel, dim3(grid), dim3(256), 0, S(stream), raw, D, Nout,
                     src_row, utt_of_row, utt_beg, utt_end, utt_norm, norm, cmvn_mode, scales, order,
                     maxoff, out);
  PKC_LAUNCH_CHECK("pkc_feat_frontend");
  return PKC_OK;
}
