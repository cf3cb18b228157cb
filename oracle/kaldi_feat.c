/* ORACLE — test infrastructure only (see oracle/__init__.py).
 *
 * Plain-C restatement of the two Kaldi programs every shipped cfg puts in its fea_opts pipe
 * (cfg/TIMIT_baselines/TIMIT_MLP_fmllr.cfg fea_opts; piped by data_io.py:18 through
 * read_mat_ark, data_io.py:645-664):
 *   apply-cmvn  — transform/cmvn.cc ApplyCmvn (Kaldi, third-party, NOT in /root/reference)
 *   add-deltas  — feat/feature-functions.cc DeltaFeatures / ComputeDeltas
 * Kaldi is absent from the image and from the reference, and the reference holds no file of its
 * output, so this restatement is "parity unpinned" against Kaldi; pkc's GPU front-end
 * (csrc/pkc_frontend.hip + pkc/frontend.py) is checked bit-exactly against it.
 *
 * Arithmetic follows Kaldi's types: statistics in double; Vector<float>::AddVec(float alpha,
 * Vector<double>) evaluates alpha * v in double and rounds once into float; the delta windows are
 * built in float; each delta term is BLAS saxpy (one fused multiply-add per term, in ascending
 * window offset).  Built with -ffp-contract=off so no other operation is fused.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ApplyCmvn's per-dimension float offset / scale from a (rows x (dim+1)) double stats matrix.
 * Returns 0, or -1 for count < 1 (KALDI_ERR "Insufficient stats"), -2 for a non-finite scale. */
int kf_cmvn_norm(const double* stats, int rows, int dim, int norm_vars, float* offset,
                 float* scale) {
  const double count = stats[dim];
  if (count < 1.0) return -1;
  if (!norm_vars) {
    const float alpha = (float)(-1.0 / count);
    for (int d = 0; d < dim; ++d) {
      float o = 0.0f;
      o = (float)((double)o + (double)alpha * stats[d]);
      offset[d] = o;
      scale[d] = 1.0f;
    }
    return 0;
  }
  if (rows < 2) return -1;
  for (int d = 0; d < dim; ++d) {
    const double mean = stats[d] / count;
    double var = stats[(dim + 1) + d] / count - mean * mean;
    const double floor_v = 1.0e-20;
    if (var < floor_v) var = floor_v;
    const double sc = 1.0 / sqrt(var);
    if (sc != sc || 1.0 / sc == 0.0) return -2;
    offset[d] = (float)(-(mean * sc));
    scale[d] = (float)sc;
  }
  return 0;
}

/* In place on one utterance (T x D float): means only x += offset; with vars x = x*scale, then
 * x += offset (MulColsVec then AddVecToRows). */
void kf_apply_cmvn(float* feats, int64_t T, int D, const float* offset, const float* scale,
                   int norm_vars) {
  for (int64_t t = 0; t < T; ++t)
    for (int d = 0; d < D; ++d) {
      float x = feats[t * D + d];
      if (norm_vars) x = x * scale[d];
      x = x + offset[d];
      feats[t * D + d] = x;
    }
}

/* DeltaFeatures::DeltaFeatures: scales for orders 0..order; window i has 2*i*window+1 taps.
 * out holds (order+1) rows of 2*order*window+1 taps, each row's window centred, zero elsewhere. */
void kf_delta_scales(int order, int window, float* out) {
  const int maxoff = order * window, W = 2 * maxoff + 1;
  float prev[2 * 7 * 999 + 1], cur[2 * 7 * 999 + 1];
  memset(out, 0, sizeof(float) * (size_t)(order + 1) * W);
  int plen = 1;
  prev[0] = 1.0f;
  out[maxoff] = 1.0f;
  for (int i = 1; i <= order; ++i) {
    const int po = (plen - 1) / 2, co = po + window, clen = plen + 2 * window;
    for (int q = 0; q < clen; ++q) cur[q] = 0.0f;
    float normalizer = 0.0f;
    for (int j = -window; j <= window; ++j) {
      normalizer += (float)(j * j);
      for (int k = -po; k <= po; ++k) cur[j + k + co] += (float)j * prev[k + po];
    }
    const float alpha = (float)(1.0 / (double)normalizer);
    for (int q = 0; q < clen; ++q) cur[q] = cur[q] * alpha;
    const int half = (clen - 1) / 2;
    for (int q = 0; q < clen; ++q) out[(size_t)i * W + maxoff - half + q] = cur[q];
    for (int q = 0; q < clen; ++q) prev[q] = cur[q];
    plen = clen;
  }
}

/* DeltaFeatures::Process for every frame of one utterance: out is T x D*(order+1). */
void kf_add_deltas(const float* feats, int64_t T, int D, int order, int window, float* out) {
  const int maxoff = order * window, W = 2 * maxoff + 1;
  float scales[8 * (2 * 7 * 999 + 1)];
  if (order > 7) return;
  kf_delta_scales(order, window, scales);
  const int Do = D * (order + 1);
  for (int64_t t = 0; t < T; ++t) {
    float* o = out + t * Do;
    for (int q = 0; q < Do; ++q) o[q] = 0.0f;
    for (int i = 0; i <= order; ++i) {
      const int mo = i * window;
      for (int j = -mo; j <= mo; ++j) {
        int64_t f = t + j;
        if (f < 0) f = 0;
        else if (f >= T) f = T - 1;
        const float sc = scales[(size_t)i * W + maxoff + j];
        if (sc != 0.0f)
          for (int d = 0; d < D; ++d) o[i * D + d] = fmaf(sc, feats[f * D + d], o[i * D + d]);
      }
    }
  }
}
