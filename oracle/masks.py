"""Oracle: sparsity masks and fake quantisation restated in numpy / torch-CPU (test only).

  hcgs_conn_mat   hcgs.py:77-143 (top level: float block counts, python-3 '/') and
                  cgs_base.py:4-58 (recursive levels: integer '//')
  quantize        quantized_modules.py:77-97  (balanced=False; clamp in place, ceil grid)
  quantize_inp    quantized_modules.py:99-119 (dynamic per-tensor max-abs, ceil grid)
  prune           quantized_modules.py:15-28  (np.percentile over |W|, strict '>')
  apply_patterns  sparsity/sparsity.py:1112-1146 (conv2d score, ties select all, conv_transpose)
  kmeans_patterns sparsity/sparsity.py:999-1049 (top-k tile candidates, sklearn KMeans, top-k of
                  each centre); sklearn is the reference's own third-party dependency
"""
import numpy as np
import torch


def _level(n_in, n_out, blocks, drops, rng, top):
    """One HCGS level; `blocks`/`drops` are the remaining levels (outermost last, already
    reversed as the reference does with reverse()+pop())."""
    if not blocks:
        return np.ones((n_in, n_out), dtype=np.float32)            # cgs_base.py:5-7
    blocks = list(blocks)
    drops = list(drops)
    bs = blocks.pop()
    dr = drops.pop()
    keep = 1 - float(dr) / 100
    if top:                                                        # hcgs.py:90-97 (float '/')
        n_rows = n_in / bs
        if n_in % bs != 0:
            n_rows += 1
        n_cols = n_out / bs
        if n_out % bs != 0:
            n_cols += 1
        n_sels = int(round(n_cols * keep))
        n_rows, n_cols = int(n_rows), int(n_cols)
    else:                                                          # cgs_base.py:12-20 ('//')
        n_rows = n_in // bs + (1 if n_in % bs else 0)
        n_cols = n_out // bs + (1 if n_out % bs else 0)
        n_sels = int(round(n_cols * keep))
    m = np.zeros((n_in, n_out), dtype=np.float32)
    for i in range(n_rows - 1):                                    # hcgs.py:99-109
        ch = rng.choice(n_cols, n_sels, False)
        for c in ch:
            c0 = c * bs
            c1 = n_out if (c == n_cols - 1 and n_out % bs != 0) else (c + 1) * bs
            sub = m[i * bs:(i + 1) * bs, c0:c1]
            m[i * bs:(i + 1) * bs, c0:c1] = _level(sub.shape[0], sub.shape[1], blocks, drops, rng, False)
    ch = rng.choice(n_cols, n_sels, False)                         # hcgs.py:110-114 (last row)
    for c in ch:
        sub = m[(n_rows - 1) * bs:n_in, c * bs:(c + 1) * bs]
        m[(n_rows - 1) * bs:n_in, c * bs:(c + 1) * bs] = _level(sub.shape[0], sub.shape[1], blocks,
                                                               drops, rng, False)
    return m


def hcgs_conn_mat(n_rows, n_cols, block_sizes, drop_ratios, rng=None):
    """HCGS connectivity mask of shape (n_rows, n_cols) = (out_features, in_features)
    (HCGS.py:28 calls conn_mat(out_features, in_features, ...)).  rng defaults to global np.random."""
    rng = np.random if rng is None else rng
    b = list(block_sizes)[::-1]
    d = list(drop_ratios)[::-1]
    return _level(n_rows, n_cols, b, d, rng, True)


def quantize(w, bits):
    """quantized_modules.py:77-97 with balanced=False, if_forward=False.  Returns (w_clamped, wq):
    the reference clamps the parameter IN PLACE (persisting) and returns a new quantised tensor."""
    w = w.clamp(-1, 1)
    s = w.sign()
    q = w.abs().mul(2 ** (bits - 1)).ceil().div(2 ** (bits - 1))
    return w, q.mul(s)


def quantize_inp(x, bits):
    """quantized_modules.py:99-119, if_forward=False (op order kept for bitwise parity)."""
    mx = x.max().abs()
    mn = x.min().abs()
    var = mx if mx > mn else mn
    if var == 0.0:
        return x
    sg = x.sign()
    y = x.div(var)
    y = y.abs().mul(2 ** (bits - 1)).ceil().div(2 ** (bits - 1))
    y = y.mul(var)
    return y.mul(sg)


def prune_mask(w, perc):
    """quantized_modules.py:15-28 for one weight matrix (its only >1-D parameter)."""
    a = np.abs(w.detach().cpu().numpy()).ravel()
    thr = np.percentile(a, perc)
    return (w.detach().abs() > float(thr)).float() if isinstance(w, torch.Tensor) else None


def kmeans_patterns(w, pattern_num, pattern_shape, pattern_nnz, random_state=None):
    """sparsity.py:999-1049 with numpy tiles: per ph x pw tile (row-major tile order, 1018-1020)
    a {0,1} candidate keeping entries >= its nnz-th largest |w| (1021-1026); KMeans with
    n_clusters = min(pattern_num, C(ph*pw, nnz)) (1004-1005, 1030) fitted on the candidates as
    float64 (the reference hands sklearn a list of float32 rows); each centre keeps the last nnz
    indices of torch's ascending sort (1036-1041: ties among equal centre entries resolve in
    torch.sort's order, which a numpy stable argsort does not reproduce).  Returns (P, ph, pw)."""
    import math

    from sklearn.cluster import KMeans
    ph, pw = pattern_shape
    a = np.abs(np.asarray(w, dtype=np.float32))
    nx, ny = (a.shape[0] - ph) // ph + 1, (a.shape[1] - pw) // pw + 1
    cands = []
    for i in range(nx):
        for j in range(ny):
            t = a[i * ph:(i + 1) * ph, j * pw:(j + 1) * pw].ravel()
            thr = np.sort(t)[-pattern_nnz]
            cands.append((t >= thr).astype(np.float64))
    n = min(pattern_num, math.comb(ph * pw, pattern_nnz))
    centres = KMeans(n_clusters=n, random_state=random_state).fit(np.array(cands)).cluster_centers_
    out = np.zeros((n, ph * pw), dtype=np.float32)
    for p, c in enumerate(centres):
        out[p, torch.from_numpy(c).sort()[1][-pattern_nnz:].numpy()] = 1.0
    return out.reshape(n, ph, pw)


def apply_patterns(w, patterns):
    """sparsity.py:1112-1146.  w: (R, C) tensor with R, C multiples of the pattern size;
    patterns: (P, ph, pw) {0,1} array.  Mask values can exceed 1 where several patterns tie."""
    w = np.abs(np.asarray(w, dtype=np.float32))
    P, ph, pw = patterns.shape
    R, C = w.shape
    tiles = w[:R // ph * ph, :C // pw * pw].reshape(R // ph, ph, C // pw, pw).transpose(0, 2, 1, 3)
    score = np.einsum("ijab,pab->pij", tiles.astype(np.float64), patterns.astype(np.float64))
    score = score.astype(np.float32)
    sel = (score >= score.max(axis=0, keepdims=True)).astype(np.float32)
    mask_t = np.einsum("pij,pab->ijab", sel, patterns.astype(np.float32))
    out = np.zeros((R, C), dtype=np.float32)
    out[:R // ph * ph, :C // pw * pw] = mask_t.transpose(0, 2, 1, 3).reshape(R // ph * ph, C // pw * pw)
    return out


def guided_conn_mat(n_rows, n_cols, block_sizes, drop_ratios, w):
    """guided_hcgs.py:9-77 / guided_cgs_base.py:5-58 / guided_choices.py:4-31 (equal_blks_for_input
    branch): per block row keep the block columns with the largest AvgPool2d mean of |W|
    (torch.nn.AvgPool2d itself computes the means here), recursively per level."""
    wabs = torch.as_tensor(np.abs(np.asarray(w, dtype=np.float32)))
    levels = list(zip(block_sizes, drop_ratios))

    def rec(a, lv):
        r, c = a.shape
        if not lv:
            return np.ones((r, c), dtype=np.float32)
        bs, drop = lv[0]
        out = np.zeros((r, c), dtype=np.float32)
        nbr = r // bs + (r % bs != 0)
        nbc = c // bs + (c % bs != 0)
        nsel = int(round(nbc * (1 - float(drop) / 100)))
        for i in range(nbr):
            rows = a[i * bs:(i + 1) * bs]
            rr = rows.shape[0]
            pool = torch.nn.AvgPool2d((rr, bs), bs) if rr != bs else torch.nn.AvgPool2d(bs, bs)
            K = pool(rows[None, None])[0, 0]
            if c % bs:
                x = (nbc - 1) * bs
                K = torch.cat([K, torch.nn.AvgPool2d((rr, c - x), c - x)(rows[None, None, :, x:])[0, 0]], 1)
            ch = np.argsort(K[0].numpy())[-nsel:]
            for j in range(nsel):
                c0 = ch[j] * bs
                out[i * bs:(i + 1) * bs, c0:c0 + bs] = rec(rows[:, c0:c0 + bs], lv[1:])
        return out

    m = rec(wabs, levels)
    assert m.shape == (n_rows, n_cols)
    return m
