"""Host-side mask generation (runs once per model build, never per step).

hcgs_mask: the HCGS connectivity matrix of HCGS.py:24-28 -> hcgs.py:77-143 -> cgs_base.py:4-58,
generated with the same numpy RNG call sequence (np.random.choice(n, k, replace=False) per block
row, depth-first) so a model built with the reference's seed gets the reference's masks.  The
block-row choices are materialised with broadcasting instead of per-block slicing.
"""
import numpy as np


def _fill(out, r0, r1, c0, c1, levels, rng, top):
    n_in, n_out = r1 - r0, c1 - c0
    if not levels:
        out[r0:r1, c0:c1] = 1.0
        return
    (bs, drop), rest = levels[0], levels[1:]
    keep = 1.0 - float(drop) / 100.0
    if top:   # hcgs.py:90-97: python-3 true division before the int() casts
        rows_f = n_in / bs + (1 if n_in % bs else 0)
        cols_f = n_out / bs + (1 if n_out % bs else 0)
        n_sel = int(round(cols_f * keep))
        n_rows, n_cols = int(rows_f), int(cols_f)
    else:     # cgs_base.py:12-20: floor division
        n_rows = n_in // bs + (1 if n_in % bs else 0)
        n_cols = n_out // bs + (1 if n_out % bs else 0)
        n_sel = int(round(n_cols * keep))
    ragged_col = n_out % bs != 0
    for i in range(n_rows):
        last = i == n_rows - 1
        rr0 = r0 + i * bs
        rr1 = r0 + n_in if last else rr0 + bs
        for c in rng.choice(n_cols, n_sel, False):
            cc0 = c0 + c * bs
            # the ragged last column block is widened to n_out except on the last block row
            # (hcgs.py:101-106 vs 110-114)
            if c == n_cols - 1 and ragged_col and not last:
                cc1 = c0 + n_out
            else:
                cc1 = min(c0 + (c + 1) * bs, c0 + n_out)
            if cc1 > cc0 and rr1 > rr0:
                _fill(out, rr0, rr1, cc0, cc1, rest, rng, False)


def hcgs_mask(out_features, in_features, block_sizes, drop_ratios, rng=None):
    """(out_features, in_features) float32 {0,1} mask; rng defaults to the global np.random."""
    if len(block_sizes) != len(drop_ratios):
        raise ValueError("block size and drop ratio should have the same length")
    rng = np.random if rng is None else rng
    m = np.zeros((out_features, in_features), dtype=np.float32)
    _fill(m, 0, out_features, 0, in_features, list(zip(block_sizes, drop_ratios)), rng, True)
    return m


# ------------------------------------------------------------------------------------------------
# guided HCGS: the connectivity is chosen by weight magnitude instead of at random
# (guided_hcgs.py:9-77 -> guided_cgs_base.py:5-58 -> guided_choices.py:4-31).  Each block row keeps
# the n_sel block columns with the largest mean |W| (torch AvgPool2d: float32 sum in window order,
# divided by the window size; np.argsort(...)[-n_sel:] picks them), recursively per level.  Used at
# model construction (from the initial W) and at chunk end (apply_ghcgs, core.py:298-300).
# ------------------------------------------------------------------------------------------------
def _window_mean(a):
    """torch.nn.AvgPool2d over one window: sequential float32 sum (row-major), / count."""
    s = np.cumsum(a.reshape(-1), dtype=np.float32)[-1] if a.size else np.float32(0)
    return np.float32(s / np.float32(a.size))


def _guided_choices(wabs, n_blk, n_sel, bs):
    """guided_choices.guided_array_rows: indices of the n_sel largest block means."""
    r, c = wabs.shape
    full = (c - bs) // bs + 1
    if full < 1:
        raise ValueError("guided HCGS: a %dx%d slice is narrower than its %d block" % (r, c, bs))
    K = [_window_mean(wabs[:, j * bs:(j + 1) * bs]) for j in range(full)]
    if c % bs != 0:
        x = (n_blk - 1) * bs
        K.append(_window_mean(wabs[:, x:c]))
    return np.argsort(np.array(K, dtype=np.float32))[-n_sel:]


def _guided_fill(out, wabs, levels):
    n_in, n_out = wabs.shape
    if not levels:
        out[...] = 1.0
        return
    (bs, drop), rest = levels[0], levels[1:]
    keep = 1.0 - float(drop) / 100.0
    n_rows = n_in // bs + (1 if n_in % bs else 0)
    n_cols = n_out // bs + (1 if n_out % bs else 0)
    n_sel = int(round(n_cols * keep))
    for i in range(n_rows):
        r0, r1 = i * bs, min((i + 1) * bs, n_in)
        ch = _guided_choices(wabs[r0:r1], n_cols, n_sel, bs)
        for c in ch[:n_sel]:          # argsort(...)[-0:] is the whole array; range(0) is empty
            c0, c1 = c * bs, min((c + 1) * bs, n_out)
            _guided_fill(out[r0:r1, c0:c1], wabs[r0:r1, c0:c1], rest)


def guided_hcgs_mask(out_features, in_features, block_sizes, drop_ratios, w):
    """(out_features, in_features) float32 {0,1} mask guided by |w| (w: (out, in) array/tensor)."""
    if len(block_sizes) != len(drop_ratios):
        raise ValueError("block size and drop ratio should have the same length")
    if hasattr(w, "detach"):
        w = w.detach().float().cpu().numpy()
    wabs = np.abs(np.asarray(w, dtype=np.float32))
    assert wabs.shape == (out_features, in_features)
    m = np.zeros((out_features, in_features), dtype=np.float32)
    _guided_fill(m, wabs, list(zip(block_sizes, drop_ratios)))
    return m


def kmeans_patterns(w, pattern_num, pattern_shape, pattern_nnz, random_state=None):
    """Pattern-set search of sparsity.find_top_k_by_kmeans (sparsity.py:999-1049), host-side and
    once per model like the reference: every non-overlapping ph x pw tile of |w| gives a {0,1}
    candidate keeping its entries >= the tile's pattern_nnz-th largest (ties keep several,
    1024-1025); sklearn KMeans(n_clusters=min(pattern_num, C(ph*pw, nnz))) clusters the candidates
    (1030) and each centre's pattern_nnz largest entries (torch.sort order, 1036-1041) become a
    pattern.  The reference passes no random_state, so its result is not reproducible (parity
    unpinned); ``random_state`` pins it for tests.  Returns a (P, ph, pw) float32 array."""
    import math

    import torch
    from sklearn.cluster import KMeans

    ph, pw = pattern_shape
    w = torch.as_tensor(w).detach().float().abs().cpu()
    nx, ny = (w.shape[0] - ph) // ph + 1, (w.shape[1] - pw) // pw + 1
    n_pat = min(int(pattern_num), math.comb(ph * pw, int(pattern_nnz)))
    tiles = w[:nx * ph, :ny * pw].reshape(nx, ph, ny, pw).permute(0, 2, 1, 3).reshape(-1, ph * pw)
    thr = torch.topk(tiles, int(pattern_nnz), dim=1).values[:, -1:]
    # the reference fits a Python list of float32 rows, which sklearn converts to float64
    cand = (tiles >= thr).to(torch.float64).numpy()
    km = KMeans(n_clusters=n_pat, random_state=random_state).fit(cand)
    out = np.zeros((n_pat, ph * pw), dtype=np.float32)
    for p, c in enumerate(km.cluster_centers_):
        idx = torch.from_numpy(c).sort()[1][-int(pattern_nnz):].numpy()
        out[p, idx] = 1.0
    return out.reshape(n_pat, ph, pw)
