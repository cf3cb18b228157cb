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
