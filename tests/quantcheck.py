"""Flip-count bound for the fake-quantised configurations.

A weight the next forward multiplies with is its 8-bit grid value k / 2^(b-1),
k = sign(w) * ceil(|clamp(w, -1, 1)| * 2^(b-1)) (quantized_modules.py:77-97, balanced=False).  Two
runs whose fp32 arithmetic differs only in summation order put a weight on a different grid point
only where its fp32 value lies within rounding of a grid boundary: a handful of elements, each ONE
quantum away.  A systematic off-by-one in a quantiser instead moves a large share of the elements,
or moves some by more than one quantum — the loose relative tolerances of those tests are only
justified together with this bound.
"""
import numpy as np


def grid_index(w, bits=8):
    w = np.clip(np.asarray(w, dtype=np.float64), -1.0, 1.0)
    return np.sign(w) * np.ceil(np.abs(w) * 2.0 ** (bits - 1))


def quantum_flips(got, ref, bits=8):
    """(elements on different grid points, largest grid distance) of two weight tensors."""
    d = grid_index(got, bits) - grid_index(ref, bits)
    return int(np.count_nonzero(d)), (float(np.abs(d).max()) if d.size else 0.0)


def assert_few_flips(got, ref, name, frac, bits=8):
    """At most `frac` of the elements (and at least one allowed) on another grid point, each by
    exactly one quantum.  Returns the flip count."""
    n, dmax = quantum_flips(got, ref, bits)
    size = np.asarray(ref).size
    assert dmax <= 1.0, "%s: a weight moved %g quanta" % (name, dmax)
    assert n <= max(1, int(frac * size)), "%s: %d of %d weights on another 8-bit grid point" % (
        name, n, size)
    return n
