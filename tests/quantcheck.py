"""Flip-count bound for the fake-quantised configurations.

A weight the next forward multiplies with is its 8-bit grid value k / 2^(b-1),
k = sign(w) * ceil(|clamp(w, -1, 1)| * 2^(b-1)) (quantized_modules.py:77-97, balanced=False).  Two
runs whose fp32 arithmetic differs only in summation order put a weight on a different grid point
only where its fp32 value lies within rounding of a grid boundary: a handful of elements, each ONE
quantum away — or, after optimizer steps, a few quanta: an RMSprop step is a sign step at first,
so a gradient within rounding of zero that changes sign moves its weight by 2 x 4.48 lr per step
(rmsprop_quanta).  A systematic off-by-one in a quantiser instead moves a large share of the elements,
or moves some by more than one quantum — the loose relative tolerances of those tests are only
justified together with this bound.  Measured shares (round 3): the C5 layer shapes after 2 steps
and the two-rank C5 DP step 0-0.2 %; the quantised run_nn chunk trained from scratch 0.7 % (35 of
4,800: its weights differ by chaos-amplified ~1e-4 after the chunk, and ~2.6 % of the elements lie
within that of a 1/128 boundary) — the callers allow 0.2 % and 5 % respectively, against the ~100 %
a systematic off-by-one moves.
"""
import numpy as np


def grid_index(w, bits=8):
    w = np.clip(np.asarray(w, dtype=np.float64), -1.0, 1.0)
    return np.sign(w) * np.ceil(np.abs(w) * 2.0 ** (bits - 1))


def quantum_flips(got, ref, bits=8):
    """(elements on different grid points, largest grid distance) of two weight tensors."""
    d = grid_index(got, bits) - grid_index(ref, bits)
    return int(np.count_nonzero(d)), (float(np.abs(d).max()) if d.size else 0.0)


def rmsprop_quanta(lr, steps, bits=8):
    """Grid distance two runs' weights can reach when a near-zero gradient takes opposite signs in
    them: RMSprop's early steps are lr * g / sqrt((1 - alpha) g^2) <= 4.48 lr (alpha = 0.95), in
    opposite directions, every step."""
    return int(np.ceil(2 * steps * 4.48 * lr * 2.0 ** (bits - 1)))


def assert_few_flips(got, ref, name, frac, bits=8, max_quanta=1):
    """At most `frac` of the elements (and at least one allowed) on another grid point, none more
    than max_quanta away.  Returns the flip count."""
    n, dmax = quantum_flips(got, ref, bits)
    size = np.asarray(ref).size
    assert dmax <= max_quanta, "%s: a weight moved %g quanta" % (name, dmax)
    assert n <= max(1, int(frac * size)), "%s: %d of %d weights on another 8-bit grid point" % (
        name, n, size)
    return n
