"""The recurrent step kernel's input quantiser (pkc_rnn_impl.h qin<FAST>) restated op for op on the
CPU and checked bit-for-bit against the reference's float32 sequence (quantized_modules.py:99-119:
x / var, abs, * 2^(b-1), ceil, / 2^(b-1), * var, * sign), over the four chained calls of an LSTM
step (neural_networks.py:1086-1091) with var shared across the chain (the kernel's proof: Q maps
the max-abs element to exactly +-var).  The FAST form divides against var_s = var 2^-(b-1) with
one Markstein fma pair and multiplies k * var_s; fma is evaluated exactly (fractions) and
rounded once to float32.  CPU only: a statement about the arithmetic, the GPU kernel is checked
against the same reference sequence by tests/test_gpu_quant_step.py."""
from fractions import Fraction

import numpy as np

f32 = np.float32


def _fma(a, b, c):
    return f32(float(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))))


def _ref(x, var, bits):
    S = f32(2.0 ** (bits - 1))
    return f32(np.ceil(np.abs(f32(x / var)) * S) / S * var * np.sign(x))


def _fast(x, var, bits):
    scale = f32(2.0 ** (bits - 1))
    rcp_s = f32(f32(1.0) / var) * scale
    var_s = var * f32(1.0 / float(scale))
    q = f32(x * rcp_s)
    e = _fma(-q, var_s, x)
    q = _fma(e, rcp_s, q)
    return f32(np.copysign(f32(np.ceil(np.abs(q)) * var_s), x))


def test_fast_quantiser_matches_reference_chain():
    rs = np.random.RandomState(0)
    n_bad = n = 0
    for trial in range(40):
        scale = 10.0 ** rs.uniform(-6, 0)
        h = (np.tanh(rs.randn(150) * 2) * scale).astype(np.float32)
        h[:3] = [0.0, -0.0, np.float32(1e-30) * scale]
        bits = 16 if trial % 4 else 8
        var = f32(max(abs(h.max()), abs(h.min())))
        qr, qf = h.copy(), h.copy()
        for _ in range(4):
            qr = np.array([_ref(v, var, bits) for v in qr], dtype=np.float32)
            qf = np.array([_fast(v, var, bits) for v in qf], dtype=np.float32)
            assert f32(max(abs(qr.max()), abs(qr.min()))) == var      # var_g == var_1
            n_bad += int((qr != qf).sum())
            n += qr.size
    assert n_bad == 0, "%d of %d quantised values differ" % (n_bad, n)
