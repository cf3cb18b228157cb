"""Bit-exactness of the quantised recurrent input inside the LSTM step kernel.

The reference re-quantises h_{t-1} in place once per gate (four QuantizeLinear calls per step,
neural_networks.py:1086-1091; Quantize_inp quantized_modules.py:99-119, each with its own per-tensor
max-abs).  The step kernel does ONE max-abs reduction (var_g = var_1 for every later call) and forms
x / var from the correctly rounded reciprocal plus an fma correction.  Both shortcuts must leave the
result bit-identical: the saved q4(h_{t-1}) (lb['hq']) is recomputed here from the saved h with the
reference's float32 op sequence in numpy (IEEE division, four reductions) and compared exactly.
"""
import configparser

import numpy as np
import pytest
import torch

from cases import LSTM_DEF

pytestmark = pytest.mark.gpu


def _quantise_like_reference(x, bits):
    S = np.float32(2.0 ** (bits - 1))
    q = x.astype(np.float32)
    for _ in range(4):
        var = np.float32(max(abs(q.max()), abs(q.min())))
        if var == 0:
            continue
        q = (np.ceil(np.abs(q / var) * S) / S * var * np.sign(q)).astype(np.float32)
    return q


@pytest.mark.parametrize("H,T,B,seed", [(24, 7, 3, 1), (512, 10, 12, 2), (1000, 5, 5, 3)])
def test_quantised_h_bit_exact(H, T, B, seed):
    import pkc.neural_networks as NN
    from test_gpu_rnn import run_block
    opts = dict(LSTM_DEF, lstm_lay="%d,%d" % (H, H), lstm_quant="True", lstm_quant_inp="True")
    cp = configparser.ConfigParser()
    cp["s"] = {k: str(v) for k, v in opts.items()}
    torch.manual_seed(seed)
    np.random.seed(seed)
    F = 40
    net = NN.LSTM(cp["s"], F).to("cuda").train()
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(T, B, F, generator=g).cuda()
    dy = torch.randn(T, B, net.out_dim, generator=g).cuda()
    eng, node, _ = run_block(net, x, dy)
    for li, lb in enumerate(node.lbuf):
        hs = lb["hs"][:(T + 1) * B * H].view(T + 1, B, H).cpu().numpy()
        hq = lb["hq"][:T * B * H].view(T, B, H).cpu().numpy()
        bits = node.layers[li]["ibits"]
        assert bits == 16
        nz = 0
        for t in range(T):
            ref = _quantise_like_reference(hs[t], bits)
            assert np.array_equal(hq[t], ref), "layer %d step %d: %d elements differ" % (
                li, t, int((hq[t] != ref).sum()))
            nz += int(np.count_nonzero(ref))
        assert nz > 0
