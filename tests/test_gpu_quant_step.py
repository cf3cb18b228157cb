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


@pytest.mark.parametrize("H,B,seed", [(512, 12, 4), (24, 3, 5), (1000, 5, 6)])
def test_qh_exact_products_match_fp32_chain(H, B, seed):
    """pkc_rnn_args.qh_exact (U on the 8-bit grid, bf16 integer MFMAs) against the exact-fp32
    chain on the same layer and inputs, over T = 2 steps: step 0 multiplies h_{-1} = 0 (identical
    outputs), step 1 multiplies the same q_g(h_0) on both paths, so its outputs differ only by the
    products' rounding — the integer form is exact up to one rounding per product, the chain rounds
    every add.  (Over longer sequences the 16-bit grid's ceil turns those last bits into one-quantum
    moves that the recurrence spreads — the oracle tests of C5 bound that regime.)"""
    import pkc.engine as E
    import pkc.neural_networks as NN
    from test_gpu_rnn import run_block
    T = 2
    opts = dict(LSTM_DEF, lstm_lay="%d,%d" % (H, H), lstm_quant="True", lstm_quant_inp="True")
    cp = configparser.ConfigParser()
    cp["s"] = {k: str(v) for k, v in opts.items()}
    outs = {}
    for exact in (True, False):
        torch.manual_seed(seed)
        np.random.seed(seed)
        net = NN.LSTM(cp["s"], 40).to("cuda").train()
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(T, B, 40, generator=g).cuda()
        dy = torch.randn(T, B, net.out_dim, generator=g).cuda()
        old = E.RNN_QH_EXACT
        E.RNN_QH_EXACT = exact
        try:
            eng, node, y = run_block(net, x, dy)
        finally:
            E.RNN_QH_EXACT = old
        assert all((lb.get("U_hq") is not None) == exact for lb in node.lbuf)
        lb = node.lbuf[0]
        outs[exact] = (lb["hs"][B * H:(T + 1) * B * H].view(T, B, H).cpu().double(),
                       lb["hq"][:T * B * H].view(T, B, H).cpu().double())
    he, hf = outs[True][0], outs[False][0]
    assert torch.equal(he[0], hf[0])                 # step 0: U * 0
    assert torch.equal(outs[True][1], outs[False][1])  # the same quantised h_{t-1} both steps
    scale = float(hf[1].abs().max())
    d = float((he[1] - hf[1]).abs().max())
    print("H %d: layer-0 step-1 h max diff %.3g of scale %.3g" % (H, d, scale))
    assert d <= 2e-6 * scale, "step-1 h differs by %.3g (scale %.3g)" % (d, scale)
