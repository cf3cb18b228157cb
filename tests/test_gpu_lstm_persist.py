"""The persistent grid-synchronised LSTM loops (csrc/pkc_rnn_lstm_persist.hip) against the per-step
launches they replace, on the same layer and inputs: every saved forward tensor (h, c, the gates, the
quantised h, the layer output), the BPTT's gate gradients, the input gradient and every weight
gradient must be bit-identical — the persistent forward keeps the per-step kernel's per-wave
contraction ranges (exact integer sums), its per-wave fmaf(256, hi, lo) * var_s and its cross-wave
summation order; the BPTT keeps the per-step fp32 MFMA chains per gate and strip and both summation
orders (pkc_rnn_lstm_persist.hip header).  The per-step form itself is pinned to the oracle
(test_gpu_configs.py::test_c5_lstm_pattern_quant_full_size, test_gpu_quant_step.py), so this makes
the persistent loops oracle-exact by transitivity.

Sizes: C5's layers (H = 512, B = 12, quantised h of 16 bits, 8-bit U; BASELINE configs[4]) and
the forward-only shapes H = 768 / 1024.  The hand-off is also exercised under uneven load (a side
stream of large matmuls running during the loops, MI355X_MICROARCH.md: hand-offs must be tested
under load), and the timeout word of every launch must stay zero.
"""
import configparser
import os

import numpy as np
import pytest
import torch

from cases import LSTM_DEF

pytestmark = pytest.mark.gpu


def _block(net, x, dy, prec):
    """test_gpu_rnn.run_block with the engine's precision (bf16: the bf16 step products)."""
    from pkc.engine import Engine
    T, B, F = x.shape
    eng = Engine({"rnn": net}, {"rnn": {"arch_opt": "sgd", "arch_lr": "0"}},
                 [["out", "compute", "rnn", "fea"]], {"fea": (0, F)}, [], batch=B, max_len=T,
                 train=False, prec=prec)
    node = eng.nodes[0]
    eng.T, eng.M = T, T * B
    eng.x[:T * B * F].copy_(x.reshape(-1))
    s = eng._stream()
    eng._rec_fwd(node, s, True)
    y = node.out[:T * B * node.N].view(T, B, node.N).clone()
    node.gslab = dy.reshape(-1).contiguous()
    node.sb = 1
    eng._rec_bwd(node, s, want_dx0=True)
    torch.cuda.synchronize()
    return eng, node, y


def _run(H, T, B, seed, persist, load=False, bf16=False, bidir=False, f32=False):
    import pkc.neural_networks as NN
    from pkc import _lib as L
    from test_gpu_rnn import dx0
    os.environ["PKC_RNN_LSTM_PERSIST"] = "1" if persist else "0"
    try:
        if bf16 or f32:                # C4's form: dense, bf16 (or exact fp32) step products
            opts = dict(LSTM_DEF, lstm_lay="%d,%d" % (H, H), lstm_drop="0.2,0.2",
                        lstm_bidir=str(bidir))
        else:                          # C5's form: quantised h, 8-bit U
            opts = dict(LSTM_DEF, lstm_lay="%d,%d" % (H, H), lstm_drop="0.2,0.2", lstm_quant="True",
                        lstm_quant_inp="True")
        cp = configparser.ConfigParser()
        cp["s"] = {k: str(v) for k, v in opts.items()}
        torch.manual_seed(seed)
        np.random.seed(seed)
        F = 40
        net = NN.LSTM(cp["s"], F).to("cuda").train()
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(T, B, F, generator=g).cuda()
        dy = torch.randn(T, B, net.out_dim, generator=g).cuda()
        side = None
        if load:                       # uneven load: large matmuls on another stream meanwhile
            side = torch.cuda.Stream()
            a = torch.randn(4096, 4096, device="cuda")
            with torch.cuda.stream(side):
                for _ in range(12):
                    a = torch.tanh(a @ a * 1e-3)
        eng, node, y = _block(net, x, dy, L.PREC_BF16 if bf16 else L.PREC_FP32)
        if side is not None:
            side.synchronize()
        forms = eng.rec_forms()
        out = {"y": y.cpu(), "dx0": dx0(eng, node).cpu(), "grad": eng.gflat.cpu()}
        for li, lb in enumerate(node.lbuf):
            n = (2 * B if bidir else B) * H
            for k in ("hs", "cs", "gates", "hq", "dgates", "hs_h", "dgates_h"):
                if lb.get(k) is not None:
                    out["%d.%s" % (li, k)] = lb[k].cpu()
            out["%d.timeout" % li] = _ctr_words(lb["rwork"], n)
        return out, forms
    finally:
        os.environ.pop("PKC_RNN_LSTM_PERSIST", None)


def _ctr_words(rwork, n):
    """[arrivals, timeout word] of a layer's last grid-synchronised launch: the step counter is
    8 shards on 128-byte lines after the [counter, timeout] words at work[4 B2 H]
    (pkc_rnn_lstm_persist.hip NSH / SHW)."""
    w = rwork[4 * n:4 * n + 9 * 32].view(torch.int32).cpu()
    return torch.stack([w[32::32][:8].sum(), w[1]])


BWD_KEYS = ("dgates", "dx0", "grad")      # what the BPTT products feed


@pytest.mark.parametrize("H,T,B,seed,load,x3", [(512, 40, 12, 1, False, True),
                                                (512, 40, 12, 1, False, False),
                                                (512, 23, 12, 2, True, True),
                                                (512, 9, 7, 3, False, False),
                                                (512, 11, 9, 6, False, False),
                                                (512, 13, 16, 7, True, False),
                                                (768, 12, 12, 4, False, True),
                                                (1024, 10, 16, 5, False, True)])
def test_lstm_persist_bit_identical_to_steps(H, T, B, seed, load, x3, monkeypatch):
    """x3 = False (PKC_RNN_LSTM_PERSIST_X3=0): the BPTT's fp32 16x16x4 chains, every tensor
    bit-identical.  x3 = True (the default): the BPTT products in three exact bf16 parts — the
    forward stays bit-identical, what the BPTT feeds (dgates, dx, the weight gradients) differs
    from the per-step launches only in the fp32 summation order of exact products: bounded at
    2e-6 of each tensor's largest element (measured in the printout)."""
    monkeypatch.setenv("PKC_RNN_LSTM_PERSIST_X3", "1" if x3 else "0")
    ref, forms_ref = _run(H, T, B, seed, False)
    got, forms = _run(H, T, B, seed, True, load)
    assert all("persistent" not in f for f in forms_ref.values()), forms_ref
    want = "persistent grid-synchronised" + ("" if H == 512 else " / BPTT fp32 steps")
    assert all(f.startswith(want) for f in forms.values()), forms
    bad, rep = [], []
    for k in ref:
        if k.endswith(".timeout"):
            # [step counter, timeout word] of the last persistent launch, the BPTT's (32 x (T - 2)
            # arrivals; B > 8 rows: four row blocks per column block, 128 x (T - 2)); with per-step
            # BPTT launches (H != 512) their gate slabs hold these words
            if H == 512:
                nwg = 32 * (4 if B > 8 else 1)
                assert int(got[k][0]) == nwg * (T - 2), "%s: arrivals %d" % (k, int(got[k][0]))
                assert int(got[k][1]) == 0, "%s: a persistent loop timed out" % k
            continue
        a, b = got[k], ref[k]
        if x3 and H == 512 and k.split(".")[-1] in BWD_KEYS:
            err = float((a.double() - b.double()).abs().max()) / float(b.double().abs().max())
            rep.append("%s %.2e" % (k, err))
            if err > 2e-6:
                bad.append("%s: max |diff| %.3g of max |ref|" % (k, err))
            continue
        if not torch.equal(a, b):
            nd = int((a != b).sum())
            first = int((a != b).reshape(-1).nonzero()[0])
            bad.append("%s: %d of %d differ (max %.3g, first at flat %d)" % (
                k, nd, a.numel(), float((a.double() - b.double()).abs().max()), first))
    print("H %d T %d B %d x3 %s forms %s; BPTT rel. diff: %s" % (H, T, B, x3, forms, ", ".join(rep)))
    assert not bad, "; ".join(bad)
    assert float(ref["grad"].abs().max()) > 0


@pytest.mark.parametrize("H,T,B,bidir,seed,load", [(1024, 14, 16, True, 11, False),
                                                   (1024, 9, 16, True, 12, True),
                                                   (512, 21, 12, False, 13, False),
                                                   (768, 8, 10, True, 14, False)])
def test_lstm_persist_bf16_bit_identical_to_steps(H, T, B, bidir, seed, load, monkeypatch):
    """The bf16 step mode's persistent loops (C4's LSTM: 4 x 1024 bidirectional, B = 16, so 32
    rows per step; and smaller shapes) with the per-step kernels' contraction chunking
    (PKC_RNN_LSTM_CO=0) against the per-step bf16 launches: bit-identical.  (The default, coalesced
    chunking sums each element's bf16 products in another grouping; tests/test_gpu_steps.py checks
    it step by step against the oracle.)"""
    monkeypatch.setenv("PKC_RNN_LSTM_CO", "0")
    ref, forms_ref = _run(H, T, B, seed, False, bf16=True, bidir=bidir)
    got, forms = _run(H, T, B, seed, True, load, bf16=True, bidir=bidir)
    assert all("persistent" not in f for f in forms_ref.values()), forms_ref
    assert all(f.startswith("persistent grid-synchronised") and "/" not in f for f in forms.values()), forms
    print("bf16 H %d T %d B %d bidir %s forms %s" % (H, T, B, bidir, forms))
    bad = []
    n = (2 * B if bidir else B) * H
    nwg = (H // 16) * (4 if (2 * B if bidir else B) > 16 else 1)   # > 16 rows: 4 BPTT row blocks
    for k in ref:
        if k.endswith(".timeout"):
            assert int(got[k][0]) == nwg * (T - 2), "%s: arrivals %d" % (k, int(got[k][0]))
            assert int(got[k][1]) == 0, "%s: a persistent loop timed out" % k
            continue
        a, b = got[k], ref[k]
        if not torch.equal(a, b):
            d = (a != b)
            bad.append("%s: %d of %d differ (first at flat %d)" % (
                k, int(d.sum()), a.numel(), int(d.reshape(-1).nonzero()[0])))
    assert not bad, "; ".join(bad)
    assert n > 0 and float(ref["grad"].abs().max()) > 0


@pytest.mark.parametrize("H,T,B,bidir,seed,load", [(1024, 10, 16, True, 21, False),
                                                   (1024, 7, 16, True, 22, True),
                                                   (512, 15, 12, False, 23, False),
                                                   (768, 8, 10, True, 24, False)])
def test_lstm_persist_fp32_bit_identical_to_steps(H, T, B, bidir, seed, load):
    """The exact-fp32 step mode's loops (C4 fp32: 4 x 1024 bidirectional, B = 16; f32_fwd_loop /
    f32_bwd_loop) against the per-step fp32 launches: the per-step 8-wave kernels' strips and chain
    order, red_sum's and rnn_bwd_epi's orders — every tensor bit-identical."""
    ref, forms_ref = _run(H, T, B, seed, False, f32=True, bidir=bidir)
    got, forms = _run(H, T, B, seed, True, load, f32=True, bidir=bidir)
    assert all("persistent" not in f for f in forms_ref.values()), forms_ref
    assert all(f.startswith("persistent grid-synchronised") and "/" not in f for f in forms.values()), forms
    print("fp32 H %d T %d B %d bidir %s forms %s" % (H, T, B, bidir, forms))
    B2 = 2 * B if bidir else B
    nwg = (H // 16) * ((B2 + 7) // 8)         # the BPTT's column blocks x 8-row blocks (f32_bwd_lds)
    bad = []
    for k in ref:
        if k.endswith(".timeout"):
            assert int(got[k][0]) == nwg * (T - 2), "%s: arrivals %d" % (k, int(got[k][0]))
            assert int(got[k][1]) == 0, "%s: a persistent loop timed out" % k
            continue
        a, b = got[k], ref[k]
        if not torch.equal(a, b):
            d = (a != b)
            bad.append("%s: %d of %d differ (first at flat %d, max %.3g)" % (
                k, int(d.sum()), a.numel(), int(d.reshape(-1).nonzero()[0]),
                float((a.double() - b.double()).abs().max())))
    assert not bad, "; ".join(bad)
    assert float(ref["grad"].abs().max()) > 0


def test_lstm_persist_repeatable():
    """Three back-to-back runs of the same persistent loops: identical outputs (the step counters
    are re-zeroed per launch; a stale counter would let a workgroup run ahead)."""
    outs = [_run(512, 17, 12, 7, True)[0] for _ in range(3)]
    for o in outs[1:]:
        for k in o:
            assert torch.equal(o[k], outs[0][k]), k


def _run_ligru(H, T, B, seed, grid, hcgs, load=False):
    import pkc.neural_networks as NN
    from pkc import _lib as L
    from cases import LIGRU_DEF
    from test_gpu_rnn import dx0
    os.environ["PKC_RNN_LIGRU_GRID"] = "1" if grid else "0"
    try:
        opts = dict(LIGRU_DEF, ligru_lay="%d,%d" % (H, H), ligru_drop="0.2,0.2")
        if hcgs:                       # C3's 16x HCGS masks on W and U
            opts.update(ligru_hcgs="True", hcgsx_block="32,2", hcgsx_sparse="75,75",
                        hcgsh_block="32,2", hcgsh_sparse="75,75")
        cp = configparser.ConfigParser()
        cp["s"] = {k: str(v) for k, v in opts.items()}
        torch.manual_seed(seed)
        np.random.seed(seed)
        F = 40
        net = NN.liGRU(cp["s"], F).to("cuda").train()
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(T, B, F, generator=g).cuda()
        dy = torch.randn(T, B, net.out_dim, generator=g).cuda()
        side = None
        if load:
            side = torch.cuda.Stream()
            a = torch.randn(4096, 4096, device="cuda")
            with torch.cuda.stream(side):
                for _ in range(12):
                    a = torch.tanh(a @ a * 1e-3)
        eng, node, y = _block(net, x, dy, L.PREC_FP32)
        if side is not None:
            side.synchronize()
        out = {"y": y.cpu(), "dx0": dx0(eng, node).cpu(), "grad": eng.gflat.cpu()}
        for li, lb in enumerate(node.lbuf):
            n = 2 * B * H
            out["%d.hs" % li] = lb["hs"][:(T + 1) * n].cpu()
            for k in ("gates", "dgates"):
                out["%d.%s" % (li, k)] = lb[k][:2 * T * n].cpu()
            out["%d.timeout" % li] = _ctr_words(lb["rwork"], n)
        return out, eng.rec_forms()
    finally:
        os.environ.pop("PKC_RNN_LIGRU_GRID", None)


@pytest.mark.parametrize("H,T,B,hcgs,seed,load", [(550, 40, 8, True, 21, False),
                                                  (550, 23, 8, True, 22, True),
                                                  (96, 17, 5, False, 23, False),
                                                  (768, 9, 8, False, 24, False),
                                                  (24, 30, 4, False, 25, False),
                                                  (24, 2, 4, False, 26, False)])
def test_ligru_fp32_grid_loops_match_steps(H, T, B, hcgs, seed, load):
    """The exact-fp32 liGRU step mode (C3 fp32: 4 x 550 bidirectional, B = 8, HCGS U) in the
    grid-synchronised loops against the per-step launches on the same layer and inputs: the same
    fp32 products summed in another order (the dense U's masked zeros included), so every tensor
    within 2e-5 of its largest element over T = 40 steps of two layers (measured values printed);
    with a dense U and H <= 256 (the per-step launches' 4-wave strips, summed in their order)
    every tensor is bit-identical; the loops' timeout word stays zero and the last launch saw
    every arrival."""
    ref, forms_ref = _run_ligru(H, T, B, seed, False, hcgs)
    got, forms = _run_ligru(H, T, B, seed, True, hcgs, load)
    assert all("grid" not in f for f in forms_ref.values()), forms_ref
    assert all(f.startswith("persistent grid-synchronised") for f in forms.values()), forms
    rep, bad = [], []
    exact = H <= 256 and not hcgs
    nwg = (H + 15) // 16 * (2 if 2 * B > 8 else 1)     # > 8 rows: two row blocks per column block
    for k in ref:
        if k.endswith(".timeout"):
            assert int(got[k][0]) == nwg * (T - 2), "%s: arrivals %d" % (k, int(got[k][0]))
            assert int(got[k][1]) == 0, "%s: a loop timed out" % k
            continue
        a, b = got[k].double(), ref[k].double()
        err = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)
        rep.append("%s %.2e" % (k, err))
        if err > 2e-5 or (exact and not torch.equal(got[k], ref[k])):
            bad.append("%s %.3g" % (k, err))
    print("liGRU fp32 H %d T %d B %d: %s" % (H, T, B, ", ".join(rep)))
    assert not bad, bad
