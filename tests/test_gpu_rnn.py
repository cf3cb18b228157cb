"""GPU parity of the recurrent layers (pkc_rnn_fwd / pkc_rnn_bwd + gate matmuls + BN) against the
reference's own golden vectors (tests/golden/rnn.npz: y, dL/dx and every parameter gradient of
sum(y * r) for random r, plus the post-forward BatchNorm running statistics)."""
import configparser
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from cases import GRU_CASES, PLAIN_CASES, LIGRU_DEF, LSTM_DEF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def section(d):
    cp = configparser.ConfigParser()
    cp["s"] = {k: str(v) for k, v in d.items()}
    return cp["s"]


def run_block(net, x, dy, drop_in=None):
    """Forward + backward of one recurrent architecture through the engine's node kernels."""
    from pkc.engine import Engine
    T, B, F = x.shape
    eng = Engine({"rnn": net}, {"rnn": {"arch_opt": "sgd", "arch_lr": "0"}},
                 [["out", "compute", "rnn", "fea"]], {"fea": (0, F)}, [], batch=B, max_len=T,
                 train=False, rnn_drop_in=drop_in)
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


def dx0(eng, node):
    from pkc.engine import _splits, MAX_SPLITS
    lb = node.lbuf[0]
    M, K, H = eng.M, lb["K"], lb["H"]
    sx = _splits(M, K, H, MAX_SPLITS)
    return lb["dx"][:node.G * sx * M * K].view(node.G * sx, M, K).sum(0)


PATTERN = dict(if_pattern="True", pattern_mode="pattern", pattern_shape="8,8", pattern_nnz="4,4",
               pattern_num="16,16")
CASES = [("ligru_bidir", "liGRU", LIGRU_DEF, 7, 3, 20, 21),
         ("ligru_uni_ln", "liGRU", dict(LIGRU_DEF, ligru_bidir="False", ligru_act="tanh,relu",
                                        ligru_orthinit="False", ligru_use_laynorm="True,False"),
          6, 2, 12, 22),
         ("lstm", "LSTM", LSTM_DEF, 7, 3, 20, 23),
         ("lstm_hcgs_quant", "LSTM", dict(LSTM_DEF, lstm_hcgs="True", lstm_quant="True",
                                          lstm_quant_inp="True"), 7, 3, 24, 24),
         ("lstm_pattern", "LSTM", dict(LSTM_DEF, **PATTERN), 5, 2, 24, 25)] + \
        [(tag, "GRU", opts, T, B, F, seed) for tag, opts, T, B, F, seed in GRU_CASES] + PLAIN_CASES


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_recurrent_layer_matches_reference(case):
    import pkc.neural_networks as NN
    tag, cls, opts, T, B, F, seed = case
    g = np.load(os.path.join(GOLDEN, "gru.npz" if cls in ("GRU", "minimalGRU", "RNN") else "rnn.npz"),
                allow_pickle=False)
    torch.manual_seed(seed)
    np.random.seed(seed)
    net = getattr(NN, cls)(section(opts), F)
    if tag == "lstm_pattern":
        net.pattern_kernels = np.load(os.path.join(GOLDEN, "quant.npz"),
                                      allow_pickle=False)["pattern_set"].reshape(16, 8, 8)
    # init parity is pinned bit-exactly on the build host (test_host_cpu); the box's LAPACK
    # rounds the orthogonal init's QR differently in the last bit, so start from the golden init
    sd = {}
    for k, v in net.state_dict().items():
        ref = torch.from_numpy(g[tag + "/init/" + k])
        np.testing.assert_allclose(v.numpy(), ref.numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
        sd[k] = ref
    net.load_state_dict(sd)
    net.to(DEV).train()
    x = torch.from_numpy(g[tag + "/x"]).to(DEV)
    r = torch.from_numpy(g[tag + "/r"]).to(DEV)
    eng, node, y = run_block(net, x, r)
    np.testing.assert_allclose(y.cpu().numpy(), g[tag + "/y"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(dx0(eng, node).cpu().numpy().reshape(T, B, F), g[tag + "/dx"],
                               rtol=1e-3, atol=1e-5)
    grads = {}
    for li, lb in enumerate(node.lbuf):
        if node.layers[li].get("ln"):        # LayerNorm of h
            H = lb["H"]
            own = lb["dgamma_ln"][0] is not None
            grads["ln.%d.gamma" % li] = lb["dgamma_ln"][0] if own else lb["ln_pg"][:H]
            grads["ln.%d.beta" % li] = lb["dbeta_ln"][0] if own else lb["ln_pg"][H:2 * H]
        for gi, gate in enumerate(net.GATES):
            if cls in ("liGRU", "GRU", "minimalGRU", "RNN"):
                if lb["db"][gi] is not None:
                    grads["w%s.%d.bias" % (gate, li)] = lb["db"][gi]
                grads["w%s.%d.weight" % (gate, li)] = lb["dW"][gi]
                grads["u%s.%d.weight" % (gate, li)] = lb["dU"][gi]
                if node.layers[li]["bn"]:
                    grads["bn_w%s.%d.weight" % (gate, li)] = lb["dgamma"][gi]
                    grads["bn_w%s.%d.bias" % (gate, li)] = lb["dbeta"][gi]
            else:
                grads["w%sx.%d.weight" % (gate, li)] = lb["dW"][gi]
                grads["u%sh.%d.weight" % (gate, li)] = lb["dU"][gi]
                grads["bn_w%sx.%d.weight" % (gate, li)] = lb["dgamma"][gi]
                grads["bn_w%sx.%d.bias" % (gate, li)] = lb["dbeta"][gi]
    for k, v in grads.items():
        ref = g[tag + "/grad/" + k]
        # with 16-bit input quantisation an fp32 last-bit difference can flip one element of a
        # quantised operand by one grid step (max|x| / 2^15); allow that much in the gradient sums
        atol = 1e-4 if "quant" in tag else 1e-5
        np.testing.assert_allclose(v.cpu().numpy(), ref, rtol=1e-3, atol=atol, err_msg=k)
    for k, v in net.state_dict().items():
        if "running" in k or k.endswith(".weight") and k[0] in "wu":
            # BN statistics, and W / U after the forward's in-place masking + clamping
            np.testing.assert_allclose(v.cpu().numpy(), g[tag + "/post/" + k], rtol=1e-4, atol=1e-6,
                                       err_msg=k)


SPARSE_CASES = [("ligru_hcgs96", "liGRU", dict(LIGRU_DEF, ligru_lay="96,80", ligru_hcgs="True",
                                               hcgsx_block="32,4", hcgsx_sparse="50,50",
                                               hcgsh_block="32,4", hcgsh_sparse="50,50"), 9, 3, 24),
                ("lstm_hcgs96", "LSTM", dict(LSTM_DEF, lstm_lay="96,64", lstm_hcgs="True",
                                             hcgsx_block="32,4", hcgsx_sparse="50,50",
                                             hcgsh_block="32,4", hcgsh_sparse="50,75"), 8, 2, 24)]


@pytest.mark.parametrize("case", SPARSE_CASES, ids=[c[0] for c in SPARSE_CASES])
def test_block_sparse_u_matches_dense(case):
    """HCGS-masked U: the step kernels that read only the 16-wide blocks holding a nonzero of the
    mask (kmap tables) give the dense kernels' outputs and gradients up to fp32 summation order."""
    import pkc.engine as E
    import pkc.neural_networks as NN
    tag, cls, opts, T, B, F = case
    res = []
    for mode in ("off", "force"):
        torch.manual_seed(7)
        np.random.seed(7)
        net = getattr(NN, cls)(section(opts), F).to(DEV).train()
        g = torch.Generator().manual_seed(3)
        x = torch.randn(T, B, F, generator=g).to(DEV)
        r = torch.randn(T, B, net.out_dim, generator=g).to(DEV)
        old = E.RNN_SPARSE
        E.RNN_SPARSE = mode
        try:
            eng, node, y = run_block(net, x, r)
        finally:
            E.RNN_SPARSE = old
        if mode == "force":
            maps = [lb["kmap_fwd"] for lb in node.lbuf]
            assert all(m is not None for m in maps)
            assert any(bool((m < 0).any()) for m in maps), "no block skipped: the case tests nothing"
        res.append([y, dx0(eng, node)] + [u for lb in node.lbuf for u in lb["dU"]] +
                   [w for lb in node.lbuf for w in lb["dW"]])
    for i, (a, b) in enumerate(zip(*res)):
        # fp32 sums in another order: differences relative to the tensor's scale
        err = (b - a).abs().max().item()
        assert err <= 2e-5 * a.abs().max().item() + 1e-7, "tensor %d: %.3g" % (i, err)
