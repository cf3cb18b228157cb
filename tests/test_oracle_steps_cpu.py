"""oracle/steps.py (one recurrent step from a given state, vectorised over t) pinned against the
autograd of oracle.nets' reference loops (liGRU neural_networks.py:1576-1584, LSTM :1087-1092),
which tests/test_oracle_golden.py pins to the reference's own outputs: run sequentially through
its own states, the per-step restatement must reproduce the loop's outputs, its dL/dU and dL/dx."""
import configparser

import numpy as np
import pytest
import torch

from cases import LIGRU_DEF, LSTM_DEF


def _net(kind, bidir, H=12, F=8):
    from oracle import nets as ON
    cfg = configparser.ConfigParser()
    if kind == "ligru":
        cfg["a"] = dict(LIGRU_DEF, ligru_lay=str(H), ligru_drop="0.3", ligru_use_batchnorm="False",
                        ligru_use_laynorm="False", ligru_bidir=str(bidir), ligru_act="relu")
        net = ON.liGRU(cfg["a"], F)
    else:
        # the reference LSTM builds W/U only with BN or LN (:681-791); BN is a separate node
        # upstream of the steps, so its output (wpre) is read back from the forward below
        cfg["a"] = dict(LSTM_DEF, lstm_lay=str(H), lstm_drop="0.3", lstm_bidir=str(bidir),
                        lstm_act="tanh")
        net = ON.LSTM(cfg["a"], F)
    return net.double()


@pytest.mark.parametrize("kind", ["ligru", "lstm"])
@pytest.mark.parametrize("bidir", [False, True])
def test_steps_match_reference_loop_autograd(kind, bidir):
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)      # (the loops' h_init = torch.zeros(...))
    try:
        _check(kind, bidir)
    finally:
        torch.set_default_dtype(old)


def _check(kind, bidir):
    from oracle import steps as S
    torch.manual_seed(5)
    H, F, T, B = 12, 8, 7, 3
    net = _net(kind, bidir, H, F)
    net.train()
    R = 2 * B if bidir else B
    mask = (torch.rand(R, H) > 0.3).double()
    x = torch.randn(T, B, F, dtype=torch.float64, requires_grad=True)
    # capture the projections the loop adds (post-BN for the LSTM) with forward hooks
    pre = {}
    if kind == "ligru":
        names = [("wz", net.wz[0]), ("wh", net.wh[0])]
        Us = [net.uz[0], net.uh[0]]
    else:
        names = [("bn_w%sx" % g, getattr(net, "bn_w%sx" % g)[0]) for g in "fioc"]
        Us = [getattr(net, "u%sh" % g)[0] for g in "fioc"]
    hooks = [m.register_forward_hook(lambda m_, i_, o_, k=k: pre.__setitem__(k, o_))
             for k, m in names]
    y = net(x, drop_masks=[mask])
    for h_ in hooks:
        h_.remove()
    dy = torch.randn_like(y)
    (y * dy).sum().backward()
    wpre = [pre[k].detach().reshape(T, R, H) for k, _ in names]
    U = [u.weight.detach() for u in Us]
    # sequential run of the one-step restatement through its own states
    h = torch.zeros(R, H, dtype=torch.float64)
    c = torch.zeros(R, H, dtype=torch.float64)
    hs, cs, gates = [h], [c], []
    for t in range(T):
        w1 = [w[t:t + 1] for w in wpre]
        if kind == "ligru":
            z, hcr, hn = S.steps_ligru_fwd(h[None], h[None], U, w1, mask, "relu")
            gates.append((z[0], hcr[0]))
        else:
            f, i, o, cc, cn, hn = S.steps_lstm_fwd(h[None], h[None], c[None], U, w1, mask, "tanh")
            gates.append((f[0], i[0], o[0], cc[0]))
            c = cn[0]
            cs.append(c)
        h = hn[0]
        hs.append(h)
    hs_t = torch.stack(hs)
    yp = hs_t[1:]
    yp = torch.cat([yp[:, :B], torch.flip(yp[:, B:], [0])], 2) if bidir else yp
    np.testing.assert_allclose(yp.numpy(), y.detach().numpy(), rtol=1e-12, atol=1e-12)
    dh = S.out_grad_proc_time(dy, B, H, bidir)
    G = torch.stack
    if kind == "ligru":
        z = G([g[0] for g in gates])
        hcr = G([g[1] for g in gates])
        # the BPTT products read the gate gradients the function itself produces: iterate to the
        # fixed point (T passes make the sequential chain exact)
        dg = [torch.zeros(T, R, H, dtype=torch.float64) for _ in range(2)]
        for _ in range(T + 1):
            dz, da, _ = S.steps_ligru_bwd(dh, dg, U, z, hcr, hs_t[:-1], mask, "relu")
            dg = [dz, da]
    else:
        f, i, o, cc = (G([g[k] for g in gates]) for k in range(4))
        cst = torch.stack(cs)
        dg = [torch.zeros(T, R, H, dtype=torch.float64) for _ in range(4)]
        for _ in range(T + 1):
            dg = S.steps_lstm_bwd(dh, dg, U, f, i, o, cc, cst[1:], cst[:-1], mask, "tanh")
    for q, u in enumerate(Us):
        np.testing.assert_allclose(S.weight_grad(dg[q], hs_t[:-1]).numpy(), u.weight.grad.numpy(),
                                   rtol=1e-10, atol=1e-12)
    # dL/dx through the projections (LSTM: through BatchNorm too; liGRU: Linear with bias)
    if kind == "ligru":
        W = [net.wz[0].weight.detach(), net.wh[0].weight.detach()]
        dx = sum(S.pre_grad_input_time(dg[q], B, bidir) @ W[q] for q in range(2))
        np.testing.assert_allclose(dx.numpy(), x.grad.numpy(), rtol=1e-10, atol=1e-12)
