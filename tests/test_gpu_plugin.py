"""The architecture plug-in contract: pkc.neural_networks classes trained by the
reference's own loop — utils.forward_model's ``net(x)`` calls, NLLLoss, ``loss.backward()`` and
torch.optim (utils.py:1884-2050, core.py:216-232; restated in oracle/run.py) — with their
forward/backward on the pkc HIP kernels (pkc.plugin), against the oracle nets run by the same loop
on the CPU.  3 steps; posteriors within 1e-4 relative (north_star tolerance), loss within 1e-4,
parameters after the 3 optimizer steps within 1e-3 of their norm (RMSprop's first steps divide
by sqrt of tiny second moments, which amplifies fp32 summation-order differences)."""
import numpy as np
import pytest
import torch

from cases import build_mlp_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _nets(cfg, secs, classes):
    import pkc.neural_networks as NN
    from oracle import nets as ON
    nets, onets, opts = {}, {}, {}
    for sec, inp in secs:
        o = cfg[sec]
        name = o["arch_name"]
        if inp is None:
            inp = next(iter(nets.values())).out_dim
        torch.manual_seed(3)
        np.random.seed(3)
        cls = classes.get(sec, "MLP")
        nets[name] = getattr(NN, cls)(o, inp)
        onets[name] = getattr(ON, cls)(o, inp)
        onets[name].load_state_dict(nets[name].state_dict())
        opts[name] = o
    for k in nets:
        nets[k].to(DEV).train()
        onets[k].train()
    return nets, onets, opts


def _compare_state(nets, onets, tol=1e-3):
    for k in nets:
        for name, v in nets[k].state_dict().items():
            if name.endswith("num_batches_tracked"):
                assert int(v.item()) == int(onets[k].state_dict()[name].item()), (k, name)
                continue
            ref = onets[k].state_dict()[name].double()
            d = (v.cpu().double() - ref).norm().item()
            assert d <= tol * ref.norm().item() + 1e-7, "%s %s %.3g" % (k, name, d)


def _run(cfg, nets, onets, opts, seq, fea_cols, lab_cols, batches, T=0, B=0, out="out_dnn2"):
    from oracle import nets as ON
    from oracle import run as OR
    from pkc.engine import torch_optimizer
    lines = OR.parse_model(cfg["model"]["model"])
    popt = {k: torch_optimizer(nets[k].parameters(), opts[k]) for k in nets}
    oopt = {k: ON.make_optimizer(onets[k].parameters(), opts[k]) for k in onets}
    for step, (inp, T_) in enumerate(batches):
        outs_p = OR.train_step(lines, nets, popt, seq, fea_cols, lab_cols, inp.to(DEV), T_, B)
        outs_o = OR.train_step(lines, onets, oopt, seq, fea_cols, lab_cols, inp, T_, B)
        np.testing.assert_allclose(outs_p["loss_final"].item(), outs_o["loss_final"].item(),
                                   rtol=1e-4)
        post, ref = outs_p[out].detach().cpu(), outs_o[out].detach()
        assert post.shape == ref.shape
        rel = ((post - ref).abs() / ref.abs().clamp_min(1e-3)).max().item()
        assert rel < 1e-4, "step %d posterior rel err %.3g" % (step, rel)
    _compare_state(nets, onets)


MLP_VARIANTS = {
    "plain": {},
    "hcgs": None,        # build_mlp_config("hcgs")
    "ln": None,
    "quant_w": dict(mlp_quant="True"),          # weight fake-quant (QuantizeLinear, STE)
    "prune": dict(mlp_prune="True", mlp_prune_perc="60,40"),
    "drop_ln_heads": "heads",
}


@pytest.mark.parametrize("variant", list(MLP_VARIANTS))
def test_plugin_mlp_trains_like_reference(variant):
    base = variant if variant in ("hcgs", "ln") else "plain"
    cfg = build_mlp_config(base)
    extra = MLP_VARIANTS[variant]
    if isinstance(extra, dict):
        cfg["architecture1"].update(extra)
        if variant == "quant_w":
            cfg["architecture2"].update(extra)
    elif extra == "heads":         # LayerNorm'd softmax head + tanh/linear body
        cfg["architecture1"].update(dnn_act="tanh,linear")
        cfg["architecture2"].update(dnn_use_laynorm="True")
    F, M = 40, 64
    nets, onets, opts = _nets(cfg, [("architecture1", F), ("architecture2", None),
                                    ("architecture3", None)], {})
    rs = np.random.RandomState(5)
    batches = []
    for rows in (M, M, 48):        # the last batch is smaller (a different row count, same engine)
        x = rs.randn(rows, F).astype(np.float32)
        lab = np.stack([rs.randint(0, 96, rows), rs.randint(0, 8, rows)], 1).astype(np.float32)
        batches.append((torch.from_numpy(np.concatenate([x, lab], 1)), 0))
    _run(cfg, nets, onets, opts, {k: False for k in nets}, {"fmllr": (0, F)},
         {"lab_cd": F, "lab_mono": F + 1}, batches)


SEQ_BODIES = {"ligru": "liGRU", "lstm": "LSTM", "lstm_bidir": "LSTM", "ligru_hcgs": "liGRU",
              "gru": "GRU", "mingru": "minimalGRU", "rnn": "RNN", "lstm_ln": "LSTM",
              "lstm_quant_w": "LSTM", "lstm_prune": "LSTM", "ligru_inpnorm": "liGRU"}


@pytest.mark.parametrize("body", list(SEQ_BODIES))
def test_plugin_seq_trains_like_reference(body):
    from test_gpu_seq import make_cfg
    cfg = make_cfg("lstm" if body == "lstm_quant_w" else body)
    a1 = cfg["a1"]
    for k in list(a1.keys()):
        if k.endswith("_drop"):      # the oracle draws torch dropout masks: no dropout here
            a1[k] = ",".join("0.0" for _ in a1[k].split(","))
    if body == "lstm_quant_w":
        a1.update(lstm_quant="True", lstm_quant_inp="False")
    F, B = 20, 4
    nets, onets, opts = _nets(cfg, [("a1", F), ("a2", None), ("a3", None)], {"a1": SEQ_BODIES[body]})
    rs = np.random.RandomState(1)
    batches = []
    for T in (9, 13, 6):             # 13 outgrows the first engine (rebuilt), 6 reuses it
        x = rs.randn(T, B, F).astype(np.float32)
        lab = np.stack([rs.randint(0, 64, (T, B)), rs.randint(0, 8, (T, B))], 2).astype(np.float32)
        batches.append((torch.from_numpy(np.concatenate([x, lab], 2)), T))
    from oracle import run as OR
    lines = OR.parse_model(cfg["model"]["model"])
    assert lines[0][1] == "compute"
    _run(cfg, nets, onets, opts, {"rnn": True, "head": False, "mono": False}, {"fea": (0, F)},
         {"lab_cd": F, "lab_mono": F + 1}, batches, B=B, out="o2")


def test_plugin_shapes_eval_and_guards():
    """(T, B, F) -> (T, B, out_dim); eval forward (running BatchNorm statistics) matches the
    oracle's eval forward; a second training forward before the backward is refused."""
    from test_gpu_seq import make_cfg
    cfg = make_cfg("ligru")
    a1 = cfg["a1"]
    a1["ligru_drop"] = "0.0,0.0"
    nets, onets, _ = _nets(cfg, [("a1", 20)], {"a1": "liGRU"})
    net, onet = nets["rnn"], onets["rnn"]
    x = torch.randn(7, 3, 20)
    net.eval()
    onet.eval()
    with torch.no_grad():
        ye = net(x.to(DEV)).cpu()
        yo = onet(x)
    assert ye.shape == (7, 3, net.out_dim)
    torch.testing.assert_close(ye, yo, rtol=1e-4, atol=1e-5)
    net.train()
    y = net(x.to(DEV))
    assert y.shape == (7, 3, net.out_dim) and y.requires_grad
    net(x.to(DEV))                   # overwrites the state the first output's backward needs
    with pytest.raises(RuntimeError):
        y.sum().backward()
    with pytest.raises(ValueError):
        net(x[0].to(DEV))
