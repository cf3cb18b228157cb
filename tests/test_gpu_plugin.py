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


def test_plugin_mlp_pattern_trains_like_reference():
    """Pattern masks through the plug-in (if_pattern, neural_networks.py:263-272, 339-361): the
    8x8/k4/n16 pattern_file set on the HCGS body and cd head, the masks computed at the first layer
    call from the weights and multiplied in once per layer call (pattern^L); 3 steps of the
    reference loop vs the oracle, posteriors <= 1e-4 relative.  The masks the plug-in computed are
    the oracle's, element for element."""
    import os

    from conftest import GOLDEN
    cfg = build_mlp_config("hcgs")
    pset = np.load(os.path.join(GOLDEN, "quant.npz"), allow_pickle=False)["pattern_set"].reshape(16, 8, 8)
    for sec in ("architecture1", "architecture2"):
        cfg[sec].update(if_pattern="True", pattern_mode="pattern", pattern_shape="8,8",
                        pattern_nnz="4,4", pattern_num="16,16")
    F, M = 40, 64
    nets, onets, opts = _nets(cfg, [("architecture1", F), ("architecture2", None),
                                    ("architecture3", None)], {})
    for k in nets:
        if nets[k].if_pattern:
            nets[k].pattern_kernels = pset
            onets[k].pattern_kernels = pset
    rs = np.random.RandomState(6)
    batches = []
    for rows in (M, M, M):
        x = rs.randn(rows, F).astype(np.float32)
        lab = np.stack([rs.randint(0, 96, rows), rs.randint(0, 8, rows)], 1).astype(np.float32)
        batches.append((torch.from_numpy(np.concatenate([x, lab], 1)), 0))
    _run(cfg, nets, onets, opts, {k: False for k in nets}, {"fmllr": (0, F)},
         {"lab_cd": F, "lab_mono": F + 1}, batches)
    for k in ("MLP_layers1", "MLP_layers2"):
        assert len(nets[k].pattern_mask) == len(onets[k].pattern_masks) > 0
        for pm, opm in zip(nets[k].pattern_mask, onets[k].pattern_masks):
            np.testing.assert_array_equal(pm.cpu().numpy(), opm.numpy())


def test_plugin_input_quant_rebinds_caller_tensor():
    """lstm_quant_inp on layer 0: the four gate projections quantise the caller's x in place in
    turn (quantized_modules.py:216-217), and after net(x) the caller's tensor holds the last
    version — as the oracle's x after onet(x).  16-bit grid of max|x| / 2^15; the values are the
    same fp32 sequence on both sides (bit-exact expected, one quantum allowed)."""
    from test_gpu_configs import build_pair
    nets, onets, _, _, _ = build_pair("c5", drop="0.0")
    net, onet = nets["rnn"].to(DEV).train(), onets["rnn"].train()
    rs = np.random.RandomState(4)
    x0 = torch.from_numpy((rs.randn(7, 3, 440) * 1.7).astype(np.float32))
    xg, xc = x0.clone().to(DEV), x0.clone()
    yg = net(xg)
    yo = onet(xc)
    assert not torch.equal(xc, x0)                  # the oracle rewrote its input
    q = float(x0.abs().max()) / 2 ** 15
    d = (xg.detach().cpu() - xc).abs().max().item()
    assert d <= q * 1.0001, "caller tensor vs oracle's in-place version: %.3g (quantum %.3g)" % (d, q)
    # an input element one quantum off (a last-bit difference in front of a ceil, counted here)
    # moves the outputs by ~quantum x |W|: compared against the output scale
    nq = int((xg.detach().cpu() != xc).sum().item())
    err = (yg.detach().cpu() - yo.detach()).abs().max().item() / yo.detach().abs().max().item()
    print("input elements one quantum off the oracle's: %d of %d; output err %.3g" % (nq, xc.numel(), err))
    assert nq <= max(1, xc.numel() // 1000), nq
    # (every step re-quantises h_{t-1} to the same 16-bit grid inside the LSTM, so a one-quantum
    # move — 2^-15 of max|h| — can happen there too, at any of the 3 layers' 7 steps)
    assert err < 1e-3, "output err %.3g with %d input elements one quantum off" % (err, nq)
    yg.sum().backward()                             # the rebinding does not upset autograd


def test_plugin_c5_lstm_pattern_quant_trains_like_reference():
    """BASELINE C5 through the architecture plug-in: LSTM 3x512 + Pattern b08b08_k04_n16 (the
    pattern_file set) + 8-bit weights + 16-bit input fake-quantisation of the arch's own input
    (rebinding the caller's x, quantized_modules.py:216-217), heads 1928 cd + 48 mono, B = 12,
    trained 3 steps by the reference loop (forward_model, NLLLoss, backward, torch.optim RMSprop)
    vs the oracle on the CPU, the oracle re-started from the plug-in's state (parameters, BN
    statistics, RMSprop state) before every step.  The 16-bit grid moves an element by one quantum
    where a last-bit difference sits in front of a ceil: posteriors 1e-3 relative, gradients 1e-3
    of the tensor's largest; each step's updates elementwise within 1e-4 of the tensor's scale
    except counted outliers: <= 0.2 % of a weight on another 8-bit grid point (tests/quantcheck.py),
    and RMSprop's amplification of the gradients' difference near g = 0 (each <= 2 x 4.48 lr, at
    most 5 % of a tensor, the counts printed) — the weights must differ by exactly their
    gradients' RMSprop updates (fp64 recomputation from each side's gradient, 1e-6 of the scale)."""
    from flipcheck import assert_counted, resync, step_outliers
    from oracle import nets as ON
    from oracle import run as OR
    from pkc.engine import torch_optimizer
    from quantcheck import assert_few_flips, rmsprop_quanta
    from test_gpu_configs import build_pair
    nets, onets, opts, model, B = build_pair("c5", drop="0.0")
    for k in nets:
        nets[k].to(DEV).train()
        onets[k].train()
    F = 440
    lines = OR.parse_model(model)
    popt = {k: torch_optimizer(nets[k].parameters(), opts[k]) for k in nets}
    oopt = {k: ON.make_optimizer(onets[k].parameters(), opts[k]) for k in onets}
    seq = {"rnn": True, "head": False, "mono": False}
    rs = np.random.RandomState(8)
    lr = float(opts["rnn"]["arch_lr"])
    flips, report, notes = {}, {}, {}
    for step, T in enumerate((10, 14, 9)):
        resync(nets, onets, {k: popt[k].state_dict() for k in nets} if step else None, oopt)
        # each parameter's RMSprop square_avg before the step (the update check below)
        pre = {}
        for k in nets:
            st = popt[k].state_dict()["state"]
            names = [nm for nm, _ in nets[k].named_parameters()]
            pre[k] = {names[i]: d["square_avg"].detach().cpu().clone() for i, d in st.items()
                      if "square_avg" in d}
        x = rs.randn(T, B, F).astype(np.float32)
        lab = np.stack([rs.randint(0, 1928, (T, B)), rs.randint(0, 48, (T, B))], 2).astype(np.float32)
        inp = torch.from_numpy(np.concatenate([x, lab], 2))
        outs_p = OR.train_step(lines, nets, popt, seq, {"fea": (0, F)},
                               {"lab_cd": F, "lab_mono": F + 1}, inp.to(DEV), T, B)
        outs_o = OR.train_step(lines, onets, oopt, seq, {"fea": (0, F)},
                               {"lab_cd": F, "lab_mono": F + 1}, inp, T, B)
        np.testing.assert_allclose(outs_p["loss_final"].item(), outs_o["loss_final"].item(), rtol=1e-4)
        post, ref = outs_p["o2"].detach().cpu(), outs_o["o2"].detach()
        rel = ((post - ref).abs() / ref.abs().clamp_min(1e-3)).max().item()
        print("c5 plug-in step %d posterior max rel err %.3g" % (step, rel))
        assert rel < 1e-3, "step %d posterior rel err %.3g" % (step, rel)
        for k in nets:
            sd_o = onets[k].state_dict()
            lrk = float(opts[k]["arch_lr"])
            for pname, v in nets[k].state_dict().items():
                if pname.endswith("num_batches_tracked"):
                    assert int(v.item()) == int(sd_o[pname].item())
                    continue
                r = sd_o[pname].double()
                tag = "%d %s/%s" % (step, k, pname)
                if k == "rnn" and pname.endswith("weight") and v.dim() == 2:
                    flips[tag] = assert_few_flips(v.cpu().numpy(), r.numpy(), tag, 2e-3,
                                                  max_quanta=rmsprop_quanta(lr, 1) + 1)
                scale = max(float(r.abs().max()), lrk)
                n, dmax, _ = step_outliers(v.cpu(), r, 1e-4, scale)
                report[tag] = n
                pp = dict(nets[k].named_parameters()).get(pname)
                po = dict(onets[k].named_parameters()).get(pname)
                if pp is None or pp.grad is None or po.grad is None:
                    # buffers (forward-only statistics) and parameters without a gradient: tight
                    assert_counted(tag, n, r.numel(), 0.0, dmax, 1e-4 * scale + 1e-7)
                    continue
                gp = pp.grad.detach().cpu().double().reshape(-1)
                go = po.grad.double().reshape(-1)
                # the gradients: one-quantum moves of the 16-bit grids (input and h_{t-1}) move a
                # gradient element by ~2^-15 of its terms; held to 1e-3 of the tensor's largest
                gn = float((gp - go).abs().max())
                assert gn <= 1e-3 * float(go.abs().max()) + 1e-12, "%s grad diff %.3g of max %.3g" % (
                    tag, gn, float(go.abs().max()))
                # the updates: RMSprop (torch.optim, alpha / eps of the config, no momentum) from
                # the common start, recomputed in fp64 from each side's own gradient — the weights
                # must differ by exactly what the gradients' difference gives through the
                # normaliser g / (sqrt(alpha s + (1 - alpha) g^2) + eps), which amplifies the noise
                # of a near-zero gradient (those elements are counted, not bounded by a ratchet)
                o = opts[k]
                al, eps = float(o["opt_alpha"]), float(o["opt_eps"])
                s0 = pre[k].get(pname)
                s0 = torch.zeros_like(go) if s0 is None else s0.double().reshape(-1)

                def upd(g):
                    return lrk * g / ((al * s0 + (1 - al) * g * g).sqrt() + eps)
                dw = (v.cpu().double() - r).reshape(-1)
                resid = float((dw + (upd(gp) - upd(go))).abs().max())
                notes[tag] = n
                assert resid <= 1e-6 * scale, "%s: weights differ by %.3g beyond their gradients' " \
                    "RMSprop updates (%d update outliers)" % (tag, resid, n)
                # the count of such moves is the share of gradient elements within the 16-bit
                # grids' noise of zero, where RMSprop's first-step normaliser turns the sign of the
                # noise into a full +-4.47 lr step (measured: up to 2.2 % of the heads' weights,
                # 0.6-1 % of the LSTM matrices, 3.3 % of a 512-wide BatchNorm beta): bounded at
                # 5 % of the tensor (at least 32 elements), each step at most 2 x 4.48 lr.  Counted
                # are the moves of at least 5 % of an lr step (from step 1 on the normaliser holds
                # the first step's g^2, and sub-percent moves of up to ~9 % of a BatchNorm beta's
                # elements are the gradients' own 1e-3 noise, already held by the residual check)
                n = int(((dw.abs() > 1e-4 * scale + 1e-7) & (dw.abs() > 0.05 * lrk)).sum())
                assert_counted(tag + " RMSprop-amplified updates", n, r.numel(),
                               max(0.05, 32.0 / r.numel()), dmax, 2 * 4.48 * lrk + 1e-7,
                               "(%d of %d)" % (n, r.numel()))
    for k in nets["rnn"].pattern_mask:
        assert len(nets["rnn"].pattern_mask[k]) == 3
    print("c5 plug-in 8-bit grid flips per step", {a: b for a, b in flips.items() if b})
    print("c5 plug-in RMSprop-amplified update outliers per step", {a: b for a, b in notes.items() if b})
