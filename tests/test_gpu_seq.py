"""Sequence-model training through the pkc engine vs the oracle: liGRU (bidirectional, BN, ReLU,
recurrent dropout) and LSTM bodies with LogSoftmax cd/mono heads, padded batches with the
reference's random left padding (core.py:183-200), three optimizer steps."""
import configparser
import random

import numpy as np
import pytest
import torch

from cases import GRU_DEF, LIGRU_DEF, LSTM_DEF, MINGRU_DEF, RNN_DEF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def make_cfg(body):
    cfg = configparser.ConfigParser()
    opt = dict(arch_opt="rmsprop", arch_lr="0.0016", opt_momentum="0.0", opt_alpha="0.95",
               opt_eps="1e-8", opt_centered="False", opt_weight_decay="0.0", arch_freeze="False")
    if body == "ligru":
        cfg["a1"] = dict(LIGRU_DEF, arch_name="rnn", ligru_lay="32,24", ligru_drop="0.2,0.2", **opt)
    elif body == "lstm_bidir":     # config C4: bidirectional LSTM, liGRU convention
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="True", **opt)
    elif body in ("ligru_hcgs", "ligru_hcgs_sparse"):   # C3: liGRU + the LSTM's HCGS hook
        cfg["a1"] = dict(LIGRU_DEF, arch_name="rnn", ligru_lay="32,24", ligru_drop="0.2,0.2",
                         ligru_hcgs="True", hcgsx_block="8,4", hcgsx_sparse="50,50",
                         hcgsh_block="8,4", hcgsh_sparse="25,50", **opt)
    elif body == "gru":            # GRU (neural_networks.py:1240-1426), bidirectional
        cfg["a1"] = dict(GRU_DEF, arch_name="rnn", gru_lay="32,24", gru_drop="0.2,0.2", **opt)
    elif body == "mingru":
        cfg["a1"] = dict(MINGRU_DEF, arch_name="rnn", minimalgru_lay="32,24",
                         minimalgru_drop="0.2,0.2", **opt)
    elif body == "rnn":
        cfg["a1"] = dict(RNN_DEF, arch_name="rnn", rnn_lay="32,24", rnn_drop="0.2,0.2",
                         rnn_act="tanh,relu", **opt)
    elif body == "lstm_ln":        # LayerNorm of h instead of BN (neural_networks.py:1093-1094)
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", lstm_use_batchnorm="False,True",
                         lstm_use_laynorm="True,True", **opt)
    elif body == "gru_nobn":       # no BN, no LN: the input Linears carry biases
        cfg["a1"] = dict(GRU_DEF, arch_name="rnn", gru_lay="32,24", gru_drop="0.2,0.2",
                         gru_use_batchnorm="False,False", **opt)
    elif body == "lstm_ln_bn":
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", lstm_use_laynorm="True,True", **opt)
    elif body == "gru_ln":
        cfg["a1"] = dict(GRU_DEF, arch_name="rnn", gru_lay="32,24", gru_drop="0.2,0.2",
                         gru_use_laynorm="True,False", gru_use_batchnorm="False,True", **opt)
    # input ln0 / bn0 over the T*B rows, padding included (neural_networks.py:1527-1532).  A
    # BatchNorm after a norm removes every per-column constant the norm adds, so that norm's beta
    # gets a gradient that is 0 up to rounding; RMSprop would blow the rounding up to full-size
    # steps, so those variants train with SGD (the optimizer is not what they test).
    elif body == "ligru_inpnorm":
        cfg["a1"] = dict(LIGRU_DEF, arch_name="rnn", ligru_lay="32,24", ligru_drop="0.2,0.2",
                         ligru_use_laynorm_inp="True", ligru_use_batchnorm_inp="True",
                         **dict(opt, arch_opt="sgd", opt_dampening="0.0", opt_nesterov="False"))
    elif body == "lstm_bninp":     # layer 0 with LN of h instead of the gate BNs
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", lstm_use_batchnorm_inp="True",
                         lstm_use_batchnorm="False,True", lstm_use_laynorm="True,False", **opt)
    elif body == "gru_lninp":
        cfg["a1"] = dict(GRU_DEF, arch_name="rnn", gru_lay="32,24", gru_drop="0.2,0.2",
                         gru_use_laynorm_inp="True", gru_use_batchnorm="False,True", **opt)
    elif body == "mingru_inpnorm":
        cfg["a1"] = dict(MINGRU_DEF, arch_name="rnn", minimalgru_lay="32,24",
                         minimalgru_drop="0.2,0.2", minimalgru_use_laynorm_inp="True",
                         minimalgru_use_batchnorm_inp="True",
                         **dict(opt, arch_opt="sgd", opt_dampening="0.0", opt_nesterov="False"))
    elif body == "lstm_gl":        # TIMIT_CGS/TIMIT_LSTM_fmllr_groupLasso.cfg: group lasso on the LSTM
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", skip_regularization="False", **opt)
    elif body in ("lstm_ghcgs_l1", "lstm_ghcgs_apply"):
        # TIMIT_CGS/TIMIT_LSTM_fmllr_ghcgs*.cfg: guided masks; before apply_guided_hcgs the L1 term
        # also trains the (unapplied) mask Parameters, after it the term is 0
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", skip_regularization="False", guided_hcgs="True",
                         apply_guided_hcgs=str(body == "lstm_ghcgs_apply"), hcgsx_block="8",
                         hcgsx_sparse="50", hcgsh_block="8,4", hcgsh_sparse="75,50", **opt)
    elif body in ("lstm_quant", "lstm_quant_ln"):
        # 8-bit weights + 16-bit quantised inputs and h (quantized_modules.py:99-119, 182-222);
        # _ln: LayerNorm of h too (:1093-1094), whose OUTPUT is what the next step quantises — the
        # exact integer step products (QX, whose max|h| partials are the cell's h) must stay off
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", lstm_quant="True", lstm_quant_inp="True",
                         param_quant="8,8", inp_quant="16",
                         lstm_use_laynorm="True,True" if body == "lstm_quant_ln" else "False,False",
                         **opt)
    elif body == "lstm_prune":     # magnitude pruning every forward (neural_networks.py:886-1005)
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", lstm_prune="True", lstm_prune_perc="60,40", **opt)
    else:
        cfg["a1"] = dict(LSTM_DEF, arch_name="rnn", lstm_lay="32,24", lstm_drop="0.2,0.2",
                         lstm_bidir="False", **opt)
    head = dict(dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False", to_do="train",
                arch_name="head", dnn_lay="64", dnn_drop="0.0", dnn_use_batchnorm="False",
                dnn_use_laynorm="False", dnn_act="softmax", **opt)
    cfg["a2"] = head
    cfg["a3"] = dict(head, arch_name="mono", dnn_lay="8", arch_lr="0.0004")
    fin = ("lt=sum(lc,lmw)\nloss_gl=cost_gl(o2,0.01,4)\nloss_final=sum(lt,loss_gl)\n"
           if body == "lstm_gl" else
           "lt=sum(lc,lmw)\nloss_l1=cost_l1(o2,0.0005)\nloss_final=sum(lt,loss_l1)\n"
           if body.startswith("lstm_ghcgs") else "loss_final=sum(lc,lmw)\n")
    cfg["model"] = {"model": "o1=compute(rnn,fea)\no2=compute(head,o1)\no3=compute(mono,o1)\n"
                             "lm=cost_nll(o3,lab_mono)\nlmw=mult_constant(lm,1.0)\n"
                             "lc=cost_nll(o2,lab_cd)\n" + fin + "err_final=cost_err(o2,lab_cd)"}
    return cfg


@pytest.mark.parametrize("body", ["ligru", "lstm", "ligru_hcgs", "lstm_bidir", "lstm_prune",
                                  "lstm_gl", "lstm_ghcgs_l1", "lstm_ghcgs_apply", "gru", "mingru",
                                  "rnn", "lstm_ln", "gru_ln", "gru_nobn", "lstm_ln_bn",
                                  "ligru_inpnorm", "lstm_bninp", "gru_lninp", "mingru_inpnorm",
                                  "ligru_hcgs_sparse", "lstm_quant", "lstm_quant_ln"])
def test_seq_engine_vs_oracle(body):
    _seq_vs_oracle(body)


QUANT_BODIES = ("lstm_quant", "lstm_quant_ln")


@pytest.mark.parametrize("body", ["ligru_hcgs", "lstm", "lstm_bidir", "gru", "ligru", "rnn",
                                  "ligru_hcgs_sparse"])
def test_seq_engine_bf16_vs_bf16_oracle(body):
    """The bf16 performance mode of the sequence configs (Engine(prec=PKC_PREC_BF16): the input
    projections W, their dX / dW, the U weight gradients and the heads on bf16-rounded operands
    with fp32 accumulation; for liGRU / LSTM / RNN layers (dense or block-sparse U) also the serial
    U products and their BPTT products (step_bf16); cell state, BN and loss fp32) against the oracle run with
    exactly that rounding (oracle.nets.use_bf16_rec_matmuls / use_bf16_matmuls), 3 SGD steps
    (RMSprop turns rounding noise of near-zero gradients into full-size sign steps; the fp32 tests
    cover it).  Only fp32 summation order differs in front of the bf16 roundings, which a last-bit
    difference can move by 2^-9: posteriors and parameters held to 1e-4 (relative / of the
    tensor's scale) except a counted share (posteriors <= 1 %, parameters <= 0.5 %) bounded by
    1e-3.  liGRU + HCGS runs the persistent time loops (pkc_rnn_persist.hip)."""
    _seq_vs_oracle(body, bf16=True)


def _seq_vs_oracle(body, bf16=False):
    import pkc.engine as E
    if bf16 and body.endswith("_sparse"):        # exercise the bf16 block-sparse step kernels
        E.RNN_BF16_SPARSE = True
    try:
        _seq_vs_oracle_run(body, bf16)
    finally:
        E.RNN_BF16_SPARSE = False


def _seq_vs_oracle_run(body, bf16):
    from flipcheck import assert_counted, resync
    import pkc.neural_networks as NN
    from oracle import nets as ON
    from oracle import run as OR
    from pkc import _lib as L
    from pkc.engine import Engine, parse_model
    cfg = make_cfg(body)
    if bf16 or body in QUANT_BODIES:
        # SGD: RMSprop's first steps are sign steps of 4.47 lr whatever |g| is, so the bf16
        # operand-rounding noise (quantised bodies: the one-quantum moves of the 16-bit input
        # grid) of a near-zero gradient element becomes a full-size step either way and later
        # steps compare chaos, not kernels (the fp32 tests keep RMSprop; the optimizer is not
        # what this test checks)
        for sec in ("a1", "a2", "a3"):
            cfg[sec].update(arch_opt="sgd", arch_lr="0.08", opt_momentum="0.0",
                            opt_dampening="0.0", opt_nesterov="False")
    F, B = 20, 4
    secs = (("a1", F), ("a2", None), ("a3", None))
    nets, onets, opts = {}, {}, {}
    for sec, inp in secs:
        o = cfg[sec]
        if inp is None:
            inp = nets["rnn"].out_dim
        torch.manual_seed(3)
        np.random.seed(3)
        cls = ({"ligru": "liGRU", "ligru_hcgs": "liGRU", "lstm": "LSTM", "lstm_bidir": "LSTM",
                "lstm_prune": "LSTM", "lstm_gl": "LSTM", "lstm_ghcgs_l1": "LSTM",
                "lstm_ghcgs_apply": "LSTM", "gru": "GRU", "mingru": "minimalGRU",
                "rnn": "RNN", "lstm_ln": "LSTM", "gru_ln": "GRU", "gru_nobn": "GRU",
                "lstm_ln_bn": "LSTM", "ligru_inpnorm": "liGRU", "lstm_bninp": "LSTM",
                "gru_lninp": "GRU", "mingru_inpnorm": "minimalGRU",
                "ligru_hcgs_sparse": "liGRU", "lstm_quant": "LSTM", "lstm_quant_ln": "LSTM"}[body]
               if sec == "a1" else "MLP")
        nets[o["arch_name"]] = getattr(NN, cls)(o, inp)
        onets[o["arch_name"]] = getattr(ON, cls)(o, inp)
        onets[o["arch_name"]].load_state_dict(nets[o["arch_name"]].state_dict())
        if bf16 and sec == "a1":        # liGRU / LSTM / RNN: bf16 step products too
            ON.use_bf16_rec_matmuls(onets[o["arch_name"]], steps=not body.startswith("gru"))
        elif bf16:
            ON.use_bf16_matmuls(onets[o["arch_name"]])
        opts[o["arch_name"]] = o
    for k in nets:
        nets[k].to(DEV).train()
        onets[k].train()
    rs = np.random.RandomState(0)
    lens = np.sort(rs.randint(5, 13, size=12))
    end = np.cumsum(lens)
    X = rs.randn(end[-1], F).astype(np.float32)
    lab = np.stack([rs.randint(0, 64, end[-1]), rs.randint(0, 8, end[-1])], 1).astype(np.int32)
    H = nets["rnn"].layer_specs()
    bid = 2 if H[0]["bidir"] else 1
    masks = {(("rnn", li)): torch.from_numpy((rs.rand(bid * B, sp["H"]) > 0.2).astype(np.float32))
             for li, sp in enumerate(H)}
    import pkc.engine as E
    old_sparse = E.RNN_SPARSE
    E.RNN_SPARSE = "force" if body.endswith("_sparse") else old_sparse
    try:
        eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fea": (0, F)},
                     ["lab_cd", "lab_mono"], batch=B, max_len=16, seed=1,
                     prec=L.PREC_BF16 if bf16 else L.PREC_FP32,
                     rnn_drop_in={k: v.to(DEV) for k, v in masks.items()})
    finally:
        E.RNN_SPARSE = old_sparse
    lbufs = next(n for n in eng.nodes if n.rec).lbuf
    if body.endswith("_sparse"):
        assert all(lb["kmap_fwd"] is not None for lb in lbufs)
    if bf16 and body == "ligru_hcgs":    # the persistent time loops (pkc_rnn_persist.hip) run
        assert all(lb.get("persist_fwd") is not None and lb.get("persist_bwd") is not None
                   for lb in lbufs), "persistent loops not taken"
    if body in QUANT_BODIES:             # exact quantised-h products only without LayerNorm
        qx = [lb.get("U_hq") is not None for lb in lbufs]
        assert qx == [body == "lstm_quant"] * len(lbufs), qx
    eng.bind_chunk(torch.from_numpy(X).to(DEV), torch.from_numpy(lab).to(DEV), end[-1], end_index=end)
    oopt = {k: ON.make_optimizer(onets[k].parameters(), opts[k]) for k in onets}
    lines = OR.parse_model(cfg["model"]["model"])
    rng_e, rng_o = random.Random(7), random.Random(7)
    snt = 0
    post_out = []
    report = {}
    for step in range(3):
        # the engine's state before this step -> the oracle's starting state (parameters, BN
        # statistics, optimizer state): each step is compared from a common start, so a rounding
        # flip of one step is counted in that step and does not compound through the next ones
        eng.sync_state()
        resync(nets, onets, {k: eng.optimizer_state_dict(k) for k in nets} if step else None, oopt)
        batch = eng.next_seq_batch(rng_e)
        begs, blens, lefts, T = batch
        # oracle batch assembly exactly as core.py:183-200
        inp = torch.zeros(T, B, F + 2)
        for k in range(B):
            n = int(lens[snt])
            left = rng_o.randint(0, T - n)
            b0 = int(end[snt] - n)
            inp[left:left + n, k, :F] = torch.from_numpy(X[b0:b0 + n])
            inp[left:left + n, k, F:] = torch.from_numpy(lab[b0:b0 + n].astype(np.float32))
            assert left == lefts[k]
            snt += 1
        body_net = onets["rnn"]
        f = body_net.forward
        body_net.forward = lambda x, _f=f: _f(x, drop_masks=[masks[("rnn", i)] for i in range(len(H))])
        outs = OR.train_step(lines, onets, oopt, {"rnn": True, "head": False, "mono": False},
                             {"fea": (0, F)}, {"lab_cd": F, "lab_mono": F + 1}, inp, T, B)
        body_net.forward = f
        eng.train_step(batch=batch)
        loss, err = eng.loss_values()
        np.testing.assert_allclose(loss, outs["loss_final"].item(), rtol=1e-3 if bf16 else 1e-4)
        if not bf16:
            np.testing.assert_allclose(err, outs["err_final"].item(), atol=1e-6)
        post = eng.head_output("o2").cpu()
        ref = outs["o2"].detach()
        relm = (post - ref).abs() / ref.abs().clamp_min(1e-3)
        rel = relm.max().item()
        # bf16 mode: a last-bit fp32 difference in front of a bf16 rounding moves that operand by
        # 2^-9; the posteriors it reaches are counted (above north_star's 1e-4) and bounded
        nout = int((relm > 1e-4).sum().item())
        post_out.append(nout)
        print("%s%s step %d posterior rel err %.3g, %d of %d above 1e-4" % (
            body, " bf16" if bf16 else "", step, rel, nout, relm.numel()))
        if bf16 or body in QUANT_BODIES:
            # a last-bit fp32 difference in front of a bf16 rounding moves that operand by 2^-9
            # (16-bit quantised h: in front of a ceil() grid step, one element by max|h| / 2^15):
            # the posteriors it moves past 1e-4 are counted (<= 1 %), none past 1e-3
            assert_counted("step %d posteriors" % step, nout, relm.numel(), 0.01, rel, 1e-3,
                           "(max rel err %.3g)" % rel)
        else:
            assert rel < 1e-4, "step %d posterior rel err %.3g (%d of %d above 1e-4)" % (
                step, rel, nout, relm.numel())
        _seq_check_update(body, bf16, step, eng, nets, onets, opts, report, post_out)
    print("%s%s parameter outliers per step and tensor: %s" % (
        body, " bf16" if bf16 else "", {k: v for k, v in report.items() if v[0]}))


def _seq_check_update(body, bf16, step, eng, nets, onets, opts, report, post_out):
    """The step's parameter updates (and BN running statistics) from the common start."""
    from flipcheck import assert_counted, step_outliers
    eng.sync_state()
    for k in nets:
        for name, v in nets[k].state_dict().items():
            if name.endswith("num_batches_tracked"):
                continue
            ref = onets[k].state_dict()[name].double()
            # the reference re-masks W / U at the next forward; pkc stores W*mask right away
            sd_o = onets[k].state_dict()
            parts = name.split(".")
            if body.startswith("ligru_hcgs") and name.endswith("weight") and parts[0] in ("wh", "wz", "uh", "uz"):
                mk = ("hcgsx" if parts[0][0] == "w" else "hcgsh") + ".%s.mask" % parts[1]
                ref = ref * sd_o[mk].double()
            if body == "lstm_ghcgs_apply" and k == "rnn" and name.endswith("weight") and \
                    len(parts[0]) == 3:
                ref = ref * sd_o["ghcgs_%s.%s.mask" % (parts[0], parts[1])].double()
            if body == "lstm_prune" and name.endswith("weight") and len(parts[0]) == 3 and k == "rnn":
                from oracle.masks import prune_mask
                perc = (60.0, 40.0)[int(parts[1])]
                ref = ref * prune_mask(sd_o[name], perc).double()
            scale = float(ref.abs().max())
            if name.endswith("running_mean") and body.endswith("inpnorm"):
                # the gate pre-activations of a BN-normalised input have column means of 0 up to
                # fp32 rounding: compare against the spread of the columns instead
                scale = float(sd_o[name.replace("running_mean", "running_var")].double().sqrt().max())
            # elementwise within 1e-4 of the tensor's scale, except counted RMSprop sign steps
            # (tests/flipcheck.py): a gradient element within rounding of zero takes the other
            # sign and moves its weight by ~9 lr in the step; each bounded by 2 x 4.48 lr
            lr = float(opts[k]["arch_lr"])
            scale = max(scale, lr)      # (a tensor whose gradient is rounding-level, e.g. ln0's
            # beta in front of bn0, stays within rounding of its init: lr is its scale)
            n, dmax, rest = step_outliers(v.cpu(), ref, 1e-4, scale)
            report["%d %s/%s" % (step, k, name)] = (n, round(dmax / scale, 6))
            sgd = opts[k]["arch_opt"] == "sgd"
            # bf16 mode (SGD): an operand-rounding flip moves a gradient element, and its update,
            # by ~2^-9 of one product — counted (<= 0.5 %), each within 1e-3 of the scale;
            # RMSprop (fp32): a sign step of one step, 2 x 4.48 lr
            noisy = bf16 or body in QUANT_BODIES
            frac = (0.005 if noisy else 0.0) if sgd else 0.02
            bound = (1e-3 if noisy else 1e-4) * scale if sgd else 2 * 4.48 * lr
            assert_counted("step %d %s %s" % (step, k, name), n, ref.numel(), frac, dmax,
                           bound + 1e-7, "(outliers, max diff / scale per tensor %s; posteriors "
                           "above 1e-4 per step %s)" % (
                               {a: b for a, b in report.items() if b[0]}, post_out))
