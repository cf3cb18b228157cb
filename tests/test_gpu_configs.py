"""Every sequence configuration of BASELINE.json at its real layer sizes, against the oracle.

The shapes are bench_seq's (scripts/bench_seq.py, the ones the bench measures):
  C3  liGRU 4x550 bidirectional, HCGS [32,2]/[75,75] (16x) on W and U, B = 8  — with the
      block-sparse U step kernels (kmap tables at these exact masks) forced on and off;
  C4  LSTM 4x1024 bidirectional (liGRU shared-weight convention), B = 16;
  C5  LSTM 3x512 + Pattern 8x8/k4/n16 (pattern_file set) + 8-bit weight / 16-bit input
      fake-quantisation, B = 12.
Short sentences (T <= 20) so the oracle's eager per-step CPU loop stays in seconds, two training
steps with injected recurrent dropout masks (the reference draws them from torch's RNG, :843-847),
heads 1928 cd + 48 mono.  Posteriors within 1e-4 relative (north_star), loss within 1e-5, weights
after the steps in relative Frobenius norm within 5e-3: RMSprop's first steps are
lr * g / sqrt((1 - alpha) g^2), so a parameter whose gradient is at rounding level (the BatchNorm
betas of the gate pre-activations) moves by a noise-determined amount of up to 4.5 lr.
"""
import os
import random
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT
from quantcheck import assert_few_flips, rmsprop_quanta

pytestmark = pytest.mark.gpu
DEV = "cuda"
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def build_pair(name, seed=2234, drop=None):
    """pkc nets + oracle nets (same state dict) for bench_seq config `name` (drop: override the
    recurrent dropout rate of every layer)."""
    import configparser

    import bench_seq as BS
    import pkc.neural_networks as NN
    from oracle import nets as ON
    cls, ropts, B = BS.rec_opts(name)
    if drop is not None:
        ropts = {k: (",".join([drop] * len(v.split(","))) if k.endswith("_drop") else v)
                 for k, v in ropts.items()}
    cfg = configparser.ConfigParser()
    cfg["a1"] = dict(ropts, arch_name="rnn", **BS.OPT)
    head = dict(dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False", arch_name="head",
                dnn_lay="1928", dnn_drop="0.0", dnn_use_batchnorm="False", dnn_use_laynorm="False",
                dnn_act="softmax", **dict(BS.OPT, arch_lr="0.0004"))
    cfg["a2"] = head
    cfg["a3"] = dict(head, arch_name="mono", dnn_lay="48")
    torch.manual_seed(seed)
    np.random.seed(seed)
    rnn = getattr(NN, cls)(cfg["a1"], 440)
    orn = getattr(ON, cls)(cfg["a1"], 440)
    orn.load_state_dict(rnn.state_dict())
    if name == "c5":
        pset = np.load(os.path.join(GOLDEN, "quant.npz"), allow_pickle=False)["pattern_set"]
        rnn.pattern_kernels = pset.reshape(16, 8, 8)
        orn.pattern_kernels = pset.reshape(16, 8, 8)
    nets = {"rnn": rnn, "head": NN.MLP(cfg["a2"], rnn.out_dim), "mono": NN.MLP(cfg["a3"], rnn.out_dim)}
    onets = {"rnn": orn, "head": ON.MLP(cfg["a2"], rnn.out_dim), "mono": ON.MLP(cfg["a3"], rnn.out_dim)}
    for k in ("head", "mono"):
        onets[k].load_state_dict(nets[k].state_dict())
    opts = {"rnn": cfg["a1"], "head": cfg["a2"], "mono": cfg["a3"]}
    model = ("o1=compute(rnn,fea)\no2=compute(head,o1)\no3=compute(mono,o1)\n"
             "lm=cost_nll(o3,lab_mono)\nlmw=mult_constant(lm,1.0)\nlc=cost_nll(o2,lab_cd)\n"
             "loss_final=sum(lc,lmw)\nerr_final=cost_err(o2,lab_cd)")
    return nets, onets, opts, model, B


def run_config(name, sparse=None, steps=2, post_tol=1e-4, w_tol=5e-3, quant_beta_bound=False,
               beta_bound=False):
    import pkc.engine as E
    from oracle import nets as ON
    from oracle import run as OR
    from pkc.engine import Engine, parse_model
    nets, onets, opts, model, B = build_pair(name)
    for k in nets:
        nets[k].to(DEV).train()
        onets[k].train()
    F = 440
    rs = np.random.RandomState(17)
    lens = np.sort(rs.randint(12, 21, size=B * steps))
    end = np.cumsum(lens)
    X = rs.randn(end[-1], F).astype(np.float32)
    lab = np.stack([rs.randint(0, 1928, end[-1]), rs.randint(0, 48, end[-1])], 1).astype(np.int32)
    specs = nets["rnn"].layer_specs()
    bid = 2 if specs[0]["bidir"] else 1
    masks = {("rnn", li): torch.from_numpy((rs.rand(bid * B, sp["H"]) > 0.2).astype(np.float32))
             for li, sp in enumerate(specs)}
    old = E.RNN_SPARSE
    if sparse is not None:
        E.RNN_SPARSE = sparse
    try:
        eng = Engine(nets, opts, parse_model(model), {"fea": (0, F)}, ["lab_cd", "lab_mono"],
                     batch=B, max_len=int(lens.max()), seed=1,
                     rnn_drop_in={k: v.to(DEV) for k, v in masks.items()})
    finally:
        E.RNN_SPARSE = old
    if sparse == "force":
        assert all(lb["kmap_fwd"] is not None for lb in eng.nodes[0].lbuf)
    if sparse == "off":
        assert all(lb["kmap_fwd"] is None for lb in eng.nodes[0].lbuf)
    eng.bind_chunk(torch.from_numpy(X).to(DEV), torch.from_numpy(lab).to(DEV), end[-1], end_index=end)
    oopt = {k: ON.make_optimizer(onets[k].parameters(), opts[k]) for k in onets}
    lines = OR.parse_model(model)
    rng_e, rng_o = random.Random(7), random.Random(7)
    snt, worst = 0, 0.0
    for step in range(steps):
        batch = eng.next_seq_batch(rng_e)
        begs, blens, lefts, T = batch
        inp = torch.zeros(T, B, F + 2)
        for k in range(B):                          # core.py:183-200
            n = int(lens[snt])
            left = rng_o.randint(0, T - n)
            b0 = int(end[snt] - n)
            inp[left:left + n, k, :F] = torch.from_numpy(X[b0:b0 + n])
            inp[left:left + n, k, F:] = torch.from_numpy(lab[b0:b0 + n].astype(np.float32))
            assert left == lefts[k]
            snt += 1
        body = onets["rnn"]
        f = body.forward
        body.forward = lambda x, _f=f: _f(x, drop_masks=[masks[("rnn", i)] for i in range(len(specs))])
        outs = OR.train_step(lines, onets, oopt, {"rnn": True, "head": False, "mono": False},
                             {"fea": (0, F)}, {"lab_cd": F, "lab_mono": F + 1}, inp, T, B)
        body.forward = f
        eng.train_step(batch=batch)
        loss, err = eng.loss_values()
        np.testing.assert_allclose(loss, outs["loss_final"].item(), rtol=1e-5)
        post = eng.head_output("o2").cpu()
        ref = outs["o2"].detach()
        rel = ((post - ref).abs() / ref.abs().clamp_min(1e-3)).max().item()
        worst = max(worst, rel)
        assert rel < post_tol, "%s step %d posterior rel err %.3g" % (name, step, rel)
    eng.sync_state()
    sd_o = onets["rnn"].state_dict()
    wworst = 0.0
    flips = {}
    for k in nets:
        osd = onets[k].state_dict()
        for pname, v in nets[k].state_dict().items():
            if pname.endswith("num_batches_tracked"):
                continue
            r = osd[pname].double()
            parts = pname.split(".")
            if k == "rnn" and pname.endswith("weight") and name == "c3" and parts[0] in ("wh", "wz", "uh", "uz"):
                # the reference re-masks W / U at the next forward; pkc stores W * mask right away
                r = r * sd_o[("hcgsx" if parts[0][0] == "w" else "hcgsh") + ".%s.mask" % parts[1]].double()
            if k == "rnn" and name == "c5" and pname.endswith("weight") and len(parts[0]) == 3:
                # pattern^L: every layer call multiplies all layers' masks in (:876-884, 1226-1237)
                r = r * onets["rnn"].pattern_masks[parts[0]][int(parts[1])].double() ** len(specs)
            if quant_beta_bound and k == "rnn" and pname.endswith("weight") and v.dim() == 2:
                # 8-bit weights: at most 0.2 % of a matrix on another grid point (+1: a weight
                # crossing zero jumps from index +1 to -1)
                nf = assert_few_flips(v.cpu().numpy(), r.numpy(), "%s %s" % (name, pname), 2e-3,
                                      max_quanta=rmsprop_quanta(float(opts[k]["arch_lr"]), steps) + 1)
                flips[pname] = nf
            d = (v.cpu().double() - r).norm().item()
            e = d / max(r.norm().item(), 1e-30)
            if (quant_beta_bound or beta_bound) and ".bias" in pname and pname.startswith("bn"):
                # gate BatchNorm betas under fake quantisation: their gradients are sums of
                # quantum-flip noise; RMSprop bounds any such noise step by
                # lr / sqrt(1 - alpha) = 4.47 lr per step (either sign).  beta_bound (C3 fp32):
                # a beta's gradient is a column sum of dgates, many elements of which sit within
                # fp32 rounding of zero — another summation order (the grid-synchronised loops')
                # flips their signs, which RMSprop's first steps turn into the same full steps
                lr = float(opts[k]["arch_lr"])
                md = (v.cpu().double() - r).abs().max().item()
                assert md <= 2 * 4.48 * lr * steps, "%s %s max abs diff %.3g" % (name, pname, md)
                continue
            wworst = max(wworst, e)
            assert d <= w_tol * r.norm().item() + 1e-6, "%s %s %s rel err %.3g" % (name, k, pname, e)
    print("%s (sparse=%s): posterior max rel err %.3g, weights max rel err %.3g, 8-bit grid flips "
          "%s" % (name, sparse, worst, wworst, flips))
    return eng


def run_config_bf16(name, steps=2, persist=True):
    """The bf16 performance mode (Engine prec PKC_PREC_BF16: bf16 projections, heads, weight
    gradients and step products — C3 through the persistent time loops) at the full layer sizes
    against the oracle run with exactly that rounding (oracle.nets.use_bf16_rec_matmuls /
    use_bf16_matmuls), SGD (as tests/test_gpu_seq.py's bf16 tests: RMSprop turns rounding noise of
    near-zero gradients into full-size sign steps), every step from a common start
    (flipcheck.resync).  Only the fp32 summation order differs in front of the bf16 roundings; a
    last-bit difference there moves one operand by 2^-9 and what it reaches is counted:
    posteriors above 1e-4 relative <= 1 % (none above 1e-3), parameter updates outside 1e-4 of the
    tensor's scale <= 0.5 % (none beyond 1e-3)."""
    import pkc.engine as E
    from flipcheck import assert_counted, resync, step_outliers
    from oracle import nets as ON
    from oracle import run as OR
    from pkc import _lib as L
    from pkc.engine import Engine, parse_model
    nets, onets, opts, model, B = build_pair(name)
    sgd = dict(arch_opt="sgd", arch_lr="0.08", opt_momentum="0.0", opt_dampening="0.0",
               opt_nesterov="False")
    for k in opts:
        opts[k].update(sgd)
    ON.use_bf16_rec_matmuls(onets["rnn"], steps=True)
    for k in ("head", "mono"):
        ON.use_bf16_matmuls(onets[k])
    for k in nets:
        nets[k].to(DEV).train()
        onets[k].train()
    F = 440
    rs = np.random.RandomState(17)
    lens = np.sort(rs.randint(12, 21, size=B * steps))
    end = np.cumsum(lens)
    X = rs.randn(end[-1], F).astype(np.float32)
    lab = np.stack([rs.randint(0, 1928, end[-1]), rs.randint(0, 48, end[-1])], 1).astype(np.int32)
    specs = nets["rnn"].layer_specs()
    bid = 2 if specs[0]["bidir"] else 1
    masks = {("rnn", li): torch.from_numpy((rs.rand(bid * B, sp["H"]) > 0.2).astype(np.float32))
             for li, sp in enumerate(specs)}
    old = (E.RNN_PERSIST, E.RNN_BF16_SPARSE)
    # (without the persistent loops C3's block-sparse U takes the per-step bf16 kernels)
    E.RNN_PERSIST, E.RNN_BF16_SPARSE = persist, not persist
    try:
        eng = Engine(nets, opts, parse_model(model), {"fea": (0, F)}, ["lab_cd", "lab_mono"],
                     batch=B, max_len=int(lens.max()), seed=1, prec=L.PREC_BF16,
                     rnn_drop_in={k: v.to(DEV) for k, v in masks.items()})
    finally:
        E.RNN_PERSIST, E.RNN_BF16_SPARSE = old
    lbufs = eng.nodes[0].lbuf
    assert all(lb.get("hs_h") is not None for lb in lbufs), "bf16 step products not taken"
    if name == "c3":
        assert all((lb.get("persist_fwd") is not None) == persist for lb in lbufs), \
            "persistent loops %s" % ("not taken" if persist else "taken")
    eng.bind_chunk(torch.from_numpy(X).to(DEV), torch.from_numpy(lab).to(DEV), end[-1], end_index=end)
    oopt = {k: ON.make_optimizer(onets[k].parameters(), opts[k]) for k in onets}
    lines = OR.parse_model(model)
    rng_e, rng_o = random.Random(7), random.Random(7)
    snt = 0
    posts, report = [], {}
    for step in range(steps):
        eng.sync_state()
        resync(nets, onets, {k: eng.optimizer_state_dict(k) for k in nets} if step else None, oopt)
        batch = eng.next_seq_batch(rng_e)
        begs, blens, lefts, T = batch
        inp = torch.zeros(T, B, F + 2)
        for k in range(B):                          # core.py:183-200
            n = int(lens[snt])
            left = rng_o.randint(0, T - n)
            b0 = int(end[snt] - n)
            inp[left:left + n, k, :F] = torch.from_numpy(X[b0:b0 + n])
            inp[left:left + n, k, F:] = torch.from_numpy(lab[b0:b0 + n].astype(np.float32))
            assert left == lefts[k]
            snt += 1
        body = onets["rnn"]
        f = body.forward
        body.forward = lambda x, _f=f: _f(x, drop_masks=[masks[("rnn", i)] for i in range(len(specs))])
        outs = OR.train_step(lines, onets, oopt, {"rnn": True, "head": False, "mono": False},
                             {"fea": (0, F)}, {"lab_cd": F, "lab_mono": F + 1}, inp, T, B)
        body.forward = f
        eng.train_step(batch=batch)
        loss, _ = eng.loss_values()
        np.testing.assert_allclose(loss, outs["loss_final"].item(), rtol=1e-3)
        post = eng.head_output("o2").cpu()
        ref = outs["o2"].detach()
        relm = (post - ref).abs() / ref.abs().clamp_min(1e-3)
        rel = relm.max().item()
        nout = int((relm > 1e-4).sum().item())
        posts.append((nout, round(rel, 6)))
        assert_counted("%s bf16 step %d posteriors" % (name, step), nout, relm.numel(), 0.01, rel,
                       1e-3, "(max rel err %.3g; per step %s)" % (rel, posts))
        eng.sync_state()
        sd_o = onets["rnn"].state_dict()
        for k in nets:
            osd = onets[k].state_dict()
            for pname, v in nets[k].state_dict().items():
                if pname.endswith("num_batches_tracked"):
                    continue
                r = osd[pname].double()
                parts = pname.split(".")
                if k == "rnn" and name == "c3" and pname.endswith("weight") and \
                        parts[0] in ("wh", "wz", "uh", "uz"):
                    r = r * sd_o[("hcgsx" if parts[0][0] == "w" else "hcgsh") + ".%s.mask" % parts[1]].double()
                scale = max(float(r.abs().max()), 0.08)
                n, dmax, _ = step_outliers(v.cpu(), r, 1e-4, scale)
                report["%d %s/%s" % (step, k, pname)] = (n, round(dmax / scale, 6))
                assert_counted("%s bf16 step %d %s %s" % (name, step, k, pname), n, r.numel(), 0.005,
                               dmax, 1e-3 * scale + 1e-7, "(outliers per tensor %s)" % (
                                   {a: b for a, b in report.items() if b[0]}))
    print("%s bf16 (persistent=%s): posteriors above 1e-4 per step (count, max rel) %s; parameter "
          "outliers %s" % (name, persist, posts, {a: b for a, b in report.items() if b[0]}))


def test_c3_ligru_hcgs_full_size_bf16():
    run_config_bf16("c3")


def test_c3_ligru_hcgs_full_size_bf16_per_step():
    run_config_bf16("c3", persist=False)


def test_c4_lstm_bidir_full_size_bf16():
    run_config_bf16("c4")


@pytest.mark.parametrize("sparse", ["force", "off"])
def test_c3_ligru_hcgs_full_size(sparse):
    run_config("c3", sparse=sparse, beta_bound=True)


def test_c4_lstm_bidir_full_size():
    run_config("c4")


def test_c5_lstm_pattern_quant_full_size():
    # 16-bit input fake-quantisation snaps to a grid of max|x| / 2^15; a last-bit difference in
    # front of a ceil() moves one element by one quantum, and the 8-bit weight grid
    # (1/128) does the same to a weight whose update lands within rounding of a grid boundary
    run_config("c5", post_tol=1e-3, w_tol=2e-2, quant_beta_bound=True)
