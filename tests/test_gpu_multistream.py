"""Multi-feature-stream chunks (reference data_io.py:184-263, utils.py:2014-2016).

The reference loads every feature stream of a chunk with its own context window and chunk
statistics, trims each to the widest window, column-stacks them in fea_dict order with the labels
after all features, and the [model] joins them with concatenate(a,b).  Checked here:
  * pkc.data_io.prepare_streams against read_lab_fea fixtures written by the reference itself
    (tests/golden/loader_multi.npz: mfcc 13 x (2,1), fbank 23 x (0,0), fmllr 40 x (5,3) — the
    TIMIT_mfcc_fbank_fmllr_liGRU_best.cfg shape with different windows), shuffled and sequential;
  * against the oracle's read_lab_fea on windows where np.roll wraps around the chunk
    (a stream whose left window exceeds the widest right window);
  * pkc.core.read_lab_fea + an Engine step on a 3-stream cfg (concatenate -> MLP -> cd / mono heads)
    against the oracle's read_lab_fea + training step, and run_nn end to end (train + forward) on
    a 3-stream liGRU cfg — core.py no longer refuses several streams.
"""
import configparser
import os
import random

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _unpack(d, prefix):
    keys, lens, data = d[prefix + "_keys"], d[prefix + "_lens"], d[prefix + "_data"]
    out, o = {}, 0
    for k, n in zip(keys, lens):
        out[str(k)] = data[o:o + n]
        o += n
    return out


@pytest.mark.parametrize("tag", ["nonseq", "seq"])
def test_prepare_streams_matches_reference_golden(tag):
    from pkc import data_io as D
    g = np.load(os.path.join(GOLDEN, "loader_multi.npz"), allow_pickle=False)
    names = [str(n) for n in g["stream_names"]]
    cd, mono = _unpack(g, "cd"), _unpack(g, "mono")
    streams = []
    for n, (dim, l, r) in zip(names, g["streams"]):
        fea = _unpack(g, "fea_" + n)
        streams.append((D.stage_chunk(fea, [cd, mono], 1000), int(l), int(r), n))
    rng = np.random.RandomState(2234) if tag == "nonseq" else None
    ch = D.prepare_streams(streams, ["lab_cd", "lab_mono"], shuffle_rng=rng)
    ref = g["rlf_%s_data" % tag]
    assert list(ch.names) == [str(x) for x in g["rlf_%s_names" % tag]]
    np.testing.assert_array_equal(ch.end_index, g["rlf_%s_end" % tag])
    fc = g["rlf_%s_feacols" % tag]
    for i, n in enumerate(names):
        assert ch.fea_cols[n] == (fc[i][0], fc[i][1]), (n, ch.fea_cols[n], fc[i])
    C_ = int(fc[-1][1])
    assert list(g["rlf_%s_labcols" % tag]) == [C_, C_ + 1]
    np.testing.assert_allclose(ch.feats.cpu().numpy(), ref[:, :C_], rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(ch.labels.cpu().numpy(), ref[:, C_:].astype(np.int32))


def test_prepare_streams_wrapping_windows_vs_oracle():
    """Windows whose np.roll wraps around the chunk (left 4 > the widest right 2; right 2 > the
    widest-left stream's...), max_seq splits, three streams in a non-sorted name order."""
    from oracle import loader as OL
    from pkc import data_io as D
    rs = np.random.RandomState(5)
    keys = ["u%02d" % i for i in range(7)]
    lens = {k: rs.randint(12, 60) for k in keys}
    spec = (("zeta", 13, 4, 0), ("alpha", 23, 0, 2), ("mid", 40, 1, 1))
    feas = {n: {k: (rs.randn(lens[k], d) * 2 + rs.randn(1, d)).astype(np.float32) for k in keys}
            for n, d, _, _ in spec}
    cd = {k: rs.randint(3, 500, lens[k]).astype(np.int32) for k in keys}
    for seq in (False, True):
        names, end, fcols, lcols, ref = OL.read_lab_fea(
            [(n, feas[n], l, r) for n, _, l, r in spec], [("lab_cd", cd)], seq, max_seq_length=40,
            rng=np.random.RandomState(9))
        streams = [(D.stage_chunk(feas[n], [cd], 40), l, r, n) for n, _, l, r in spec]
        ch = D.prepare_streams(streams, ["lab_cd"],
                               shuffle_rng=None if seq else np.random.RandomState(9))
        assert list(ch.names) == list(names)
        np.testing.assert_array_equal(ch.end_index, end)
        assert ch.fea_cols == fcols, (ch.fea_cols, fcols)
        C_ = max(c1 for _, c1 in fcols.values())
        np.testing.assert_allclose(ch.feats.cpu().numpy(), ref[:, :C_], rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(ch.labels.cpu().numpy()[:, 0], ref[:, C_].astype(np.int32))


STREAMS = (("mfcc", 13, 2, 1), ("fbank", 23, 0, 0), ("fmllr", 40, 3, 3))


def _write_streams(d, seed, n_utt=16):
    from pkc import data_io as D
    rs = np.random.RandomState(seed)
    ali = os.path.join(d, "ali_%d" % seed)
    os.makedirs(ali, exist_ok=True)
    scps, raw = {}, {n: {} for n, _, _, _ in STREAMS}
    keys = ["spk%d_u%03d" % (seed, i) for i in range(n_utt)]
    lens = {k: rs.randint(30, 80) for k in keys}
    for n, dim, _, _ in STREAMS:
        ark, scp = os.path.join(d, "feats_%s_%d.ark" % (n, seed)), os.path.join(d, "feats_%s_%d.scp" % (n, seed))
        with open(scp, "w") as f:
            for i, k in enumerate(keys):
                m = (rs.randn(lens[k], dim) * (1 + dim / 20) + rs.randn(1, dim)).astype(np.float32)
                raw[n][k] = m
                D.write_mat_path(ark, m, k, append=i > 0)
                f.write("%s %s\n" % (k, ark))
        scps[n] = scp
    cd, mono = {}, {}
    for i, k in enumerate(keys):
        cd[k] = rs.randint(0, 64, lens[k]).astype(np.int32)
        mono[k] = rs.randint(1, 9, lens[k]).astype(np.int32)
        D.write_vec_int_path(os.path.join(ali, "ali_pdf.ark"), cd[k], k, append=i > 0)
        D.write_vec_int_path(os.path.join(ali, "ali_phones.ark"), mono[k], k, append=i > 0)
    return scps, ali, raw, cd, mono


def _cfg(d, name, to_do, scps, ali, body="mlp", counts=None, pretrain=None):
    cfg = configparser.ConfigParser()
    cfg["exp"] = {"seed": "2234", "out_folder": d, "use_cuda": "True", "multi_gpu": "False",
                  "to_do": to_do, "out_info": os.path.join(d, name + ".info"), "save_gpumem": "False",
                  "production": "False", "run_nn_script": "run_nn.py"}
    cfg["batches"] = {"batch_size_train": "32" if body == "mlp" else "4",
                      "batch_size_valid": "32" if body == "mlp" else "4",
                      "max_seq_length_train": "1000", "max_seq_length_valid": "1000"}
    cfg["data_chunk"] = {
        "fea": "\n".join("fea_name=%s\nfea_lst=%s\nfea_opts=\ncw_left=%d\ncw_right=%d\n"
                         % (n, scps[n], l, r) for n, _, l, r in STREAMS),
        "lab": "lab_name=lab_cd\nlab_folder=%s\nlab_opts=ali-to-pdf\n\n"
               "lab_name=lab_mono\nlab_folder=%s\nlab_opts=ali-to-phones --per-frame=true\n" % (ali, ali)}
    base = dict(arch_library="pkc.neural_networks", arch_pretrain_file="none", arch_freeze="False",
                arch_seq_model="False", dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False",
                arch_opt="rmsprop", opt_momentum="0.0", opt_alpha="0.95", opt_eps="1e-8",
                opt_centered="False", opt_weight_decay="0.0")
    if body == "mlp":
        cfg["architecture1"] = dict(base, arch_class="MLP", arch_name="MLP_layers1", dnn_lay="96,96",
                                    dnn_drop="0.0,0.0", dnn_use_batchnorm="True,True",
                                    dnn_use_laynorm="False,False", dnn_act="relu,relu",
                                    arch_lr="0.08", arch_opt="sgd", opt_dampening="0.0",
                                    opt_nesterov="False")
    else:
        cfg["architecture1"] = dict(base, arch_class="liGRU", arch_name="MLP_layers1",
                                    arch_seq_model="True", arch_lr="0.0016", ligru_lay="32,32",
                                    ligru_drop="0.2,0.2", ligru_use_laynorm_inp="False",
                                    ligru_use_batchnorm_inp="False", ligru_use_laynorm="False,False",
                                    ligru_use_batchnorm="True,True", ligru_bidir="True",
                                    ligru_act="relu,relu", ligru_orthinit="True")
    cfg["architecture2"] = dict(base, arch_class="MLP", arch_name="MLP_layers2", dnn_lay="64",
                                dnn_drop="0.0", dnn_use_batchnorm="False", dnn_use_laynorm="False",
                                dnn_act="softmax", arch_lr="0.0004")
    cfg["architecture3"] = dict(cfg["architecture2"], arch_name="MLP_layers3", dnn_lay="8")
    if pretrain:
        for i in (1, 2, 3):
            cfg["architecture%d" % i]["arch_pretrain_file"] = pretrain % i
    cfg["model"] = {"model": "conc1=concatenate(mfcc,fbank)\nconc2=concatenate(conc1,fmllr)\n"
                             "out_dnn1=compute(MLP_layers1,conc2)\n"
                             "out_dnn2=compute(MLP_layers2,out_dnn1)\n"
                             "out_dnn3=compute(MLP_layers3,out_dnn1)\n"
                             "loss_mono=cost_nll(out_dnn3,lab_mono)\n"
                             "loss_mono_w=mult_constant(loss_mono,1.0)\n"
                             "loss_cd=cost_nll(out_dnn2,lab_cd)\n"
                             "loss_final=sum(loss_cd,loss_mono_w)\nerr_final=cost_err(out_dnn2,lab_cd)"}
    cfg["forward"] = {"forward_out": "out_dnn2", "normalize_posteriors": "True",
                      "normalize_with_counts_from": counts or "none", "save_out_file": "True",
                      "require_decoding": "True"}
    path = os.path.join(d, name + ".cfg")
    with open(path, "w") as f:
        cfg.write(f)
    return path


def test_read_lab_fea_three_streams_and_engine_step(tmp_path):
    """pkc.core.read_lab_fea's six items on a 3-stream cfg vs the oracle's read_lab_fea, then one
    training step of concatenate -> MLP -> heads through the Engine vs the oracle's step."""
    import pkc.neural_networks as NN
    from oracle import loader as OL
    from oracle import nets as ON
    from oracle import run as OR
    from pkc import core
    from pkc.engine import Engine, parse_model
    d = str(tmp_path)
    scps, ali, raw, cd, mono = _write_streams(d, 0)
    path = _cfg(d, "train", "train", scps, ali)
    np.random.seed(2234)
    shared = []
    core.read_lab_fea(path, False, shared, d)
    names, chunk, end, fea_dict, lab_dict, arch_dict = core._finish_chunk(shared)
    labs = {"lab_cd": cd, "lab_mono": mono}        # in lab_dict order (the [model] line order)
    onames, oend, ofc, olc, ref = OL.read_lab_fea(
        [(n, raw[n], l, r) for n, _, l, r in STREAMS], [(ln, labs[ln]) for ln in lab_dict], False,
        rng=np.random.RandomState(2234))
    assert list(names) == list(onames)
    np.testing.assert_array_equal(end, oend)
    for n, _, _, _ in STREAMS:
        assert tuple(fea_dict[n][5:7]) == ofc[n] and fea_dict[n][7] == ofc[n][1] - ofc[n][0]
    assert {k: v[3] for k, v in lab_dict.items()} == olc
    data = np.asarray(chunk)                 # the reference's float64 [features | labels] rows
    np.testing.assert_allclose(data, ref, rtol=1e-6, atol=1e-6)
    # one training step on the first batch, concatenate resolved to the stacked column range
    cfg = configparser.ConfigParser()
    cfg.read(path)
    lines = parse_model(cfg["model"]["model"])
    F = max(c1 for _, c1 in ofc.values())
    torch.manual_seed(3)
    nets, onets, opts, oopt = {}, {}, {}, {}
    inp = {"MLP_layers1": F, "MLP_layers2": 96, "MLP_layers3": 96}
    for i in (1, 2, 3):
        o = cfg["architecture%d" % i]
        a = o["arch_name"]
        nets[a] = NN.MLP(o, inp[a])
        onets[a] = ON.MLP(o, inp[a])
        onets[a].load_state_dict(nets[a].state_dict())
        nets[a].to(DEV).train()
        onets[a].train()
        opts[a] = o
        oopt[a] = ON.make_optimizer(onets[a].parameters(), o)
    fea_cols = {k: (v[5], v[6]) for k, v in fea_dict.items()}
    lab_names = sorted(lab_dict, key=lambda k: lab_dict[k][3])
    eng = Engine(nets, opts, lines, fea_cols, lab_names, batch=32, seed=1)
    eng.bind_chunk(chunk.feats, chunk.labels, chunk.n_rows)
    eng.train_step()
    post = eng.head_output("out_dnn2").cpu().double()
    # the oracle's forward_model concatenates the stream slices itself (utils.py:2014-2016)
    outs = OR.train_step(OR.parse_model(cfg["model"]["model"]), onets, oopt,
                         {a: False for a in onets}, fea_cols, {k: v[3] for k, v in lab_dict.items()},
                         torch.from_numpy(ref[:32].astype(np.float32)))
    o = outs["out_dnn2"].detach().double()
    rel = ((post - o).abs() / o.abs().clamp_min(1e-3)).max().item()
    np.testing.assert_allclose(eng.loss_values()[0], outs["loss_final"].item(), rtol=1e-5)
    assert rel < 1e-4, "posterior rel err %.3g" % rel


def test_run_nn_three_streams_ligru_train_forward(tmp_path):
    """run_nn end to end on a 3-stream liGRU cfg (the TIMIT_mfcc_fbank_fmllr_liGRU_best.cfg feature
    shape): training chunk -> .info / .pkl, forward -> a posterior ark for every utterance."""
    from oracle import loader as OL
    from pkc.core import run_nn
    d = str(tmp_path)
    scps, ali, _, _, _ = _write_streams(d, 1)
    counts = os.path.join(d, "counts")
    with open(counts, "w") as f:
        f.write("[ " + " ".join(str(i + 3) for i in range(64)) + " ]\n")
    c_tr = _cfg(d, "train_ck0", "train", scps, ali, body="ligru")
    c_va = _cfg(d, "valid", "valid", scps, ali, body="ligru")
    data, _, _ = run_nn(None, None, None, None, None, None, c_tr, True, c_va)
    info = configparser.ConfigParser()
    info.read(os.path.join(d, "train_ck0.info"))
    assert 0 < float(info["results"]["loss"]) < 20
    # the next chunk's six items carry the three streams' column ranges
    fea_dict = data[3]
    assert [tuple(fea_dict[n][5:8]) for n, _, _, _ in STREAMS] == [(0, 52, 52), (52, 75, 23),
                                                                   (75, 355, 280)]
    c_fw = _cfg(d, "forward", "forward", scps, ali, body="ligru", counts=counts,
                pretrain=os.path.join(d, "train_ck0_architecture%d.pkl"))
    random.seed(0)
    run_nn(None, None, None, None, None, None, c_fw, True, c_fw)
    with open(os.path.join(d, "forward_out_dnn2_to_decode.ark"), "rb") as f:
        mats = OL.parse_mat_ark(f.read())
    assert len(mats) == 16
    c = np.arange(3, 67, dtype=np.float64)
    for k, m in mats:
        np.testing.assert_allclose(np.exp(m + np.log(c / c.sum())).sum(1), 1.0, rtol=1e-4)


def test_concat_mlp_ligru_mlp_engine_vs_oracle():
    """The TIMIT_mfcc_fbank_fmllr_liGRU_best.cfg model graph (cfg :260-270): two feature streams
    concatenated -> MLP_layers_first (feed-forward over the T*B rows of the sentence batch) ->
    liGRU (bidirectional) -> MLP_layers_second -> cd / mono LogSoftmax heads, three training steps
    against the oracle's forward_model (utils.py:1905-1934: a feed-forward arch on a 3-D input is
    viewed as (T*B, F), a recurrent one reading a 2-D output as (T, B, F)), every step from a common
    start (flipcheck.resync), posteriors within 1e-4 and updates elementwise within 1e-4 of their
    scale except counted RMSprop sign steps."""
    import pkc.neural_networks as NN
    from cases import LIGRU_DEF, MLP_DEF
    from flipcheck import assert_counted, resync, step_outliers
    from oracle import nets as ON
    from oracle import run as OR
    from pkc.engine import Engine, parse_model
    opt = dict(arch_opt="rmsprop", arch_lr="0.0016", opt_momentum="0.0", opt_alpha="0.95",
               opt_eps="1e-8", opt_centered="False", opt_weight_decay="0.0", arch_freeze="False")
    cfg = configparser.ConfigParser()
    # (the feed-forward archs with SGD, as the TIMIT MLP cfgs: their BatchNorm'd Linear biases have
    # gradients at rounding level, which RMSprop's first sign steps would blow up to 4.5 lr)
    sgd = dict(opt, arch_opt="sgd", arch_lr="0.08", opt_dampening="0.0", opt_nesterov="False")
    cfg["pre"] = dict(MLP_DEF, arch_name="pre", dnn_lay="48,40", dnn_drop="0.0,0.0",
                      dnn_use_batchnorm="True,True", dnn_use_laynorm="False,False",
                      dnn_act="relu,relu", **sgd)
    cfg["rnn"] = dict(LIGRU_DEF, arch_name="rnn", ligru_lay="32,24", ligru_drop="0.2,0.2", **opt)
    cfg["post"] = dict(MLP_DEF, arch_name="post", dnn_lay="36", dnn_drop="0.0",
                       dnn_use_batchnorm="True", dnn_use_laynorm="False", dnn_act="relu", **sgd)
    head = dict(MLP_DEF, arch_name="head", dnn_lay="64", dnn_drop="0.0", dnn_use_batchnorm="False",
                dnn_use_laynorm="False", dnn_act="softmax", **opt)
    cfg["head"] = head
    cfg["mono"] = dict(head, arch_name="mono", dnn_lay="8", arch_lr="0.0004")
    model = ("conc=concatenate(mfcc,fmllr)\no0=compute(pre,conc)\no1=compute(rnn,o0)\n"
             "o2=compute(post,o1)\no3=compute(head,o2)\no4=compute(mono,o2)\n"
             "lm=cost_nll(o4,lab_mono)\nlmw=mult_constant(lm,1.0)\nlc=cost_nll(o3,lab_cd)\n"
             "loss_final=sum(lc,lmw)\nerr_final=cost_err(o3,lab_cd)")
    F1, F2, B = 8, 12, 4
    F = F1 + F2
    dims = {"pre": F, "rnn": 40, "post": 48, "head": 36, "mono": 36}
    cls = {"pre": "MLP", "rnn": "liGRU", "post": "MLP", "head": "MLP", "mono": "MLP"}
    nets, onets, opts = {}, {}, {}
    for a in ("pre", "rnn", "post", "head", "mono"):
        torch.manual_seed(7)
        nets[a] = getattr(NN, cls[a])(cfg[a], dims[a])
        onets[a] = getattr(ON, cls[a])(cfg[a], dims[a])
        onets[a].load_state_dict(nets[a].state_dict())
        nets[a].to(DEV).train()
        onets[a].train()
        opts[a] = cfg[a]
    seqd = {a: a == "rnn" for a in nets}
    rs = np.random.RandomState(0)
    lens = np.sort(rs.randint(5, 13, size=12))
    end = np.cumsum(lens)
    X = rs.randn(end[-1], F).astype(np.float32)
    lab = np.stack([rs.randint(0, 64, end[-1]), rs.randint(0, 8, end[-1])], 1).astype(np.int32)
    masks = [torch.from_numpy((rs.rand(2 * B, h) > 0.2).astype(np.float32)) for h in (32, 24)]
    fea_cols = {"mfcc": (0, F1), "fmllr": (F1, F)}
    eng = Engine(nets, opts, parse_model(model), fea_cols, ["lab_cd", "lab_mono"], batch=B,
                 max_len=16, seed=1, rnn_drop_in={("rnn", i): m.to(DEV) for i, m in enumerate(masks)})
    eng.bind_chunk(torch.from_numpy(X).to(DEV), torch.from_numpy(lab).to(DEV), end[-1], end_index=end)
    oopt = {k: ON.make_optimizer(onets[k].parameters(), opts[k]) for k in onets}
    lines = OR.parse_model(model)
    rng_e, rng_o = random.Random(7), random.Random(7)
    snt, report = 0, {}
    for step in range(3):
        eng.sync_state()
        resync(nets, onets, {k: eng.optimizer_state_dict(k) for k in nets} if step else None, oopt)
        batch = eng.next_seq_batch(rng_e)
        _, _, lefts, T = batch
        inp = torch.zeros(T, B, F + 2)
        for k in range(B):                          # core.py:183-200
            n = int(lens[snt])
            left = rng_o.randint(0, T - n)
            b0 = int(end[snt] - n)
            inp[left:left + n, k, :F] = torch.from_numpy(X[b0:b0 + n])
            inp[left:left + n, k, F:] = torch.from_numpy(lab[b0:b0 + n].astype(np.float32))
            assert left == lefts[k]
            snt += 1
        f = onets["rnn"].forward
        onets["rnn"].forward = lambda x, _f=f: _f(x, drop_masks=masks)
        outs = OR.train_step(lines, onets, oopt, seqd, fea_cols, {"lab_cd": F, "lab_mono": F + 1},
                             inp, T, B)
        onets["rnn"].forward = f
        eng.train_step(batch=batch)
        np.testing.assert_allclose(eng.loss_values()[0], outs["loss_final"].item(), rtol=1e-4)
        post = eng.head_output("o3").cpu()
        ref = outs["o3"].detach()
        rel = ((post - ref).abs() / ref.abs().clamp_min(1e-3)).max().item()
        assert rel < 1e-4, "step %d posterior rel err %.3g" % (step, rel)
        eng.sync_state()
        for k in nets:
            lr = float(opts[k]["arch_lr"])
            sgd_k = opts[k]["arch_opt"] == "sgd"
            for name, v in nets[k].state_dict().items():
                if name.endswith("num_batches_tracked"):
                    continue
                r = onets[k].state_dict()[name].double()
                scale = max(float(r.abs().max()), lr)
                n, dmax, _ = step_outliers(v.cpu(), r, 1e-4, scale)
                report["%d %s/%s" % (step, k, name)] = (n, round(dmax / scale, 6))
                # RMSprop: counted sign steps of near-zero gradients; SGD: 1e-4 of the scale
                assert_counted("step %d %s %s" % (step, k, name), n, r.numel(),
                               0.0 if sgd_k else 0.02, dmax,
                               (1e-4 * scale if sgd_k else 2 * 4.48 * lr) + 1e-7, "(outliers %s)" % (
                                   {a: b for a, b in report.items() if b[0]}))
    print("concat -> MLP -> liGRU -> MLP: RMSprop sign-step outliers %s" % (
        {a: b for a, b in report.items() if b[0]}))
