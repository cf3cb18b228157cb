"""Drop-in run_nn (pkc.core.run_nn) end to end on synthetic Kaldi arks: train chunk -> .info + .pkl,
next-chunk hand-off, valid, forward -> posterior ark readable by the reference's reader layout."""
import configparser
import os

import numpy as np
import pytest
import torch

from oracle import loader as OL

pytestmark = pytest.mark.gpu


def write_data(d, seed, n_utt=24):
    from pkc import data_io as D
    rs = np.random.RandomState(seed)
    fea_ark, scp = os.path.join(d, "feats_%d.ark" % seed), os.path.join(d, "feats_%d.scp" % seed)
    ali = os.path.join(d, "ali_%d" % seed)
    os.makedirs(ali, exist_ok=True)
    with open(scp, "w") as f:
        for i in range(n_utt):
            k = "spk%d_u%03d" % (seed, i)
            T = rs.randint(30, 90)
            D.write_mat_path(fea_ark, (rs.randn(T, 40) + rs.randn(1, 40)).astype(np.float32), k,
                             append=i > 0)
            D.write_vec_int_path(os.path.join(ali, "ali_pdf.ark"), rs.randint(0, 64, T), k, append=i > 0)
            D.write_vec_int_path(os.path.join(ali, "ali_phones.ark"), rs.randint(1, 9, T), k,
                                 append=i > 0)
            f.write("%s %s\n" % (k, fea_ark))
    return scp, ali


def chunk_cfg(d, name, to_do, scp, ali, pretrain="none", counts=None):
    cfg = configparser.ConfigParser()
    cfg["exp"] = {"seed": "2234", "out_folder": d, "use_cuda": "True", "multi_gpu": "False",
                  "to_do": to_do, "out_info": os.path.join(d, name + ".info"), "save_gpumem": "False",
                  "production": "False", "run_nn_script": "run_nn.py"}
    cfg["batches"] = {"batch_size_train": "32", "batch_size_valid": "32",
                      "max_seq_length_train": "1000", "max_seq_length_valid": "1000"}
    cfg["data_chunk"] = {
        "fea": "fea_name=fmllr\nfea_lst=%s\nfea_opts=\ncw_left=5\ncw_right=5\n" % scp,
        "lab": "lab_name=lab_cd\nlab_folder=%s\nlab_opts=ali-to-pdf\n\n"
               "lab_name=lab_mono\nlab_folder=%s\nlab_opts=ali-to-phones --per-frame=true\n" % (ali, ali)}
    base = dict(arch_library="pkc.neural_networks", arch_class="MLP", arch_pretrain_file=pretrain,
                arch_freeze="False", arch_seq_model="False", dnn_use_laynorm_inp="False",
                dnn_use_batchnorm_inp="False", arch_opt="rmsprop", opt_momentum="0.0",
                opt_alpha="0.95", opt_eps="1e-8", opt_centered="False", opt_weight_decay="0.0")
    cfg["architecture1"] = dict(base, arch_name="MLP_layers1", dnn_lay="96,96", dnn_drop="0.15,0.15",
                                dnn_use_batchnorm="True,True", dnn_use_laynorm="False,False",
                                dnn_act="relu,relu", arch_lr="0.08", arch_opt="sgd",
                                opt_dampening="0.0", opt_nesterov="False")
    cfg["architecture2"] = dict(base, arch_name="MLP_layers2", dnn_lay="64", dnn_drop="0.0",
                                dnn_use_batchnorm="False", dnn_use_laynorm="False", dnn_act="softmax",
                                arch_lr="0.0004")
    cfg["architecture3"] = dict(cfg["architecture2"], arch_name="MLP_layers3", dnn_lay="8")
    cfg["model"] = {"model": "out_dnn1=compute(MLP_layers1,fmllr)\nout_dnn2=compute(MLP_layers2,out_dnn1)\n"
                             "out_dnn3=compute(MLP_layers3,out_dnn1)\nloss_mono=cost_nll(out_dnn3,lab_mono)\n"
                             "loss_mono_w=mult_constant(loss_mono,1.0)\nloss_cd=cost_nll(out_dnn2,lab_cd)\n"
                             "loss_final=sum(loss_cd,loss_mono_w)\nerr_final=cost_err(out_dnn2,lab_cd)"}
    cfg["forward"] = {"forward_out": "out_dnn2", "normalize_posteriors": "True",
                      "normalize_with_counts_from": counts or "none", "save_out_file": "True",
                      "require_decoding": "True"}
    path = os.path.join(d, name + ".cfg")
    with open(path, "w") as f:
        cfg.write(f)
    return path


def make_seq(path):
    """Turn a chunk cfg into a liGRU (2 x 32, bidirectional) body cfg."""
    cfg = configparser.ConfigParser()
    cfg.read(path)
    a1 = cfg["architecture1"]
    keep = {k: a1[k] for k in ("arch_name", "arch_pretrain_file", "arch_freeze", "arch_opt",
                               "opt_momentum", "opt_alpha", "opt_eps", "opt_centered",
                               "opt_weight_decay")}
    cfg["architecture1"] = dict(keep, arch_library="pkc.neural_networks", arch_class="liGRU",
                                arch_seq_model="True", arch_lr="0.0016", ligru_lay="32,32",
                                ligru_drop="0.2,0.2", ligru_use_laynorm_inp="False",
                                ligru_use_batchnorm_inp="False", ligru_use_laynorm="False,False",
                                ligru_use_batchnorm="True,True", ligru_bidir="True",
                                ligru_act="relu,relu", ligru_orthinit="True", arch_opt="rmsprop")
    cfg["batches"]["batch_size_train"] = "4"
    cfg["batches"]["batch_size_valid"] = "4"
    with open(path, "w") as f:
        cfg.write(f)
    return path


def test_run_nn_ligru_train_forward(tmp_path):
    from pkc.core import run_nn
    d = str(tmp_path)
    scp0, ali0 = write_data(d, 0)
    counts = os.path.join(d, "counts")
    with open(counts, "w") as f:
        f.write("[ " + " ".join(str(i + 3) for i in range(64)) + " ]\n")
    c_tr = make_seq(chunk_cfg(d, "train_ck0", "train", scp0, ali0))
    c_va = make_seq(chunk_cfg(d, "valid", "valid", scp0, ali0))
    data, _, _ = run_nn(None, None, None, None, None, None, c_tr, True, c_va)
    info = configparser.ConfigParser()
    info.read(os.path.join(d, "train_ck0.info"))
    assert 0 < float(info["results"]["loss"]) < 20
    c_fw = make_seq(chunk_cfg(d, "forward", "forward", scp0, ali0, counts=counts))
    cfg = configparser.ConfigParser()
    cfg.read(c_fw)
    for i in (1, 2, 3):
        cfg["architecture%d" % i]["arch_pretrain_file"] = os.path.join(d, "train_ck0_architecture%d.pkl" % i)
    with open(c_fw, "w") as f:
        cfg.write(f)
    run_nn(None, None, None, None, None, None, c_fw, True, c_fw)
    with open(os.path.join(d, "forward_out_dnn2_to_decode.ark"), "rb") as f:
        mats = OL.parse_mat_ark(f.read())
    assert len(mats) == 24
    c = np.arange(3, 67, dtype=np.float64)
    for k, m in mats:
        np.testing.assert_allclose(np.exp(m + np.log(c / c.sum())).sum(1), 1.0, rtol=1e-4)


def test_run_nn_train_valid_forward(tmp_path):
    from pkc.core import run_nn
    d = str(tmp_path)
    scp0, ali0 = write_data(d, 0)
    scp1, ali1 = write_data(d, 1)
    counts = os.path.join(d, "counts")
    with open(counts, "w") as f:
        f.write("[ " + " ".join(str(i + 3) for i in range(64)) + " ]\n")
    c_tr0 = chunk_cfg(d, "train_ck0", "train", scp0, ali0)
    c_tr1 = chunk_cfg(d, "train_ck1", "train", scp1, ali1)
    data, pats, pmasks = run_nn(None, None, None, None, None, None, c_tr0, True, c_tr1)
    info = configparser.ConfigParser()
    info.read(os.path.join(d, "train_ck0.info"))
    loss0 = float(info["results"]["loss"])
    assert np.isfinite(loss0) and 0 < loss0 < 20 and 0 <= float(info["results"]["err"]) <= 1
    pk = {a: os.path.join(d, "train_ck0_architecture%d.pkl" % i) for i, a in
          ((1, "MLP_layers1"), (2, "MLP_layers2"), (3, "MLP_layers3"))}
    for a, p in pk.items():
        ck = torch.load(p, weights_only=True)
        assert set(ck) == {"model_par", "optimizer_par"}
        assert ck["optimizer_par"]["param_groups"][0]["lr"] > 0
    # the returned chunk is the prefetched next one (chunk 1), already prepared on the GPU
    assert data[0][0].startswith("spk1_")
    c_tr1b = chunk_cfg(d, "train_ck1", "train", scp1, ali1)
    cfg = configparser.ConfigParser()
    cfg.read(c_tr1b)
    for i in (1, 2, 3):
        cfg["architecture%d" % i]["arch_pretrain_file"] = pk[["MLP_layers1", "MLP_layers2", "MLP_layers3"][i - 1]]
    with open(c_tr1b, "w") as f:
        cfg.write(f)
    c_va = chunk_cfg(d, "valid", "valid", scp0, ali0)
    data, _, _ = run_nn(*data, c_tr1b, False, c_va)
    info.read(os.path.join(d, "train_ck1.info"))
    assert np.isfinite(float(info["results"]["loss"]))
    # forward with the trained model -> posterior ark
    c_fw = chunk_cfg(d, "forward", "forward", scp0, ali0, counts=counts)
    cfg = configparser.ConfigParser()
    cfg.read(c_fw)
    for i, a in ((1, "MLP_layers1"), (2, "MLP_layers2"), (3, "MLP_layers3")):
        cfg["architecture%d" % i]["arch_pretrain_file"] = os.path.join(d, "train_ck1_architecture%d.pkl" % i)
    with open(c_fw, "w") as f:
        cfg.write(f)
    data, _, _ = run_nn(None, None, None, None, None, None, c_fw, True, c_fw)
    ark = os.path.join(d, "forward_out_dnn2_to_decode.ark")
    with open(ark, "rb") as f:
        mats = OL.parse_mat_ark(f.read())
    assert len(mats) == 24
    for k, m in mats:
        assert m.shape[1] == 64 and np.isfinite(m).all()
        # log-posteriors minus log prior: exp(m + logprior) sums to one per frame
        c = np.arange(3, 67, dtype=np.float64)
        p = np.exp(m + np.log(c / c.sum()))
        np.testing.assert_allclose(p.sum(1), 1.0, rtol=1e-4)
