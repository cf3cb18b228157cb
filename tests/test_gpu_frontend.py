"""Kaldi feature front-end on the GPU (pkc_feat_frontend) vs the plain-C oracle restatement of
apply-cmvn / add-deltas (oracle/kaldi_feat.c), bit for bit, through the chunk staging of the
loader (sorted / split utterance order, deltas across split points, dropped utterances), and end
to end through pkc.core.read_lab_fea with the shipped cfgs' fea_opts pipe.  Parity against Kaldi
itself is unpinned (Kaldi is not in the reference or the image)."""
import configparser
import os

import numpy as np
import pytest
import torch

import frontend_data as FD
from oracle import kaldi_feat as OK
from oracle import loader as OL

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("order", [0, 2, 3])
@pytest.mark.parametrize("norm_vars", [False, True])
@pytest.mark.parametrize("max_seq", [-1, 40])
def test_frontend_matches_oracle(tmp_path, order, norm_vars, max_seq):
    from pkc import data_io as D
    from pkc import frontend as F
    fea, u2s, stats, lab = FD.make(seed=order * 7 + int(norm_vars))
    cm, us = FD.write_files(str(tmp_path), stats, u2s)
    fe = F.FeaFrontend.parse(FD.fea_opts(cm, us, order=order, norm_vars=norm_vars))
    st = D.stage_chunk(fea, [lab], max_seq, frontend=fe)
    torch.cuda.current_stream().wait_event(st.done)
    got = st.raw_d.cpu().numpy()
    proc = OK.pipeline(fea, stats, u2s, norm_vars=norm_vars, order=order)
    names, ref, _, end = OL.load_dataset(proc, lab, max_seq)
    assert st.names == names
    np.testing.assert_array_equal(st.end_index, end)
    assert got.shape == ref.shape == (ref.shape[0], 13 * (order + 1))
    assert np.array_equal(got.view(np.uint32), ref.astype(np.float32).view(np.uint32))


def test_frontend_large_chunk_property():
    """TIMIT-sized chunk (740 utterances, 40-dim, order 2): the first-order block of an utterance's
    interior frame is the window-2 regression of the cmvn'd static block around it (checked on a
    sample against the oracle), and every row is finite."""
    from pkc import data_io as D
    from pkc import frontend as F
    rs = np.random.RandomState(5)
    fea = {"s%02d_u%04d" % (i % 50, i): rs.randn(rs.randint(150, 450), 40).astype(np.float32)
           for i in range(740)}
    u2s = {k: k.split("_")[0] for k in fea}
    stats = {}
    for spk in set(u2s.values()):
        x = np.concatenate([fea[k] for k in fea if u2s[k] == spk]).astype(np.float64)
        s = np.zeros((2, 41))
        s[0, :40], s[1, :40], s[0, 40] = x.sum(0), (x * x).sum(0), len(x)
        stats[spk] = s
    fe = F.FeaFrontend()
    fe.cmvn = dict(stats=stats, utt2spk=u2s, norm_vars=False, norm_means=True)
    fe.order = 2
    st = D.stage_chunk(fea, [], 1000, frontend=fe)
    torch.cuda.current_stream().wait_event(st.done)
    got = st.raw_d.cpu().numpy()
    assert got.shape == (sum(len(v) for v in fea.values()), 120) and np.isfinite(got).all()
    sample = sorted(fea)[::97]
    proc = OK.pipeline({k: fea[k] for k in sample}, stats, u2s, order=2)
    for k in sample:
        i = st.names.index(k)
        b = st.end_index[i - 1] if i else 0
        assert np.array_equal(got[b:st.end_index[i]], proc[k])


def _cfg(d, scp, ali, fea_opts):
    cfg = configparser.ConfigParser()
    cfg["exp"] = {"seed": "2234", "out_folder": d, "use_cuda": "True", "to_do": "train",
                  "out_info": os.path.join(d, "c.info"), "run_nn_script": "run_nn.py"}
    cfg["batches"] = {"batch_size_train": "16", "max_seq_length_train": "1000"}
    cfg["data_chunk"] = {
        "fea": "fea_name=mfcc\nfea_lst=%s\nfea_opts=%s\ncw_left=2\ncw_right=2\n" % (scp, fea_opts),
        "lab": "lab_name=lab_cd\nlab_folder=%s\nlab_opts=ali-to-pdf\n" % ali}
    cfg["architecture1"] = dict(arch_name="MLP_layers1", arch_seq_model="False")
    cfg["model"] = {"model": "out_dnn1=compute(MLP_layers1,mfcc)\nloss_final=cost_nll(out_dnn1,lab_cd)"}
    path = os.path.join(d, "c.cfg")
    with open(path, "w") as f:
        cfg.write(f)
    return path


def test_read_lab_fea_with_cmvn_deltas_pipe(tmp_path):
    """pkc.core.read_lab_fea on a cfg whose fea_opts is the shipped `apply-cmvn --utt2spk ... |
    add-deltas --delta-order=2` pipe == the oracle loader (read_lab_fea, frame shuffle included)
    over the oracle front-end's output."""
    from pkc import core
    from pkc import data_io as D
    d = str(tmp_path)
    fea, u2s, stats, lab = FD.make(seed=3)
    cm, us = FD.write_files(d, stats, u2s)
    ark, scp, ali = os.path.join(d, "f.ark"), os.path.join(d, "f.scp"), os.path.join(d, "ali")
    os.makedirs(ali)
    with open(scp, "w") as f:
        for i, (k, m) in enumerate(fea.items()):
            D.write_mat_path(ark, m, k, append=i > 0)
            f.write("%s %s\n" % (k, ark))
    for i, (k, v) in enumerate(lab.items()):
        D.write_vec_int_path(os.path.join(ali, "ali_pdf.ark"), v, k, append=i > 0)
    cfg = _cfg(d, scp, ali, FD.fea_opts(cm, us, order=2))
    shared = []
    np.random.seed(2234)
    core.read_lab_fea(cfg, False, shared, d)
    out = core._finish_chunk(shared)
    ch = out[1]
    proc = OK.pipeline(fea, stats, u2s, order=2)
    names, end, fcols, lcols, ref = OL.read_lab_fea([("mfcc", proc, 2, 2)], [("lab_cd", lab)], False,
                                                    rng=np.random.RandomState(2234))
    assert ch.names == names
    np.testing.assert_array_equal(ch.end_index, end)
    C_ = 39 * 5
    assert ch.feats.shape == (ref.shape[0], C_)
    np.testing.assert_allclose(ch.feats.cpu().numpy(), ref[:, :C_].astype(np.float32), rtol=1e-6,
                               atol=1e-6)
    np.testing.assert_array_equal(ch.labels.cpu().numpy()[:, 0], ref[:, C_].astype(np.int32))
