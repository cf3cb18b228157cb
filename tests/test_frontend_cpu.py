"""Kaldi feature front-end, host side (no GPU): fea_opts parsing, the CMVN statistics archive
readers, and the host-computed tables (ApplyCmvn offsets / scales, DeltaFeatures windows) against
the plain-C oracle restatement (oracle/kaldi_feat.c; parity unpinned against Kaldi itself)."""
import numpy as np
import pytest

from oracle import kaldi_feat as OK
from pkc import data_io as D
from pkc import frontend as F

import frontend_data as FD


@pytest.mark.parametrize("order,window", [(0, 2), (1, 2), (2, 2), (3, 2), (2, 1), (2, 3), (7, 2)])
def test_delta_scales_match_oracle(order, window):
    got, maxoff = F.delta_scales(order, window)
    assert maxoff == order * window
    assert got.tobytes() == OK.delta_scales(order, window).tobytes()


def test_delta_scales_known_values():
    # the add-deltas windows every Kaldi recipe uses (order 2, window 2)
    tab, _ = F.delta_scales(2, 2)
    np.testing.assert_allclose(tab[1, 2:7], [-0.2, -0.1, 0, 0.1, 0.2], rtol=1e-6)
    np.testing.assert_allclose(tab[2], [.04, .04, .01, -.04, -.1, -.04, .01, .04, .04], rtol=1e-5,
                               atol=1e-8)


@pytest.mark.parametrize("norm_vars", [False, True])
def test_cmvn_norm_matches_oracle(norm_vars):
    _, _, stats, _ = FD.make()
    for s in stats.values():
        a, b = F.cmvn_norm(s, norm_vars), OK.cmvn_norm(s, norm_vars)
        assert a[0].tobytes() == b[0].tobytes() and a[1].tobytes() == b[1].tobytes()


def test_cmvn_norm_errors():
    with pytest.raises(ValueError):
        F.cmvn_norm(np.zeros((2, 5)), False)         # count < 1 (KALDI_ERR in ApplyCmvn)


@pytest.mark.parametrize("text", [False, True])
def test_parse_pipe_and_stats(tmp_path, text):
    _, u2s, stats, _ = FD.make()
    cm, us = FD.write_files(str(tmp_path), stats, u2s, text_stats=text)
    opts = FD.fea_opts(cm, us, order=2)
    assert F.is_native_pipe(opts)
    fe = F.FeaFrontend.parse(opts)
    assert fe.order == 2 and fe.window == 2 and not fe.cmvn["norm_vars"]
    assert fe.cmvn["utt2spk"] == u2s
    for k, m in stats.items():
        np.testing.assert_array_equal(fe.cmvn["stats"][k], m)
    assert fe.out_dim(13) == 39
    fe0 = F.FeaFrontend.parse(FD.fea_opts(cm, us, order=0, norm_vars=True))
    assert fe0.order == 0 and fe0.cmvn["norm_vars"]


def test_parse_rejects_unknown_stages(tmp_path):
    _, u2s, stats, _ = FD.make()
    cm, us = FD.write_files(str(tmp_path), stats, u2s)
    assert not F.is_native_pipe("splice-feats --left-context=3 ark:- ark:- |")
    with pytest.raises(NotImplementedError):
        F.FeaFrontend.parse("splice-feats ark:- ark:- |")
    with pytest.raises(NotImplementedError):
        F.FeaFrontend.parse("add-deltas --bogus=1 ark:- ark:- |")
    with pytest.raises(ValueError):
        F.FeaFrontend.parse("apply-cmvn --norm-means=false --norm-vars=true ark:%s ark:- ark:- |" % cm)
    assert F.FeaFrontend.parse("") is None


def test_norm_tables_drop_utterances_without_stats(tmp_path):
    fea, u2s, stats, _ = FD.make()
    cm, us = FD.write_files(str(tmp_path), stats, u2s)
    fe = F.FeaFrontend.parse(FD.fea_opts(cm, us))
    kept, norm, idx, mode = fe.norm_tables(sorted(fea), 13)
    assert "spkX_u999" not in kept and "spk1_nolab" in kept and mode == 1
    assert norm.shape == (4, 2, 13)
    for k, i in zip(kept, idx):
        off, sc = OK.cmvn_norm(stats[u2s[k]], False)
        assert norm[i, 0].tobytes() == off.tobytes()


@pytest.mark.parametrize("max_seq", [-1, 40])
def test_frontend_row_maps(max_seq):
    """The row maps the GPU kernel reads reproduce the sorted / split layout of load_dataset: the
    source frame of output row r, looked up through them, is the r-th frame load_dataset emits."""
    fea, _, _, lab = FD.make()
    names, pieces, labs, end = D.dataset_pieces({k: len(v) for k, v in fea.items()}, [lab], max_seq)
    fe = F.FeaFrontend()
    fe.order = 0
    fa = D.frontend_args(fea, pieces, fe)
    srow, urow, ubeg, uend = fa["arrays"][:4]
    names2, raw2, labs2, end2 = D.load_dataset(fea, [lab], max_seq)
    np.testing.assert_array_equal(fa["raw"][srow], raw2)
    assert names == names2 and (end == end2).all() and (labs[0] == labs2[0]).all()
    assert np.all(srow >= ubeg[urow]) and np.all(srow < uend[urow])


@pytest.mark.parametrize("max_seq", [-1, 40, 25])
def test_load_dataset_split_order_matches_oracle(max_seq):
    """pkc's load_dataset == data_io.load_dataset restated (oracle, golden-pinned) with pieces
    split by max_seq_length: frames / labels / end_index in the re-sorted order, names in the
    order of the first sort (the reference re-sorts the data but not snt_name)."""
    from oracle import loader as OL
    fea, _, _, lab = FD.make(seed=11)
    n1, raw1, l1, e1 = D.load_dataset(fea, [lab], max_seq)
    n2, raw2, l2, e2 = OL.load_dataset(fea, lab, max_seq)
    assert n1 == n2
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_array_equal(raw1, raw2)
    np.testing.assert_array_equal(l1[0], l2)
