"""CPU-only checks of the product's host side: the C ABI library loads and exports every symbol
declared in include/pkc.h, host-side mask generation and module construction match the reference
(golden vectors), and the host ark writer/reader is byte-compatible with data_io.write_mat."""
import configparser
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT
from cases import GHCGS, build_mlp_config

HDR = os.path.join(ROOT, "include", "pkc.h")


def G(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int64_t|int|const char\*)\s+(pkc_\w+)\(", txt, re.M)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "pkc_gemm" in syms and "pkc_optim_step" in syms and len(syms) >= 18


def test_library_exports_every_declared_symbol():
    from pkc import _lib
    lib = _lib.lib()
    for s in declared_symbols():
        assert hasattr(lib, s), s
    assert lib.pkc_abi_version() == _lib.ABI_VERSION == 9


def test_gemm_split_policy():
    from pkc import _lib
    lib = _lib.lib()
    for M, N, K in [(128, 1024, 1024), (128, 1928, 1024), (128, 48, 1024), (1024, 440, 128),
                    (7, 9, 5), (128, 1024, 440)]:
        s = lib.pkc_gemm_pick_splits(M, N, K)
        assert 1 <= s <= 16
        kchunk = -(-(-(-K // s)) // 32) * 32
        assert (s - 1) * kchunk < K      # every split owns a non-empty k range


HCGS = [((1024, 440), [128, 4], [25, 62.5], 1), ((1024, 1024), [128, 4], [25, 62.5], 2),
        ((512, 512), [32, 2], [75, 75], 3), ((512, 440), [32, 2], [75, 75], 4),
        ((550, 550), [64, 4], [50, 25], 5), ((550, 440), [64, 4], [50, 25], 6),
        ((100, 70), [16, 4], [50, 50], 7), ((64, 48), [16], [50], 8),
        ((96, 40), [32, 8, 2], [50, 50, 50], 9)]


@pytest.mark.parametrize("i", range(len(HCGS)))
def test_product_hcgs_mask_matches_reference(i):
    from pkc.cgs import hcgs_mask
    g = G("hcgs.npz")
    (r, c), bl, dr, seed = HCGS[i]
    m = hcgs_mask(r, c, bl, dr, rng=np.random.RandomState(seed))
    ref = np.unpackbits(g["m%d" % i])[:r * c].reshape(r, c)
    np.testing.assert_array_equal(m.astype(np.uint8), ref)


@pytest.mark.parametrize("variant", ["plain", "hcgs", "quant", "ln"])
def test_product_mlp_init_matches_reference(variant):
    """Same seed -> same weights, masks, BN buffers and state_dict keys as the reference."""
    from pkc.neural_networks import MLP
    g = G("mlp_%s.npz" % variant)
    cfg = build_mlp_config(variant)
    torch.manual_seed(2234)
    np.random.seed(2234)
    for sec, inp in (("architecture1", 40), ("architecture2", 32), ("architecture3", 32)):
        o = cfg[sec]
        net = MLP(o, inp)
        sd = net.state_dict()
        ref_keys = sorted(k.split("/", 2)[2] for k in g.files if k.startswith("init/%s/" % o["arch_name"]))
        assert sorted(sd.keys()) == ref_keys
        for k, v in sd.items():
            np.testing.assert_array_equal(v.numpy(), g["init/%s/%s" % (o["arch_name"], k)], err_msg=k)


@pytest.mark.parametrize("tag,cls,kind,F,seed", [
    ("ligru_bidir", "liGRU", "ligru", 20, 21), ("lstm", "LSTM", "lstm", 20, 23),
    ("lstm_hcgs_quant", "LSTM", "lstm_hq", 24, 24)])
def test_product_recurrent_init_matches_reference(tag, cls, kind, F, seed):
    import pkc.neural_networks as NN
    from cases import LIGRU_DEF, LSTM_DEF
    opts = {"ligru": LIGRU_DEF, "lstm": LSTM_DEF,
            "lstm_hq": dict(LSTM_DEF, lstm_hcgs="True", lstm_quant="True", lstm_quant_inp="True")}[kind]
    cp = configparser.ConfigParser()
    cp["s"] = {k: str(v) for k, v in opts.items()}
    g = G("rnn.npz")
    torch.manual_seed(seed)
    np.random.seed(seed)
    net = getattr(NN, cls)(cp["s"], F)
    sd = net.state_dict()
    ref_keys = sorted(k[len(tag) + 6:] for k in g.files if k.startswith(tag + "/init/"))
    assert sorted(sd) == ref_keys
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), g[tag + "/init/" + k], err_msg=k)


def test_ark_writer_bytes_match_reference(tmp_path):
    from pkc import data_io
    gi = G("post_inputs.npz")
    counts = gi["counts"].astype(np.float32)
    path = str(tmp_path / "post.ark")
    for i, (k, m) in enumerate(zip(["spkA_utt1", "spkB_utt2"], [gi["m0"], gi["m1"]])):
        data_io.write_mat_path(path, m - np.log(counts / np.sum(counts)), k, append=i > 0)
    with open(os.path.join(GOLDEN, "post.ark"), "rb") as f:
        ref = f.read()
    with open(path, "rb") as f:
        assert f.read() == ref


def test_ark_reader_roundtrip(tmp_path):
    from pkc import data_io
    rs = np.random.RandomState(0)
    mats = {"a_1": rs.randn(5, 7).astype(np.float32), "b_2": rs.randn(1, 7).astype(np.float32),
            "c_3": rs.randn(11, 7).astype(np.float32)}
    path = str(tmp_path / "f.ark")
    for i, (k, m) in enumerate(mats.items()):
        data_io.write_mat_path(path, m, k, append=i > 0)
    got = dict(data_io.read_mat_ark_path(path))
    assert list(got) == list(mats)
    for k in mats:
        np.testing.assert_array_equal(got[k], mats[k])


def test_product_ligru_hcgs_init_matches_oracle():
    """liGRU + HCGS (config C3, pkc extension reusing the LSTM hook): the product module draws
    its masks and weights in the same order as the oracle restatement."""
    import configparser
    import numpy as np
    import torch
    import pkc.neural_networks as NN
    from oracle import nets as ON
    from cases import LIGRU_DEF
    cp = configparser.ConfigParser()
    cp["s"] = dict(LIGRU_DEF, ligru_hcgs="True", hcgsx_block="8,4", hcgsx_sparse="50,50",
                   hcgsh_block="8,4", hcgsh_sparse="25,50")
    sds = []
    for cls in (NN.liGRU, ON.liGRU):
        torch.manual_seed(9)
        np.random.seed(9)
        sds.append(cls(cp["s"], 20).state_dict())
    assert sds[0].keys() == sds[1].keys()
    assert any("hcgsx" in k for k in sds[0])
    for k in sds[0]:
        assert torch.equal(sds[0][k], sds[1][k]), k


@pytest.mark.parametrize("i", range(len(GHCGS)))
def test_product_guided_mask_matches_reference(i):
    """guided_hcgs.conn_mat known answers (AvgPool2d float32 block means, argsort selection)."""
    from pkc.cgs import guided_hcgs_mask
    g = G("ghcgs.npz")
    (r, c), bl, dr = GHCGS[i]
    np.testing.assert_array_equal(guided_hcgs_mask(r, c, bl, dr, g["w%d" % i]), g["mask%d" % i])


@pytest.mark.parametrize("cls", ["MLP", "LSTM"])
def test_product_guided_init_matches_oracle(cls):
    """guided_hcgs=True: the guidedHCGS mask Parameters are built from the initial W / U under
    the reference's names, and apply_ghcgs regenerates them from the current weights."""
    import pkc.neural_networks as NN
    from oracle import nets as ON
    from cases import LSTM_DEF, MLP_DEF
    cp = configparser.ConfigParser()
    if cls == "MLP":
        cp["s"] = dict(MLP_DEF, dnn_lay="64,32", dnn_drop="0,0", dnn_use_batchnorm="True,True",
                       dnn_use_laynorm="False,False", dnn_act="relu,relu", guided_hcgs="True",
                       hcgs_block="16,4", hcgs_sparse="50,50")
    else:
        cp["s"] = dict(LSTM_DEF, guided_hcgs="True", hcgsx_block="8,4", hcgsx_sparse="50,50",
                       hcgsh_block="8", hcgsh_sparse="75")
    nets = []
    for c in (getattr(NN, cls), getattr(ON, cls)):
        torch.manual_seed(4)
        np.random.seed(4)
        nets.append(c(cp["s"], 40 if cls == "MLP" else 20))
    sds = [n.state_dict() for n in nets]
    assert sds[0].keys() == sds[1].keys()
    assert any("ghcgs" in k for k in sds[0])
    for k in sds[0]:
        assert torch.equal(sds[0][k], sds[1][k]), k
    for n in nets:                       # new weights -> regenerated masks agree
        torch.manual_seed(5)
        for pn, p in n.named_parameters():
            if "mask" not in pn:
                p.data.normal_()
    nets[0].apply_ghcgs()
    nets[1].apply_ghcgs()
    for k, v in nets[0].state_dict().items():
        if "ghcgs" in k:
            assert torch.equal(v, nets[1].state_dict()[k]), k


@pytest.mark.parametrize("case", ["gru_bidir", "gru_uni_nobn", "mingru_bidir", "mingru_uni_nobn",
                                  "rnn_bidir", "rnn_uni_nobn"])
def test_product_gru_init_matches_reference(case):
    import pkc.neural_networks as NN
    from cases import GRU_CASES, PLAIN_CASES
    allc = [(t, "GRU", o, T, B, F, sd) for t, o, T, B, F, sd in GRU_CASES] + PLAIN_CASES
    tag, cls, opts, T, B, F, seed = [c for c in allc if c[0] == case][0]
    cp = configparser.ConfigParser()
    cp["s"] = {k: str(v) for k, v in opts.items()}
    g = G("gru.npz")
    torch.manual_seed(seed)
    np.random.seed(seed)
    sd = getattr(NN, cls)(cp["s"], F).state_dict()
    ref_keys = sorted(k[len(tag) + 6:] for k in g.files if k.startswith(tag + "/init/"))
    assert sorted(sd) == ref_keys
    for k, v in sd.items():
        np.testing.assert_array_equal(v.numpy(), g[tag + "/init/" + k], err_msg=k)


def test_product_cm_decode_matches_reference(tmp_path):
    """Kaldi CM compressed feature matrices (data_io.py:729-766) through the C ABI, from an ark
    file and from pipe bytes."""
    from pkc import data_io as D
    g = G("cm.npz")
    ark = b""
    for i in range(3):
        ark += b"utt%d \0BCM " % i + g["blob%d" % i].tobytes()
    path = str(tmp_path / "cm.ark")
    open(path, "wb").write(ark)
    got = list(D.read_mat_ark_path(path))
    assert [k for k, _ in got] == ["utt0", "utt1", "utt2"]
    for i, (_, m) in enumerate(got):
        np.testing.assert_array_equal(m, g["mat%d" % i])
    for i, (_, m) in enumerate(D.parse_mat_ark_bytes(ark)):
        np.testing.assert_array_equal(m, g["mat%d" % i])


@pytest.mark.parametrize("tag", ["mat", "vec", "mixed"])
def test_product_text_ark_matches_reference(tag, tmp_path):
    """Text-form (`ark,t:`) Kaldi arks (data_io.py:680-681 + 714-726 for matrices, 446-453 for int
    vectors), and a mixed ark whose text entries sit between binary FM / DM ones: the pkc readers
    (file path and pipe bytes) return exactly what the reference's read_mat_ark /
    read_vec_int_ark returned on the same bytes (golden text_ark.npz, float32 values bit-equal)."""
    from pkc import data_io as D
    g = G("text_ark.npz")
    blob = g[tag + "_bytes"].tobytes()
    keys = list(g[tag + "_keys"])
    path = str(tmp_path / "t.ark")
    open(path, "wb").write(blob)
    if tag == "vec":
        runs = [list(D.read_vec_int_ark_path(path)), list(D.parse_vec_int_ark_bytes(blob))]
    else:
        runs = [list(D.read_mat_ark_path(path)), D.parse_mat_ark_bytes(blob)]
    for got in runs:
        assert [k for k, _ in got] == keys
        for i, (_, v) in enumerate(got):
            ref = g["%s_%d" % (tag, i)]
            if tag == "vec":
                assert v.dtype == np.int32
                np.testing.assert_array_equal(v, ref)
            else:
                assert v.dtype == np.float32
                np.testing.assert_array_equal(v, ref.astype(np.float32))
                assert np.signbit(v).tolist() == np.signbit(ref.astype(np.float32)).tolist()


@pytest.mark.parametrize("tag", ["a", "b", "c", "d"])
def test_product_kmeans_pattern_search_matches_reference(tag):
    """pkc.cgs.kmeans_patterns vs sparsity.find_top_k_by_kmeans (sparsity.py:999-1049), both with
    sklearn KMeans seeded (random_state=0): candidates with ties (case c), ragged tiles (b) and a
    pattern_num capped at C(ph*pw, nnz) (d) give the reference's pattern set exactly."""
    from pkc.cgs import kmeans_patterns
    g = G("kmeans.npz")
    num, ph, pw, nnz = (int(v) for v in g[tag + "_args"])
    k = kmeans_patterns(torch.from_numpy(g[tag + "_w"]), num, [ph, pw], nnz, random_state=0)
    np.testing.assert_array_equal(k, g[tag + "_kernel"])
    assert (k.reshape(k.shape[0], -1).sum(1) == nnz).all()


def test_dropin_core_module_replaces_run_nn(tmp_path):
    """pytorch-kaldi-cgs_amd/dropin/core.py ahead of a reference checkout on sys.path: run_exp's
    `importlib.import_module('core')` (run_exp.py:81-83) gets pkc's run_nn and every other name of
    the reference's core.py (a stand-in file here, so the test needs no reference)."""
    import importlib
    import subprocess
    import sys
    ref = tmp_path / "ref"
    ref.mkdir()
    (ref / "core.py").write_text("def run_nn(*a):\n    return 'reference'\n"
                                 "def read_next_chunk_into_shared_list_with_subprocess():\n"
                                 "    return 'helper'\n")
    code = ("import importlib, sys; m = importlib.import_module('core'); "
            "import pkc.core; assert m.run_nn is pkc.core.run_nn; "
            "assert m.read_next_chunk_into_shared_list_with_subprocess() == 'helper'; print('ok')")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([
        os.path.join(ROOT, "pytorch-kaldi-cgs_amd", "dropin"), os.path.join(ROOT, "pytorch-kaldi-cgs_amd"),
        str(ref)]))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       cwd=str(tmp_path))
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]


def test_sync_bn_refuses_per_rank_batchnorm():
    """[exp] sync_bn synchronises the MLP layers' BatchNorm only: an input BatchNorm
    (dnn_use_batchnorm_inp) would keep per-rank statistics, so the engine refuses it instead of
    silently breaking the R-ranks-equal-one-process recipe."""
    from pkc.engine import Engine, parse_model
    from pkc.neural_networks import MLP
    cfg = build_mlp_config("plain")
    cfg["architecture1"]["dnn_use_batchnorm_inp"] = "True"
    torch.manual_seed(0)
    nets = {cfg[s]["arch_name"]: MLP(cfg[s], k) for s, k in
            (("architecture1", 40), ("architecture2", 32), ("architecture3", 32))}
    opts = {cfg[s]["arch_name"]: cfg[s] for s in ("architecture1", "architecture2", "architecture3")}

    class Sync:
        world, rank = 2, 0

    with pytest.raises(NotImplementedError, match="input BatchNorm"):
        Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fmllr": (0, 40)},
               ["lab_cd", "lab_mono"], batch=8, device="cpu", sync_bn=Sync())


def test_quantcheck_flip_bound():
    """The flip-count helper of the quantised-config GPU tests: summation-order noise near a grid
    boundary moves few weights by one quantum; an off-by-one quantiser moves most of them."""
    from quantcheck import grid_index, quantum_flips
    rs = np.random.RandomState(0)
    w = rs.uniform(-0.99, 0.99, size=(64, 64)).astype(np.float32)
    assert quantum_flips(w, w) == (0, 0.0)
    k = grid_index(w)
    near = np.clip(w, -1, 1) * 128
    e = w.copy()
    e[0, 0] = np.float32(np.sign(w[0, 0]) * (np.floor(abs(near[0, 0])) / 128))   # onto the boundary
    assert quantum_flips(e, w)[1] <= 1.0
    shifted = (np.sign(w) * (np.abs(np.clip(w, -1, 1)) + 1.0 / 128)).astype(np.float32)
    n, dmax = quantum_flips(shifted, w)
    assert n > 0.9 * w.size and dmax == 1.0
    assert (np.abs(k) <= 128).all()


def test_forward_update_placement_respects_deadlines():
    """PKC_OPT_FWD: Engine._place_fwd_opt puts each weight update of step k into a launch of
    step k+1's forward BEFORE the first launch that reads that node's parameters (the gather launch
    = key None, then one launch per matmul node; two heads reading the same tensor share one), at
    most 8 operations per launch, balanced by bytes.  Host logic only (mock nodes)."""
    from pkc.engine import Engine

    class NS:                         # hashable by identity, like the engine's node objects
        def __init__(self, **kw):
            self.__dict__.update(kw)
    fea = ("fea", 0)
    body = []
    src = fea
    for i in range(5):
        n = NS(name="L%d" % i, rec=False, W=object(), head=False, src=src)
        body.append(n)
        src = ("node", n)
    heads = [NS(name="H%d" % i, rec=False, W=object(), head=True, src=src) for i in range(2)]
    nodes = body + heads
    ops = []
    for n in nodes:
        for part in range(2 if n in body else 3):
            ops.append((n, ("opt %s [%d]" % (n.name, part), 0.0, 7e6 if n in body else 15e6, None)))
    slots = Engine._place_fwd_opt(NS(nodes=nodes), ops)
    order = [None] + body + [heads[0]]
    seen = {}
    for pos, key in enumerate(order):
        for op in slots.get(key, []):
            seen[op[0]] = pos
        assert len(slots.get(key, [])) + (2 if key is heads[0] else 1) <= 8
    assert len(seen) == len(ops)
    for n, op in ops:
        first = order.index(heads[0] if n in heads else n)
        assert seen[op[0]] < first, (op[0], seen[op[0]], first)
    # the gather launch takes layer 0's update (nothing else can) and the load is spread
    assert any(op[0].startswith("opt L0") for op in slots[None])
    assert len([k for k in slots if slots[k]]) >= 4
