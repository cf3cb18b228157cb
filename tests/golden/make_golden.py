"""Generate golden vectors by importing the *reference* (hellboywyh/pytorch-kaldi-CGS) on CPU.

Runs ONLY in the build container (where /root/reference exists).  Only data leaves: every
fixture is an .npz of inputs and expected outputs (plus one .bin of ark bytes).  No reference
source or bytecode is copied.  Shims used (all monkeypatches of *this* process only):

  * torch.Tensor.cuda -> identity           (reference hard-codes .cuda(), e.g. sparsity.py:1045)
  * hcgs.conn_mat(...) -> for_test=True path (hcgs.py:134-137 returns numpy instead of .to("cuda"))
  * data_io.read_mat_ark / read_vec_int_ark -> synthetic dicts  (Kaldi binaries are absent)
  * neural_networks.liGRU.{prune, guided_hcgs, if_pattern} = False (class attributes core.run_nn
    reads and the reference's liGRU never defines; only for the run_nn golden cases)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import configparser
import os
import sys
import tempfile

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

torch.Tensor.cuda = lambda t, *a, **k: t          # noqa: E731  (CPU-only container)

import data_io            # noqa: E402
import hcgs               # noqa: E402
import neural_networks    # noqa: E402
import quantized_modules  # noqa: E402
import utils              # noqa: E402
from sparsity import sparsity  # noqa: E402

sys.path.insert(0, OUT)
from cases import (LIGRU_DEF, LSTM_DEF, MLP_DEF, RUN_NN_CASES, build_mlp_config,  # noqa: E402,F401
                   run_nn_cfg)

_TMP = tempfile.mkdtemp(prefix="pkc_golden_")
_orig_conn_mat = hcgs.conn_mat


def _conn_mat_cpu(n_in, n_out, block_sizes, drop_ratios, mat_num="1", *a, **k):
    return torch.from_numpy(_orig_conn_mat(n_in, n_out, block_sizes, drop_ratios, mat_num,
                                           dir=_TMP, for_test=True))


hcgs.conn_mat = _conn_mat_cpu


def synth_utts(rs, n_utt, lmin, lmax, dim=40, n_cd=1928, n_mono=48, cd_min=0):
    names = ["utt%03d" % rs.randint(0, 1000) + "_%d" % i for i in range(n_utt)]
    fea, cd, mono = {}, {}, {}
    for n in names:
        T = rs.randint(lmin, lmax + 1)
        off = rs.normal(0, 0.3, size=(1, dim))
        fea[n] = (rs.normal(0, 1, size=(T, dim)) + off).astype(np.float32)
        cd[n] = rs.randint(cd_min, n_cd, size=T).astype(np.int32)
        mono[n] = rs.randint(1, n_mono + 1, size=T).astype(np.int32)
    return names, fea, cd, mono


def pack_dict(prefix, d, out):
    keys = sorted(d.keys())
    out[prefix + "_keys"] = np.array(keys)
    out[prefix + "_lens"] = np.array([len(d[k]) for k in keys], dtype=np.int64)
    out[prefix + "_data"] = np.concatenate([d[k] for k in keys])


# ----------------------------------------------------------------------------------------------
# G1: loader (data_io.load_dataset / context_window / load_chunk / read_lab_fea)
# ----------------------------------------------------------------------------------------------
def gen_loader():
    out = {}
    rs = np.random.RandomState(11)
    names, fea, cd, mono = synth_utts(rs, 5, 6, 24, cd_min=3)
    # a feature-only utterance with no alignment (must be dropped, data_io.py:20-24)
    fea["zz_noali"] = rs.normal(size=(12, 40)).astype(np.float32)
    pack_dict("fea", fea, out)
    pack_dict("cd", cd, out)
    pack_dict("mono", mono, out)

    cur = {}

    def fake_read_mat_ark(spec, output_folder):
        for k, v in cur["fea"].items():
            yield k, v

    def fake_read_vec_int_ark(spec, output_folder):
        src = cur["mono"] if "phones" in spec else cur["cd"]
        for k, v in src.items():
            yield k, v

    data_io.read_mat_ark = fake_read_mat_ark
    data_io.read_vec_int_ark = fake_read_vec_int_ark
    cur.update(fea=fea, cd=cd, mono=mono)
    cases = {"A": (5, 5, -1), "B": (2, 1, 8), "C": (0, 0, 10), "D": (3, 3, 1000)}
    fea13 = {k: v[:, :13].copy() for k, v in fea.items()}
    pack_dict("fea13", fea13, out)
    for tag, (L, R, msl) in cases.items():
        cur["fea"] = fea if tag == "A" else fea13
        name, ds, end = data_io.load_chunk("x.scp", "", "alidir", "ali-to-pdf", L, R, msl, _TMP)
        out["chunk%s_names" % tag] = np.array(name)
        out["chunk%s_data" % tag] = ds.astype(np.float32)
        out["chunk%s_end" % tag] = np.asarray(end)
        out["chunk%s_cfg" % tag] = np.array([L, R, msl])

    # full read_lab_fea with two label streams (cd + mono), non-sequential -> shuffled
    cfg = configparser.ConfigParser()
    cfg["exp"] = {"to_do": "train", "seed": "2234"}
    cfg["batches"] = {"max_seq_length_train": "1000"}
    cfg["data_chunk"] = {
        "fea": "fea_name=fmllr\nfea_lst=x.scp\nfea_opts=\ncw_left=5\ncw_right=5\n",
        "lab": "lab_name=lab_cd\nlab_folder=alidir\nlab_opts=ali-to-pdf\n\n"
               "lab_name=lab_mono\nlab_folder=alidir\nlab_opts=ali-to-phones --per-frame=true\n"}
    cfg["architecture1"] = {"arch_name": "MLP_layers1", "arch_seq_model": "False"}
    cfg["model"] = {"model": "out_dnn1=compute(MLP_layers1,fmllr)\n"
                             "loss_cd=cost_nll(out_dnn1,lab_cd)\nloss_mono=cost_nll(out_dnn1,lab_mono)"}
    cfg_path = os.path.join(_TMP, "chunk.cfg")
    with open(cfg_path, "w") as f:
        cfg.write(f)
    for seq, tag in ((False, "nonseq"), (True, "seq")):
        cur["fea"] = fea
        cfg["architecture1"]["arch_seq_model"] = str(seq)
        with open(cfg_path, "w") as f:
            cfg.write(f)
        np.random.seed(2234)
        shared = []
        data_io.read_lab_fea(cfg_path, False, shared, _TMP)
        out["rlf_%s_names" % tag] = np.array(shared[0])
        out["rlf_%s_end" % tag] = np.asarray(shared[1])
        out["rlf_%s_data" % tag] = shared[5].astype(np.float32)
        out["rlf_%s_feacols" % tag] = np.array(shared[2]["fmllr"][5:8], dtype=np.int64)
        out["rlf_%s_labcols" % tag] = np.array([shared[3]["lab_cd"][3], shared[3]["lab_mono"][3]])
    np.savez_compressed(os.path.join(OUT, "loader.npz"), **out)


# multi-stream chunks (data_io.py:184-263): three feature streams of different widths and context
# windows (the TIMIT_mfcc_fbank_fmllr_liGRU_best.cfg shape), column-stacked after a per-stream
# trim to the widest window, labels (cd + mono) after all features
MULTI_STREAMS = (("mfcc", 13, 2, 1), ("fbank", 23, 0, 0), ("fmllr", 40, 5, 3))


def gen_loader_multi():
    out = {}
    rs = np.random.RandomState(12)
    names, fea0, cd, mono = synth_utts(rs, 6, 9, 30, cd_min=2)
    streams = {}
    for name, dim, _, _ in MULTI_STREAMS:
        streams[name] = {k: (rs.normal(0, 1, size=(len(v), dim)) * (1 + 0.1 * dim) +
                             rs.normal(0, 0.5, size=(1, dim))).astype(np.float32)
                         for k, v in fea0.items()}
        pack_dict("fea_" + name, streams[name], out)
    pack_dict("cd", cd, out)
    pack_dict("mono", mono, out)

    def fake_read_mat_ark(spec, output_folder):
        name = next(n for n, _, _, _ in MULTI_STREAMS if "feats_%s.scp" % n in spec)
        for k, v in streams[name].items():
            yield k, v

    def fake_read_vec_int_ark(spec, output_folder):
        src = mono if "phones" in spec else cd
        for k, v in src.items():
            yield k, v

    data_io.read_mat_ark = fake_read_mat_ark
    data_io.read_vec_int_ark = fake_read_vec_int_ark
    cfg = configparser.ConfigParser()
    cfg["exp"] = {"to_do": "train", "seed": "2234"}
    cfg["batches"] = {"max_seq_length_train": "1000"}
    cfg["data_chunk"] = {
        "fea": "\n".join("fea_name=%s\nfea_lst=feats_%s.scp\nfea_opts=\ncw_left=%d\ncw_right=%d\n"
                         % (n, n, l, r) for n, _, l, r in MULTI_STREAMS),
        "lab": "lab_name=lab_cd\nlab_folder=alidir\nlab_opts=ali-to-pdf\n\n"
               "lab_name=lab_mono\nlab_folder=alidir\nlab_opts=ali-to-phones --per-frame=true\n"}
    cfg["architecture1"] = {"arch_name": "MLP_layers1", "arch_seq_model": "False"}
    cfg["model"] = {"model": "conc1=concatenate(mfcc,fbank)\nconc2=concatenate(conc1,fmllr)\n"
                             "out_dnn1=compute(MLP_layers1,conc2)\n"
                             "loss_cd=cost_nll(out_dnn1,lab_cd)\nloss_mono=cost_nll(out_dnn1,lab_mono)"}
    cfg_path = os.path.join(_TMP, "chunk_multi.cfg")
    for seq, tag in ((False, "nonseq"), (True, "seq")):
        cfg["architecture1"]["arch_seq_model"] = str(seq)
        with open(cfg_path, "w") as f:
            cfg.write(f)
        np.random.seed(2234)
        shared = []
        data_io.read_lab_fea(cfg_path, False, shared, _TMP)
        out["rlf_%s_names" % tag] = np.array(shared[0])
        out["rlf_%s_end" % tag] = np.asarray(shared[1])
        out["rlf_%s_data" % tag] = shared[5].astype(np.float32)
        out["rlf_%s_feacols" % tag] = np.array([shared[2][n][5:8] for n, _, _, _ in MULTI_STREAMS],
                                               dtype=np.int64)
        out["rlf_%s_labcols" % tag] = np.array([shared[3]["lab_cd"][3], shared[3]["lab_mono"][3]])
    out["streams"] = np.array([[d, l, r] for _, d, l, r in MULTI_STREAMS], dtype=np.int64)
    out["stream_names"] = np.array([n for n, _, _, _ in MULTI_STREAMS])
    np.savez_compressed(os.path.join(OUT, "loader_multi.npz"), **out)


# ----------------------------------------------------------------------------------------------
# G2: HCGS masks (hcgs.conn_mat + cgs_base.conn_mat), seeded global np.random
# ----------------------------------------------------------------------------------------------
HCGS_CASES = [
    # (rows=out, cols=in, blocks, drops, seed)
    (1024, 440, [128, 4], [25, 62.5], 1),
    (1024, 1024, [128, 4], [25, 62.5], 2),
    (512, 512, [32, 2], [75, 75], 3),
    (512, 440, [32, 2], [75, 75], 4),
    (550, 550, [64, 4], [50, 25], 5),
    (550, 440, [64, 4], [50, 25], 6),
    (100, 70, [16, 4], [50, 50], 7),
    (64, 48, [16], [50], 8),
    (96, 40, [32, 8, 2], [50, 50, 50], 9),
]


def gen_hcgs():
    out = {}
    for i, (r, c, bl, dr, seed) in enumerate(HCGS_CASES):
        np.random.seed(seed)
        m = _orig_conn_mat(r, c, list(bl), list(dr), "g%d" % i, dir=_TMP, for_test=True)
        out["m%d" % i] = np.packbits(m.astype(np.uint8).ravel())
        out["shape%d" % i] = np.array([r, c])
        out["density%d" % i] = np.array([m.mean()])
    np.savez_compressed(os.path.join(OUT, "hcgs.npz"), **out)


# ----------------------------------------------------------------------------------------------
# G3: quantisation / prune / pattern known answers
# ----------------------------------------------------------------------------------------------
def gen_quant():
    out = {}
    g = torch.Generator().manual_seed(5)
    w = (torch.rand(64, 48, generator=g) * 2.6 - 1.3)
    out["w"] = w.numpy().copy()
    for b in (8, 4, 16):
        wq = quantized_modules.Quantize(w.clone(), numBits=b, balanced=False)
        out["wq%d" % b] = wq.numpy()
        wq_f = quantized_modules.Quantize(w.clone(), numBits=b, if_forward=True, balanced=False)
        out["wqf%d" % b] = wq_f.numpy()
    x = torch.randn(37, 29, generator=g) * 3.0
    out["x"] = x.numpy().copy()
    for b in (16, 8):
        out["xq%d" % b] = quantized_modules.Quantize_inp(x.clone(), b).numpy()
        out["xqf%d" % b] = quantized_modules.Quantize_inp(x.clone(), b, if_forward=True).numpy()
    # double quantisation (the LSTM quantises the same input tensor 4x, in place)
    xx = x.clone()
    for _ in range(4):
        xx = quantized_modules.Quantize_inp(xx, 16)
    out["xq16x4"] = xx.numpy()
    # prune (percentile over all >1-D params of a Linear)
    lin = torch.nn.Linear(48, 64)
    with torch.no_grad():
        lin.weight.copy_(w)
    for perc in (70.0, 33.3, 0.0, 100.0):
        out["prune%g" % perc] = quantized_modules.prune(lin, perc)[0].numpy()
    # pattern application with the fixed pattern set shipped by the reference
    pat = np.load(os.path.join(REF, "pattern_file", "b08b08_k04_n16_pattern.npy"))
    kernel = torch.from_numpy(pat.reshape(16, 1, 8, 8).astype(np.float32))
    out["pattern_set"] = pat
    out["pmask"] = sparsity.apply_patterns(w, kernel).numpy()
    wz = w.clone()
    wz[:8, :16] = 0.0                    # an all-zero tile -> every pattern ties (mask > 1)
    out["wz"] = wz.numpy()
    out["pmask_z"] = sparsity.apply_patterns(wz, kernel).numpy()
    np.savez_compressed(os.path.join(OUT, "quant.npz"), **out)


def gen_kmeans():
    """find_top_k_by_kmeans (sparsity.py:999-1049) with sklearn's KMeans given random_state=0
    (the reference passes none; seeding it is the only way to pin the search), on weights with
    ties, a ragged edge and a pattern_num above C(ph*pw, nnz)."""
    import functools

    from sklearn.cluster import KMeans
    orig = sparsity.KMeans
    sparsity.KMeans = functools.partial(KMeans, random_state=0)
    try:
        out = {}
        g = torch.Generator().manual_seed(11)
        cases = [("a", torch.randn(64, 48, generator=g), 16, (8, 8), 4),
                 ("b", torch.randn(44, 36, generator=g), 8, (8, 8), 2),
                 ("c", torch.randn(32, 32, generator=g).round(), 16, (8, 8), 6),
                 ("d", torch.randn(16, 16, generator=g), 12, (2, 2), 1)]
        for tag, w, num, shape, nnz in cases:
            k = sparsity.find_top_k_by_kmeans(w.clone(), num, list(shape), nnz, list(shape))
            out[tag + "_w"] = w.numpy().copy()
            out[tag + "_args"] = np.array([num, shape[0], shape[1], nnz])
            out[tag + "_kernel"] = k.numpy()[:, 0]
    finally:
        sparsity.KMeans = orig
    np.savez_compressed(os.path.join(OUT, "kmeans.npz"), **out)


# ----------------------------------------------------------------------------------------------
# guided HCGS masks (guided_hcgs.py:9-77): deterministic functions of |W|
# ----------------------------------------------------------------------------------------------
from cases import GHCGS  # noqa: E402


def gen_ghcgs():
    import guided_hcgs
    out = {}
    rs = np.random.RandomState(11)
    for i, (shape, blocks, drops) in enumerate(GHCGS):
        w = torch.from_numpy(rs.randn(*shape).astype(np.float32))
        if i == 4:                                   # exact ties: equal block means
            w[:, 32:64] = w[:, 0:32]
        m = guided_hcgs.conn_mat(shape[0], shape[1], list(blocks), list(drops), w, str(i),
                                 dir=_TMP, for_test=True)
        out["w%d" % i] = w.numpy().copy()
        out["mask%d" % i] = np.asarray(m, dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, "ghcgs.npz"), **out)


# ----------------------------------------------------------------------------------------------
# helpers to build reference modules from option dicts
# ----------------------------------------------------------------------------------------------
def section(d):
    cp = configparser.ConfigParser()
    cp["s"] = {k: str(v) for k, v in d.items()}
    return cp["s"]


def sd_np(module, prefix, out):
    for k, v in module.state_dict().items():
        out[prefix + k] = v.detach().numpy().copy()


# ----------------------------------------------------------------------------------------------
# G4: MLP training steps through the reference's utils.model_init/optimizer_init/forward_model
# ----------------------------------------------------------------------------------------------
def gen_mlp(variant, steps=3, B=16, F=40):
    out = {}
    cfg = build_mlp_config(variant)
    arch_dict = {"MLP_layers1": ["architecture1", "MLP_layers1", 0],
                 "MLP_layers2": ["architecture2", "MLP_layers2", 0],
                 "MLP_layers3": ["architecture3", "MLP_layers3", 0]}
    fea_dict = {"fmllr": ["fmllr", "x.scp", "", "5", "5", 0, F, F]}
    lab_dict = {"lab_cd": ["lab_cd", "a", "ali-to-pdf", F], "lab_mono": ["lab_mono", "a", "p", F + 1]}
    model = cfg["model"]["model"].split("\n")
    rs = np.random.RandomState(7)
    data = np.zeros((steps * B, F + 2), dtype=np.float32)
    data[:, :F] = rs.normal(size=(steps * B, F))
    data[:, F] = rs.randint(0, 96, size=steps * B)
    data[:, F + 1] = rs.randint(0, 8, size=steps * B)
    data = torch.from_numpy(data)
    out["data"] = data.numpy().copy()
    torch.manual_seed(2234)
    np.random.seed(2234)
    inp_out = dict(fea_dict)
    nns, costs = utils.model_init(inp_out, model, cfg, arch_dict, False, False, "train")
    opts = utils.optimizer_init(nns, cfg, arch_dict)
    for n, net in nns.items():
        sd_np(net, "init/%s/" % n, out)
    for s in range(steps):
        inp = data[s * B:(s + 1) * B].contiguous()
        outs = utils.forward_model(fea_dict, lab_dict, arch_dict, model, nns, costs, inp, inp_out,
                                   0, B, "train", ["out_dnn2"])
        for o in opts.values():
            o.zero_grad()
        outs["loss_final"].backward()
        for n, net in nns.items():
            for pn, p in net.named_parameters():
                if p.grad is not None:
                    out["step%d/grad/%s/%s" % (s, n, pn)] = p.grad.numpy().copy()
        for o in opts.values():
            o.step()
        out["step%d/loss" % s] = np.array([outs["loss_final"].item(), outs["loss_cd"].item(),
                                           outs["loss_mono"].item()])
        out["step%d/err" % s] = np.array([outs["err_final"].item()])
        out["step%d/out_dnn2" % s] = outs["out_dnn2"].detach().numpy().copy()
        out["step%d/out_dnn1" % s] = outs["out_dnn1"].detach().numpy().copy()
        if s == steps - 1:
            for n, net in nns.items():
                sd_np(net, "step%d/sd/%s/" % (s, n), out)
    # optimizer state after the last step (RMSprop square_avg)
    for n, o in opts.items():
        for gi, group in enumerate(o.param_groups):
            for pi, p in enumerate(group["params"]):
                st = o.state.get(p, {})
                if "square_avg" in st:
                    out["opt/%s/%d" % (n, pi)] = st["square_avg"].numpy().copy()
    np.savez_compressed(os.path.join(OUT, "mlp_%s.npz" % variant), **out)


# ----------------------------------------------------------------------------------------------
# G5: recurrent layers (liGRU bidir, LSTM uni with/without HCGS+quant, LSTM pattern)
# ----------------------------------------------------------------------------------------------
def run_rnn(cls, opts_d, T, B, F, seed, out, tag, extra=None):
    torch.manual_seed(seed)
    np.random.seed(seed)
    net = cls(section(opts_d), F)
    if extra:
        extra(net)
    sd_np(net, tag + "/init/", out)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(T, B, F, generator=g)
    r = torch.randn(T, B, net.out_dim, generator=g)
    out[tag + "/x"] = x.numpy().copy()
    out[tag + "/r"] = r.numpy().copy()
    xi = x.clone().requires_grad_(True)
    y = net(xi)
    (y * r).sum().backward()
    out[tag + "/y"] = y.detach().numpy().copy()
    out[tag + "/dx"] = xi.grad.numpy().copy()
    for pn, p in net.named_parameters():
        if p.grad is not None:
            out[tag + "/grad/" + pn] = p.grad.numpy().copy()
    sd_np(net, tag + "/post/", out)     # in-place mask/clamp side effects + BN running stats


def gen_rnn():
    out = {}
    run_rnn(neural_networks.liGRU, LIGRU_DEF, 7, 3, 20, 21, out, "ligru_bidir")
    run_rnn(neural_networks.liGRU, dict(LIGRU_DEF, ligru_bidir="False", ligru_act="tanh,relu",
                                        ligru_orthinit="False", ligru_use_laynorm="True,False"),
            6, 2, 12, 22, out, "ligru_uni_ln")
    run_rnn(neural_networks.LSTM, LSTM_DEF, 7, 3, 20, 23, out, "lstm")
    run_rnn(neural_networks.LSTM, dict(LSTM_DEF, lstm_hcgs="True", lstm_quant="True",
                                       lstm_quant_inp="True"), 7, 3, 24, 24, out, "lstm_hcgs_quant")
    pat = np.load(os.path.join(REF, "pattern_file", "b08b08_k04_n16_pattern.npy"))
    kernel = torch.from_numpy(pat.reshape(16, 1, 8, 8).astype(np.float32))

    def with_pattern(net):
        for key in net.pattern:
            net.pattern[key] = [kernel for _ in range(net.N_lstm_lay)]
    run_rnn(neural_networks.LSTM, dict(LSTM_DEF, if_pattern="True", pattern_mode="pattern",
                                       pattern_shape="8,8", pattern_nnz="4,4", pattern_num="16,16"),
            5, 2, 24, 25, out, "lstm_pattern", extra=with_pattern)
    np.savez_compressed(os.path.join(OUT, "rnn.npz"), **out)


def gen_cm():
    """Kaldi CM compressed matrices (data_io.py:729-766): hand-built blobs decoded by the
    reference's _read_compressed_mat."""
    import io
    out = {}
    rs = np.random.RandomState(17)
    for i, (rows, cols) in enumerate([(7, 5), (40, 13), (1, 3)]):
        gh = np.array([(rs.randn() * 3, abs(rs.randn()) * 10 + 0.5, rows, cols)],
                      dtype=[("minvalue", "<f4"), ("range", "<f4"), ("num_rows", "<i4"), ("num_cols", "<i4")])
        ph = np.sort(rs.randint(0, 65536, size=(cols, 4)), axis=1).astype("<u2")
        data = rs.randint(0, 256, size=cols * rows).astype(np.uint8)
        data[:min(6, data.size)] = [0, 64, 65, 192, 193, 255][:min(6, data.size)]
        blob = gh.tobytes() + ph.tobytes() + data.tobytes()
        m = data_io._read_compressed_mat(io.BytesIO(blob), "CM ")
        out["blob%d" % i] = np.frombuffer(blob, dtype=np.uint8).copy()
        out["mat%d" % i] = np.asarray(m, dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, "cm.npz"), **out)


def text_ark_inputs():
    """Kaldi text-form arks (`ark,t:` — copy-feats / copy-int-vector output, kaldi-matrix.cc
    Matrix::Write text branch): float matrices as "key  [\n  v v v \n  v v v ]\n", int vectors as
    "key v v v \n", a bracketed int vector, formats %g-style with exponents and negative zero; plus a
    mixed ark (text entries between binary FM / DM ones)."""
    import struct
    rs = np.random.RandomState(23)
    mats = []
    txt = b""
    for i, (r, c) in enumerate([(3, 4), (1, 6), (5, 2)]):
        m = (rs.randn(r, c) * 10.0 ** rs.randint(-6, 4, size=(r, c))).astype(np.float32)
        m[0, 0] = -0.0
        rows = ["  " + " ".join(("%g" if (j + k) % 2 else "%.7g") % v for k, v in enumerate(row))
                for j, row in enumerate(m)]
        txt += ("utt%d  [\n" % i + " \n".join(rows) + " ]\n").encode()
        mats.append(m)
    vtxt = b"".join(("a%d " % i + " ".join(str(v) for v in rs.randint(0, 1928, size=n)) + " \n")
                    .encode() for i, n in enumerate((5, 1, 9)))
    vtxt += b"b0 [ 3 1 4 1 5 ]\n"
    fm = rs.randn(2, 3).astype(np.float32)
    dm = rs.randn(3, 2)
    mixed = (b"bin0 \0BFM \x04" + struct.pack("<i", 2) + b"\x04" + struct.pack("<i", 3) + fm.tobytes()
             + b"txt0  [\n  1.5 -2 3e-07 \n  4 5 6 ]\n"
             + b"bin1 \0BDM \x04" + struct.pack("<i", 3) + b"\x04" + struct.pack("<i", 2) + dm.tobytes())
    return txt, vtxt, mixed


def gen_text_ark():
    """Text-form arks read by the reference's read_mat_ark / read_vec_int_ark (data_io.py:645-726,
    412-455): the input bytes and the reference's decoded matrices / vectors."""
    out = {}
    for tag, blob in zip(("mat", "vec", "mixed"), text_ark_inputs()):
        path = os.path.join(_TMP, "text_%s.ark" % tag)
        with open(path, "wb") as f:
            f.write(blob)
        out[tag + "_bytes"] = np.frombuffer(blob, dtype=np.uint8).copy()
        reader = data_io.read_vec_int_ark if tag == "vec" else data_io.read_mat_ark
        items = list(reader("ark:" + path, _TMP))
        out[tag + "_keys"] = np.array([k for k, _ in items])
        for i, (k, v) in enumerate(items):
            out["%s_%d" % (tag, i)] = np.asarray(v)
    np.savez_compressed(os.path.join(OUT, "text_ark.npz"), **out)


def gen_gru():
    from cases import GRU_CASES
    out = {}
    for tag, opts, T, B, F, seed in GRU_CASES:
        run_rnn(neural_networks.GRU, opts, T, B, F, seed, out, tag)
    from cases import PLAIN_CASES
    for tag, cls, opts, T, B, F, seed in PLAIN_CASES:
        run_rnn(getattr(neural_networks, cls), opts, T, B, F, seed, out, tag)
    np.savez_compressed(os.path.join(OUT, "gru.npz"), **out)


# ----------------------------------------------------------------------------------------------
# G6: posterior ark bytes (data_io.write_mat) incl. count normalisation (core.py:242-249)
# ----------------------------------------------------------------------------------------------
def gen_ark():
    rs = np.random.RandomState(3)
    counts = rs.randint(1, 500, size=10).astype(np.float32)
    cpath = os.path.join(_TMP, "counts")
    with open(cpath, "w") as f:
        f.write("[ " + " ".join(str(int(c)) for c in counts) + " ]\n")
    mats = [np.log(rs.dirichlet(np.ones(10), size=n)).astype(np.float32) for n in (3, 5)]
    cnt = data_io.load_counts(cpath)
    with open(os.path.join(OUT, "post.ark"), "wb") as f:
        for k, m in zip(["spkA_utt1", "spkB_utt2"], mats):
            data_io.write_mat(_TMP, f, m - np.log(cnt / np.sum(cnt)), k)
    np.savez_compressed(os.path.join(OUT, "post_inputs.npz"), counts=counts, m0=mats[0], m1=mats[1])


# ----------------------------------------------------------------------------------------------
# G9: the reference's own core.run_nn over a chunk lifecycle (train ck0 -> train ck1 resumed from
# the reference-written .pkl -> valid -> forward ark), on CPU with the Kaldi reads shimmed
# ----------------------------------------------------------------------------------------------
def gen_run_nn(case):
    import core
    out = {}
    rs = np.random.RandomState({"mlp": 41, "ligru": 42, "lstm_quant": 43}[case])
    data = {}
    for tag, n in (("ck0", 14), ("ck1", 14)):
        names, fea, cd, mono = synth_utts(rs, n, 12, 40, n_cd=48, n_mono=8)
        data[tag] = (fea, cd, mono)
        pack_dict(tag + "_fea", fea, out)
        pack_dict(tag + "_cd", cd, out)
        pack_dict(tag + "_mono", mono, out)
    counts = rs.randint(1, 500, size=48)
    out["counts"] = counts
    d = tempfile.mkdtemp(prefix="pkc_runnn_")
    cpath = os.path.join(d, "counts")
    with open(cpath, "w") as f:
        f.write("[ " + " ".join(str(int(c)) for c in counts) + " ]\n")

    def fake_read_mat_ark(spec, output_folder):
        tag = spec.split("scp:")[1].split()[0]
        for k, v in data[os.path.basename(tag)][0].items():
            yield k, v

    def fake_read_vec_int_ark(spec, output_folder):
        tag = os.path.basename(spec.split("gunzip -c ")[1].split("/ali*")[0]).replace(".ali", "")
        src = data[tag][2] if "phones" in spec else data[tag][1]
        for k, v in src.items():
            yield k, v

    data_io.read_mat_ark = fake_read_mat_ark
    data_io.read_vec_int_ark = fake_read_vec_int_ark
    # the reference's liGRU lacks the .prune / .guided_hcgs / .if_pattern attributes core.run_nn
    # reads (core.py:123, 299, 304): run_nn raises AttributeError on any liGRU cfg.  Shim them as
    # class attributes with the value every other architecture has when the feature is off
    for attr in ("prune", "guided_hcgs", "if_pattern"):
        if not hasattr(neural_networks.liGRU, attr):
            setattr(neural_networks.liGRU, attr, False)
    secs = ("architecture1", "architecture2", "architecture3")
    pk0 = {s: os.path.join(d, "train_ck0_%s.pkl" % s) for s in secs}
    pk1 = {s: os.path.join(d, "train_ck1_%s.pkl" % s) for s in secs}
    c_tr0 = run_nn_cfg(d, "train_ck0", "train", "ck0", case)
    c_tr1 = run_nn_cfg(d, "train_ck1", "train", "ck1", case, pretrain=pk0)
    c_va = run_nn_cfg(d, "valid", "valid", "ck0", case, pretrain=pk1)
    c_fw = run_nn_cfg(d, "forward", "forward", "ck0", case, pretrain=pk1, counts=cpath)
    nxt, pats, pms = core.run_nn(None, None, None, None, None, None, c_tr0, True, c_tr1)
    nxt, pats, pms = core.run_nn(*nxt, c_tr1, False, c_va, patterns=pats, pattern_masks=pms)
    nxt, pats, pms = core.run_nn(*nxt, c_va, False, c_fw, patterns=pats, pattern_masks=pms)
    core.run_nn(*nxt, c_fw, False, c_fw, patterns=pats, pattern_masks=pms)
    for tag in ("train_ck0", "train_ck1", "valid"):
        info = configparser.ConfigParser()
        info.read(os.path.join(d, tag + ".info"))
        out["info_" + tag] = np.array([float(info["results"]["loss"]), float(info["results"]["err"])])
    sub = os.path.join(OUT, "run_nn_" + case)
    os.makedirs(sub, exist_ok=True)
    import shutil
    for s in secs:       # the reference-written checkpoints: ck0 is the resume input of the test
        shutil.copy(pk0[s], os.path.join(sub, "train_ck0_%s.pkl" % s))
        ck = torch.load(pk1[s], weights_only=True)
        for k, v in ck["model_par"].items():
            out["ck1/%s/model/%s" % (s, k)] = v.numpy().copy()
        for pi, st in ck["optimizer_par"]["state"].items():
            for k, v in st.items():
                if torch.is_tensor(v):
                    out["ck1/%s/opt/%d/%s" % (s, pi, k)] = v.numpy().copy()
    shutil.copy(os.path.join(d, "forward_out_dnn2_to_decode.ark"),
                os.path.join(sub, "forward_out_dnn2_to_decode.ark"))
    np.savez_compressed(os.path.join(sub, "expected.npz"), **out)


if __name__ == "__main__":
    if len(sys.argv) > 1:          # e.g. `make_golden.py mlp:l1 mlp:l2 mlp:gl`
        for a in sys.argv[1:]:
            kind, _, v = a.partition(":")
            {"mlp": gen_mlp, "ghcgs": lambda _v: gen_ghcgs(), "gru": lambda _v: gen_gru(),
             "cm": lambda _v: gen_cm(), "run_nn": gen_run_nn,
             "kmeans": lambda _v: gen_kmeans(), "text_ark": lambda _v: gen_text_ark(),
             "loader_multi": lambda _v: gen_loader_multi()}[kind](v)
        sys.exit(0)
    gen_loader()
    gen_loader_multi()
    gen_hcgs()
    gen_ghcgs()
    gen_quant()
    gen_kmeans()
    for v in ("plain", "hcgs", "quant", "ln", "l1", "l2", "gl"):
        gen_mlp(v)
    gen_rnn()
    gen_gru()
    gen_cm()
    gen_ark()
    gen_text_ark()
    for c in RUN_NN_CASES:
        gen_run_nn(c)
    total = sum(os.path.getsize(os.path.join(OUT, f)) for f in os.listdir(OUT))
    print("golden fixtures written to %s (%.1f KB)" % (OUT, total / 1024))
