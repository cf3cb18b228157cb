"""pkc.core.run_nn — drop-in for the reference's core.run_nn (core.py:24-362).

Same signature, same return value ([data_name, data_set, data_end_index, fea_dict, lab_dict,
arch_dict], patterns, pattern_masks) and the same side files:
  * ``<info>``: [results] loss= err= elapsed_time_chunk= (core.py:338-345; forward: time only),
  * one ``<info>_<arch>.pkl`` per architecture in train mode ({'model_par', 'optimizer_par'},
    core.py:285-322),
  * ``<info>_<out>_to_decode.ark`` posteriors in forward mode (core.py:134-145, 238-249) in the
    byte format of data_io.write_mat, consumed unchanged by kaldi_decoding_scripts/decode_dnn.sh.

The chunk lives in HBM between calls: ``data_set`` is a pkc.data_io.Chunk (the reference returns a
CUDA tensor; run_exp only hands it back to the next call).  Everything per batch runs on the HIP
kernels through pkc.engine; the host only parses arks and bookkeeps utterances.
"""
import configparser
import importlib
import os
import random
import re
import sys
import threading
import time

import numpy as np
import torch

from . import data_io as D
from . import dist as DP
from . import frontend as FE
from . import _lib as L
from . import neural_networks as NN
from .engine import Engine, ForwardRunner, parse_model
from .neural_networks import strtobool


def _cfg_item2sec(config, field, value):
    for sec in config.sections():
        if field in config[sec] and config[sec][field] == value:
            return sec
    raise KeyError("%s=%s not found in cfg" % (field, value))


def dict_fea_lab_arch(config):
    """utils.py:1611-1711: feature / label / architecture descriptors used by the [model]."""
    lines = parse_model(config["model"]["model"])
    fea_field = config["data_chunk"]["fea"]
    lab_field = config["data_chunk"]["lab"]
    fea_names = re.findall(r"fea_name=(.*)\n", fea_field.replace(" ", "") + "\n")
    lab_names = re.findall(r"lab_name=(.*)\n", lab_field.replace(" ", "") + "\n")
    fea_dict, lab_dict, arch_dict = {}, {}, {}
    for out, op, a, b in lines:
        for inp in (a, b):
            if inp in fea_names and inp not in fea_dict:
                m = re.findall("fea_name=" + inp + r"\nfea_lst=(.*)\nfea_opts=(.*)\ncw_left=(.*)\ncw_right=(.*)",
                               fea_field)[0]
                fea_dict[inp] = [inp] + list(m)
            if inp in lab_names and inp not in lab_dict:
                m = re.findall("lab_name=" + inp + r"\nlab_folder=(.*)\nlab_opts=(.*)", lab_field)[0]
                lab_dict[inp] = [inp] + list(m)
        if op == "compute" and a not in arch_dict:
            sec = _cfg_item2sec(config, "arch_name", a)
            arch_dict[a] = [sec, a, strtobool(config[sec]["arch_seq_model"])]
    return fea_dict, lab_dict, arch_dict


def _read_features(fea_scp, fea_opts, output_folder):
    """Feature stream of one chunk: ``copy-feats scp:<scp> ark:- |<opts>`` as data_io.py:18.

    The scp's binary arks ("key path:offset" or "key path") are read directly.  An
    ``apply-cmvn ... | add-deltas ...`` fea_opts pipe (every shipped cfg) is parsed into a
    pkc.frontend.FeaFrontend that pkc_feat_frontend applies on the GPU after the upload; any other
    pipe is run through Kaldi exactly as the reference does.  Returns (feats, frontend or None)."""
    if fea_opts.strip() and not FE.is_native_pipe(fea_opts):
        import subprocess
        cmd = "copy-feats scp:" + fea_scp + " ark:- |" + fea_opts
        out = subprocess.run(cmd, shell=True, capture_output=True, check=True).stdout
        return dict(D.parse_mat_ark_bytes(out)), None
    frontend = FE.FeaFrontend.parse(fea_opts) if fea_opts.strip() else None
    feats = {}
    by_file = {}
    with open(fea_scp) as f:
        for line in f:
            if not line.strip():
                continue
            key, spec = line.split(None, 1)
            path = spec.strip().rsplit(":", 1)[0] if re.search(r":\d+$", spec.strip()) else spec.strip()
            by_file.setdefault(path, set()).add(key)
    for path, keys in by_file.items():
        for k, m in D.read_mat_ark_path(path):
            if k in keys:
                feats[k] = m
    return feats, frontend


def _read_labels(lab_folder, lab_opts, output_folder):
    """``gunzip -c ali*.gz | <lab_opts> final.mdl ark:- ark:-|`` (data_io.py:19-21); a
    pre-converted ``<lab_folder>/<lab_opts-tag>.ark`` int-vector ark (binary or text) is read
    directly."""
    tag = "pdf" if "pdf" in lab_opts else "phones"
    pre = os.path.join(lab_folder, "ali_%s.ark" % tag)
    if os.path.exists(pre):
        return dict(D.read_vec_int_ark_path(pre))
    import subprocess
    cmd = "gunzip -c " + lab_folder + "/ali*.gz | " + lab_opts + " " + lab_folder + "/final.mdl ark:- ark:-|"
    out = subprocess.run(cmd[:-1], shell=True, capture_output=True, check=True).stdout
    return dict(D.parse_vec_int_ark_bytes(out))


def read_lab_fea(cfg_file, fea_only, shared_list, output_folder):
    """data_io.read_lab_fea (data_io.py:155-282) on the host side: parse arks, hand raw frames to
    the GPU chunk preparation.  Appends the same six items to shared_list; item 5 is a Chunk."""
    config = configparser.ConfigParser()
    config.read(cfg_file)
    to_do = config["exp"]["to_do"]
    max_seq = {"train": int(config["batches"].get("max_seq_length_train", "-1")),
               "valid": int(config["batches"].get("max_seq_length_valid", "-1"))}.get(to_do, -1)
    fea_dict, lab_dict, arch_dict = dict_fea_lab_arch(config)
    labs, lab_names = [], []
    if not fea_only:
        for lname, ld in lab_dict.items():
            labs.append(_read_labels(ld[1], ld[2], output_folder))
            lab_names.append(lname)
    seq = any(a[2] for a in arch_dict.values())
    rng = np.random if (not seq and to_do != "forward") else None
    # every feature stream (data_io.py:184-263: fea_dict order) sorted / split and its pinned-memory
    # upload started on a side stream here, in the loader thread, so it overlaps the current chunk's
    # training.  The GPU half of load_chunk (context windows, normalisation, stream stacking, frame
    # shuffle) is item 5's finish(): run_nn calls it where the reference's thread shuffles (after
    # the model init draws), keeping np.random's draw order
    streams = []
    for fname, fd in fea_dict.items():
        fea, frontend = _read_features(fd[1], fd[2], output_folder)
        staged = D.stage_chunk(fea, labs, max_seq, frontend=frontend)
        streams.append((staged, int(fd[3]), int(fd[4]), fname))
    data_set = D.PendingChunk(streams, labs, lab_names, max_seq, rng)
    for fname in fea_dict:
        c0, c1 = data_set.fea_cols[fname]
        fea_dict[fname] = fea_dict[fname][:5] + [c0, c1, c1 - c0]    # data_io.py:225-240
    c_end = max(c1 for _, c1 in data_set.fea_cols.values())
    for i, ln in enumerate(lab_names):
        lab_dict[ln] = lab_dict[ln][:3] + [c_end + i]                 # data_io.py:259-261
    # data_io.py:277-282: [data_name, data_end_index, fea_dict, lab_dict, arch_dict, data_set]
    shared_list.extend([data_set.names, data_set.end_index, fea_dict, lab_dict, arch_dict, data_set])


def _finish_chunk(shared_list):
    """core.py:349-362: the six loader items in run_nn's return order, the chunk prepared."""
    data_name, data_end_index, fea_dict, lab_dict, arch_dict, data_set = shared_list
    return [data_name, data_set.finish(), data_end_index, fea_dict, lab_dict, arch_dict]


def model_init(config, arch_dict, fea_dims, to_do):
    """utils.model_init (utils.py:1749-1830) restricted to pkc architectures."""
    nns = {}
    out_dims = dict(fea_dims)
    for out, op, a, b in parse_model(config["model"]["model"]):
        if op == "concatenate":                          # utils.py:1805-1809
            out_dims[out] = out_dims[a] + out_dims[b]
        if op != "compute":
            continue
        sec = arch_dict[a][0]
        o = config[sec]
        lib = o.get("arch_library", "pkc.neural_networks")
        cls_name = o["arch_class"]
        mod = importlib.import_module(lib) if lib.startswith("pkc") else NN
        cls = getattr(mod, cls_name, None) or getattr(NN, cls_name)
        config.set(sec, "use_cuda", config["exp"].get("use_cuda", "True"))
        config.set(sec, "to_do", to_do)
        net = cls(config[sec], out_dims[b])
        net.cuda()
        if to_do == "train" and not strtobool(o.get("arch_freeze", "False")):
            net.train()
        else:
            net.eval()
        nns[a] = net
        out_dims[out] = net.out_dim
    return nns


def run_nn(data_name, data_set, data_end_index, fea_dict, lab_dict, arch_dict, cfg_file,
           processed_first, next_config_file, if_prune=False, patterns=None, pattern_masks=None,
           if_apply_ghcgs=False, if_pattern_search=False):
    patterns = {} if patterns is None else patterns
    pattern_masks = {} if pattern_masks is None else pattern_masks
    if if_pattern_search:
        # core.py:149-151 imports pattern_prun_model from pattern_search, which the reference does
        # not define (pattern_search.py has no such function): the call cannot run there either
        raise NotImplementedError("if_pattern_search: pattern_search.pattern_prun_model does not "
                                  "exist in the reference")
    # if_apply_ghcgs is accepted and unused, as in the reference (core.py:25)
    if not os.path.exists(cfg_file):
        sys.stderr.write("ERROR: The config file %s does not exist!\n" % cfg_file)
        sys.exit(0)
    config = configparser.ConfigParser()
    config.read(cfg_file)
    seed = int(config["exp"]["seed"])
    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)
    output_folder = config["exp"]["out_folder"]
    to_do = config["exp"]["to_do"]
    info_file = config["exp"]["out_info"]
    is_production = strtobool(config["exp"].get("production", "False"))
    forward_outs = config["forward"]["forward_out"].split(",")
    forward_norm = list(map(strtobool, config["forward"]["normalize_posteriors"].split(",")))
    forward_counts = config["forward"]["normalize_with_counts_from"].split(",")
    require_dec = list(map(strtobool, config["forward"]["require_decoding"].split(",")))
    batch_size = {"train": int(config["batches"]["batch_size_train"]),
                  "valid": int(config["batches"]["batch_size_valid"])}.get(to_do, 1)
    # [exp] pkc_prec = bf16 (a pkc key): bf16 matmul operands with fp32 accumulation, master
    # weights, BatchNorm, loss and optimizer; bf16x3: compensated bf16 matmuls
    # (fp32-class products on the bf16 MFMA); default fp32, the reference's
    # arithmetic
    prec = {"fp32": L.PREC_FP32, "bf16": L.PREC_BF16, "bf16x3": L.PREC_BF16X3}.get(
        config["exp"].get("pkc_prec", "fp32").strip().lower())
    if prec is None:
        raise ValueError("[exp] pkc_prec must be fp32, bf16 or bf16x3, not %r"
                         % config["exp"]["pkc_prec"])

    if processed_first:
        shared = []
        read_lab_fea(cfg_file, is_production, shared, output_folder)
        data_name, data_set, data_end_index, fea_dict, lab_dict, arch_dict = _finish_chunk(shared)
    shared_next = []
    th = threading.Thread(target=read_lab_fea, args=(next_config_file, is_production, shared_next,
                                                     output_folder))
    th.start()

    fea_dims = {k: v[-1] for k, v in fea_dict.items()}
    nns = model_init(config, arch_dict, fea_dims, to_do)
    for net_name in nns:
        pt = config[arch_dict[net_name][0]]["arch_pretrain_file"]
        if pt != "none":
            ck = torch.load(pt, map_location="cuda", weights_only=True)
            nns[net_name].load_state_dict(ck["model_par"])
        if getattr(nns[net_name], "prune", False) and if_prune:       # core.py:122-127
            nns[net_name].prune_parameters()
        if net_name in patterns:          # pattern sets / masks carried between chunks (129-131)
            nns[net_name].pattern = patterns[net_name]
            nns[net_name].pattern_mask = pattern_masks[net_name]
    seq_model = any(arch_dict[a][2] for a in arch_dict)
    lines = parse_model(config["model"]["model"])
    arch_opts = {a: config[arch_dict[a][0]] for a in nns}
    chunk = data_set
    fea_cols = {k: (v[5], v[6]) for k, v in fea_dict.items()}
    lab_names = sorted(lab_dict, key=lambda k: lab_dict[k][3])

    start = time.time()
    loss_tot = err_tot = 0.0
    lens = np.diff(np.concatenate([[0], np.asarray(chunk.end_index)]))
    # chunk-level data parallelism (pkc.dist): every rank trains on its share of the chunk, one
    # gradient all-reduce per step; forward mode runs on rank 0 only (one posterior ark per chunk)
    rank, ws = DP.world()
    ws_eff = 1 if to_do == "forward" else ws
    allreduce = DP.GradAllReduce() if (ws_eff > 1 and to_do == "train") else None
    eseed = seed + 7919 * rank          # per-rank dropout streams
    if to_do == "forward" and rank != 0:
        pass
    elif seq_model:
        eng = Engine(nns, arch_opts, lines, fea_cols, lab_names, batch=batch_size, seed=eseed,
                     train=(to_do == "train"), max_len=int(lens.max()), grad_scale=1.0 / ws_eff,
                     prec=prec)
        for net_name in nns:
            pt = config[arch_dict[net_name][0]]["arch_pretrain_file"]
            if pt != "none" and to_do == "train":
                ck = torch.load(pt, map_location="cpu", weights_only=True)
                eng.load_optimizer_state_dict(net_name, ck["optimizer_par"])
                eng.set_lr(net_name, float(config[arch_dict[net_name][0]]["arch_lr"]))
        eng.bind_chunk(chunk.feats, chunk.labels, chunk.n_rows, end_index=chunk.end_index,
                       sentences=DP.shard_sentences(chunk.end_index, rank, ws_eff))
        if ws_eff > 1:
            eng.n_batches = DP.agree_min(eng.n_batches, device=eng.dev)
            if to_do == "train":        # frame-weighted sequence DP: the chunk's loss scales
                eng.frame_scales = DP.frame_weights(eng.sent_len, eng.B, eng.n_batches,
                                                    device=eng.dev)
        post_files, priors = {}, {}
        if to_do == "forward":
            for oi, out in enumerate(forward_outs):
                suffix = "_to_decode.ark" if require_dec[oi] else ".ark"
                post_files[out] = info_file.replace(".info", "_" + out + suffix)
                open(post_files[out], "wb").close()
                if forward_norm[oi]:
                    counts = D.load_counts(forward_counts[oi])
                    priors[out] = np.log(counts / np.sum(counts)).astype(np.float32)
        for i in range(eng.n_batches):
            if to_do == "train":
                eng.train_step(allreduce)   # python random draws the padding offsets (core.py:193)
            else:
                eng.eval_step()
            if to_do == "forward":
                for out in forward_outs:
                    post = eng.head_output(out).cpu().numpy()
                    if out in priors:                       # core.py:242-245, host side as there
                        post = post - priors[out]
                    D.write_mat_path(post_files[out], post, chunk.names[i], append=True)
        if to_do != "forward":
            loss_sum, err_sum = DP.sum_scalars(eng.chunk_totals(), device=eng.dev)
            nb = max(1, eng.n_batches * ws_eff)
            loss_tot, err_tot = loss_sum / nb, err_sum / nb
        if to_do == "train":
            eng.sync_state()
    elif to_do in ("train", "valid"):
        # SyncBN (pkc extension): [exp] sync_bn = True synchronises the MLP layers'
        # BatchNorm statistics over the ranks (default: per-rank statistics, as each reference
        # batch is normalised by its own)
        sbn = None
        if ws_eff > 1 and to_do == "train" and config["exp"].get("sync_bn", "False") == "True":
            sbn = DP.SyncBatchNorm()
        eng = Engine(nns, arch_opts, lines, fea_cols, lab_names, batch=batch_size, seed=eseed,
                     train=(to_do == "train"), grad_scale=1.0 / ws_eff, sync_bn=sbn, prec=prec)
        for net_name in nns:
            pt = config[arch_dict[net_name][0]]["arch_pretrain_file"]
            if pt != "none" and to_do == "train":
                ck = torch.load(pt, map_location="cpu", weights_only=True)
                eng.load_optimizer_state_dict(net_name, ck["optimizer_par"])
                eng.set_lr(net_name, float(config[arch_dict[net_name][0]]["arch_lr"]))
        r0, r1 = DP.shard_rows(chunk.n_rows, rank, ws_eff)
        eng.bind_chunk(chunk.feats[r0:r1], chunk.labels[r0:r1], r1 - r0)
        n_batches = DP.agree_min((r1 - r0) // batch_size, device=eng.dev)
        eng.n_batches = n_batches
        if to_do == "train":
            # 32-step graph replays when the chunk is long enough: one replay boundary (≈ 9 µs of
            # GPU idle) per 32 batches instead of per 8 (profiles/r04_graph_steps_ab.txt)
            eng.capture(split_optimizer=allreduce is not None,
                        steps_per_graph=32 if n_batches >= 128 else 8)
            eng.train_steps(n_batches, allreduce)
        else:
            for i in range(n_batches):
                eng.eval_step()
        loss_sum, err_sum = DP.sum_scalars(eng.chunk_totals(), device=eng.dev)
        nb = max(1, n_batches * ws_eff)
        loss_tot, err_tot = loss_sum / nb, err_sum / nb
        if to_do == "train":
            eng.sync_state()
    else:
        runner = ForwardRunner(nns, lines, fea_cols, forward_outs)
        post_files = {}
        for oi, out in enumerate(forward_outs):
            suffix = "_to_decode.ark" if require_dec[oi] else ".ark"
            post_files[out] = info_file.replace(".info", "_" + out + suffix)
            open(post_files[out], "wb").close()
        priors = {}
        for oi, out in enumerate(forward_outs):
            if forward_norm[oi]:
                counts = D.load_counts(forward_counts[oi])
                priors[out] = np.log(counts / np.sum(counts)).astype(np.float32)
        beg = 0
        for i, end in enumerate(chunk.end_index):
            outs = runner.forward(chunk.feats, int(beg), int(end), priors)
            for out in forward_outs:
                D.write_mat_path(post_files[out], outs[out], chunk.names[i], append=True)
            beg = end
    torch.cuda.synchronize()
    elapsed = time.time() - start

    if to_do == "train" and ws_eff > 1:
        DP.average_buffers(list(nns.values()))
    if to_do == "train":
        for net in nns.values():
            if getattr(net, "prune", False) and if_prune:       # chunk-end pruning (291-296)
                net.prune_parameters()
            if getattr(net, "guided_hcgs", False) and not net.apply_guided_hcgs:   # (298-300)
                net.apply_ghcgs()
    if to_do == "train":
        patterns, pattern_masks = {}, {}                             # core.py:287-288
        for net_name, net in nns.items():
            if getattr(net, "if_pattern", False):                    # core.py:304-306
                patterns[net_name] = net.pattern
                pattern_masks[net_name] = net.pattern_mask
    if rank == 0:
        if to_do == "train":
            for net_name, net in nns.items():
                ck = {"model_par": net.state_dict(),
                      "optimizer_par": eng.optimizer_state_dict(net_name)}
                torch.save(ck, info_file.replace(".info", "_" + arch_dict[net_name][0] + ".pkl"))
        with open(info_file, "w") as f:
            f.write("[results]\n")
            if to_do != "forward":
                f.write("loss=%s\n" % np.float32(loss_tot))
                f.write("err=%s\n" % np.float32(err_tot))
            f.write("elapsed_time_chunk=%f\n" % elapsed)

    th.join()
    nxt = _finish_chunk(shared_next)
    return nxt, patterns, pattern_masks
