"""Calibrate the CPU baseline: the oracle restatement that bench.py times on the GPU
box's host cores against the REFERENCE itself (imported from /root/reference, build container
only) on the same cores and the same C1 MLP training step (TIMIT_MLP_fmllr.cfg shape, B = 128),
with all 8 threads and with 1.  Writes profiles/r03_cpu_calibration.json (the C1 MLP step
and, since round 3, a sequence step: liGRU 4x550 bidirectional).  The reference never
travels to the GPU box; only this ratio does.

Shims (this process only): torch.Tensor.cuda -> identity (the reference hard-codes .cuda()).
Usage: PYTHONDONTWRITEBYTECODE=1 python scripts/cpu_calibrate.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def steps_per_s(step, seconds):
    for _ in range(2):
        step()
    n, t0 = 0, time.time()
    while time.time() - t0 < seconds:
        step()
        n += 1
    return n / (time.time() - t0)


def oracle_step(B):
    from oracle import nets as ON
    from oracle import run as OR
    cfg = bench.c1_cfg()
    torch.manual_seed(0)
    nets, opts = {}, {}
    for sec, inp in bench.DIMS:
        o = cfg[sec]
        nets[o["arch_name"]] = ON.MLP(o, inp).train()
        opts[o["arch_name"]] = ON.make_optimizer(nets[o["arch_name"]].parameters(), o)
    lines = OR.parse_model(cfg["model"]["model"])
    rs = np.random.RandomState(1)
    inp = torch.from_numpy(np.concatenate([rs.randn(B, 440), rs.randint(0, 48, (B, 2))],
                                          1).astype(np.float32))
    seq = {k: False for k in nets}
    fc, lc = {"fmllr": (0, 440)}, {"lab_cd": 440, "lab_mono": 441}
    return lambda: OR.train_step(lines, nets, opts, seq, fc, lc, inp)


def reference_step(B):
    if not os.path.isdir(REF):
        raise SystemExit("the reference is only present in the build container")
    torch.Tensor.cuda = lambda t, *a, **k: t      # noqa: E731
    sys.path.insert(0, REF)
    import utils
    cfg = bench.c1_cfg()
    cfg["exp"] = {"use_cuda": "False", "to_do": "train", "seed": "2234"}
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from cases import MLP_DEF               # the reference MLP's remaining option keys
    for sec, _ in bench.DIMS:                 # the reference's plug-in keys (utils.py:1768-1779)
        nl = len(cfg[sec]["dnn_lay"].split(","))
        for k, v in MLP_DEF.items():
            if k not in cfg[sec]:
                cfg[sec][k] = ",".join([v.split(",")[0]] * nl) if k in ("param_quant", "mlp_prune_perc") else v
        cfg[sec].update(arch_library="neural_networks", arch_class="MLP", arch_seq_model="False",
                        arch_pretrain_file="none", use_cuda="False")
    arch_dict = {"MLP_layers1": ["architecture1", "MLP_layers1", 0],
                 "MLP_layers2": ["architecture2", "MLP_layers2", 0],
                 "MLP_layers3": ["architecture3", "MLP_layers3", 0]}
    fea_dict = {"fmllr": ["fmllr", "x.scp", "", "5", "5", 0, 440, 440]}
    lab_dict = {"lab_cd": ["lab_cd", "a", "ali-to-pdf", 440], "lab_mono": ["lab_mono", "a", "p", 441]}
    model = cfg["model"]["model"].split("\n")
    torch.manual_seed(0)
    inp_out = dict(fea_dict)
    nns, costs = utils.model_init(inp_out, model, cfg, arch_dict, False, False, "train")
    opts = utils.optimizer_init(nns, cfg, arch_dict)
    rs = np.random.RandomState(1)
    inp = torch.from_numpy(np.concatenate([rs.randn(B, 440), rs.randint(0, 48, (B, 2))],
                                          1).astype(np.float32))

    def step():            # core.py:216-232
        outs = utils.forward_model(fea_dict, lab_dict, arch_dict, model, nns, costs, inp, inp_out,
                                   0, B, "train", [])
        for o in opts.values():
            o.zero_grad()
        outs["loss_final"].backward()
        for o in opts.values():
            o.step()
    return step


SEQ_MODEL = ("o1=compute(rnn,fea)\no2=compute(head,o1)\no3=compute(mono,o1)\n"
             "lm=cost_nll(o3,lab_mono)\nlmw=mult_constant(lm,1.0)\nlc=cost_nll(o2,lab_cd)\n"
             "loss_final=sum(lc,lmw)\nerr_final=cost_err(o2,lab_cd)")


def seq_cfg():
    """C3 without HCGS (the reference liGRU has no HCGS hooks): liGRU 4x550
    bidirectional, ReLU, BN, dropout 0.2, heads 1928 cd + 48 mono (scripts/bench_seq.py)."""
    import configparser
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_seq as BS
    _, ropts, B = BS.rec_opts("c3")
    ropts = {k: v for k, v in ropts.items() if "hcgs" not in k}
    cfg = configparser.ConfigParser()
    cfg["a1"] = dict(ropts, arch_name="rnn", **BS.OPT)
    head = dict(dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False", arch_name="head",
                dnn_lay="1928", dnn_drop="0.0", dnn_use_batchnorm="False", dnn_use_laynorm="False",
                dnn_act="softmax", **dict(BS.OPT, arch_lr="0.0004"))
    cfg["a2"] = head
    cfg["a3"] = dict(head, arch_name="mono", dnn_lay="48")
    return cfg, B


def seq_input(T, B):
    rs = np.random.RandomState(1)
    return torch.from_numpy(np.concatenate([rs.randn(T, B, 440), rs.randint(0, 48, (T, B, 2))],
                                           2).astype(np.float32))


def oracle_seq_step(T):
    from oracle import nets as ON
    from oracle import run as OR
    cfg, B = seq_cfg()
    torch.manual_seed(0)
    rnn = ON.liGRU(cfg["a1"], 440)
    nets = {"rnn": rnn, "head": ON.MLP(cfg["a2"], rnn.out_dim), "mono": ON.MLP(cfg["a3"], rnn.out_dim)}
    opts = {k: ON.make_optimizer(nets[k].parameters(), cfg[s]) for k, s in
            (("rnn", "a1"), ("head", "a2"), ("mono", "a3"))}
    for n in nets.values():
        n.train()
    lines = OR.parse_model(SEQ_MODEL)
    inp = seq_input(T, B)
    seq = {"rnn": True, "head": False, "mono": False}
    return (lambda: OR.train_step(lines, nets, opts, seq, {"fea": (0, 440)},
                                  {"lab_cd": 440, "lab_mono": 441}, inp, T, B)), B


def reference_seq_step(T):
    if not os.path.isdir(REF):
        raise SystemExit("the reference is only present in the build container")
    torch.Tensor.cuda = lambda t, *a, **k: t      # noqa: E731
    sys.path.insert(0, REF)
    import utils
    cfg, B = seq_cfg()
    cfg["exp"] = {"use_cuda": "False", "to_do": "train", "seed": "2234"}
    cfg["model"] = {"model": SEQ_MODEL}
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from cases import MLP_DEF
    for sec in ("a2", "a3"):
        for k, v in MLP_DEF.items():
            if k not in cfg[sec]:
                cfg[sec][k] = v
        cfg[sec].update(arch_library="neural_networks", arch_class="MLP", arch_seq_model="False",
                        arch_pretrain_file="none", use_cuda="False")
    cfg["a1"].update(arch_library="neural_networks", arch_class="liGRU", arch_seq_model="True",
                     arch_pretrain_file="none", use_cuda="False")
    arch_dict = {"rnn": ["a1", "rnn", 1], "head": ["a2", "head", 0], "mono": ["a3", "mono", 0]}
    fea_dict = {"fea": ["fea", "x.scp", "", "5", "5", 0, 440, 440]}
    lab_dict = {"lab_cd": ["lab_cd", "a", "ali-to-pdf", 440], "lab_mono": ["lab_mono", "a", "p", 441]}
    model = SEQ_MODEL.split("\n")
    torch.manual_seed(0)
    inp_out = dict(fea_dict)
    nns, costs = utils.model_init(inp_out, model, cfg, arch_dict, False, False, "train")
    opts = utils.optimizer_init(nns, cfg, arch_dict)
    inp = seq_input(T, B)

    def step():            # core.py:216-232
        outs = utils.forward_model(fea_dict, lab_dict, arch_dict, model, nns, costs, inp, inp_out,
                                   T, B, "train", [])
        for o in opts.values():
            o.zero_grad()
        outs["loss_final"].backward()
        for o in opts.values():
            o.step()
    return step, B


def main():
    B, seconds = 128, float(os.environ.get("CAL_SECONDS", "10"))
    out = {"workload": "C1/C2 MLP training step 440-5x1024-{1928,48}, B=128, fp32, torch-CPU eager",
           "container_cpus": os.cpu_count(), "results": {}}
    for threads in (os.cpu_count(), 1):
        torch.set_num_threads(threads)
        r_ref = steps_per_s(reference_step(B), seconds) * B
        r_orc = steps_per_s(oracle_step(B), seconds) * B
        out["results"][str(threads)] = {"reference_frames_per_s": round(r_ref, 1),
                                        "oracle_frames_per_s": round(r_orc, 1),
                                        "oracle_over_reference": round(r_orc / r_ref, 3)}
        print(threads, out["results"][str(threads)], flush=True)
    # a sequence configuration: liGRU 4x550 bidirectional (C3 without HCGS), B = 8, T = 60
    T = int(os.environ.get("CAL_T", "60"))
    out["sequence"] = {"workload": "liGRU 4x550 bidir (C3 without HCGS: the reference liGRU has no "
                                   "HCGS hooks), B=8 sentences x T=%d, fp32, torch-CPU eager" % T,
                       "results": {}}
    for threads in (os.cpu_count(), 1):
        torch.set_num_threads(threads)
        st, Bs = reference_seq_step(T)
        r_ref = steps_per_s(st, seconds) * Bs * T
        st, Bs = oracle_seq_step(T)
        r_orc = steps_per_s(st, seconds) * Bs * T
        out["sequence"]["results"][str(threads)] = {
            "reference_frames_per_s": round(r_ref, 1), "oracle_frames_per_s": round(r_orc, 1),
            "oracle_over_reference": round(r_orc / r_ref, 3)}
        print("seq", threads, out["sequence"]["results"][str(threads)], flush=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", "r03_cpu_calibration.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
