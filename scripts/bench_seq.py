"""Training throughput of the sequence configurations of BASELINE.json (informational; the headline
bench.py line is the C2 MLP):

  C3  liGRU 4x550 bidirectional + HCGS [32,2]/[75,75] (16x) on W and U, B = 8 sentences, ReLU, BN,
      dropout 0.2, heads 1100 -> 1928 cd + 48 mono                       (TIMIT_CGS liGRU)
  C4  LSTM 4x1024 bidirectional (liGRU shared-weight convention), B = 16, tanh, BN, T <= 500
                                                                          (Librispeech_baselines)
  C5  LSTM 3x512 + Pattern 8x8/k4/n16 + 8-bit weights + 16-bit inputs, B = 12, T <= 200
                                                                          (LibriSpeech_CGS)
  plus GRU 4x550 bidirectional (north_star's GRU family) at the C3 shape.

Synthetic TIMIT-shaped chunk: utterance lengths U[150, 450] (C5: U[100, 200]), 440-dim
context-expanded features.  Metric: real (unpadded) frames / s of the batch loop, one sentence
batch = one step (core.py:183-232), plus microseconds per recurrent time step and layer.

Usage: python scripts/bench_seq.py [--configs c3,c4,c5,gru] [--steps K] [--warmup W]
"""
import argparse
import configparser
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

OPT = dict(arch_opt="rmsprop", arch_lr="0.0016", opt_momentum="0.0", opt_alpha="0.95",
           opt_eps="1e-8", opt_centered="False", opt_weight_decay="0.0", arch_freeze="False",
           to_do="train", skip_regularization="True")


def rec_opts(cfg_name):
    """c3b: C3 with the secondary HCGS setting of SURVEY 8 a13 (blocks [128, 4], sparsity
    [25, 62.5] %: density ~0.42 instead of C3's 16x masks) — where the persistent loops' fragment
    plans stop fitting and the layers fall back to the per-step launches (rec_forms)."""
    n = {"c3": 4, "c3b": 4, "c4": 4, "c5": 3, "gru": 4}[cfg_name]
    if cfg_name in ("c3", "c3b", "gru"):
        p = "ligru" if cfg_name != "gru" else "gru"
        d = {p + "_lay": ",".join(["550"] * n), p + "_drop": ",".join(["0.2"] * n),
             p + "_use_laynorm_inp": "False", p + "_use_batchnorm_inp": "False",
             p + "_use_laynorm": ",".join(["False"] * n),
             p + "_use_batchnorm": ",".join(["True"] * n), p + "_bidir": "True",
             p + "_act": ",".join(["relu"] * n), p + "_orthinit": "True"}
        if cfg_name == "c3":
            d.update(ligru_hcgs="True", hcgsx_block="32,2", hcgsx_sparse="75,75",
                     hcgsh_block="32,2", hcgsh_sparse="75,75")
        elif cfg_name == "c3b":
            d.update(ligru_hcgs="True", hcgsx_block="128,4", hcgsx_sparse="25,62.5",
                     hcgsh_block="128,4", hcgsh_sparse="25,62.5")
        return ("liGRU" if cfg_name != "gru" else "GRU"), d, 8
    H = "1024" if cfg_name == "c4" else "512"
    d = dict(lstm_lay=",".join([H] * n), lstm_drop=",".join(["0.2"] * n),
             lstm_use_laynorm_inp="False", lstm_use_batchnorm_inp="False",
             lstm_use_laynorm=",".join(["False"] * n), lstm_use_batchnorm=",".join(["True"] * n),
             lstm_bidir="True" if cfg_name == "c4" else "False", lstm_act=",".join(["tanh"] * n),
             lstm_orthinit="True", lstm_hcgs="False")
    if cfg_name == "c5":
        d.update(if_pattern="True", pattern_mode="pattern", pattern_shape="8,8",
                 pattern_nnz=",".join(["4"] * n), pattern_num=",".join(["16"] * n),
                 lstm_quant="True", lstm_quant_inp="True", param_quant=",".join(["8"] * n),
                 inp_quant="16")
    return "LSTM", d, (16 if cfg_name == "c4" else 12)


def build(cfg_name, seed=2234, rank=0, world=1, prec="fp32"):
    """Engine + nets of `cfg_name` bound to a synthetic length-sorted chunk of 64 * B sentences.
    Data parallelism (world > 1): every rank builds the same model from the same seeds and draws
    its OWN chunk (weak scaling: B sentences per rank and step), its loss scaled per batch by its
    share of the global batch's padded rows (pkc.dist.frame_weights, one collective per chunk)."""
    import pkc.neural_networks as NN
    from pkc import _lib as L
    from pkc.engine import Engine, parse_model
    cls, ropts, B = rec_opts(cfg_name)
    cfg = configparser.ConfigParser()
    cfg["a1"] = dict(ropts, arch_name="rnn", **OPT)
    head = dict(dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False", arch_name="head",
                dnn_lay="1928", dnn_drop="0.0", dnn_use_batchnorm="False", dnn_use_laynorm="False",
                dnn_act="softmax", **dict(OPT, arch_lr="0.0004"))
    cfg["a2"] = head
    cfg["a3"] = dict(head, arch_name="mono", dnn_lay="48")
    model = ("o1=compute(rnn,fea)\no2=compute(head,o1)\no3=compute(mono,o1)\n"
             "lm=cost_nll(o3,lab_mono)\nlmw=mult_constant(lm,1.0)\nlc=cost_nll(o2,lab_cd)\n"
             "loss_final=sum(lc,lmw)\nerr_final=cost_err(o2,lab_cd)")
    torch.manual_seed(seed)
    np.random.seed(seed)
    rnn = getattr(NN, cls)(cfg["a1"], 440)
    if cfg_name == "c5":
        pset = np.load(os.path.join(ROOT, "tests", "golden", "quant.npz"),
                       allow_pickle=False)["pattern_set"]
        rnn.pattern_kernels = pset.reshape(16, 8, 8)
    nets = {"rnn": rnn, "head": NN.MLP(cfg["a2"], rnn.out_dim), "mono": NN.MLP(cfg["a3"], rnn.out_dim)}
    for n in nets.values():
        n.cuda().train()
    opts = {"rnn": cfg["a1"], "head": cfg["a2"], "mono": cfg["a3"]}
    rs = np.random.RandomState(seed + 1000 * rank)
    lo, hi = (100, 200) if cfg_name == "c5" else (150, 450)
    n_utt = 64 * B
    lens = np.sort(rs.randint(lo, hi + 1, size=n_utt))          # length-sorted, as the loader
    end = np.cumsum(lens)
    N = int(end[-1])
    g = torch.Generator(device="cuda")
    g.manual_seed(seed + 1000 * rank)
    feats = torch.randn(N, 440, device="cuda", generator=g)
    labs = torch.stack([torch.randint(0, 1928, (N,), device="cuda", generator=g),
                        torch.randint(0, 48, (N,), device="cuda", generator=g)],
                       1).to(torch.int32).contiguous()
    # the chunk's longest sentence over all ranks sizes the buffers (the same on every rank)
    max_len = int(lens.max())
    if world > 1:
        from pkc import dist as DP
        max_len = -DP.agree_min(-max_len, device="cuda")
    eng = Engine(nets, opts, parse_model(model), {"fea": (0, 440)}, ["lab_cd", "lab_mono"],
                 batch=B, max_len=max_len, seed=seed + rank, grad_scale=1.0 / world,
                 prec=L.PREC_BF16 if prec == "bf16" else L.PREC_FP32)
    eng.bind_chunk(feats, labs, N, end_index=end)
    if world > 1:
        from pkc import dist as DP
        eng.n_batches = DP.agree_min(eng.n_batches, device="cuda")
        eng.frame_scales = DP.frame_weights(eng.sent_len, eng.B, eng.n_batches, device="cuda")
    return eng, nets, B


def alg_flops_per_row(nets):
    """Algorithmic training flops per padded (T x B x direction) row of a step, SURVEY 8d: the
    W and U products of every recurrent layer scaled by their HCGS / pattern mask density, the
    heads' products; x3 for forward + the two backward products.  Returns (flops per row of the
    first recurrent layer's T*B*dirs rows, flops per frame row of the heads)."""
    specs = nets["rnn"].layer_specs()
    per_dir_row = 0.0
    K = nets["rnn"].input_dim if hasattr(nets["rnn"], "input_dim") else 440
    for sp in specs:
        H = sp["H"]
        G = len(sp["W"])
        dW = float(sp["Wmask"].detach().float().mean()) if sp.get("Wmask") is not None else 1.0
        dU = float(sp["Umask"].detach().float().mean()) if sp.get("Umask") is not None else 1.0
        per_dir_row += 3 * 2 * G * H * (K * dW + H * dU)
        K = 2 * H if sp["bidir"] else H
    head = 3 * 2 * (nets["head"].out_dim + nets["mono"].out_dim) * nets["rnn"].out_dim
    return per_dir_row, head


def run(cfg_name, steps, warmup, allreduce=None, rank=0, world=1, prec="fp32", graphs=False):
    """Times `steps` sentence batches after `warmup` (barrier + synchronize on both sides of the
    timed region; the max over ranks).  frames_per_s is the whole job's: every rank's real frames
    over that time.  graphs: the steps replay per-T captured graphs (Engine.capture), captured in
    an untimed pass over the timed batches first (steady state: every T seen before); the
    capture pass's rate is reported beside it."""
    eng, nets, B = build(cfg_name, rank=rank, world=world, prec=prec)
    cap_s = None
    if graphs:
        import pkc.engine as E
        E.SEQ_CAPTURE_AFTER = 1           # the capture pass below sees each timed T once
        assert world == 1 and eng.capture()
    rng = random.Random(7)
    # sample the batches across the length-sorted chunk (short and long sentences alike)
    nb = eng.n_batches
    order = [int(i) for i in np.linspace(0, nb - 1, warmup + steps)]
    batches = []
    for i in order:
        eng.snt = i * B
        batches.append(eng.next_seq_batch(rng))
    for i, b in zip(order[:warmup], batches[:warmup]):
        eng.batch_i = i                   # the frame weight of batch i (data parallelism)
        eng.train_step(allreduce, batch=b)
    if graphs:                            # capture pass (each timed T once)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in batches[warmup:]:
            eng.train_step(batch=b)
        torch.cuda.synchronize()
        cap_s = time.perf_counter() - t0
    frames, tsteps = 0, 0
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i, b in zip(order[warmup:], batches[warmup:]):
        eng.batch_i = i
        eng.train_step(allreduce, batch=b)
        frames += int(b[1].sum())
        tsteps += int(b[3])
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        from pkc import dist as DP
        t = torch.tensor([dt], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
        frames, tsteps = DP.sum_scalars([frames, tsteps], device="cuda")
        frames, tsteps = int(frames), tsteps / world   # padded lengths vary: the mean over ranks
    specs = nets["rnn"].layer_specs()
    nl = len(specs)
    dirs = 2 if specs[0]["bidir"] else 1
    per_row, head = alg_flops_per_row(nets)
    flops = world * tsteps * B * (dirs * per_row + head)  # padded rows, as the reference computes
    extra = {}
    if graphs:
        extra = {"graphs": True, "captures": eng.seq_captures,
                 "capture_pass_ms_per_step": cap_s * 1e3 / steps}
    return {"config": cfg_name, "prec": prec, **extra, "batch_sentences": B, "steps": steps,
            "n_ranks": world,
            "frames_per_s": frames / dt, "ms_per_step": dt * 1e3 / steps,
            "us_per_time_step_per_layer_fwd_bwd": dt * 1e6 / (tsteps * nl),
            "mean_T": tsteps / steps, "alg_tflops_per_s": flops / dt / 1e12,
            "alg_gflop_per_step": flops / steps / 1e9, "rec_forms": eng.rec_forms()}


def parity(cfg_name, prec="fp32", seed=2234, lo=12, hi=20):
    """First-step posterior error of a configuration at its full layer sizes (BASELINE metric:
    "posterior max-abs-err vs ref"): the engine's first training step at `prec` on one batch of B
    sentences of U[lo, hi] frames (short, so the oracle's eager CPU loop takes seconds), same
    initial weights, same injected recurrent dropout masks and left padding, against the oracle
    (the reference's algorithm in fp32 on the CPU).  The oracle is the checker here only."""
    import pkc.neural_networks as NN
    from oracle import nets as ON
    from oracle import run as OR
    from pkc import _lib as L
    from pkc.engine import Engine, parse_model
    cls, ropts, B = rec_opts(cfg_name)
    cfg = configparser.ConfigParser()
    cfg["a1"] = dict(ropts, arch_name="rnn", **OPT)
    head = dict(dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False", arch_name="head",
                dnn_lay="1928", dnn_drop="0.0", dnn_use_batchnorm="False", dnn_use_laynorm="False",
                dnn_act="softmax", **dict(OPT, arch_lr="0.0004"))
    cfg["a2"] = head
    cfg["a3"] = dict(head, arch_name="mono", dnn_lay="48")
    model = ("o1=compute(rnn,fea)\no2=compute(head,o1)\no3=compute(mono,o1)\n"
             "lm=cost_nll(o3,lab_mono)\nlmw=mult_constant(lm,1.0)\nlc=cost_nll(o2,lab_cd)\n"
             "loss_final=sum(lc,lmw)\nerr_final=cost_err(o2,lab_cd)")
    torch.manual_seed(seed)
    np.random.seed(seed)
    rnn = getattr(NN, cls)(cfg["a1"], 440)
    orn = getattr(ON, cls)(cfg["a1"], 440)
    orn.load_state_dict(rnn.state_dict())
    if cfg_name == "c5":
        pset = np.load(os.path.join(ROOT, "tests", "golden", "quant.npz"),
                       allow_pickle=False)["pattern_set"].reshape(16, 8, 8)
        rnn.pattern_kernels = orn.pattern_kernels = pset
    nets = {"rnn": rnn, "head": NN.MLP(cfg["a2"], rnn.out_dim), "mono": NN.MLP(cfg["a3"], rnn.out_dim)}
    onets = {"rnn": orn, "head": ON.MLP(cfg["a2"], rnn.out_dim), "mono": ON.MLP(cfg["a3"], rnn.out_dim)}
    for k in ("head", "mono"):
        onets[k].load_state_dict(nets[k].state_dict())
    opts = {"rnn": cfg["a1"], "head": cfg["a2"], "mono": cfg["a3"]}
    for k in nets:
        nets[k].cuda().train()
        onets[k].train()
    rs = np.random.RandomState(seed)
    lens = np.sort(rs.randint(lo, hi + 1, size=B))
    end = np.cumsum(lens)
    X = rs.randn(end[-1], 440).astype(np.float32)
    lab = np.stack([rs.randint(0, 1928, end[-1]), rs.randint(0, 48, end[-1])], 1).astype(np.int32)
    specs = rnn.layer_specs()
    R = 2 * B if specs[0]["bidir"] else B
    masks = {("rnn", li): torch.from_numpy((rs.rand(R, sp["H"]) > 0.2).astype(np.float32))
             for li, sp in enumerate(specs)}
    eng = Engine(nets, opts, parse_model(model), {"fea": (0, 440)}, ["lab_cd", "lab_mono"],
                 batch=B, max_len=int(lens.max()), seed=1,
                 prec=L.PREC_BF16 if prec == "bf16" else L.PREC_FP32,
                 rnn_drop_in={k: v.cuda() for k, v in masks.items()})
    eng.bind_chunk(torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda(), end[-1], end_index=end)
    batch = eng.next_seq_batch(random.Random(7))
    _, _, lefts, T = batch
    inp = torch.zeros(T, B, 442)
    for k in range(B):                              # core.py:183-200, the engine's left pads
        n, b0, left = int(lens[k]), int(end[k] - lens[k]), int(lefts[k])
        inp[left:left + n, k, :440] = torch.from_numpy(X[b0:b0 + n])
        inp[left:left + n, k, 440:] = torch.from_numpy(lab[b0:b0 + n].astype(np.float32))
    eng.train_step(batch=batch)
    post = eng.head_output("o2").cpu().double()
    f = orn.forward
    orn.forward = lambda x, _f=f: _f(x, drop_masks=[masks[("rnn", i)] for i in range(len(specs))])
    outs = OR.forward_model(OR.parse_model(model), onets, {"rnn": True, "head": False, "mono": False},
                            {"fea": (0, 440)}, {"lab_cd": 440, "lab_mono": 441}, inp, T, B)
    orn.forward = f
    ref = outs["o2"].detach().double()
    d = (post - ref).abs()
    del eng
    torch.cuda.empty_cache()
    return {"posterior_max_abs_err": float(d.max()),
            "posterior_max_rel_err": float((d / ref.abs().clamp_min(1e-3)).max()),
            "posterior_ref": "oracle fp32 (reference algorithm), first training step, %d layers at "
                             "full size, B=%d sentences, T=%d" % (len(specs), B, T)}


def gpu_like_T(cfg_name, seed=5):
    """A padded batch length drawn like the GPU's: the longest of B sentence lengths from the
    config's distribution (U[150, 450]; C5 U[100, 200])."""
    _, _, B = rec_opts(cfg_name)
    lo, hi = (100, 200) if cfg_name == "c5" else (150, 450)
    return int(np.random.RandomState(seed).randint(lo, hi + 1, size=B).max())


def _cpu_rate(cfg_name, T, threads, seconds):
    """(frames/s, steps, seconds) of the oracle's eager torch-CPU restatement of the training step
    (the reference's per-time-step algorithm, neural_networks.py:1523-1599 / 1077-1097) on one
    padded batch of B sentences x T frames; at least one timed step."""
    import configparser

    from oracle import nets as ON
    from oracle import run as OR
    torch.set_num_threads(threads)
    cls, ropts, B = rec_opts(cfg_name)
    cfg = configparser.ConfigParser()
    cfg["a1"] = dict(ropts, arch_name="rnn", **OPT)
    head = dict(dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False", arch_name="head",
                dnn_lay="1928", dnn_drop="0.0", dnn_use_batchnorm="False", dnn_use_laynorm="False",
                dnn_act="softmax", **dict(OPT, arch_lr="0.0004"))
    cfg["a2"] = head
    cfg["a3"] = dict(head, arch_name="mono", dnn_lay="48")
    torch.manual_seed(0)
    np.random.seed(0)
    rnn = getattr(ON, cls)(cfg["a1"], 440)
    if cfg_name == "c5":
        pset = np.load(os.path.join(ROOT, "tests", "golden", "quant.npz"),
                       allow_pickle=False)["pattern_set"]
        rnn.pattern_kernels = pset.reshape(16, 8, 8)
    nets = {"rnn": rnn, "head": ON.MLP(cfg["a2"], rnn.out_dim), "mono": ON.MLP(cfg["a3"], rnn.out_dim)}
    opts = {k: ON.make_optimizer(nets[k].parameters(), cfg[s]) for k, s in
            (("rnn", "a1"), ("head", "a2"), ("mono", "a3"))}
    for n in nets.values():
        n.train()
    lines = OR.parse_model("o1=compute(rnn,fea)\no2=compute(head,o1)\no3=compute(mono,o1)\n"
                           "lm=cost_nll(o3,lab_mono)\nlmw=mult_constant(lm,1.0)\n"
                           "lc=cost_nll(o2,lab_cd)\nloss_final=sum(lc,lmw)\n"
                           "err_final=cost_err(o2,lab_cd)")
    rs = np.random.RandomState(1)
    inp = torch.from_numpy(np.concatenate([rs.randn(T, B, 440), rs.randint(0, 48, (T, B, 2))],
                                          2).astype(np.float32))
    seq = {"rnn": True, "head": False, "mono": False}

    def step():
        OR.train_step(lines, nets, opts, seq, {"fea": (0, 440)}, {"lab_cd": 440, "lab_mono": 441},
                      inp, T, B)

    step()                                   # warm-up (allocations, pattern masks)
    n, t0 = 0, time.time()
    while n == 0 or time.time() - t0 < seconds:
        step()
        n += 1
    dt = time.time() - t0
    return n * T * B / dt, n, dt


# all-core sample length cap: C4's eager step at the GPU-like T = 381 takes 105 s on 8 threads
# (its per-frame cost GROWS with T: 58 frames/s there against 122 on ONE thread at T = 24 — every
# time step's U-gradient accumulation streams the 4 x 1024 x 1024 fp32 U matrices through DRAM), so
# the bench's bounded sample runs C4 at T = 96; profiles/r03_cpu_seq_baselines.json holds the
# full-T figures measured in the build container
T_CAP = {"c4": 96}


def cpu_baseline(cfg_name, seconds=10.0, T=None, T1=24):
    """CPU baseline of a sequence configuration on the host cores: the oracle restatement (kind
    "port"; its speed against the reference itself: profiles/r03_cpu_calibration.json) on all
    cores at a padded length drawn like the GPU's (gpu_like_T, capped by T_CAP), and on ONE core
    (cores_1) at a short batch T1 (one core at T ~ 300 takes minutes per step)."""
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    threads = min(threads, os.cpu_count())
    _, _, B = rec_opts(cfg_name)
    T = T or min(gpu_like_T(cfg_name), T_CAP.get(cfg_name, 10 ** 9))
    v, n, dt = _cpu_rate(cfg_name, T, threads, seconds)
    v1, n1, dt1 = _cpu_rate(cfg_name, T1, 1, seconds / 2)
    torch.set_num_threads(threads)
    return {"value": round(v, 1), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": "%d training steps of %s (B=%d sentences x T=%d frames, T drawn like the "
                      "GPU's%s, oracle restatement, torch-CPU eager, %d threads, %.1f s)"
                      % (n, cfg_name, B, T, " and capped" if cfg_name in T_CAP else "", threads,
                         dt),
            "cores_1": {"value": round(v1, 1), "unit": "frames/s", "cores": 1,
                        "sample": "%d training steps (B=%d x T=%d, 1 thread, %.1f s)"
                                  % (n1, B, T1, dt1)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c4,c5,gru")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--prec", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--graphs", action="store_true", help="replay per-T captured step graphs")
    a = ap.parse_args()
    out = []
    for c in a.configs.split(","):
        r = run(c, a.steps, a.warmup, prec=a.prec, graphs=a.graphs)
        print(json.dumps(r), flush=True)
        out.append(r)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
