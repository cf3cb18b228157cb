"""bench.py — training throughput (acoustic frames/s) of the pkc run_nn hot path on MI355X.

Workload (BASELINE.json configs[1], "TIMIT_baselines MLP 5x1024 bf16 on 1 MI355X, dense MFMA
path"): cfg/TIMIT_baselines/TIMIT_MLP_fmllr.cfg architecture — fMLLR 40 x 11 context = 440 inputs,
5 x 1024 ReLU+BN+dropout 0.15 (SGD lr 0.08), heads 1928 cd + 48 mono LogSoftmax (RMSprop 4e-4),
batch_size_train = 128 frames, loss = NLL(cd) + 1.0 NLL(mono), err = cost_err(cd).
Synthetic "TIMIT-shaped fMLLR" chunk: ~740 utterances of 150-450 frames x 40 dims,
prepared on the GPU (context window + chunk normalisation + frame shuffle) like a real chunk.

A step = one batch of the chunk: batch gather, forward, fused LogSoftmax/NLL heads, backward,
[RCCL all-reduce of the flat gradient buffer when N > 1], optimizer — replayed from hipGraphs.
Multi-GPU: one process per GPU (torch.distributed.run), chunk-level data parallelism: every rank
trains its own chunk slice at the cfg batch size (weak scaling), gradients averaged every step.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# dense MFMA peaks (spec); the compensated bf16 form (PKC_PREC_BF16X3) issues 3 bf16 MFMAs per
# product: its peak in algorithmic flops is a third of bf16's
MFMA_PEAK_TFLOPS = {"fp32": 157.3, "bf16": 2500.0, "bf16x3": 2500.0 / 3}
PREC_NAMES = {"fp32": 0, "bf16": 1, "bf16x3": 3}          # pkc._lib.PREC_*


def c1_cfg(drop="0.15"):
    import configparser
    base = dict(dnn_use_laynorm_inp="False", dnn_use_batchnorm_inp="False", to_do="train",
                mlp_hcgs="False", mlp_quant="False", mlp_prune="False", guided_hcgs="False",
                apply_guided_hcgs="False", skip_regularization="False", arch_freeze="False")
    cfg = configparser.ConfigParser()
    cfg["architecture1"] = dict(base, arch_name="MLP_layers1", dnn_lay="1024,1024,1024,1024,1024",
                                dnn_drop=",".join([drop] * 5), dnn_use_batchnorm="True,True,True,True,True",
                                dnn_use_laynorm="False,False,False,False,False",
                                dnn_act="relu,relu,relu,relu,relu", arch_lr="0.08", arch_opt="sgd",
                                opt_momentum="0.0", opt_weight_decay="0.0", opt_dampening="0.0",
                                opt_nesterov="False")
    head = dict(base, arch_name="MLP_layers2", dnn_lay="1928", dnn_drop="0.0",
                dnn_use_batchnorm="False", dnn_use_laynorm="False", dnn_act="softmax",
                arch_lr="0.0004", arch_opt="rmsprop", opt_momentum="0.0", opt_alpha="0.95",
                opt_eps="1e-8", opt_centered="False", opt_weight_decay="0.0")
    cfg["architecture2"] = head
    cfg["architecture3"] = dict(head, arch_name="MLP_layers3", dnn_lay="48")
    cfg["model"] = {"model": "out_dnn1=compute(MLP_layers1,fmllr)\n"
                             "out_dnn2=compute(MLP_layers2,out_dnn1)\n"
                             "out_dnn3=compute(MLP_layers3,out_dnn1)\n"
                             "loss_mono=cost_nll(out_dnn3,lab_mono)\n"
                             "loss_mono_w=mult_constant(loss_mono,1.0)\n"
                             "loss_cd=cost_nll(out_dnn2,lab_cd)\n"
                             "loss_final=sum(loss_cd,loss_mono_w)\n"
                             "err_final=cost_err(out_dnn2,lab_cd)"}
    return cfg


DIMS = (("architecture1", 440), ("architecture2", 1024), ("architecture3", 1024))


def synth_chunk(seed, n_utt):
    """lengths U[150,450], 40-dim N(0,1) + per-utterance offset N(0,0.3),
    cd labels U[0,1928), mono U[1,48]."""
    rs = np.random.RandomState(seed)
    fea, cd, mono = {}, {}, {}
    for i in range(n_utt):
        k = "spk%03d_utt%05d" % (i % 462, i)
        T = rs.randint(150, 451)
        fea[k] = (rs.randn(T, 40) + rs.randn(1, 40) * 0.3).astype(np.float32)
        cd[k] = rs.randint(0, 1928, size=T).astype(np.int32)
        mono[k] = rs.randint(1, 49, size=T).astype(np.int32)
    return fea, cd, mono


def build(prec, batch, rank, world, seed=2234):
    from pkc import _lib
    from pkc.data_io import prepare_chunk
    from pkc.engine import Engine, parse_model
    from pkc.neural_networks import MLP
    cfg = c1_cfg()
    torch.manual_seed(seed)
    np.random.seed(seed)
    nets, opts = {}, {}
    for sec, inp in DIMS:
        o = cfg[sec]
        nets[o["arch_name"]] = MLP(o, inp).cuda().train()
        opts[o["arch_name"]] = o
    # chunk-level DP: rank r prepares its own chunk slice (different utterances)
    fea, cd, mono = synth_chunk(seed + 1000 * rank, 740)
    t0 = time.time()
    chunk = prepare_chunk(fea, [cd, mono], ["lab_cd", "lab_mono"], 5, 5, 1000,
                          shuffle_rng=np.random.RandomState(seed), fea_name="fmllr")
    torch.cuda.synchronize()
    prep_s = time.time() - t0
    eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), chunk.fea_cols, chunk.lab_names,
                 batch=batch, prec=prec, seed=seed + rank, grad_scale=1.0 / world)
    eng.bind_chunk(chunk.feats, chunk.labels, chunk.n_rows)
    return eng, chunk, prep_s, nets


def cpu_baseline(batch, seconds=12.0):
    """The oracle (reference algorithm restated in PyTorch-CPU eager) on the host cores, and on
    one core (cores_1)."""
    from oracle import nets as ON
    from oracle import run as OR
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    threads = min(threads, os.cpu_count())
    cfg = c1_cfg()
    lines = OR.parse_model(cfg["model"]["model"])
    rs = np.random.RandomState(1)
    inp = torch.from_numpy(np.concatenate([rs.randn(batch, 440), rs.randint(0, 48, (batch, 2))],
                                          1).astype(np.float32))
    fc, lc = {"fmllr": (0, 440)}, {"lab_cd": 440, "lab_mono": 441}

    def rate(nthreads, secs):
        torch.set_num_threads(nthreads)
        torch.manual_seed(0)
        nets, opts = {}, {}
        for sec, inp_dim in DIMS:
            o = cfg[sec]
            nets[o["arch_name"]] = ON.MLP(o, inp_dim).train()
            opts[o["arch_name"]] = ON.make_optimizer(nets[o["arch_name"]].parameters(), o)
        seq = {k: False for k in nets}
        for _ in range(2):
            OR.train_step(lines, nets, opts, seq, fc, lc, inp)
        n, t0 = 0, time.time()
        while n == 0 or time.time() - t0 < secs:
            OR.train_step(lines, nets, opts, seq, fc, lc, inp)
            n += 1
        dt = time.time() - t0
        return n * batch / dt, n, dt

    v, n, dt = rate(threads, seconds)
    v1, n1, dt1 = rate(1, seconds / 2)
    torch.set_num_threads(threads)
    out = {"value": round(v, 1), "unit": "frames/s", "cores": threads, "kind": "port",
           "sample": "%d training steps of the C1 MLP at B=%d (oracle restatement, torch-CPU eager, "
                     "%d threads, %.1f s)" % (n, batch, threads, dt),
           "cores_1": {"value": round(v1, 1), "unit": "frames/s", "cores": 1,
                       "sample": "%d training steps at B=%d, 1 thread, %.1f s" % (n1, batch, dt1)}}
    try:   # the restatement's speed relative to the reference itself (scripts/cpu_calibrate.py)
        cal = json.load(open(os.path.join(ROOT, "profiles", "r03_cpu_calibration.json")))
        out["calibration_port_over_reference"] = {
            "mlp": {k: v["oracle_over_reference"] for k, v in cal["results"].items()},
            "ligru_seq": {k: v["oracle_over_reference"] for k, v in cal["sequence"]["results"].items()}}
    except (OSError, ValueError, KeyError):
        pass
    return out


def pmc_traffic(label):
    """HBM bytes per launch of `label` from the committed rocprofv3 PMC summary
    (scripts/gpu.sh pmc -> profiles/*pmc_traffic.json): (2 x FETCH_SIZE + WRITE_SIZE) KiB, the
    gfx950 FETCH_SIZE half-count correction applied as MI355X_MICROARCH.md's HBM section
    prescribes (it is exact for 128-byte coalesced reads; for 64-byte row segments it can
    over-count the reads up to 2x — the summary keeps the raw counters).  None when the summary
    is for another launch."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("label") == label and d.get("traffic_bytes_per_launch"):
            return d["traffic_bytes_per_launch"]
    return None


def batch_sweep(prec, batches=(1024, 4096), steps=150):
    """Informational: the same step at larger frame batches — not `value`.
    (150 steps: with 30, the 20-40 ms timed regions read 10-20 % low against bench.py --batch runs
    of the same build, profiles/r04_bench_latest.json vs r04_bn_bwd_epi_ab.txt)"""
    out = {}
    for b in batches:
        eng, _, _, _ = build(prec, b, 0, 1)
        for _ in range(3):
            eng.train_step()
        eng.capture(steps_per_graph=graph_steps(steps))
        eng.train_steps(16)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.train_steps(steps)
        torch.cuda.synchronize()
        out[str(b)] = round(steps * b / (time.perf_counter() - t0), 1)
        del eng
        torch.cuda.empty_cache()
    return out


def launch_ranks(n):
    """`bench.py --gpus N` started as one process (no WORLD_SIZE): run N ranks through
    torch.distributed.run as child processes — before this process touches the GPU — and return
    their exit status (rank 0 prints the line)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def parity_leg(prec, batch, seed=2234):
    """Posterior error of the measured configuration (BASELINE metric: "posterior max-abs-err vs
    ref"): the engine's first training step on one batch of the C2 model — same initial weights,
    same injected dropout masks — against the oracle (the reference's algorithm in fp32 on the
    CPU).  Part of the CPU-baseline leg: the oracle is the checker here, never the thing timed.
    Returns max abs / max relative error of the cd head's log-posteriors (the first step: later
    steps of this model at init are chaotic, tests/test_gpu_mlp.py::test_engine_c2_bf16_vs_oracle)."""
    from oracle import nets as ON
    from oracle import run as OR
    from pkc.engine import Engine, parse_model
    from pkc.neural_networks import MLP
    cfg = c1_cfg()
    torch.manual_seed(seed)
    nets, onets, opts, oopt = {}, {}, {}, {}
    for sec, inp in DIMS:
        o = cfg[sec]
        a = o["arch_name"]
        nets[a] = MLP(o, inp)
        onets[a] = ON.MLP(o, inp)
        onets[a].load_state_dict(nets[a].state_dict())
        onets[a].train()
        nets[a].cuda().train()
        opts[a] = o
        oopt[a] = ON.make_optimizer(onets[a].parameters(), o)
    rs = np.random.RandomState(seed)
    X = rs.randn(batch, 440).astype(np.float32)
    lab = np.stack([rs.randint(0, 1928, batch), rs.randint(0, 48, batch)], 1).astype(np.int32)
    keeps = {"MLP_layers1.%d" % i: torch.from_numpy((rs.rand(batch, 1024) > 0.15).astype(np.uint8))
             for i in range(5)}
    eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fmllr": (0, 440)},
                 ["lab_cd", "lab_mono"], batch=batch, prec=prec, seed=1,
                 drop_keep_in={k: v.cuda() for k, v in keeps.items()})
    eng.bind_chunk(torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda(), batch)
    eng.train_step()
    head = [l for l in eng.layers if l.arch == "MLP_layers2"][-1]
    post = head.out.view(batch, -1).cpu().double()
    inp = torch.from_numpy(np.concatenate([X, lab.astype(np.float32)], 1))
    body = onets["MLP_layers1"]
    f = body.forward
    dm = [keeps["MLP_layers1.%d" % i].float() for i in range(5)]
    body.forward = lambda x, _f=f: _f(x, drop_masks=dm)
    outs = OR.train_step(OR.parse_model(cfg["model"]["model"]), onets, oopt,
                         {a: False for a in onets}, {"fmllr": (0, 440)},
                         {"lab_cd": 440, "lab_mono": 441}, inp)
    ref = outs["out_dnn2"].detach().double()
    d = (post - ref).abs()
    return {"posterior_max_abs_err": float(d.max()),
            "posterior_max_rel_err": float((d / ref.abs().clamp_min(1e-3)).max()),
            "posterior_ref": "oracle fp32 (reference algorithm), first training step, B=%d" % batch}


def graph_steps(steps):
    """Steps per multi-step graph replay: the largest divisor of the timed step count in [8, 50]
    (8 when none), so the timed region is whole replays.  Each replay boundary leaves the GPU idle
    ≈ 9 µs before the next graph's first launch (profiles/r04_bench_step_timeline.txt); PKC_GRAPH_STEPS
    overrides."""
    env = os.environ.get("PKC_GRAPH_STEPS")
    if env:
        return int(env)
    divs = [d for d in range(8, 51) if steps % d == 0]
    return max(divs) if divs else 8


def time_steps(eng, steps, warmup, allreduce=None, world=1):
    eng.train_steps(warmup, allreduce)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.train_steps(steps, allreduce)        # exactly `steps` batches
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device="cuda")
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        dt = float(tt.item())
    return dt


REC_KERNELS = ("rnn_fwd_mm", "rnn_bwd_mm", "persist::", "lstmp::")   # the recurrences' step / loop kernels


def mfma_profile(name, prec="fp32"):
    """MFMA figures of a configuration from its committed rocprofv3 counter pass at `prec`
    (scripts/gpu.sh mfma -> profiles/r*_mfma_<name>[_bf16].json, scripts/mfma_summary.py); None
    without one.  "all_kernels": busy-cycle utilisation, MFMA-flop weighted over the kernels whose
    counter window is trustworthy (the large projection / weight-gradient GEMMs dominate it);
    "recurrent": the serial recurrence's own kernels (per-step launches or persistent loops) —
    their MFMA flops over their time, against the dense peak of the pass's dtype."""
    import glob
    suffix = "" if prec == "fp32" else "_" + prec
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_mfma_%s%s.json" % (name, suffix))),
                    reverse=True):
        try:
            rows = json.load(open(f))
            out = {"source": os.path.relpath(f, ROOT), "prec": prec}
            fl = sum(r["mfma_gflop"] for r in rows if r.get("mfma_util_pct") is not None)
            if fl > 0:
                out["all_kernels"] = {"mfma_util_pct": round(sum(
                    r["mfma_util_pct"] * r["mfma_gflop"] for r in rows
                    if r.get("mfma_util_pct") is not None) / fl, 2), "weighting": "mfma flops"}
            rec = [r for r in rows if any(k in r["kernel"] for k in REC_KERNELS)]
            if rec:
                gf = sum(r["mfma_gflop"] for r in rec)
                sec = sum(r["mfma_gflop"] / r["tflops"] * 1e-3 for r in rec if r.get("tflops"))
                tf = gf / sec * 1e-3 if sec > 0 else None
                peak = MFMA_PEAK_TFLOPS["bf16" if rows and rec[0].get("mfma_dtype") == "bf16"
                                        else "fp32"]
                out["recurrent"] = {"tflops": round(tf, 2) if tf else None,
                                    "pct_of_peak": round(100 * tf / peak, 3) if tf else None,
                                    "kernels": sorted({r["kernel"].split("(")[0] for r in rec})}
            if len(out) > 2:
                return out
        except (OSError, ValueError, KeyError, TypeError, ZeroDivisionError):
            continue
    return None


def seq_entry(name, steps, warmup, with_cpu, cpu_seconds, prec="fp32"):
    """A BASELINE sequence configuration measured like the headline: frames/s over `steps` timed
    sentence batches, its roofline (max(F_alg / MFMA peak, B_alg / HBM peak) over the
    measured time, and the serial-step figure) and a CPU baseline.  prec "fp32": the parity
    precision; "bf16": the performance mode (W projections, weight gradients and heads on bf16
    MFMA, the serial U products exact fp32), priced against the bf16 peak."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_seq
    r = bench_seq.run(name, steps=steps, warmup=warmup, prec=prec)
    achieved = r["alg_tflops_per_s"]
    peak = MFMA_PEAK_TFLOPS[prec]
    out = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if k != "config"}
    out["dtype"] = prec
    out["roofline"] = {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak,
                       "unit": "TFLOP/s", "frac": round(achieved / peak, 5),
                       "note": "algorithmic flops (W, U scaled by mask density, heads; x3 for "
                               "training) over padded rows / measured step time; the recurrence "
                               "is serial-latency-bound: see us_per_time_step_per_layer_fwd_bwd"}
    prof = mfma_profile(name, prec)
    if prof:
        out["roofline"]["mfma_util"] = prof
    # first-step posterior error of this mode at the config's layer sizes against the fp32 oracle
    # (after the timed region; the oracle is the checker, never the thing timed)
    out.update(bench_seq.parity(name, prec=prec))
    if with_cpu:
        out["cpu_baseline"] = bench_seq.cpu_baseline(name, seconds=cpu_seconds)
    return out


def measure_mlp(prec, args, rank, world, allreduce):
    """The C2 step at `prec`: live per-launch profile -> dominant entry point, the captured
    step's timed region (exactly args.steps batches), the dominant launch's roofline."""
    from pkc import _lib
    eng, chunk, prep_s, nets = build(prec, args.batch, rank, world)
    # per-launch device times of warm eager steps -> dominant kernel + its roofline inputs
    for _ in range(3):
        eng.train_step(allreduce)
    agg = {}
    NPROF = 5
    for _ in range(NPROF):
        prof = eng.profile_step()
        for label, fn, fl, nb, ms in prof:
            a = agg.setdefault(label, [0, 0.0, 0.0, 0.0])
            a[0] += 1
            a[1] += ms / NPROF
            a[2] += fl
            a[3] += nb
    for v in agg.values():
        v[0] //= NPROF
    # dominant kernel = the libpkc entry point with the largest in-step device time, measured
    # live with HIP events as (step graph) - (step graph without its launches) for the three
    # largest candidates by eager time (after this the weights are stale: it runs after the
    # timed region, or alone in a counter run)
    by_fn = {}
    for label, fn, fl, nb, ms in prof:
        f = by_fn.setdefault(fn, {"labels": set(), "launches": 0, "flops": 0.0, "bytes": 0.0,
                                  "eager_ms": 0.0})
        f["labels"].add(label)
        f["launches"] += 1
        f["flops"] += fl
        f["bytes"] += nb
        f["eager_ms"] += ms
    cands = sorted(by_fn, key=lambda k: -by_fn[k]["eager_ms"])[:3]

    def pick_dominant():
        costs = {fn: eng.step_cost_of(by_fn[fn]["labels"])[0] for fn in cands}
        fn = max(costs, key=costs.get)
        return fn, costs[fn]

    if args.pmc_replay:
        # counter runs (scripts/gpu.sh pmc): the dominant kernel's launches, N rounds, last
        dom_fn = args.pmc_kernel or pick_dominant()[0]
        nl = eng.replay_launches(dom_fn, args.pmc_replay)
        tag = dom_fn + ("" if prec == _lib.PREC_BF16 else
                        "@" + {v: k for k, v in PREC_NAMES.items()}[prec])
        print(json.dumps({"pmc_replay": tag, "launches": nl * args.pmc_replay}), flush=True)
        sys.exit(0)
    eng.capture(split_optimizer=world > 1, steps_per_graph=graph_steps(args.steps))
    graph_lps = eng.graph_launches_per_step
    dt = time_steps(eng, args.steps, args.warmup, allreduce, world)
    loss_sum, err_sum = eng.chunk_totals()
    n_done = args.warmup + args.steps
    dom_fn, dom_us = pick_dominant()
    d = by_fn[dom_fn]
    cnt = d["launches"]
    per_launch_fl = d["flops"] / cnt
    per_launch_nb = d["bytes"] / cnt
    avg_ms = dom_us / cnt * 1e-3
    pname = {v: k for k, v in PREC_NAMES.items()}[prec]
    traffic = pmc_traffic(dom_fn if pname == "bf16" else dom_fn + "@" + pname)
    del eng
    torch.cuda.empty_cache()
    # MFMA-bound only where the launch's arithmetic intensity exceeds the machine balance
    balance = MFMA_PEAK_TFLOPS[pname] * 1e12 / (HBM_PEAK_GBS * 1e9)
    if "gemm" in dom_fn and per_launch_fl / max(per_launch_nb, 1.0) > balance:
        bound, peak, unit = "mfma", MFMA_PEAK_TFLOPS[pname], "TFLOP/s"
        achieved = per_launch_fl / (avg_ms * 1e-3) / 1e12
    else:
        bound, peak, unit = "hbm", HBM_PEAK_GBS, "GB/s"
        achieved = per_launch_nb / (avg_ms * 1e-3) / 1e9
    frames = args.steps * args.batch * world
    return {"value": round(frames / dt, 1), "ms_per_step": round(dt / args.steps * 1e3, 4),
            "dtype": pname,
            "roofline": {"kernel": dom_fn, "labels": sorted(d["labels"]), "bound": bound,
                         "achieved": round(achieved, 2), "peak": peak, "unit": unit,
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "avg_launch_us": round(avg_ms * 1e3, 3), "launches_per_step": cnt,
                         "algorithmic_bytes_per_launch": per_launch_nb,
                         "algorithmic_flops_per_launch": per_launch_fl,
                         "mfma_tflops_per_launch": round(per_launch_fl / (avg_ms * 1e-3) / 1e12, 2)},
            "launches_per_step": len(prof),
            "graph_launches_per_step": graph_lps,
            "step_breakdown_us": {k: round(v[1] * 1e3, 2) for k, v in
                                  sorted(agg.items(), key=lambda kv: -kv[1][1])},
            "chunk_frames_per_rank": chunk.n_rows, "chunk_prep_s": round(prep_s, 3),
            "mean_loss": round(loss_sum / max(1, n_done), 4)}


WORKLOADS = {
    "c2": "TIMIT_baselines MLP 440-5x1024-{1928,48} (TIMIT_MLP_fmllr.cfg), batch_size_train=128, "
          "dropout 0.15, SGD body + RMSprop heads",
    "c3": "TIMIT_CGS liGRU 4x550 bidirectional + HCGS [32,2]/[75,75] on W and U, B=8 sentences, "
          "heads 1928 cd + 48 mono",
    "c4": "Librispeech_baselines LSTM 4x1024 bidirectional, B=16 sentences per rank, T<=450, "
          "heads 1928 cd + 48 mono, chunk DP (frame-weighted all-reduce)",
    "c5": "LibriSpeech_CGS LSTM 3x512 + Pattern b08b08_k04_n16 + 8-bit weight / 16-bit input "
          "fake-quant, B=12 sentences per rank, T<=200, chunk DP (frame-weighted all-reduce)",
}


def seq_main(args, rank, world, allreduce):
    """`--config c3|c4|c5`: the sequence configuration measured as THE line (one rank per GPU,
    every rank its own synthetic chunk, B sentences per rank and step: weak scaling)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import bench_seq
    r = bench_seq.run(args.config, steps=args.steps, warmup=args.warmup, allreduce=allreduce,
                      rank=rank, world=world)
    if rank != 0:
        return
    peak = MFMA_PEAK_TFLOPS["fp32"]
    res = {"metric": "acoustic frames/sec (train)", "value": round(r["frames_per_s"], 1),
           "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(r["ms_per_step"], 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic TIMIT-shaped chunk per rank (64 x B length-sorted sentences, "
                   "440-dim features), random-init weights",
           "config": {"workload": WORKLOADS[args.config],
                      "global_batch": r["batch_sentences"] * world,
                      "parallelism": "dp%d" % world},
           "roofline": {"bound": "mfma", "achieved": round(r["alg_tflops_per_s"], 3),
                        "peak": peak, "unit": "TFLOP/s",
                        "frac": round(r["alg_tflops_per_s"] / peak, 5), "traffic": None,
                        "note": "whole step: algorithmic flops (W, U scaled by mask density, "
                                "heads; x3 for training) over padded rows / measured time; the "
                                "recurrence is serial-latency-bound (us_per_time_step...)"},
           "us_per_time_step_per_layer_fwd_bwd": round(r["us_per_time_step_per_layer_fwd_bwd"], 3),
           "mean_T": round(r["mean_T"], 1)}
    prof = mfma_profile(args.config)
    if prof:
        res["roofline"]["mfma_util"] = prof
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = bench_seq.cpu_baseline(args.config, seconds=args.cpu_seconds)
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2: the headline MLP (default); c3/c4/c5: a sequence configuration "
                         "as the line (with --gpus N: N data-parallel ranks of it)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--prec", choices=["bf16", "fp32", "bf16x3"], default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-batch-sweep", action="store_true")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 value of the headline")
    ap.add_argument("--no-seq-configs", action="store_true",
                    help="skip the informational C3/C4/C5 sequence-model throughputs")
    ap.add_argument("--pmc-replay", type=int, default=0,
                    help="only replay the dominant launch N times (for rocprofv3 --pmc passes)")
    ap.add_argument("--pmc-kernel", default="",
                    help="entry point to replay with --pmc-replay (default: pick the dominant one)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PKC_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks sharing one GPU
    backend = os.environ.get("PKC_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    allreduce = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

        def allreduce(t, async_op=False):
            return dist.all_reduce(t, async_op=async_op)
    if args.config != "c2":
        seq_main(args, rank, world, allreduce)
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    from pkc import _lib
    prec = PREC_NAMES[args.prec]
    head = measure_mlp(prec, args, rank, world, allreduce)
    extra = {}
    if rank == 0 and world == 1 and args.prec == "bf16" and not args.no_fp32:
        # the same configuration in fp32 (the reference's precision) and in compensated bf16
        # (bf16 MFMA, fp32-class products): the entries whose posteriors meet north_star's 1e-4,
        # measured the same way, each with its own roofline
        extra["fp32_entry"] = measure_mlp(_lib.PREC_FP32, args, 0, 1, None)
        extra["fp32_value"] = extra["fp32_entry"]["value"]
        extra["bf16x3_entry"] = measure_mlp(_lib.PREC_BF16X3, args, 0, 1, None)
        extra["bf16x3_value"] = extra["bf16x3_entry"]["value"]
        if not args.no_cpu_baseline:
            extra["fp32_entry"].update(parity_leg(_lib.PREC_FP32, args.batch))
            extra["bf16x3_entry"].update(parity_leg(_lib.PREC_BF16X3, args.batch))
    sweep = {}
    if rank == 0 and world == 1 and not args.no_batch_sweep:
        sweep = batch_sweep(prec)
        if args.prec == "bf16" and not args.no_fp32:
            # the reference-precision modes at the large batches: exact fp32 and compensated bf16
            # (fp32-class products on the bf16 MFMA), with the first-step posterior error of each
            # batch against the oracle (north_star: 1e-4)
            by = {"bf16": sweep}
            for name, pr in (("fp32", _lib.PREC_FP32), ("bf16x3", _lib.PREC_BF16X3)):
                by[name] = batch_sweep(pr)
                torch.cuda.empty_cache()
            by["bf16x3_over_fp32"] = {b: round(by["bf16x3"][b] / by["fp32"][b], 3) for b in by["fp32"]}
            if not args.no_cpu_baseline:
                by["bf16x3_posterior_max_rel_err"] = {
                    b: parity_leg(_lib.PREC_BF16X3, int(b))["posterior_max_rel_err"] for b in by["fp32"]}
            extra["batch_sweep_by_prec"] = by
    seq = {}
    if rank == 0 and world == 1 and not args.no_seq_configs:
        # BASELINE configs C3-C5: C3 (the largest single-GPU config) measured like the headline,
        # C4 / C5 informational
        seq["c3"] = seq_entry("c3", max(20, args.steps), 3, False, 0)
        torch.cuda.empty_cache()
        seq["c3"]["bf16_entry"] = seq_entry("c3", max(20, args.steps), 3, False, 0, "bf16")
        torch.cuda.empty_cache()
        for c in ("c4", "c5"):
            seq[c] = seq_entry(c, 8, 2, False, 0)
            torch.cuda.empty_cache()
            seq[c]["bf16_entry"] = seq_entry(c, 8, 2, False, 0, "bf16")
            torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        extra.update(parity_leg(prec, args.batch))
    if rank == 0:
        res = {
            "metric": "acoustic frames/sec (train)",
            "value": head["value"],
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.prec,
            "data": "synthetic TIMIT-shaped fMLLR chunk (740 utts x U[150,450] frames x 40 dims, "
                    "context +-5, GPU-prepared), random-init weights",
            "config": {"workload": WORKLOADS["c2"],
                       "global_batch": args.batch * world, "parallelism": "dp%d" % world,
                       "chunk_frames_per_rank": head["chunk_frames_per_rank"]},
            "roofline": head["roofline"],
            "launches_per_step": head["launches_per_step"],
            "graph_launches_per_step": head["graph_launches_per_step"],
            "step_breakdown_us": head["step_breakdown_us"],
            "batch_sweep_frames_per_s": sweep,
            "sequence_configs": seq,
            "chunk_prep_s": head["chunk_prep_s"],
            "mean_loss": head["mean_loss"],
        }
        res.update(extra)
        if not args.no_cpu_baseline and world == 1:
            res["cpu_baseline"] = cpu_baseline(args.batch, args.cpu_seconds)
            sys.path.insert(0, os.path.join(ROOT, "scripts"))
            import bench_seq
            for c, e in seq.items():          # after every timed region: CPU legs last
                e["cpu_baseline"] = bench_seq.cpu_baseline(c, seconds=args.cpu_seconds)
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    _a = [a for a in sys.argv[1:]]
    _n = 1
    for i, a in enumerate(_a):
        if a == "--gpus" and i + 1 < len(_a):
            _n = int(_a[i + 1])
        elif a.startswith("--gpus="):
            _n = int(a.split("=", 1)[1])
    if _n > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(_n))
    main()
