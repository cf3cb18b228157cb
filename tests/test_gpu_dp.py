"""Chunk-level data parallelism through the Engine (SURVEY 8e parity check): 2 ranks (gloo,
sharing the one GPU; on a node the same code runs over RCCL) each train their half of every
global batch with Engine(grad_scale = 1/2) and the bucketed, overlapped gradient all-reduce
(pkc.dist.GradAllReduce) — eagerly and from the split hipGraphs — against one process training
the full global batch.  No BatchNorm (per-rank batch statistics differ by design), dropout 0.

Checked: the two replicas are bit-identical after every run; they equal the single-process
full-batch training within fp32 summation-order tolerance; the summed loss equals the full-batch
loss.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT
from quantcheck import assert_few_flips, rmsprop_quanta

pytestmark = pytest.mark.gpu
STEPS, B = 3, 32


def full_batch_reference(bn=False, prec=None, wide=False, b=B):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dp_engine_worker as W
    X, lab = W.data(STEPS, 2 * b, *((1928, 48) if wide else (32, 8)))
    eng, nets = W.build(W.dp_config(bn=bn, wide=wide), 1, 2 * b, X, lab, prec=prec)
    for _ in range(STEPS):
        eng.train_step()
    torch.cuda.synchronize()
    loss, _ = eng.chunk_totals()
    return loss, {a + "/" + k: v.detach().cpu().numpy() for a in nets
                  for k, v in nets[a].state_dict().items()}


@pytest.mark.parametrize("mode", ["eager", "graph", "syncbn", "bf16graph", "wide", "widegraph"])
def test_dp_engine_two_ranks_equal_full_batch(mode, tmp_path):
    """syncbn: the body layers carry BatchNorm, its statistics synchronised over the ranks
    (pkc.dist.SyncBatchNorm, SURVEY 8e's DP parity recipe): then the split global batch still
    equals the one-process full batch, running statistics included.  bf16graph: the bench's
    precision (bf16-stored operands, the optimizer refreshing the bf16 weight copies after the
    all-reduce) from the split graphs: replicas bit-identical; against the one-process bf16 run
    the fp32 sums differ in order, which can flip a weight's bf16 rounding: 1e-2 / 1e-3 on the
    weights and 1e-3 on the loss (a stale bf16 copy moves the loss by far more).  wide / widegraph:
    1024 rows per rank, hidden 2048, heads 1928 (one dW matmul) and 48 (split-K dW): the first
    all-reduce bucket, cut at the cd head, must wait for the mono head's slab sum."""
    wide = mode.startswith("wide")
    b = 1024 if wide else B
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000 +
                                                            {"graph": 7, "syncbn": 13,
                                                             "bf16graph": 19, "wide": 23,
                                                             "widegraph": 29}.get(mode, 0)),
           os.path.join(ROOT, "tests", "dp_engine_worker.py"), str(tmp_path), mode, str(STEPS),
           str(b)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    g0 = np.load(os.path.join(tmp_path, "rank0_%s.npz" % mode))
    g1 = np.load(os.path.join(tmp_path, "rank1_%s.npz" % mode))
    assert int(g0["calls"]) == 2 * STEPS          # two buckets per step
    from pkc import _lib as L
    bf = mode == "bf16graph"
    loss, ref = full_batch_reference(bn=mode == "syncbn", prec=L.PREC_BF16 if bf else None,
                                     wide=wide, b=b)
    for k, v in ref.items():
        np.testing.assert_array_equal(g0[k], g1[k], err_msg="replicas differ: " + k)
        if k.endswith("num_batches_tracked"):
            continue
        np.testing.assert_allclose(g0[k], v, rtol=1e-2 if bf else 1e-4, atol=1e-3 if bf else 1e-6,
                                   err_msg=k)
    np.testing.assert_allclose(float(g0["loss"]), loss, rtol=1e-3 if bf else 1e-5)


def test_dp_c_abi_allreduce_world1():
    """The C-ABI data-parallel exchange (include/pkc.h pkc_dp_*: RCCL communicator inside libpkc,
    for hosts without torch.distributed) on a one-rank world: the all-reduce is the identity, and
    an Engine step that exchanges its gradients through it equals a step without exchange."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dp_engine_worker as W
    from pkc import dist as DP
    ar = DP.CAbiAllReduce(device=0)
    try:
        x = torch.randn(1000003, device="cuda")
        ref = x.clone()
        ar(x)
        torch.cuda.synchronize()
        assert torch.equal(x, ref)
        X, lab = W.data(STEPS, B)
        states = []
        for use in (False, True):
            eng, nets = W.build(W.dp_config(), 1, B, X, lab)
            for _ in range(STEPS):
                eng.train_step(ar if use else None)
            torch.cuda.synchronize()
            states.append({a + "/" + k: v.detach().cpu() for a in nets
                           for k, v in nets[a].state_dict().items()})
        for k in states[0]:
            assert torch.equal(states[0][k], states[1][k]), k
        assert ar.calls >= STEPS + 1
    finally:
        ar.close()


SEQ_STEPS = 2


def _oracle_seq_dp(name, ranks, X, lab):
    """SURVEY 8e's sequence-DP step restated on the oracle: one model replica per rank, each
    running its own padded sentence batch (its own BatchNorm statistics, T_r), its loss scaled by
    its frame weight; the replicas' gradients summed (the all-reduce), ONE optimizer step, the
    result copied to every replica; BatchNorm running statistics averaged at the chunk end
    (pkc.dist.average_buffers)."""
    from oracle import nets as ON
    from oracle import run as OR
    from test_gpu_configs import build_pair
    reps = []
    for _ in ranks:
        _, onets, opts, model, B = build_pair(name, drop="0.0")
        for n in onets.values():
            n.train()
        reps.append(onets)
    oopt = {k: ON.make_optimizer(reps[0][k].parameters(), opts[k]) for k in reps[0]}
    lines = OR.parse_model(model)
    F = 440
    loss_sum = 0.0
    for s in range(SEQ_STEPS):
        for rep in reps:
            for n in rep.values():
                n.zero_grad(set_to_none=True)
        for rep, g in zip(reps, ranks):
            T = int(g["T"][s])
            inp = torch.zeros(T, B, F + 2)
            for k in range(B):
                b0, n, left = int(g["begs"][s][k]), int(g["lens"][s][k]), int(g["lefts"][s][k])
                inp[left:left + n, k, :F] = torch.from_numpy(X[b0:b0 + n])
                inp[left:left + n, k, F:] = torch.from_numpy(lab[b0:b0 + n].astype(np.float32))
            outs = OR.forward_model(lines, rep, {"rnn": True, "head": False, "mono": False},
                                    {"fea": (0, F)}, {"lab_cd": F, "lab_mono": F + 1}, inp, T, B)
            (outs["loss_final"] * float(g["scales"][s])).backward()
            loss_sum += float(outs["loss_final"])
        for k in reps[0]:
            for ps in zip(*[rep[k].parameters() for rep in reps]):
                if ps[0].grad is None:
                    continue
                for p in ps[1:]:
                    ps[0].grad += p.grad
        for o in oopt.values():
            o.step()
        for k in reps[0]:
            for ps in zip(*[rep[k].parameters() for rep in reps]):
                for p in ps[1:]:
                    p.data.copy_(ps[0].data)
    for k in reps[0]:
        for bufs in zip(*[rep[k].named_buffers() for rep in reps]):
            if bufs[0][0].endswith("running_mean") or bufs[0][0].endswith("running_var"):
                bufs[0][1].copy_(sum(b for _, b in bufs) / len(bufs))
    return reps[0], loss_sum, opts


@pytest.mark.parametrize("name", ["c4", "c5"])
def test_dp_seq_two_ranks_equal_oracle_dp(name, tmp_path):
    """Sequence-model chunk DP through the Engine: 2 gloo ranks on one GPU
    train the C4 / C5 layer shapes (LSTM 4x1024 bidirectional; LSTM 3x512 + pattern + 8/16-bit
    quantisation) on their round-robin halves of a length-sorted chunk — unequal padded T per rank,
    so each rank's loss carries its frame weight T_r / sum T (pkc.dist.frame_weights, one
    collective per chunk) — with the gradient all-reduce.  Checked: the frame weights, the two
    replicas bit-identical, and the replica equal to the same data-parallel step restated on the
    oracle (fp32): loss within 1e-5, weights within the tolerances of test_gpu_configs (C5: the
    fake-quantisation grids, see there)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dp_seq_worker as SW
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port",
           str(29500 + os.getpid() % 1000 + {"c4": 31, "c5": 37}[name]),
           os.path.join(ROOT, "tests", "dp_seq_worker.py"), str(tmp_path), name, str(SEQ_STEPS)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    g = [np.load(os.path.join(tmp_path, "seq_rank%d_%s.npz" % (k, name))) for k in range(2)]
    # two buckets per step: the first cut after a recurrent layer's weight gradients
    # (Engine._bucket_cut on a RecNode), overlapping the lower layers' BPTT
    assert int(g[0]["calls"]) == 2 * SEQ_STEPS
    # unequal padded lengths, frame weights T_r / (T_0 + T_1)
    T = np.stack([gi["T"] for gi in g])
    assert (T[0] != T[1]).any()
    for k in range(2):
        np.testing.assert_allclose(g[k]["scales"][:SEQ_STEPS], T[k] / T.sum(0), rtol=1e-12)
    keys = [k for k in g[0].files if "/" in k]
    for k in keys:
        np.testing.assert_array_equal(g[0][k], g[1][k], err_msg="replicas differ: " + k)
    lens, end, X, lab, B = SW.chunk(name, SEQ_STEPS, 2)
    onets, oloss, opts = _oracle_seq_dp(name, g, X, lab)
    np.testing.assert_allclose(float(g[0]["loss"]), oloss, rtol=1e-5)
    w_tol = 2e-2 if name == "c5" else 5e-3
    nl = len(onets["rnn"].pattern_masks[next(iter(onets["rnn"].pattern_masks))]) if name == "c5" else 0
    for key in keys:
        if key.endswith("num_batches_tracked"):
            continue
        arch, pname = key.split("/", 1)
        ref = onets[arch].state_dict()[pname].double()
        parts = pname.split(".")
        if arch == "rnn" and name == "c5" and pname.endswith("weight") and len(parts[0]) == 3:
            ref = ref * onets["rnn"].pattern_masks[parts[0]][int(parts[1])].double() ** nl
        got = torch.from_numpy(g[0][key]).double()
        if name == "c5" and arch == "rnn" and pname.endswith("weight") and got.dim() == 2:
            assert_few_flips(got.numpy(), ref.numpy(), key, 2e-3,     # quantcheck
                             max_quanta=rmsprop_quanta(float(opts[arch]["arch_lr"]), SEQ_STEPS) + 1)
        if name == "c5" and ".bias" in pname and pname.startswith("bn"):
            lr = float(opts[arch]["arch_lr"])          # quantum-flip noise, bounded by RMSprop
            assert (got - ref).abs().max().item() <= 2 * 4.48 * lr * SEQ_STEPS, key
            continue
        d = (got - ref).norm().item()
        assert d <= w_tol * ref.norm().item() + 1e-6, "%s rel err %.3g" % (key, d / ref.norm().item())
