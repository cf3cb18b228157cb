"""Data-parallel path (pkc.dist) on CPU: world_size-2 gloo process groups.

Covers the sharding rules, the per-step collective (one SUM all-reduce of the flat gradient
buffer with the loss gradient pre-scaled by 1/R), the per-chunk reductions (loss/err totals, BN
running-statistics averaging), the replica check, and the DP identity the design relies on:
with the loss scaled by 1/R, the all-reduced gradient of R half-batches equals the single-process
full-batch gradient (oracle MLP without BatchNorm, dropout 0 — SURVEY.md §8e parity check).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cases import build_mlp_config


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, ws=2, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_entry, args=(fn, r, ws, port, q) + args) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = {}
    while not q.empty():
        r, v = q.get()
        res[r] = v
    for p in procs:
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
    return [res[r] for r in range(ws)]


def _entry(fn, rank, ws, port, q, *args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from pkc import dist as DP
    DP.init_from_env(backend="gloo")
    try:
        q.put((rank, fn(rank, ws, *args)))
    finally:
        dist.destroy_process_group()


def test_shard_rows_partition():
    from pkc import dist as DP
    for n, ws in ((1000, 2), (1001, 4), (7, 8)):
        rs = [DP.shard_rows(n, r, ws) for r in range(ws)]
        sizes = {b - a for a, b in rs}
        assert len(sizes) == 1                       # equal shares: equal step counts
        assert all(rs[i][1] == rs[i + 1][0] for i in range(ws - 1))
        assert rs[-1][1] <= n and rs[0][0] == 0


def test_shard_sentences_round_robin():
    from pkc import dist as DP
    lens = np.array([3, 4, 4, 5, 7, 9, 9, 12, 15])
    end = np.cumsum(lens)
    seen = []
    for r in range(3):
        b, l = DP.shard_sentences(end, r, 3)
        np.testing.assert_array_equal(l, lens[r::3])
        np.testing.assert_array_equal(b + l, end[r::3])
        seen += list(b)
    assert sorted(seen) == sorted(np.concatenate([[0], end[:-1]]).tolist())


def _collectives(rank, ws):
    from pkc import dist as DP
    out = {}
    out["min"] = DP.agree_min(10 + rank)
    out["sum"] = DP.sum_scalars([1.5 * (rank + 1), rank])
    g = torch.full((5,), float(rank + 1))
    ar = DP.GradAllReduce()
    ar(g)
    out["grad"] = g.tolist()
    bn = torch.nn.BatchNorm1d(3)
    bn.running_mean.fill_(rank)
    bn.running_var.fill_(2.0 * rank + 1)
    DP.average_buffers([bn])
    out["rm"] = bn.running_mean.tolist()
    out["rv"] = bn.running_var.tolist()
    lin = torch.nn.Linear(4, 3)
    torch.manual_seed(0)
    lin.reset_parameters()
    out["same"] = DP.check_replicas([lin])
    if rank == 1:
        with torch.no_grad():
            lin.weight[0, 0] += 1e-3
    out["diff"] = DP.check_replicas([lin])
    return out


def test_collectives_world2():
    r0, r1 = _run(_collectives)
    for r in (r0, r1):
        assert r["min"] == 10
        assert r["sum"] == [4.5, 1.0]
        assert r["grad"] == [3.0] * 5
        assert r["rm"] == [0.5] * 3 and r["rv"] == [2.0] * 3
        assert r["same"] is True and r["diff"] is False


def _mlp_grads(rank, ws, B):
    """Gradients of the oracle MLP (no BN) on this rank's share of one global batch of B frames."""
    from oracle import nets as ON
    from pkc import dist as DP
    cfg = build_mlp_config("plain")
    body = dict(cfg["architecture1"])
    body.update(dnn_use_batchnorm="False,False")
    cfg["architecture1"] = body
    torch.manual_seed(5)
    np.random.seed(5)
    net1 = ON.MLP(cfg["architecture1"], 40)
    net2 = ON.MLP(cfg["architecture2"], 32)
    rs = np.random.RandomState(11)
    x = torch.from_numpy(rs.normal(size=(B, 40)).astype(np.float32))
    y = torch.from_numpy(rs.randint(0, 96, size=B).astype(np.int64))
    r0, r1 = DP.shard_rows(B, rank, ws)
    logp = net2(net1(x[r0:r1]))
    loss, _ = ON.nll_err(logp, y[r0:r1])
    (loss / ws).backward()                       # Engine(grad_scale=1/R) does this scaling
    params = list(net1.parameters()) + list(net2.parameters())
    flat = torch.cat([p.grad.reshape(-1) for p in params if p.grad is not None])
    if ws > 1:
        DP.GradAllReduce()(flat)
    return flat.numpy()


def test_dp_gradient_equals_full_batch():
    full = _mlp_grads(0, 1, 32)
    g0, g1 = _run(_mlp_grads, 2, 32)
    np.testing.assert_array_equal(g0, g1)        # replicas receive identical gradients
    np.testing.assert_allclose(g0, full, rtol=1e-5, atol=1e-8)


def _mlp_grads_uneven(rank, ws, cuts):
    """Frame-weighted DP (pkc.dist.frame_weight, the sequence-model scaling): rank r holds rows
    [cuts[r], cuts[r+1]) of one global batch (unequal shares, as unequal padded T_r * B), scales
    its mean loss by its share of the rows, and the summed gradient is the full-batch gradient."""
    from oracle import nets as ON
    from pkc import dist as DP
    cfg = build_mlp_config("plain")
    body = dict(cfg["architecture1"])
    body.update(dnn_use_batchnorm="False,False")
    cfg["architecture1"] = body
    torch.manual_seed(5)
    np.random.seed(5)
    net1 = ON.MLP(cfg["architecture1"], 40)
    net2 = ON.MLP(cfg["architecture2"], 32)
    rs = np.random.RandomState(12)
    B = cuts[-1]
    x = torch.from_numpy(rs.normal(size=(B, 40)).astype(np.float32))
    y = torch.from_numpy(rs.randint(0, 96, size=B).astype(np.int64))
    r0, r1 = (cuts[rank], cuts[rank + 1]) if ws > 1 else (0, B)
    w = DP.frame_weight(r1 - r0)
    logp = net2(net1(x[r0:r1]))
    loss, _ = ON.nll_err(logp, y[r0:r1])
    (loss * w).backward()
    flat = torch.cat([p.grad.reshape(-1) for p in list(net1.parameters()) + list(net2.parameters())
                      if p.grad is not None])
    if ws > 1:
        DP.GradAllReduce()(flat)
    return w, flat.numpy()


def test_dp_frame_weighted_gradient_equals_full_batch():
    cuts = [0, 30, 40]
    _, full = _mlp_grads_uneven(0, 1, cuts)
    (w0, g0), (w1, g1) = _run(_mlp_grads_uneven, 2, cuts)
    assert (w0, w1) == (0.75, 0.25)
    np.testing.assert_array_equal(g0, g1)
    np.testing.assert_allclose(g0, full, rtol=1e-5, atol=1e-8)


def _frame_weights(rank, ws, lens, B):
    from pkc import dist as DP
    return DP.frame_weights(lens[rank], B, 2).tolist()


def test_frame_weights_one_collective_per_chunk():
    """pkc.dist.frame_weights: every batch's loss scale of a chunk from the sentence lengths
    alone (T_r[i] = the longest of rank r's i-th B sentences; scale T_r[i] / sum_r T_r[i]), in one
    all-reduce at bind time instead of one host-blocking scalar all-reduce per step."""
    lens = [[5, 9, 3, 3, 7, 2, 30], [4, 4, 10, 1, 1, 1, 1]]       # B = 3: T = [9, 7] and [10, 1]
    w0, w1 = _run(_frame_weights, 2, lens, 3)
    np.testing.assert_allclose(w0, [9 / 19, 7 / 8], rtol=1e-15)
    np.testing.assert_allclose(w1, [10 / 19, 1 / 8], rtol=1e-15)
    assert _frame_weights(0, 1, lens, 3) == [1.0, 1.0]
