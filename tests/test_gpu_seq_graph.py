"""Sequence training steps replayed from captured graphs (Engine.capture on a sequence model: one
graph per padded length T, captured at its first batch) against the same steps issued eagerly:
bit-identical losses, posteriors and trained parameters, for liGRU + HCGS (block-sparse U), LSTM,
bidirectional LSTM and LSTM with 8-bit weights / 16-bit inputs (exact quantised-h products), and
in bf16 mode liGRU + HCGS (the persistent time loops) and the bidirectional LSTM (bf16 steps).  The batch metadata reaches the
device through the pinned ring (no host synchronisation per batch), and a batch's data-parallel
frame weight follows the batch it belongs to (SeqBatch.index)."""
import copy
import random

import numpy as np
import pytest
import torch

from test_gpu_seq import make_cfg

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _build(body):
    import pkc.neural_networks as NN
    cfg = make_cfg("lstm" if body == "lstm_quant" else body)
    if body == "lstm_quant":
        cfg["a1"].update(lstm_quant="True", lstm_quant_inp="True", param_quant="8,8", inp_quant="16")
    cls = {"ligru_hcgs_sparse": "liGRU", "lstm": "LSTM", "lstm_bidir": "LSTM",
           "lstm_quant": "LSTM"}[body]
    nets, opts = {}, {}
    for sec, inp in (("a1", 20), ("a2", None), ("a3", None)):
        o = cfg[sec]
        inp = inp or nets["rnn"].out_dim
        torch.manual_seed(3)
        np.random.seed(3)
        nets[o["arch_name"]] = getattr(NN, cls if sec == "a1" else "MLP")(o, inp)
        opts[o["arch_name"]] = o
    for n in nets.values():
        n.to(DEV).train()
    return cfg, nets, opts


@pytest.mark.parametrize("body", ["ligru_hcgs_sparse", "lstm", "lstm_bidir", "lstm_quant",
                                  "ligru_hcgs_sparse:bf16", "lstm_bidir:bf16"])
def test_seq_graph_replay_equals_eager(body):
    import pkc.engine as E
    from pkc import _lib as L
    from pkc.engine import Engine, parse_model
    body, _, mode = body.partition(":")
    prec = L.PREC_BF16 if mode == "bf16" else L.PREC_FP32
    cfg, nets0, opts = _build(body)
    F, B = 20, 4
    rs = np.random.RandomState(0)
    # 4 batches of 4 sentences whose longest are 12, 9, 12, 9: each length eager at its first
    # batch, captured and replayed at its second (SEQ_CAPTURE_AFTER = 2)
    lens = np.array([5, 7, 12, 9, 6, 9, 8, 9, 12, 12, 10, 5, 7, 9, 9, 6])
    end = np.cumsum(lens)
    X = torch.from_numpy(rs.randn(end[-1], F).astype(np.float32)).to(DEV)
    lab = torch.from_numpy(np.stack([rs.randint(0, 64, end[-1]), rs.randint(0, 8, end[-1])],
                                    1).astype(np.int32)).to(DEV)
    runs = []
    old_sparse = E.RNN_SPARSE
    E.RNN_SPARSE = "force" if body.endswith("_sparse") else old_sparse
    try:
        for graphs in (False, True):
            nets = copy.deepcopy(nets0)
            eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fea": (0, F)},
                         ["lab_cd", "lab_mono"], batch=B, max_len=16, seed=1, prec=prec)
            if mode == "bf16" and body.startswith("ligru"):
                assert all(lb.get("persist_fwd") is not None for lb in eng.nodes[0].lbuf)
            if body == "lstm_quant":
                assert all(lb.get("U_hq") is not None for lb in eng.nodes[0].lbuf)
            if graphs:
                assert eng.capture()
            eng.bind_chunk(X, lab, end[-1], end_index=end)
            rng = random.Random(7)
            trace = []
            for _ in range(4):
                batch = eng.next_seq_batch(rng)
                eng.train_step(batch=batch)
                trace.append((eng.loss_values(), eng.head_output("o2").cpu().clone()))
            if graphs:
                assert eng.seq_captures == 2 and sorted(eng.seq_graphs) == [9, 12]
            eng.sync_state()
            runs.append((trace, {k: {n: v.detach().cpu().clone() for n, v in m.state_dict().items()}
                                 for k, m in nets.items()}))
    finally:
        E.RNN_SPARSE = old_sparse
    (te, se), (tg, sg) = runs
    for step, ((le, pe), (lg, pg)) in enumerate(zip(te, tg)):
        assert le == lg, (step, le, lg)
        assert torch.equal(pe, pg), step
    for k in se:
        for n in se[k]:
            assert torch.equal(se[k][n], sg[k][n]), (k, n)


def test_seq_batch_carries_its_index():
    """The data-parallel loss scale of a batch is that batch's frame weight even when another
    batch was drawn in between (a stale Engine.batch_i)."""
    from pkc.engine import Engine, parse_model
    cfg, nets, opts = _build("lstm")
    F, B = 20, 4
    lens = np.array([5, 7, 12, 9, 6, 9, 8, 9])
    end = np.cumsum(lens)
    X = torch.randn(int(end[-1]), F, device=DEV)
    lab = torch.zeros(int(end[-1]), 2, dtype=torch.int32, device=DEV)
    eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fea": (0, F)},
                 ["lab_cd", "lab_mono"], batch=B, max_len=16, seed=1)
    eng.bind_chunk(X, lab, end[-1], end_index=end)
    eng.frame_scales = np.array([0.25, 0.75])
    b0 = eng.next_seq_batch(random.Random(1))
    b1 = eng.next_seq_batch(random.Random(2))
    assert (b0.index, b1.index, eng.batch_i) == (0, 1, 1)
    eng.train_step(batch=b0)
    assert eng.grad_scale == 0.25
    eng.train_step(batch=b1)
    assert eng.grad_scale == 0.75
