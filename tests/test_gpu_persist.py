"""The persistent liGRU time loops (pkc_rnn_persist.hip: one launch per layer for the whole forward
and BPTT loop, U blocks held in registers / LDS, no per-step launch) against the per-step launches
of the same bf16 step arithmetic (PKC_RNN_BF16_SPARSE: block-sparse bf16 step kernels), at the
BASELINE C3 layer shape (liGRU 4 x 550 bidirectional, HCGS [32,2]/[75,75] U masks, B = 8).  The
two forms differ only in the order of the fp32 block sums, which can move a bf16 copy of h (or of
dgates) by one bf16 rounding where its fp32 value sits on a rounding tie: counted here, the rest
held to fp32-sum tolerance.  The oracle comparisons of the same mode: tests/test_gpu_seq.py
test_seq_engine_bf16_vs_bf16_oracle[ligru_hcgs] (persistent loops asserted on, small layers),
tests/test_gpu_steps.py (every time step of every layer at the C3 shape vs oracle/steps.py) and
tests/test_gpu_configs.py::test_c3_ligru_hcgs_full_size_bf16 (training steps vs the bf16 oracle)."""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(persist, steps=2, lo=40, hi=61):
    import pkc.engine as E
    from pkc import _lib as L
    from pkc.engine import Engine, parse_model
    from test_gpu_configs import build_pair
    nets, _, opts, model, B = build_pair("c3", drop="0.2")
    for k in nets:
        nets[k].to(DEV).train()
    F = 440
    rs = np.random.RandomState(21)
    lens = np.sort(rs.randint(lo, hi, size=B * steps))
    end = np.cumsum(lens)
    X = torch.from_numpy(rs.randn(end[-1], F).astype(np.float32)).to(DEV)
    lab = torch.from_numpy(np.stack([rs.randint(0, 1928, end[-1]), rs.randint(0, 48, end[-1])], 1)
                           .astype(np.int32)).to(DEV)
    specs = nets["rnn"].layer_specs()
    masks = {("rnn", li): torch.from_numpy((rs.rand(2 * B, sp["H"]) > 0.2).astype(np.float32)).to(DEV)
             for li, sp in enumerate(specs)}
    old = (E.RNN_PERSIST, E.RNN_BF16_SPARSE)
    E.RNN_PERSIST, E.RNN_BF16_SPARSE = persist, not persist
    try:
        eng = Engine(nets, opts, parse_model(model), {"fea": (0, F)}, ["lab_cd", "lab_mono"],
                     batch=B, max_len=int(lens.max()), seed=1, prec=L.PREC_BF16, rnn_drop_in=masks)
        used = [lb.get("persist_fwd") is not None and lb.get("persist_bwd") is not None
                for lb in eng.nodes[0].lbuf]
        eng.bind_chunk(X, lab, end[-1], end_index=end)
        rng = random.Random(3)
        out = []
        for _ in range(steps):
            eng.train_step(batch=eng.next_seq_batch(rng))
            torch.cuda.synchronize()
            out.append((eng.head_output("o2").cpu().clone(), eng.gflat.detach().cpu().clone(),
                        eng.loss_values()))
        lb = eng.nodes[0].lbuf[-1]
        y = lb["y"].detach().cpu().clone()
    finally:
        E.RNN_PERSIST, E.RNN_BF16_SPARSE = old
    return used, out, y


def test_persistent_ligru_matches_per_step_launches():
    used_p, out_p, y_p = _run(True)
    used_s, out_s, y_s = _run(False)
    assert all(used_p) and not any(used_s), (used_p, used_s)
    for s, ((pp, gp, lp), (ps, gs, ls)) in enumerate(zip(out_p, out_s)):
        rel = ((pp - ps).abs() / ps.abs().clamp_min(1e-3)).max().item()
        nout = int(((pp - ps).abs() / ps.abs().clamp_min(1e-3) > 1e-4).sum())
        gerr = (gp - gs).norm().item() / gs.norm().item()
        print("step %d: posterior max rel diff %.3g (%d of %d above 1e-4), flat gradient rel "
              "diff %.3g, loss %.6f vs %.6f" % (s, rel, nout, pp.numel(), gerr, lp[0], ls[0]))
        if s == 0:      # the forward: same bf16 operands, fp32 sums in another order
            assert rel < 1e-3 and nout <= pp.numel() // 100, (rel, nout)
        np.testing.assert_allclose(lp[0], ls[0], rtol=1e-4)
    # (the BPTT's bf16 dgates copies inherit the fp32 order differences over all T steps and 4
    # layers, so the full-size gradients of the two forms drift apart by the bf16 mode's own
    # precision (5.5e-3 in gpurun_out/r5_persist.log): they are checked per time step against
    # oracle/steps.py — tests/test_gpu_steps.py::test_c3_bf16_persistent_loops_per_time_step —
    # and the size of the gap against the bf16 oracle's distance to the fp32 oracle in
    # tests/test_gpu_steps.py::test_bf16_chain_gap_is_the_modes_precision)


def test_persistent_ligru_bptt_matches_per_step_short():
    """The BPTT of both forms from the same forward, short sentences (T <= 8) so that the bf16
    dgates copies — where a last-bit fp32 difference can move one copy by a bf16 rounding — have
    few steps to compound over: every gradient within 1e-3 of its norm (measured on the print)."""
    used_p, out_p, _ = _run(True, steps=1, lo=5, hi=9)
    used_s, out_s, _ = _run(False, steps=1, lo=5, hi=9)
    assert all(used_p) and not any(used_s)
    (pp, gp, lp), (ps, gs, ls) = out_p[0], out_s[0]
    gerr = (gp - gs).norm().item() / gs.norm().item()
    rel = ((pp - ps).abs() / ps.abs().clamp_min(1e-3)).max().item()
    print("T <= 8: posterior max rel diff %.3g, flat gradient rel diff %.3g" % (rel, gerr))
    assert rel < 1e-3 and gerr < 1e-3, (rel, gerr)


def test_persistent_ligru_very_short_sentences():
    """Edge lengths: padded batches of T = 1..3 steps (the BPTT loop then runs 0-2 steps and the
    carry hand-off at its end is skipped or taken) — forward and gradients as the per-step form."""
    used_p, out_p, _ = _run(True, steps=2, lo=1, hi=4)
    used_s, out_s, _ = _run(False, steps=2, lo=1, hi=4)
    assert all(used_p) and not any(used_s)
    for s, ((pp, gp, lp), (ps, gs, ls)) in enumerate(zip(out_p, out_s)):
        gerr = (gp - gs).norm().item() / gs.norm().item()
        rel = ((pp - ps).abs() / ps.abs().clamp_min(1e-3)).max().item()
        print("T <= 3 step %d: posterior max rel diff %.3g, flat gradient rel diff %.3g" % (s, rel, gerr))
        assert rel < 1e-3 and gerr < 1e-3, (s, rel, gerr)
