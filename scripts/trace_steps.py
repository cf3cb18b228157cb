"""Phase breakdown of the recurrent forward step kernel (measurement only).

Runs the sequence bench's config on the phase-trace build of libpkc (pkc/libpkc_trace.so, built
with `python pytorch-kaldi-cgs_amd/pkc/_build.py --trace`; its step kernels stamp s_memtime at
their phase boundaries, pkc_rnn_impl.h PKC_TR) and prints, over the workgroups of the last traced
launch, the median duration of every phase in shader-clock cycles and in ns (the cycle counter's
rate taken from the 100 MHz real-time stamps of the same workgroups).  The stamps drain the
outstanding memory operations at each boundary, so the phases add up to somewhat more than the
untraced kernel; their proportions are the point.

Usage: PKC_LIB=pytorch-kaldi-cgs_amd/pkc/libpkc_trace.so python scripts/trace_steps.py --config c5
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))

PHASES = ["entry", "operand + epilogue-input loads", "var max-abs reduction",
          "quantise + MFMA chains", "4-wave tile reduction (LDS)", "cell update + stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--persist", action="store_true",
                    help="the persistent liGRU loops' per-wave phase sums instead (C3, bf16)")
    ap.add_argument("--lstm-persist", action="store_true",
                    help="the persistent LSTM loops' per-wave phase sums instead (C5)")
    a = ap.parse_args()
    if a.persist:
        return persist(a)
    if a.lstm_persist:
        return lstm_persist(a)
    assert "libpkc_trace" in os.environ.get("PKC_LIB", ""), "set PKC_LIB to the trace build"
    import torch
    import bench_seq
    from pkc import _lib as L
    bench_seq.run(a.config, a.steps, 1, prec=a.prec)
    torch.cuda.synchronize()
    n = 4096 * 8
    buf = (C.c_ulonglong * n)()
    assert L.lib().pkc_trace_read(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
    t = t[(t[:, 0] > 0) & (t[:, 7] > 0)]
    if not (t[:, 3] > 0).any():         # no quantised-h phase (stamp 3): an empty phase
        t[:, 3] = t[:, 2]
    cyc = np.diff(t[:, 1:7], axis=1)                        # phases 1..5 in shader cycles
    real_ns = (t[:, 7] - t[:, 0]) * 10.0                    # 100 MHz
    ghz = (t[:, 6] - t[:, 1]) / np.maximum(real_ns, 1)
    clk = float(np.median(ghz))
    span_ns = float((t[:, 7].max() - t[:, 0].min()) * 10.0)
    out = {"config": a.config, "prec": a.prec, "workgroups": int(len(t)),
           "clock_ghz_median": round(clk, 3), "launch_span_ns": span_ns,
           "workgroup_ns_median": float(np.median(real_ns)),
           "phases": {PHASES[i + 1]: {"cycles_median": float(np.median(cyc[:, i])),
                                      "ns_median": round(float(np.median(cyc[:, i])) / clk, 1),
                                      "cycles_max": float(cyc[:, i].max())}
                      for i in range(5)}}
    print(json.dumps(out, indent=1))


PPHASES = ["fragment loop (MFMAs)", "products barrier wait", "cell-update values",
           "store issue", "step-end barrier wait"]


def persist(a):
    """Per step and wave (workgroup 0 of the last forward / BPTT loop launched): cycles of each
    phase, averaged over the loop's steps."""
    import torch
    import bench_seq
    from pkc import _lib as L
    bench_seq.run(a.config, a.steps, 1, prec=a.prec)
    torch.cuda.synchronize()
    n = 2 * 8 * 8
    buf = (C.c_ulonglong * n)()
    assert L.lib().pkc_trace_read_persist(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(2, 8, 8).astype(np.int64)
    out = {"config": a.config, "prec": a.prec}
    for k, name in enumerate(("forward loop", "BPTT loop")):
        T = int(t[k, 0, 5])
        steps = T if k == 0 else max(T - 1, 1)
        per = t[k, :, :5] / float(steps)
        out[name] = {"T": T, "cycles_per_step_by_wave": {
            PPHASES[i]: [round(float(v), 1) for v in per[:, i]] for i in range(5)},
            "cycles_per_step_wave_mean": {PPHASES[i]: round(float(per[:, i].mean()), 1)
                                          for i in range(5)}}
    print(json.dumps(out, indent=1))


LPHASES = {"forward loop": ["wait for the step's arrivals", "h_{t-1} loads + var",
                            "quantise + MFMA + partials", "cell update + stores", "arrive"],
           "BPTT loop": ["wait for the step's arrivals", "dgates loads + MFMA + partials",
                         "gate gradients + stores", "arrive", "-"]}


def lstm_persist(a):
    """Per step and wave (workgroup 0 of the last persistent LSTM forward / BPTT launch): cycles
    of each phase averaged over the loop's steps, and ns at the clock measured beside it."""
    import torch
    import bench_seq
    from pkc import _lib as L
    bench_seq.run(a.config, a.steps, 1, prec=a.prec)
    torch.cuda.synchronize()
    n = 2 * 16 * 8
    buf = (C.c_ulonglong * n)()
    assert L.lib().pkc_trace_read_lstm_persist(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(2, 16, 8).astype(np.int64)
    out = {"config": a.config, "prec": a.prec, "clock_ghz_assumed": 2.4}
    if a.prec == "bf16" or a.config == "c4":   # the bf16 / fp32 dense loops' phases
        LPHASES["forward loop"] = ["wait for the step's arrivals", "h_{t-1} load issue",
                                   "load wait + MFMA + partials", "cell update + stores", "arrive"]
        LPHASES["BPTT loop"] = ["wait for the step's arrivals", "dgates loads + MFMA + partials",
                                "gate gradients + stores", "arrive", "-"]
    for k, name in enumerate(("forward loop", "BPTT loop")):
        live = t[k, :, 5] > 0                 # the waves the last launch of that loop stamped
        nw = int(live.sum())
        T = int(t[k, live, 5][0]) if nw else 0
        steps = T if k == 0 else max(T - 1, 1)
        per = t[k, live, :5] / float(steps)
        mean = per.mean(0)
        out[name] = {"T": T, "waves": nw,
                     "cycles_per_step_wave_mean": {LPHASES[name][i]: round(float(mean[i]), 1)
                                                   for i in range(5)},
                     "cycles_per_step_total": round(float(per.sum(1).mean()), 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
