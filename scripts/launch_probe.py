"""Composition of the C2 step's grouped backward launches: each launch's operations recorded from
one step, then the launch re-issued alone and with subsets of its operations (matmuls only, the
dX problem only, updates only), timed as graph replays of back-to-back copies.  Says which part
of a grouped launch sets its duration.  Usage: python scripts/launch_probe.py [--prec fp32]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from pkc import _lib as L  # noqa: E402
from pkc.engine import Engine  # noqa: E402


def main():
    prec = L.PREC_FP32 if "--prec" in sys.argv and sys.argv[-1] == "fp32" else L.PREC_BF16
    eng, _, _, _ = bench.build(prec, 128, 0, 1)
    for _ in range(3):
        eng.train_step()
    torch.cuda.synchronize()
    launches = []
    orig = Engine._gemms

    def rec(self, probs, s):
        launches.append([tuple(q) for q in probs])
        return orig(self, probs, s)

    Engine._gemms = rec
    eng.train_step()
    Engine._gemms = orig
    torch.cuda.synchronize()

    def t_us(ops, reps=20):
        if not ops:
            return 0.0
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                eng._gemms(list(ops), eng._stream())
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
        return best

    for i, ops in enumerate(launches):
        if len(ops) < 2:
            continue
        labels = [q[0] for q in ops]
        gem = [q for q in ops if q[3].kind == L.OP_GEMM]
        dx = [q for q in gem if q[0].startswith("dX")]
        rest = [q for q in ops if q[3].kind != L.OP_GEMM]
        row = {"all": t_us(ops), "matmuls": t_us(gem), "dX": t_us(dx),
               "non-matmul": t_us(rest)}
        for q in ops:
            row[q[0][:28]] = t_us([q])
        print("launch %d [%s]" % (i, ", ".join(labels)), flush=True)
        print("   " + "  ".join("%s %.2f" % (k, v) for k, v in row.items()), flush=True)


if __name__ == "__main__":
    main()
