"""Where two runs of the same C5-shaped LSTM block differ: per-step vs per-step, persistent vs
persistent and per-step vs persistent (tests/test_gpu_lstm_persist.py's runner), reporting per layer
and gate the first time step with a difference.  Usage: python scripts/lstm_persist_probe.py [H T B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "pytorch-kaldi-cgs_amd"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from test_gpu_lstm_persist import _run  # noqa: E402


def first_steps(a, b, T, B, H):
    out = {}
    for k in a:
        if k.endswith(".timeout") or torch.equal(a[k], b[k]):
            continue
        d = (a[k] != b[k])
        if k.endswith(".gates") or k.endswith(".dgates"):
            d = d[:4 * T * B * H].view(4, T, B * H).any(2)
            out[k] = [int(d[g].nonzero()[0]) if d[g].any() else None for g in range(4)]
        elif k.endswith(".hs") or k.endswith(".cs"):
            d = d[:(T + 1) * B * H].view(T + 1, B * H).any(1)
            out[k] = int(d.nonzero()[0])
        elif k.endswith(".hq"):
            d = d[:T * B * H].view(T, B * H).any(1)
            out[k] = int(d.nonzero()[0])
        else:
            out[k] = int(d.sum())
    return out


def main():
    H, T, B = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (512, 12, 12)))
    r1, _ = _run(H, T, B, 1, False)
    r2, _ = _run(H, T, B, 1, False)
    p1, _ = _run(H, T, B, 1, True)
    p2, _ = _run(H, T, B, 1, True)
    print("steps vs steps", first_steps(r1, r2, T, B, H), flush=True)
    print("persistent vs persistent", first_steps(p1, p2, T, B, H), flush=True)
    print("steps vs persistent", first_steps(r1, p1, T, B, H), flush=True)


if __name__ == "__main__":
    main()
