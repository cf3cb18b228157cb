"""Error budget of the bf16 C2 step's posteriors: which bf16-rounded operand
puts the cd head's log-posteriors at ~1.4e-4 relative from the fp32 reference (north_star: 1e-4).

The bf16 engine multiplies bf16-rounded operands (round-to-nearest-even of the fp32 values: the
gathered batch x, each layer's output, the weights) with fp32 accumulation; everything else
(bias, BatchNorm, activations, dropout, LogSoftmax) runs in fp32.  This restates that on the CPU:
the oracle's C1 MLP (reference algorithm, fp32) with the inputs and / or weights of chosen Linear
layers rounded to bf16 before their fp32 product, against the unrounded oracle, first training
step's forward (the quantity bench.py's parity_leg checks), same seeds and dropout masks as
parity_leg.  The GPU line's own figure (posterior_max_rel_err in BENCH) sits beside the 'all' row.

CPU only: python scripts/bf16_error_budget.py [--seeds 3] > profiles/r04_bf16_error_budget.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def run(seed, which, batch=128):
    """Log-posteriors of the cd head after the first forward, with the Linear layers named in
    `which` (set of (layer key, 'x' | 'w')) fed bf16-rounded operands."""
    import bench
    from oracle import nets as ON
    cfg = bench.c1_cfg()
    torch.manual_seed(seed)
    nets = {}
    from pkc.neural_networks import MLP
    for sec, inp in bench.DIMS:
        o = cfg[sec]
        a = o["arch_name"]
        ref = MLP(o, inp)                       # pkc's init draws = the reference's
        nets[a] = ON.MLP(o, inp)
        nets[a].load_state_dict(ref.state_dict())
        nets[a].train()
    rs = np.random.RandomState(seed)
    X = torch.from_numpy(rs.randn(batch, 440).astype(np.float32))
    rs.randint(0, 1928, batch), rs.randint(0, 48, batch)          # the labels' draws (unused)
    keeps = [torch.from_numpy((rs.rand(batch, 1024) > 0.15).astype(np.float32)) for _ in range(5)]
    hooks = []
    names = {}
    for a, net in nets.items():
        for i, lin in enumerate(net.wx):
            names[id(lin)] = "head_cd" if a == "MLP_layers2" else (
                "head_mono" if a == "MLP_layers3" else "body%d" % i)
    orig = nn.Linear.forward

    def fwd(self, x):
        k = names.get(id(self))
        if ("*", "x3") in which:              # compensated: x_hi w_hi + x_hi w_lo + x_lo w_hi
            xh, wh = bf(x), bf(self.weight)
            xl, wl = bf(x - xh), bf(self.weight - wh)
            return F.linear(xh, wh) + (F.linear(xh, wl) + F.linear(xl, wh)) + self.bias
        xx = bf(x) if (k, "x") in which or ("*", "x") in which else x
        w = bf(self.weight) if (k, "w") in which or ("*", "w") in which else self.weight
        return F.linear(xx, w, self.bias)

    nn.Linear.forward = fwd
    try:
        with torch.no_grad():
            h = nets["MLP_layers1"](X, drop_masks=keeps)
            post = nets["MLP_layers2"](h)
    finally:
        nn.Linear.forward = orig
    for hk in hooks:
        hk.remove()
    return post.double()


CASES = {
    "all (the bf16 engine)": {("*", "x"), ("*", "w")},
    "body only (fp32 heads)": {("body%d" % i, s) for i in range(5) for s in "xw"},
    "heads only": {(h, s) for h in ("head_cd", "head_mono") for s in "xw"},
    "weights only": {("*", "w")},
    "activations only": {("*", "x")},
    "input batch x only": {("body0", "x")},
    "body except layer 0": {("body%d" % i, s) for i in range(1, 5) for s in "xw"},
    "last body layer + heads": {(k, s) for k in ("body4", "head_cd", "head_mono") for s in "xw"},
    "body layers 3-4 + heads": {(k, s) for k in ("body3", "body4", "head_cd", "head_mono")
                                for s in "xw"},
    "body layers 2-4 + heads": {(k, s) for k in ("body2", "body3", "body4", "head_cd", "head_mono")
                                for s in "xw"},
    "compensated bf16 (3 products of hi/lo bf16 parts, every layer)": {("*", "x3")},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=3)
    a = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    out = {"what": "max relative error (|d| / max(|ref|, 1e-3), bench.parity_leg's measure) of "
                   "the cd head's log-posteriors, C1 step 1 forward, B = 128, vs the fp32 oracle; "
                   "per seed", "cases": {}}
    refs = {s: run(s, set()) for s in range(a.seeds)}
    for name, which in CASES.items():
        rows = []
        for s in range(a.seeds):
            p = run(s, which)
            d = (p - refs[s]).abs()
            rows.append({"seed": s, "max_rel": float((d / refs[s].abs().clamp_min(1e-3)).max()),
                         "max_abs": float(d.max()), "rms_abs": float(d.pow(2).mean().sqrt())})
        out["cases"][name] = {"max_rel_over_seeds": max(r["max_rel"] for r in rows), "seeds": rows}
        print(name, ["%.3g" % r["max_rel"] for r in rows], file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
