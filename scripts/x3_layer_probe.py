"""GPU diagnostic (not a test): C1 one step at fp32 and at compensated bf16 (bf16x3), per-layer
comparison of activations and gradients against the fp32 oracle. Used to show that the bf16x3
C1 gradient gap is ReLU-branch flips (dbeta moves, dgamma does not), DESIGN.md round-4 budget.
Run on the GPU box: python scripts/x3_layer_probe.py"""
import sys, os
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd")); sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import copy
import numpy as np, torch
from test_gpu_mlp import c1_config, C1_DIMS, build_nets
from pkc import _lib as L
from pkc.engine import Engine, parse_model
cfg = c1_config(drop="0.15")
nets0, opts = build_nets(cfg, C1_DIMS)
B = 128
rs = np.random.RandomState(5)
X = rs.randn(B, 440).astype(np.float32)
lab = np.stack([rs.randint(0, 1928, B), rs.randint(0, 48, B)], 1).astype(np.int32)
keeps = {"MLP_layers1.%d" % i: torch.from_numpy((rs.rand(B, 1024) > 0.15).astype(np.uint8)) for i in range(5)}
res = {}
for name, prec, spread in (("fp32", L.PREC_FP32, True), ("x3", L.PREC_BF16X3, True)):
    nets = copy.deepcopy(nets0)
    for n in nets.values(): n.cuda().train()
    eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fmllr": (0, 440)}, ["lab_cd", "lab_mono"],
                 batch=B, seed=1, prec=prec, drop_keep_in={k: v.cuda() for k, v in keeps.items()})
    eng.bind_chunk(torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda(), B)
    eng.train_step()
    torch.cuda.synchronize()
    res[name] = {}
    for n in eng.nodes:
        for (p, key, _m) in n.params():
            if isinstance(key, str):
                res[name]["%s.%s" % (n.name, key)] = getattr(n, key).detach().double().cpu().clone()
    res[name]["_outs"] = {nn_.name: nn_.out.detach().double().cpu().clone() for nn_ in eng.nodes if getattr(nn_, "out", None) is not None}
for k in res["fp32"]:
    if k == "_outs": continue
    a, b = res["fp32"][k], res["x3"][k]
    print("grad %-28s rel %.3e" % (k, ((a - b).norm() / max(a.norm(), 1e-30)).item()))
for k in res["fp32"]["_outs"]:
    a, b = res["fp32"]["_outs"][k], res["x3"]["_outs"][k]
    print("out  %-28s rel %.3e" % (k, ((a - b).norm() / max(a.norm(), 1e-30)).item()))
