"""Diagnostic: per-parameter gradient comparison engine vs oracle at the C1 shape, one step."""
import sys, os
sys.path[:0] = ['.', 'tests', 'tests/golden', 'pytorch-kaldi-cgs_amd']
import numpy as np, torch
from test_gpu_mlp import c1_config, build_nets, C1_DIMS
from oracle import nets as ON, run as OR
from pkc.engine import Engine, parse_model
drop = sys.argv[1] if len(sys.argv) > 1 else "0.15"
cfg = c1_config(drop=drop)
nets, opts = build_nets(cfg, C1_DIMS)
onets, _ = build_nets(cfg, C1_DIMS, cls=ON.MLP)
for a in nets:
    onets[a].load_state_dict(nets[a].state_dict()); nets[a].cuda().train(); onets[a].train()
B = 128
rs = np.random.RandomState(5)
X = rs.randn(B, 440).astype(np.float32)
lab = np.stack([rs.randint(0, 1928, B), rs.randint(0, 48, B)], 1).astype(np.int32)
keeps = {"MLP_layers1.%d" % i: torch.from_numpy((rs.rand(B, 1024) > float(drop)).astype(np.uint8)) for i in range(5)}
eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fmllr": (0, 440)}, ["lab_cd", "lab_mono"], batch=B,
             drop_keep_in={k: v.cuda() for k, v in keeps.items()})
eng.bind_chunk(torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda(), B)
# oracle forward/backward without optimizer step
lines = OR.parse_model(cfg["model"]["model"])
dm = [keeps["MLP_layers1.%d" % i].float() for i in range(5)]
inp = torch.from_numpy(np.concatenate([X, lab.astype(np.float32)], 1))
body = onets["MLP_layers1"]; f = body.forward
body.forward = lambda x, _f=f: _f(x, drop_masks=dm)
outs = OR.forward_model(lines, onets, {a: False for a in nets}, {"fmllr": (0, 440)}, {"lab_cd": 440, "lab_mono": 441}, inp)
outs["loss_final"].backward()
eng._forward_kernels(eng._stream(), True); eng._backward_kernels(eng._stream()); torch.cuda.synchronize()
for lay in eng.layers:
    net = onets[lay.arch]
    ref = {"W": net.wx[lay.idx].weight.grad, "b": net.wx[lay.idx].bias.grad}
    got = {"W": lay.dW.cpu(), "b": lay.db.cpu()}
    if lay.bn:
        ref["g"] = net.bn[lay.idx].weight.grad; got["g"] = lay.dgamma.cpu()
        ref["be"] = net.bn[lay.idx].bias.grad; got["be"] = lay.dbeta.cpu()
    for k in ref:
        d = (got[k] - ref[k]).abs().max().item(); m = ref[k].abs().max().item()
        print("%-16s %-3s maxdiff %.3e  refmax %.3e  rel %.2e" % (lay.name, k, d, m, d / max(m, 1e-30)))
# element-level look at the first mismatching layer
body.debug_z = []
for n in onets.values():
    n.zero_grad()
outs = OR.forward_model(lines, onets, {a: False for a in nets}, {"fmllr": (0, 440)}, {"lab_cd": 440, "lab_mono": 441}, inp)
outs["loss_final"].backward()
for i in range(5):
    lay = eng.layers[i]
    ref = body.debug_z[i].grad
    got = lay.dz.view(B, -1).cpu()
    d = (got - ref).abs()
    bad = (d > 1e-3 * ref.abs().max()).nonzero()
    xh = lay.xhat.view(B, -1).cpu()
    print("layer", i, "bad elems", bad.shape[0], "cols", sorted(set(bad[:, 1].tolist()))[:10])
    if bad.shape[0]:
        c = bad[0, 1].item()
        zc = body.debug_z[i][:, c].detach()
        print("  col", c, "z std", zc.std().item(), "xhat range", xh[:, c].min().item(), xh[:, c].max().item(),
              "ref dz", ref[:4, c].tolist(), "got", got[:4, c].tolist())
