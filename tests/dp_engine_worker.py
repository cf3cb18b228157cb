"""Worker of tests/test_gpu_dp.py (not collected by pytest): one rank of a chunk-level
data-parallel Engine run, launched by torch.distributed.run with the gloo backend (several ranks
sharing one GPU).  Each rank trains its half of every global batch with Engine(grad_scale=1/R)
and the bucketed all-reduce of pkc.dist.GradAllReduce (the first bucket overlapping the rest of the
backward), eagerly or replayed from the split hipGraphs (mode "graph"), and saves its state.

argv: out_dir mode (eager | graph | syncbn | bf16graph | wide | widegraph) steps B_per_rank

wide*: a 2048-wide hidden layer under a 1928-wide cd head and a 48-wide mono head at >= 1024 rows
per rank: the cd head's dW is one matmul while the mono head's is split over K (pkc.engine
_dw_splits), and the first all-reduce bucket is cut at the cd head — both heads' gradients must be
final (the split one's slab sum included) before it goes out.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def dp_config(bn=False, wide=False):
    """Body 40 -> 64 (LayerNorm, no BatchNorm: the local batch statistics of BN differ per rank;
    bn=True: BatchNorm on both layers, for the SyncBN runs), SGD; cd head 32 (RMSprop), mono head 8
    (RMSprop); dropout 0."""
    from cases import build_mlp_config
    cfg = build_mlp_config("plain")
    if bn:
        cfg["architecture1"].update(dnn_lay="64,64", dnn_use_batchnorm="True,True",
                                    dnn_use_laynorm="False,False", dnn_act="relu,tanh")
    else:
        cfg["architecture1"].update(dnn_lay="64,64", dnn_use_batchnorm="False,False",
                                    dnn_use_laynorm="True,False", dnn_act="relu,tanh")
    cfg["architecture2"].update(dnn_lay="32")
    if wide:
        cfg["architecture1"].update(dnn_lay="2048", dnn_use_batchnorm="False",
                                    dnn_use_laynorm="False", dnn_act="relu", dnn_drop="0.0")
        cfg["architecture2"].update(dnn_lay="1928")
        cfg["architecture3"].update(dnn_lay="48")
    return cfg


def dims(cfg):
    h = int(cfg["architecture1"]["dnn_lay"].split(",")[-1])
    return (("architecture1", 40), ("architecture2", h), ("architecture3", h))


def data(steps, B_total, ncd=32, nmono=8):
    rs = np.random.RandomState(3)
    X = rs.randn(steps * B_total, 40).astype(np.float32)
    lab = np.stack([rs.randint(0, ncd, steps * B_total), rs.randint(0, nmono, steps * B_total)],
                   1).astype(np.int32)
    return X, lab


def build(cfg, world, B, X, lab, sync_bn=None, prec=None):
    from pkc import _lib as L
    from pkc.engine import Engine, parse_model
    from pkc.neural_networks import MLP
    torch.manual_seed(2234)
    np.random.seed(2234)
    nets, opts = {}, {}
    for sec, inp in dims(cfg):
        o = cfg[sec]
        nets[o["arch_name"]] = MLP(o, inp).cuda().train()
        opts[o["arch_name"]] = o
    eng = Engine(nets, opts, parse_model(cfg["model"]["model"]), {"fmllr": (0, 40)},
                 ["lab_cd", "lab_mono"], batch=B, seed=1, grad_scale=1.0 / world, sync_bn=sync_bn,
                 prec=L.PREC_FP32 if prec is None else prec)
    eng.bind_chunk(torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda(), X.shape[0])
    return eng, nets


def main():
    out, mode, steps, B = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    from pkc import dist as DP
    dist.init_process_group("gloo")
    rank, world = DP.world()
    torch.cuda.set_device(0)
    wide = mode.startswith("wide")
    X, lab = data(steps, B * world, *((1928, 48) if wide else (32, 8)))
    # rank r's rows of global batch s: [s*B*R + r*B, +B) — laid out so the engine's batch counter
    # walks them in order
    rows = np.concatenate([np.arange(s * B * world + rank * B, s * B * world + (rank + 1) * B)
                           for s in range(steps)])
    sbn = DP.SyncBatchNorm() if mode == "syncbn" else None
    from pkc import _lib as L
    eng, nets = build(dp_config(bn=mode == "syncbn", wide=wide), world, B, X[rows], lab[rows],
                      sync_bn=sbn,
                      prec=L.PREC_BF16 if mode == "bf16graph" else None)
    ar = DP.GradAllReduce()
    if wide:
        heads = [n for n in eng.nodes if n.head]
        assert [n.sdw for n in heads] == [1, 4], [n.sdw for n in heads]
        assert eng._bucket_cut()[0] is heads[0]
    if mode in ("graph", "bf16graph", "widegraph"):
        assert eng.capture(split_optimizer=True)
        assert eng.graph_tail is not None        # bucketed: two backward graphs
    for _ in range(steps):
        eng.train_step(ar)
    torch.cuda.synchronize()
    loss, err = DP.sum_scalars(eng.chunk_totals())
    sd = {a + "/" + k: v.detach().cpu().numpy() for a in nets for k, v in nets[a].state_dict().items()}
    np.savez(os.path.join(out, "rank%d_%s.npz" % (rank, mode)), loss=loss / world, calls=ar.calls,
             **sd)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
