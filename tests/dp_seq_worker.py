"""Worker of tests/test_gpu_dp.py::test_dp_seq_* (not collected by pytest): one rank of sequence-
model chunk-level data parallelism through the Engine, launched by torch.distributed.run with the
gloo backend (the ranks share the one GPU; on a node the same code runs over RCCL).

The rank builds the bench_seq configuration (C4: LSTM 4x1024 bidirectional, C5: LSTM 3x512 +
pattern + 8/16-bit fake quantisation; recurrent dropout 0) from the common seeds, takes its
round-robin share of a length-sorted chunk of short sentences (pkc.dist.shard_sentences, as
pkc.core.run_nn does), gets the chunk's per-batch frame weights in ONE collective
(pkc.dist.frame_weights), and trains `steps` sentence batches with the bucketed gradient
all-reduce.  It saves its parameters, its batches (begin rows, lengths, left pads, T) and its
frame weights, so the test can restate the same data-parallel step on the oracle.

argv: out_dir config (c4 | c5) steps
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "pytorch-kaldi-cgs_amd"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "scripts")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def chunk(name, steps, world):
    """A length-sorted chunk of world * steps * B short sentences (T in [8, 22]), 440-dim
    features, cd / mono labels; the same on every rank."""
    import bench_seq as BS
    B = BS.rec_opts(name)[2]
    rs = np.random.RandomState(29)
    lens = np.sort(rs.randint(8, 21, size=world * steps * B))
    # the last sentence of every global batch (rank world-1's) 2 frames longer: unequal padded
    # T per rank in every step, whatever the draw
    lens[world * B - 1::world * B] += 2
    end = np.cumsum(lens)
    X = rs.randn(end[-1], 440).astype(np.float32)
    lab = np.stack([rs.randint(0, 1928, end[-1]), rs.randint(0, 48, end[-1])], 1).astype(np.int32)
    return lens, end, X, lab, B


def main():
    out, name, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    from pkc import dist as DP
    from pkc.engine import Engine, parse_model
    from test_gpu_configs import build_pair
    dist.init_process_group("gloo")
    rank, world = DP.world()
    torch.cuda.set_device(0)
    nets, _, opts, model, B = build_pair(name, drop="0.0")
    for n in nets.values():
        n.cuda().train()
    lens, end, X, lab, B = chunk(name, steps, world)
    eng = Engine(nets, opts, parse_model(model), {"fea": (0, 440)}, ["lab_cd", "lab_mono"],
                 batch=B, max_len=int(lens.max()), seed=1 + rank, grad_scale=1.0 / world)
    eng.bind_chunk(torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda(), end[-1],
                   end_index=end, sentences=DP.shard_sentences(end, rank, world))
    eng.n_batches = DP.agree_min(eng.n_batches, device=eng.dev)
    eng.frame_scales = DP.frame_weights(eng.sent_len, eng.B, eng.n_batches, device=eng.dev)
    ar = DP.GradAllReduce()
    rng = random.Random(7 + rank)
    rec = []
    for _ in range(steps):
        b = eng.next_seq_batch(rng)
        rec.append(b)
        eng.train_step(ar, batch=b)
    torch.cuda.synchronize()
    eng.sync_state()
    DP.average_buffers(list(nets.values()))
    loss, err = DP.sum_scalars(eng.chunk_totals())
    sd = {a + "/" + k: v.detach().cpu().numpy() for a in nets for k, v in nets[a].state_dict().items()}
    np.savez(os.path.join(out, "seq_rank%d_%s.npz" % (rank, name)), loss=loss, calls=ar.calls,
             scales=eng.frame_scales,
             begs=np.stack([b[0] for b in rec]), lens=np.stack([b[1] for b in rec]),
             lefts=np.stack([b[2] for b in rec]), T=np.array([b[3] for b in rec]), **sd)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
