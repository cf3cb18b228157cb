"""host issue time vs wall time per sequence step (diagnostic; run as python <tree>/scripts/host_probe.py c3)"""
import os, sys, time, random
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pytorch-kaldi-cgs_amd")); sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np, torch
import bench_seq as BS
cfg = sys.argv[1]
eng, nets, B = BS.build(cfg)
rng = random.Random(7)
nb = eng.n_batches
order = [int(i) for i in np.linspace(0, nb - 1, 8)]
batches = []
for i in order:
    eng.snt = i * B
    batches.append(eng.next_seq_batch(rng))
for b in batches[:2]:
    eng.train_step(batch=b)
torch.cuda.synchronize()
host, wall, ts = 0.0, 0.0, 0
for b in batches[2:]:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.train_step(batch=b)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    host += t1 - t0; wall += t2 - t0; ts += int(b[3])
print("%s %s host %.2f ms/step  wall %.2f ms/step  host us per T-step %.2f  wall us per T-step %.2f" % (
    ROOT.split("/")[-1], cfg, host * 1e3 / 6, wall * 1e3 / 6, host * 1e6 / ts, wall * 1e6 / ts))
