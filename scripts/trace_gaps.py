"""Per-step kernel timeline from a rocprofv3 kernel trace: duration of each kernel and the gap
before it, averaged over the steps of the timed (graph-replayed) region."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "batch_gather"
# optional: keep only steps with a kernel whose name contains this (e.g. the bf16 instances, so
# the fp32 leg of the same bench command is not the one summarised)
need = sys.argv[3] if len(sys.argv) > 3 else None
# optional: drop steps holding a kernel whose name contains this (the bench's multi-step graphs
# run the batch gather inside the first grouped launch; a standalone batch_gather_kernel marks a
# single-step graph replay — warmup, parity and per-launch probes — or a replay's first step)
skip = sys.argv[4] if len(sys.argv) > 4 else None
starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
# the bench's own steps: the most common launch count between consecutive gathers (other
# workloads in the same trace — batch sweep, sequence configs — have other shapes)
pairs = list(zip(starts, starts[1:]))
lens = defaultdict(int)
for a, b in pairs:
    lens[b - a] += 1
if need or skip:
    pairs = [(a, b) for a, b in pairs
             if (not need or any(need in r["Kernel_Name"] for r in rows[a:b]))
             and not (skip and any(skip in r["Kernel_Name"] for r in rows[a:b]))]
    lens = defaultdict(int)
    for a, b in pairs:
        lens[b - a] += 1
# optional: the step's launch count (the bench line's graph_launches_per_step), else the mode
L = int(sys.argv[5]) if len(sys.argv) > 5 else max(lens, key=lens.get)
# the graph-replayed steps of the timed region: of the steps with the common shape, the 200
# shortest from first launch start to last launch end (eager steps of the same command — the
# parity leg, per-launch cost probes — carry host launch gaps)
cand = [rows[a:b] for a, b in pairs if b - a == L]
cand.sort(key=lambda st: int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"]))
steps = sorted(cand[:200], key=lambda st: int(st[0]["Start_Timestamp"]))
agg = defaultdict(lambda: [0.0, 0.0, 0])
order = []
tot = []
for st in steps:
    t0 = int(st[0]["Start_Timestamp"])
    t1 = int(st[-1]["End_Timestamp"])
    tot.append((t1 - t0) / 1e3)
    prev_end = None
    for i, r in enumerate(st):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:60]
        key = "%02d %s g%sx%sx%s" % (i, name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e
        a = agg[key]
        a[0] += (e - s) / 1e3
        a[1] += gap
        a[2] += 1
        if key not in order:
            order.append(key)
n = len(steps)
sd = sg = 0
for k in order:
    d, g, c = agg[k]
    sd += d / c
    sg += g / c
    print("%-90s dur %7.2f  gap %6.2f" % (k, d / c, g / c))
print("steps %d  mean step %.1f us  sum dur %.1f  sum gap %.1f" % (n, sum(tot) / n, sd, sg))
