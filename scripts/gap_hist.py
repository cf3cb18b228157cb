"""Distribution of the idle gap before each step's first launch (batch gather) in a rocprofv3
kernel trace of bench.py: tells graph-replay boundaries (every k-th step) from in-graph gaps."""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "batch_gather"
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"] and i > 0]
gaps = np.array([(int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3 for i in idx])
lens = np.array([b - a for a, b in zip(idx, idx[1:])])
steady = gaps[-400:]
print("steps", len(gaps), "launches per step (mode)", np.bincount(lens).argmax() if len(lens) else 0)
print("gap before %s over the last %d steps: p10 %.2f p50 %.2f p90 %.2f max %.2f mean %.2f us" % (
    first, len(steady), *np.percentile(steady, [10, 50, 90]), steady.max(), steady.mean()))
print("last 24 gaps:", " ".join("%.1f" % g for g in gaps[-24:]))
