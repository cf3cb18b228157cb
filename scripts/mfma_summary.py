"""Summarise an MFMA-utilisation PMC pass (scripts/gpu_mfma.sh): per kernel name over the pass's
dispatches, SQ_INSTS_VALU_MFMA_MOPS_{BF16,F32} x 512 = MFMA flops, SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE x 1024 SIMDs) = MfmaUtil (rocprofv3's own derived-metric formula), and the
kernel's achieved TF/s from its dispatch timestamps.  Usage: mfma_summary.py <pass dir> [top]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
SIMDS = 256 * 4
# per dispatch: SQ counters summed over their instances, GRBM_GUI_ACTIVE the max over its
# instances (rocprofv3's reduce(GRBM_GUI_ACTIVE, max)), then summed over the kernel's dispatches
disp = collections.defaultdict(lambda: collections.defaultdict(float))
names, dur = {}, {}
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        d = (f, r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        dur[d] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        c, v = r["Counter_Name"], float(r["Counter_Value"])
        disp[d][c] = max(disp[d][c], v) if c == "GRBM_GUI_ACTIVE" else disp[d][c] + v
acc = collections.defaultdict(lambda: collections.defaultdict(float))
seen = collections.defaultdict(set)
for d, cs in disp.items():
    k = names[d]
    seen[k].add(d)
    acc[k]["ns"] += dur[d]
    for c, v in cs.items():
        acc[k][c] += v
rows = []
for k, c in acc.items():
    fl = 512.0 * (c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) + c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0))
    if fl == 0.0:
        continue
    busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), c.get("GRBM_GUI_ACTIVE", 0.0)
    rows.append({"kernel": k[:110], "dispatches": len(seen[k]), "mfma_gflop": round(fl / 1e9, 3),
                 "tflops": round(fl / c["ns"] / 1e3, 1) if c["ns"] else None,
                 "mfma_util_pct": round(100.0 * busy / (gui * SIMDS), 2) if gui else None})
rows.sort(key=lambda r: -r["mfma_gflop"])
print(json.dumps(rows[:top], indent=1))
