"""Summarise an MFMA-utilisation PMC pass (scripts/gpu.sh mfma): per kernel name over the pass's
dispatches, SQ_INSTS_VALU_MFMA_MOPS_{BF16,F32} x 512 = MFMA flops, and MfmaUtil = the MFMA busy
cycles over the SIMD cycles the kernel had:

    util = SQ_VALU_MFMA_BUSY_CYCLES / ((GRBM_GUI_ACTIVE / 8) x 1024 SIMDs)

SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD (32 per v_mfma_f32_32x32x16_bf16,
MI355X_MICROARCH.md's SQ-units row); GRBM_GUI_ACTIVE as rocprofv3 reports it is the SUM over the 8
XCDs' GRBMs (its DVFS paragraph: clock = GUI_ACTIVE / 8 / wall time), so the kernel's cycles are
GUI_ACTIVE / 8.  (Round 2 divided by the whole GUI_ACTIVE: utilisation 8x too low, VERDICT r2
weak #6.)  Beside it the kernel's achieved TF/s from its dispatch timestamps and that over the
dense peak of the dtype it issues (tflops_pct_of_peak); the two agree up to the clock the chip
ran at (util counts cycles, TF/s counts nanoseconds at the 2.4 GHz the peak assumes).

The kernel's cycles: GUI_ACTIVE / 8 counts the whole counter-collection window, which for a
kernel of a few microseconds is wider than its dispatch (start, end) timestamps — round 3 read
4.1-5.9 GHz "clocks" off it.  Where GUI_ACTIVE / 8 / ns exceeds the chip's
2.4 GHz the window is not the kernel, so the counters do not say how many cycles the kernel had:
mfma_util_pct is null there (a clamp made it a copy of tflops_pct_of_peak)
and only the timestamp-based tflops_pct_of_peak is reported.  The raw window figure stays in
window_clock_ghz.
Usage: mfma_summary.py <pass dir> [top]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
SIMDS = 256 * 4
XCDS = 8
PEAK_TFLOPS = {"bf16": 2516.6, "f32": 157.3}     # dense MFMA at 2.4 GHz, 256 CUs
MAX_CLOCK_GHZ = 2.4
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
    dt = "bf16" if c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) >= c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) else "f32"
    tf = fl / c["ns"] / 1e3 if c["ns"] else None
    wclk = gui / XCDS / c["ns"] if c["ns"] else None          # GHz over the counter window
    clk = wclk if (wclk and wclk <= MAX_CLOCK_GHZ) else None     # the window is the kernel
    cycles = c["ns"] * clk if clk else 0.0
    rows.append({"kernel": k[:110], "dispatches": len(seen[k]), "mfma_gflop": round(fl / 1e9, 3),
                 "mfma_dtype": dt, "tflops": round(tf, 1) if tf is not None else None,
                 "tflops_pct_of_peak": round(100.0 * tf / PEAK_TFLOPS[dt], 2) if tf else None,
                 "mfma_util_pct": round(100.0 * busy / (cycles * SIMDS), 2) if cycles else None,
                 "effective_clock_ghz": round(clk, 3) if clk else None,
                 "window_clock_ghz": round(wclk, 3) if wclk else None})
rows.sort(key=lambda r: -r["mfma_gflop"])
print(json.dumps(rows[:top], indent=1))
