"""Summarise the two PMC passes of scripts/gpu.sh pmc: the last N dispatches of each pass are
the replayed dominant launch; traffic = (2 x FETCH_SIZE + WRITE_SIZE) KiB per dispatch (gfx950
FETCH_SIZE counts half of a wide coalesced read, MI355X_MICROARCH.md HBM section)."""
import csv
import glob
import json
import os
import sys

root, n = sys.argv[1], int(sys.argv[2])   # n: replaced by the launch count the run reports


def per_dispatch(pass_dir, counter):
    files = glob.glob(os.path.join(root, pass_dir, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        rows += [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
    tail = rows[-n:]
    vals = [float(r["Counter_Value"]) for r in tail]
    names = sorted({r["Kernel_Name"] for r in tail})     # every instance the replayed launches use
    return names, (sum(vals) / len(vals)) if vals else None


label, labels = None, set()
for logname in ("fetch.log", "write.log"):
    for line in open(os.path.join(root, logname)):
        if line.startswith("{") and "pmc_replay" in line:
            d = json.loads(line)
            label, n = d["pmc_replay"], int(d["launches"])
            labels.add(label)
if len(labels) > 1:
    sys.exit("the two passes replayed different kernels: %s" % sorted(labels))
kf, fetch = per_dispatch("fetch", "FETCH_SIZE")
kw, write = per_dispatch("write", "WRITE_SIZE")
out = {"label": label, "kernels": kf, "dispatches": n, "FETCH_SIZE_KiB": fetch,
       "WRITE_SIZE_KiB": write,
       "traffic_bytes_per_launch": (2 * fetch + write) * 1024 if fetch is not None and write is not None
       else None}
print(json.dumps(out, indent=1))
