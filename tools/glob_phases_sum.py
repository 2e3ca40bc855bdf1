"""Per-phase HBM bytes and duration of k_chains_glob from tools/glob_phases.py runs.

usage: python tools/glob_phases_sum.py OUTDIR
OUTDIR holds pmc_fetch/, pmc_write/ (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE) and trace/ (--kernel-trace).
"""
import csv
import glob
import os
import sys

STOPS = [1, 2, 3, 4, 5, 6, 7, 8, 0]
NAMES = {1: "H* compact + ranks", 2: "adjacency", 3: "up/down sweeps", 4: "maxes + bucket + bp",
         5: "prefix ranks", 6: "preorder + heads", 7: "reps", 8: "order sort", 0: "output"}


def glob_rows(pattern, key, kernel="k_chains_glob"):
    out = []
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r.get("Kernel_Name", ""):
                out.append(r)
    out.sort(key=lambda r: int(r[key]))
    return out


d = sys.argv[1]
fetch = [float(r["Counter_Value"]) for r in glob_rows(f"{d}/pmc_fetch/**/*counter_collection.csv", "Dispatch_Id")]
write = [float(r["Counter_Value"]) for r in glob_rows(f"{d}/pmc_write/**/*counter_collection.csv", "Dispatch_Id")]
tr = glob_rows(f"{d}/trace/**/*kernel_trace.csv", "Start_Timestamp")
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tr]
print(f"dispatches: fetch {len(fetch)} write {len(write)} trace {len(dur)}")
cum = {}
for i, k in enumerate(STOPS):
    f = fetch[i] * 1024 if i < len(fetch) else float("nan")
    w = write[i] * 1024 if i < len(write) else float("nan")
    ms = dur[i] if i < len(dur) else float("nan")
    cum[k] = (2 * f + w, w, ms)
prev = (0.0, 0.0, 0.0)
print(f"| phase | HBM GB (2xFETCH+WRITE) | of which writes GB | ms | cumulative GB | cumulative ms |")
print("|---|---|---|---|---|---|")
for k in STOPS:
    b, w, ms = cum[k]
    print(f"| {NAMES[k]} | {(b - prev[0]) / 1e9:.1f} | {(w - prev[1]) / 1e9:.1f} | {ms - prev[2]:.1f} | {b / 1e9:.1f} | {ms:.1f} |")
    prev = cum[k]

pf = [float(r["Counter_Value"]) for r in glob_rows(f"{d}/pmc_fetch/**/*counter_collection.csv", "Dispatch_Id", "k_glob_prep")]
pw = [float(r["Counter_Value"]) for r in glob_rows(f"{d}/pmc_write/**/*counter_collection.csv", "Dispatch_Id", "k_glob_prep")]
pt = glob_rows(f"{d}/trace/**/*kernel_trace.csv", "Start_Timestamp", "k_glob_prep")
pd = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in pt]
if pf:
    n = len(pf)
    f = sum(pf) / n * 1024
    w = sum(pw) / max(1, len(pw)) * 1024
    print(f"\nk_glob_prep (before every k_chains_glob, {n} dispatches): {(2 * f + w) / 1e9:.1f} GB per launch "
          f"({w / 1e9:.1f} GB writes), {sum(pd) / max(1, len(pd)):.1f} ms")
