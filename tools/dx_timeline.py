"""Diagnostic: kernel timeline (us) of the last multi-entry diff call in a rocprofv3 kernel trace."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
i0 = [i for i, r in enumerate(rows) if "k_dx_label" in r["Kernel_Name"]][-1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + 10]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'][:48]:48s} start {(s - t0) / 1000:8.2f}  dur {(e - s) / 1000:8.2f}")
