"""One C3 step's kernel timeline from a rocprofv3 kernel trace: per queue, every kernel of the last step
(from the last k_build launch to the end of the trace's last step), start/duration relative to the step
start, and the gaps on the main queue.  usage: python tools/timeline.py kt_kernel_trace.csv [anchor]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_build"
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
       r["Queue_Id"]) for r in rows]
ks.sort()
starts = [i for i, k in enumerate(ks) if anchor in k[2]]
a, b = starts[-2], starts[-1]  # the second-to-last step (the last may run into teardown)
t0 = ks[a][0]
step = ks[a:b]
main_q = ks[a][3]
print(f"step {((ks[b][0] - t0) / 1e3):.1f} us, main queue {main_q}")
last_end = t0
busy = 0
for s, e, n, q in step:
    gap = (s - last_end) / 1e3 if q == main_q else 0
    print(f"{q:>3} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f}  {'gap %.1f' % gap if q == main_q and gap > 2 else '':>10}  {n[:70]}")
    if q == main_q:
        busy += e - max(s, last_end) if e > last_end else 0
        last_end = max(last_end, e)
print(f"main queue busy {busy / 1e3:.1f} us of {(ks[b][0] - t0) / 1e3:.1f}")
