"""Diagnostic: cumulative HBM traffic and time of k_chains_glob's phases at the C5 shape.

usage (stamps build, under rocprofv3 --pmc or --kernel-trace):
    python tools/glob_phases.py RUNS
Runs rebuild + mark + simplify once per stop k = 1..8 and 0 (the whole kernel), in that order, with
option chains_glob_stop = k (k_chains_glob returns after phase k).  The i-th k_chains_glob dispatch of the
profile is stop STOPS[i]; tools/glob_phases_sum.py differences them into per-phase figures.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E  # noqa: E402

E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from tools import synth  # noqa: E402

STOPS = [1, 2, 3, 4, 5, 6, 7, 8, 0]
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 320
t = time.time()
corpus, _ = synth.generate(runs, threads=16, **synth.CONFIGS["c5"])
print(f"generated {runs} runs in {time.time() - t:.1f}s", flush=True)
eng = E.Engine(0)
eng.load(corpus)
eng.synchronize()
print("loaded", flush=True)
for k in STOPS:
    eng.set_option("chains_glob_stop", k)
    t = time.time()
    eng.rebuild()
    eng.mark()
    eng.simplify()
    eng.synchronize()
    print(f"stop {k}: {time.time() - t:.2f}s", flush=True)
eng.close()
