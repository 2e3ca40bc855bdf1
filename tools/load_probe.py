"""Diagnostic: nemo_load_corpus of one C5 batch (143 runs of 1M-node graphs, page-locked), wall time per
load, alone and with the library's kernel timings.  Usage: load_probe.py [runs] [option=value ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

import nemo_amd.engine as E  # noqa: E402
from tools import synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 143
c, _ = synth.generate(runs, prepend_run0=True, threads=16, **synth.CONFIGS["c5"])
pin = E.pin_corpus(c)
eng = E.Engine(0)
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    eng.set_option(k, int(v))
eng.set_timing(True)
for rep in range(4):
    eng.reset_timings()
    t = time.perf_counter()
    eng.load(c)
    eng.synchronize()
    dt = time.perf_counter() - t
    tm = eng.timings()
    print(f"load {rep}: {dt * 1e3:.1f} ms;", {k: round(v["ms"], 1) for k, v in tm.items()}, flush=True)
E.unpin_corpus(pin)
eng.close()
