"""Profiling driver: the bench step on a C3-shaped corpus, for rocprofv3 runs.

usage: python tools/prof_pipeline.py [runs] [steps] [option=value ...]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nemo_amd.corpus import DIFF_PER_RUN  # noqa: E402
from nemo_amd.engine import Engine  # noqa: E402
from tools import synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
opts = dict(a.split("=") for a in sys.argv[3:])
corpus, _ = synth.generate(runs, threads=16)
succ = corpus.success_iters()
fail = corpus.failed_iters()
eng = Engine(0)
for k, v in opts.items():
    eng.set_option(k, int(v))
eng.load(corpus)
eng.set_timing(True)
for s in range(steps):
    t = time.perf_counter()
    eng.rebuild()
    eng.mark()
    eng.simplify()
    eng.prototypes(succ)
    eng.diffprov(fail, DIFF_PER_RUN)
    eng.triggers()
    eng.pull(1)
    eng.pull(2)
    eng.synchronize()
    print(f"step {s}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
for k, v in sorted(eng.timings().items(), key=lambda kv: -kv[1]["ms"]):
    print(f"{k:16s} {v['launches']:4d} {v['ms'] / v['launches']:9.3f} ms/launch")
