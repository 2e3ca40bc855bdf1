"""Wall-clock breakdown of bench.py's step, synchronising after every call.

usage: python tools/step_breakdown.py [runs] [steps]
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nemo_amd.corpus import DIFF_PER_RUN  # noqa: E402
from nemo_amd.engine import Engine  # noqa: E402
from tools import synth  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
corpus, _ = synth.generate(runs, prepend_run0=True, threads=16)
succ, fail = corpus.success_iters(), corpus.failed_iters()
eng = Engine(0)
eng.load(corpus)
acc = {}


def t(name, f):
    t0 = time.perf_counter()
    r = f()
    eng.synchronize()
    acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
    return r


for s in range(steps + 1):
    if s == 1:
        acc.clear()
    t("rebuild", eng.rebuild)
    t("mark", eng.mark)
    t("simplify", eng.simplify)
    t("stage", eng.stage_simplified)
    t("prototypes", lambda: eng.prototypes(succ))
    t("run_tables", lambda: eng.run_tables(1))
    t("diffprov", lambda: eng.diffprov(fail, DIFF_PER_RUN))
    t("triggers", eng.triggers)
    t("trigger_rows", eng.trigger_rows)
    t("pull1", lambda: eng.pull(1))
    t("pull2", lambda: eng.pull(2))
    t("diff_masks", lambda: eng.diff_masks(len(fail)))
    t("missing", eng.missing)
    t("view", eng.simplified_view)
tot = sum(acc.values())
for k, v in acc.items():
    print(f"{k:14s} {1e3 * v / steps:9.2f} ms  {100 * v / tot:5.1f}%")
print(f"{'total':14s} {1e3 * tot / steps:9.2f} ms")
