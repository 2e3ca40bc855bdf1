"""Diagnostic: per-phase ticks of the multi-entry diff's walks (k_dx_walk) from the stamps build.

usage: python tools/stamps_dx.py [c3|c5] [RUNS] [P_FAULT]
Reach workgroups (chunk x direction) and depth workgroups (2 sources each), wave 0's view: the first window's
staging, the walks, the waits for the worker waves (finalize k-1 / stage k+1) at the window barriers, the missing
rows pass; windows; total.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402

import nemo_amd.engine as E  # noqa: E402

E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from nemo_amd.corpus import DIFF_PER_RUN  # noqa: E402
from tools import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
runs = int(sys.argv[2]) if len(sys.argv) > 2 else (10000 if cfg == "c3" else 64)
pf = float(sys.argv[3]) if len(sys.argv) > 3 else (0.15 if cfg == "c3" else 0.6)
corpus, _ = synth.generate(runs, p_fault=pf, prepend_run0=True, **synth.CONFIGS[cfg])
f = corpus.failed_iters()
eng = E.Engine(0)
eng.load(corpus)
eng.mark()
eng.diffprov(f, DIFF_PER_RUN)
eng.synchronize()
nu = len(f)
nch = (nu + 63) // 64
nd = (nu + 1) // 2
n = 16 * max(2 * nch, nd)
st = eng.debug_copy("stamps", 0, 8 * n).view(np.uint64).reshape(-1, 16).astype(np.int64)
names = ["stage0", "-", "-", "walk", "wait", "rows", "windows", "total"]
for label, rows, off in (("reach", st[:2 * nch], 0), ("depth", st[:nd], 8)):
    blk = rows[:, off:off + 8]
    print(f"{label}: {len(blk)} workgroups")
    for i, nm in enumerate(names):
        print(f"  {nm:9s} median {np.median(blk[:, i]):14.0f}  max {blk[:, i].max():14.0f}")
eng.close()
