"""Diagnostic: per-phase ticks (s_memtime) of the whole-graph walks (k_dx_walks) from the stamps build.

usage: python tools/stamps_dx.py [RUNS] [P_FAULT] [FUSE]
Bwd* workgroups (one per 64-source chunk): stage, walk, finalize, leaf candidates, publish.
Longest-path workgroups: stage, walk, finalize, wait for the chunk's Bwd*, LP pass, missing rows.
Ticks from each workgroup's start; the launch's first start is the origin of "start".
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

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
pf = float(sys.argv[2]) if len(sys.argv) > 2 else 0.15
fuse = int(sys.argv[3]) if len(sys.argv) > 3 else 1
corpus, _ = synth.generate(runs, p_fault=pf, prepend_run0=True, **synth.CONFIGS["c3"])
f = corpus.failed_iters()
eng = E.Engine(0)
eng.load(corpus)
eng.mark()
eng.set_option("diff_fuse", fuse)
for _ in range(3):
    eng.diffprov(f, DIFF_PER_RUN)
eng.synchronize()
nu = len(f)
nch = (nu + 63) // 64
nb = nch * (1 + 11)
st = eng.debug_copy("stamps", 0, 8 * 16 * nb).view(np.uint64).reshape(-1, 16).astype(np.int64)
t0 = st[:, 0].min()
for label, rows, names in (("bwd", st[:nch], ["stage", "walk", "finalize", "lc", "publish"]),
                           ("depth", st[nch:nb], ["stage", "walk", "finalize", "wait", "lp", "rows"])):
    rows = rows[rows[:, 0] > 0]
    print(f"{label}: {len(rows)} workgroups; start median {np.median(rows[:, 0] - t0):.0f} max {(rows[:, 0] - t0).max()}")
    d = np.diff(rows[:, :len(names) + 1], axis=1)
    for i, nm in enumerate(names):
        print(f"  {nm:9s} median {np.median(d[:, i]):10.0f}  max {d[:, i].max():10.0f}")
    print(f"  end       median {np.median(rows[:, len(names)] - t0):10.0f}  max {(rows[:, len(names)] - t0).max()}")
eng.close()
# k_dx_label (slots 10-14 of its block index x + y * gridDim.x): start, loads issued+landed (tick at first
# use is after the wait), dense lookups, marks, bitmap store
eng = E.Engine(0)
eng.load(corpus)
eng.mark()
eng.diffprov(f, DIFF_PER_RUN)
eng.synchronize()
st = eng.debug_copy("stamps", 0, 8 * 16 * nu).view(np.uint64).reshape(-1, 16).astype(np.int64)[:, 10:15]
st = st[st[:, 0] > 0]
d = np.diff(st, axis=1)
print(f"label: {len(st)} workgroups")
for i, nm in enumerate(["loads", "dense", "marks", "store"]):
    print(f"  {nm:9s} median {np.median(d[:, i]):10.0f}  max {d[:, i].max():10.0f}")
eng.close()
