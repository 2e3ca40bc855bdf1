"""Diagnostic: k_diff global tier (windowed sweeps) per-phase ticks from the stamps build.

usage: python tools/stamps_diff.py [RUNS] [NODES] [EOT]
"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E
E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from nemo_amd.corpus import DIFF_PER_RUN
from tools import synth
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 40
nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
eot = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
corpus, _ = synth.generate(runs, target_nodes=nodes, eot=eot, threads=16, body_extra=6, nval=3, nloc=4)
s, f = corpus.success_iters(), corpus.failed_iters()
if not f:  # entries only need a label source: take successful runs
    f = [i for i in s if i != 0][:4]
eng = E.Engine(0)
eng.load(corpus); eng.mark(); eng.simplify(); eng.synchronize()
eng.set_timing(True)
eng.diffprov(f, DIFF_PER_RUN); eng.synchronize()
print("entries", len(f), {k: round(v["ms"], 2) for k, v in eng.timings().items() if v["ms"] > 0.01})
st = eng.debug_copy("stamps", 0, 16 * 8 * len(f)).view(np.uint64).reshape(len(f), 16).astype(np.int64)
names = ["F stage", "F levels", "F write", "B stage", "B levels", "B write", "D stage", "D levels", "D write"]
tot = st[:, :9].sum(1)
print("ticks per entry: median", np.median(tot))
for i, nm in enumerate(names):
    print(f"{nm:10s} median {np.median(st[:, i]):12.0f}  share {st[:, i].sum() / tot.sum():.3f}")
d = np.diff(st[:, 9:13], axis=1)
for i, nm in enumerate(["clear + failGoals", "three sweeps", "mask + leaves + missing"]):
    print(f"{nm:24s} median {np.median(d[:, i]):12.0f}")
eng.close()
