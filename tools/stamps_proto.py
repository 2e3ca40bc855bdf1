"""Diagnostic: per-phase cycles of k_proto_lds from the stamps build (slots 0-7 of run r)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E
E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from tools import synth
corpus, _ = synth.generate(int(sys.argv[1]) if len(sys.argv) > 1 else 2000, threads=16, **synth.CONFIGS["c3"])
eng = E.Engine(0)
eng.load(corpus); eng.mark(); eng.simplify()
eng.prototypes(corpus.success_iters()); eng.synchronize()
R = corpus.n_runs
st = eng.debug_copy("stamps", 0, 16 * 8 * R).view(np.uint64).reshape(R, 16).astype(np.int64)[:, :8]
ok = st[:, 7] > 0
st = st[ok]
d = np.diff(st, axis=1)
names = ["stage", "chain fixup", "root/hasrc", "R1", "G2", "sweep", "out"]
print("runs", ok.sum(), "cycles per WG median", np.median(st[:, 7] - st[:, 0]))
for i, nm in enumerate(names):
    print(f"{nm:12s} median {np.median(d[:, i]):10.0f} mean {d[:, i].mean():10.0f} share {d[:, i].sum() / d.sum():.3f}")
t0, t1 = st[:, 0], st[:, 7]
span = t1.max() - t0.min()
print("kernel span cycles", span, "mean concurrency", (t1 - t0).sum() / span)
