"""Diagnostic: k_chains fast-front compaction (stamps 0, 10-13, 1; stamps build)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E
E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from tools import synth
corpus, _ = synth.generate(int(sys.argv[1]) if len(sys.argv) > 1 else 2000, threads=16, **synth.CONFIGS["c3"])
eng = E.Engine(0)
eng.load(corpus); eng.mark(); eng.simplify(); eng.synchronize()
G = corpus.n_graphs
st = eng.debug_copy("stamps", 0, 16 * 8 * G).view(np.uint64).reshape(G, 16).astype(np.int64)
cols = [0, 10, 11, 1]
ok = np.all(st[:, cols] > 0, axis=1)
d = np.diff(st[ok][:, cols], axis=1)
for i, nm in enumerate(["init", "count (loads)", "scan + place"]):
    print(f"{nm:22s} median {np.median(d[:, i]):8.0f} p90 {np.percentile(d[:, i], 90):8.0f}")
