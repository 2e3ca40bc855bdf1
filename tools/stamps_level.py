"""Diagnostic: one prefix-rank level of k_chains (stamps 10-14, stamps build)."""
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
ok = (st[:, 14] > 0) & (st[:, 10] > 0)
d = np.diff(st[ok][:, 10:15], axis=1)
for i, nm in enumerate(["bk keys", "barrier 1", "count", "barrier 2"]):
    print(f"{nm:10s} median {np.median(d[:, i]):8.0f} p10 {np.percentile(d[:, i], 10):8.0f} p90 {np.percentile(d[:, i], 90):8.0f}")
