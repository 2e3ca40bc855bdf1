"""Diagnostic: per-phase cycle shares of k_build from the stamps build."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E  # noqa: E402

E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from tools import synth  # noqa: E402

corpus, _ = synth.generate(int(sys.argv[1]) if len(sys.argv) > 1 else 500, threads=16, **synth.CONFIGS["c3"])
eng = E.Engine(0)
eng.load(corpus)
eng.synchronize()
G = corpus.n_graphs
st = eng.debug_copy("stamps", 0, 16 * 8 * G).view(np.uint64).reshape(G, 16).astype(np.int64)
nlev = eng.debug_copy("nlev", 0, 4 * G).view(np.uint32)
names = ["input+bitmap", "reverse CSR", "forward CSR", "sources", "Kahn levels"]
d = np.diff(st[:, 10:16], axis=1)
ok = st[:, 15] > 0
d = d[ok]
print("graphs", ok.sum(), "cycles per graph: median", np.median(d.sum(1)), "p90", np.percentile(d.sum(1), 90))
for i, nm in enumerate(names):
    print(f"{nm:14s} median {np.median(d[:, i]):10.0f}  share {d[:, i].sum() / d.sum():.3f}")
print("levels per graph: median", np.median(nlev), "max", nlev.max())
sub = ["zero ptr", "count atomics", "indeg pack", "scan", "row ptr store", "scatter", "row sort+dedupe", "col store"]
b = np.concatenate([st[:, 11:12], st[:, 0:7], st[:, 12:13]], axis=1)[ok]
db = np.diff(b, axis=1)
for i, nm in enumerate(sub):
    print(f"  rev {nm:16s} median {np.median(db[:, i]):9.0f}")
# the Kahn phase split: the level loop itself, then the Kahn-order copy and (post graphs) e2 emission
kl = (st[:, 7] - st[:, 14])[ok]
ke = (st[:, 15] - st[:, 7])[ok]
print(f"  Kahn loop         median {np.median(kl):9.0f}")
print(f"  topo copy + e2    median {np.median(ke):9.0f}")
