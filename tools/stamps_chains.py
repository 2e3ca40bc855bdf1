"""Diagnostic: per-phase cycle shares of k_chains from the stamps build."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E
E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from tools import synth
corpus, _ = synth.generate(int(sys.argv[1]) if len(sys.argv) > 1 else 500, threads=16, **synth.CONFIGS["c3"])
eng = E.Engine(0)
eng.load(corpus); eng.mark(); eng.simplify(); eng.synchronize()
G = corpus.n_graphs
st = eng.debug_copy("stamps", 0, 16 * 8 * G).view(np.uint64).reshape(G, 16).astype(np.int64)
idx = [0, 1, 2, 3, 4, 5, 6, 8, 9]
names = ["compact", "ranks", "adjacency", "up/down", "prefix ranks", "reps", "sort", "tail lists"]
d = np.diff(st[:, idx], axis=1)
ok = (st[:, 9] > 0)
d = d[ok]
print("graphs", ok.sum(), "total cycles per graph: median", np.median(d.sum(1)), "p90", np.percentile(d.sum(1), 90))
for i, nm in enumerate(names):
    print(f"{nm:14s} median {np.median(d[:, i]):10.0f}  mean {d[:, i].mean():10.0f}  share {d[:, i].sum() / d.sum():.3f}")
sub = st[ok]
for a, b, nm in [(0, 10, "  zero maps"), (10, 11, "  loads+hist"), (11, 1, "  scan+scatter")]:
    print(f"{nm:14s} median {np.median(sub[:, b] - sub[:, a]):10.0f}")
nch = []
ch = eng.chains()
import collections
cnt = collections.Counter(int(g) for g in ch[:, 0])
keys = collections.Counter((int(r[0]), int(r[2]), int(r[4])) for r in ch)
print("chains per graph mean", len(ch) / G, "max", max(cnt.values()), "records with (len, head) ties:", sum(v for v in keys.values() if v > 1), "of", len(ch))
# level statistics of H* (maxup = longest chain prefix) from the chain records
lens = ch[:, 4] if ch.shape[1] > 4 else None
print("chain length: mean", float(np.mean(ch[:, 4])), "max", int(np.max(ch[:, 4])))
