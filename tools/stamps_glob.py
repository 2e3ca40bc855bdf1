"""Diagnostic: per-phase cycle shares of k_chains_glob (deep graphs) from the stamps build.

usage: python tools/stamps_glob.py [RUNS] [NODES] [EOT] [dense]
"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E
E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from tools import synth
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
eot = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
dense = len(sys.argv) > 4 and sys.argv[4] == "dense"  # C5's ~4 edges per node (tools/synth.py CONFIGS["c5"])
extra = {"body_extra": 6, "nval": 3, "nloc": 4} if dense else {}
corpus, _ = synth.generate(runs, target_nodes=nodes, eot=eot, threads=16, **extra)
eng = E.Engine(0)
if os.environ.get("NEMO_GLOB_BLOCK"):
    eng.set_option("chains_glob_block", int(os.environ["NEMO_GLOB_BLOCK"]))
eng.load(corpus); eng.mark(); eng.simplify(); eng.synchronize()
G = corpus.n_graphs
st = eng.debug_copy("stamps", 0, 16 * 8 * G).view(np.uint64).reshape(G, 16).astype(np.int64)
names = ["H* compact + ranks", "adjacency", "up/down", "bucket + bp", "prefix ranks", "preorder + heads",
         "reps", "order sort", "output + tail lists"]
ok = st[:, 9] > 0
d = np.diff(st[ok][:, :10], axis=1)
print("graphs", int(ok.sum()), "total ticks per graph: median", np.median(d.sum(1)))
for i, nm in enumerate(names):
    print(f"{nm:22s} median {np.median(d[:, i]):12.0f}  share {d[:, i].sum() / d.sum():.3f}")
for i, nm in enumerate(["up stage", "up sweep", "down stage", "down sweep"]):
    print(f"{nm:22s} median {np.median(st[ok][:, 10 + i]):12.0f}")
print("sweep iterations (up)", np.median(st[ok][:, 14] & 0xFFFFFFFF), "with a node of > 8 in-ring links", np.median(st[ok][:, 14] >> 32), "H* nodes", np.median(st[ok][:, 15]))
ch = eng.chains()
print("chains per graph", len(ch) / G, "max chain length", int(np.max(ch[:, 4])) if len(ch) else 0)
eng.close()
