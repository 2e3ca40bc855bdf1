"""Diagnostic: k_topo_deep per-phase ticks (stamps build) on deep graphs.

usage: python tools/stamps_topo.py [RUNS] [NODES] [EOT]
"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nemo_amd.engine as E
E.LIB_PATH = os.path.join(os.path.dirname(E.LIB_PATH), "libnemohip_stamps.so")
from tools import synth
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
eot = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
corpus, _ = synth.generate(runs, target_nodes=nodes, eot=eot, threads=16, body_extra=6, nval=3, nloc=4)
eng = E.Engine(0)
eng.load(corpus); eng.synchronize()
G = corpus.n_graphs
st = eng.debug_copy("stamps", 0, 16 * 8 * G).view(np.uint64).reshape(G, 16).astype(np.int64)
names = ["frontier + row ptrs", "child loads", "atomics", "append", "barrier"]
tot = st[:, :5].sum(1)
print("ticks per graph: median", np.median(tot))
for i, nm in enumerate(names):
    print(f"{nm:20s} median {np.median(st[:, i]):12.0f}  share {st[:, i].sum() / tot.sum():.3f}")
eng.close()
