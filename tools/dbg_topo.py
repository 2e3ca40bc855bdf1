import os, sys, numpy as np
sys.path.insert(0, '/root/repo')
from nemo_amd import engine as E
from tools import synth
corpus, _ = synth.generate(24, target_nodes=2500)
eng = E.Engine(0)
V, G = int(corpus.node_off[-1]), corpus.n_graphs
src = np.asarray(corpus.edge_src).astype(np.int64); dst = np.asarray(corpus.edge_dst).astype(np.int64)
goff = np.repeat(np.asarray(corpus.node_off[:-1]).astype(np.int64), np.diff(np.asarray(corpus.edge_off).astype(np.int64)))
for blk in (256, 1024, 1024):
    for k, v in (("graph_lds_max", 0), ("build_lds_max", 0), ("global_block", blk)):
        eng.set_option(k, v)
    eng.load(corpus); eng.synchronize()
    nlv = eng.debug_copy("nlv", 0, 4 * V).view(np.uint32).astype(np.int64)
    topo = eng.debug_copy("topo", 0, 4 * V).view(np.uint32).astype(np.int64)
    bad = int((nlv[goff + src] >= nlv[goff + dst]).sum())
    perm = all(len(np.unique(topo[int(corpus.node_off[g]):int(corpus.node_off[g + 1])])) == int(corpus.node_off[g + 1] - corpus.node_off[g]) for g in range(G))
    print(blk, "edges with nlv[src] >= nlv[dst]:", bad, "topo permutation:", perm, flush=True)
eng.close()
