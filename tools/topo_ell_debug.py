"""Debug k_topo_ell: load a deep-shape corpus with every big graph on the child-record Kahn kernel, and
on a refusal dump the state of the first graph in error against a host Kahn pass."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nemo_amd import engine as E  # noqa: E402
from tools import synth  # noqa: E402

corpus, _ = synth.generate(9, run_base=0, prepend_run0=True, target_nodes=12000, eot=16, body_extra=6, nval=3,
                           nloc=4, p_fault=0.4)
V, G = int(corpus.node_off[-1]), corpus.n_graphs
eng = E.Engine(0)
for k, v in (("graph_lds_max", 0), ("build_lds_max", 0), ("chains_glob_min_v", 0), ("global_block", 1024)):
    eng.set_option(k, v)
for ell in (1,) if os.environ.get("NEMO_LIB") else (0, 1):
    eng.set_option("topo_ell", ell)
    try:
        eng.load(corpus)
        print("ell", ell, "load ok")
        continue
    except E.NemoError as ex:
        print("ell", ell, "load failed:", ex)
    err = eng.debug_copy("err", 0, 4 * G).view(np.uint32)
    nlev = eng.debug_copy("nlev", 0, 4 * G).view(np.uint32)
    bad = [g for g in range(G) if err[g]]
    print("graphs in error", bad, "nlev", nlev[bad].tolist())
    g = bad[0]
    n0, n1 = int(corpus.node_off[g]), int(corpus.node_off[g + 1])
    e0, e1 = int(corpus.edge_off[g]), int(corpus.edge_off[g + 1])
    nv = n1 - n0
    nlv = eng.debug_copy("nlv", 4 * n0, 4 * nv).view(np.uint32)
    cnt = eng.debug_copy("s_a", 4 * (n0 + g), 4 * nv).view(np.uint32)
    lvl = eng.debug_copy("lvl", 4 * (n0 + g), 4 * (int(nlev[g]) + 1)).view(np.uint32)
    src = corpus.edge_src[e0:e1].astype(np.int64)
    dst = corpus.edge_dst[e0:e1].astype(np.int64)
    indeg = np.bincount(dst, minlength=nv)
    # host levels
    lev = np.full(nv, -1)
    order = np.argsort(src, kind="stable")
    fp = np.zeros(nv + 1, np.int64)
    np.add.at(fp, src + 1, 1)
    fp = np.cumsum(fp)
    fc = dst[order]
    c = indeg.copy()
    front = [v for v in range(nv) if c[v] == 0]
    L = 0
    for v in front:
        lev[v] = 0
    while front:
        nxt = []
        for u in front:
            for w in fc[fp[u]:fp[u + 1]]:
                c[w] -= 1
                if c[w] == 0:
                    nxt.append(w)
                    lev[w] = L + 1
        front = nxt
        L += 1
    print("host levels", L, "device levels", int(nlev[g]), "placed", int(lvl[-1]) if len(lvl) else 0, "of", nv)
    hs = np.bincount(lev[lev >= 0], minlength=L)
    print("level sizes host  ", hs[:26].tolist())
    print("level sizes device", np.diff(lvl.astype(np.int64))[:26].tolist())
    ovf = int(((fp[1:] - fp[:-1]) > 8).sum())
    print("rows past 8 children:", ovf, "of", nv)
    placed = set()
    # nodes the device placed: level offsets give count; nlv valid for placed nodes only
    unplaced = [v for v in range(nv) if cnt[v] != 0]
    print("nodes with cnt != 0:", len(unplaced), unplaced[:10], "their cnt", [int(cnt[v]) for v in unplaced[:10]],
          "host level", [int(lev[v]) for v in unplaced[:10]], "indeg", [int(indeg[v]) for v in unplaced[:10]])
    for v in unplaced[:3]:
        par = src[dst == v]
        print("  node", v, "parents", par.tolist(), "parent dev nlv", [int(nlv[p]) for p in par],
              "parent host lev", [int(lev[p]) for p in par], "parent outdeg", [int(fp[p + 1] - fp[p]) for p in par])
    gsoff = eng.debug_copy("gs_off", 8 * g, 8).view(np.uint64)[0]
    for v in unplaced[:3]:
        for p in src[dst == v][:2]:
            rec = eng.debug_copy("gscratch", 4 * (int(gsoff) + 8 * int(p)), 32).view(np.uint32)
            print("  record of parent", int(p), rec.tolist(), "row", fc[fp[p]:fp[p + 1]].tolist())
eng.close()
