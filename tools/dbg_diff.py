import os, sys, numpy as np
sys.path.insert(0, '/root/repo')
from nemo_amd import engine as E
from nemo_amd.corpus import DIFF_PER_RUN
from oracle import oracle as O
from tools import synth
corpus, _ = synth.generate(24, target_nodes=2500)
s, f = corpus.success_iters(), corpus.failed_iters()
orc = O.analyze(corpus, s, f, diff_mode=DIFF_PER_RUN)
g0 = 1; n0 = int(corpus.node_off[g0]); V = int(corpus.node_off[g0+1]) - n0
e0, e1 = int(corpus.edge_off[g0]), int(corpus.edge_off[g0+1])
src = np.asarray(corpus.edge_src[e0:e1]).astype(int); dst = np.asarray(corpus.edge_dst[e0:e1]).astype(int)
word = np.asarray(corpus.node_word[n0:n0+V]); label = np.asarray(corpus.label[n0:n0+V])
isrule = (word >> 31) & 1
par = [[] for _ in range(V)]; chl = [[] for _ in range(V)]
for a_, b_ in zip(src, dst): par[b_].append(a_); chl[a_].append(b_)
fr = corpus.run_index(f[0]); gs = 2 * fr + 1
flab = set(int(corpus.label[x]) for x in range(int(corpus.node_off[gs]), int(corpus.node_off[gs+1])) if not (int(corpus.node_word[x]) >> 31) & 1)
good = np.array([(not isrule[v]) and int(label[v]) not in flab for v in range(V)])
eng = E.Engine(0)
for blk in (256, 1024):
    for k, v in (("graph_lds_max", 0), ("build_lds_max", 0), ("global_block", blk)):
        eng.set_option(k, v)
    eng.load(corpus); eng.mark(); eng.simplify(); eng.diffprov(f, DIFF_PER_RUN); eng.synchronize()
    topo = eng.debug_copy("topo", 4 * n0, 4 * V).view(np.uint32)
    tpos = eng.debug_copy("diff_tpos", 0, 4 * V).view(np.uint32)
    bits = eng.debug_copy("dbits", 0, V).view(np.uint8)
    tp_ok = np.array_equal(tpos[topo], np.arange(V))
    F = (bits & 1) != 0; Bb = (bits & 2) != 0
    # check local consistency of F and B against the rules
    badF = [v for v in range(V) if F[v] != (good[v] or any(F[p] for p in par[v]))]
    badB = [v for v in range(V) if Bb[v] != (good[v] or any(Bb[c] for c in chl[v]))]
    print(blk, "tpos ok", tp_ok, "F viol", len(badF), badF[:8], "B viol", len(badB), badB[:8], flush=True)
    for v in badB[:4]:
        print("  B node", v, "rule", isrule[v], "children", [(c, int(tpos[c]), bool(Bb[c])) for c in chl[v]], "tpos", int(tpos[v]), flush=True)
    for v in badF[:4]:
        print("  F node", v, "rule", isrule[v], "parents", [(c, int(tpos[c]), bool(F[c])) for c in par[v]], "tpos", int(tpos[v]), flush=True)
eng.close()
