"""GPU parity: libnemohip (gfx950 kernels, called through the C ABI) vs the CPU oracle.

Integer/index/bit work throughout, so the bar is bit-exact on every output
(flags, chains incl. acceptance order k, table bitsets, inter/union, diff
masks, missing events, trigger rows, simplified-graph edge multisets).
"""
import numpy as np
import pytest

from nemo_amd import engine as E
from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE, corpus_from_graphs
from oracle import oracle as O
from tests.compare import assert_same
from tests.small import random_corpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def _check(eng, corpus, mode=DIFF_REFERENCE, pulls=True):
    s, f = corpus.success_iters(), corpus.failed_iters()
    orc = O.analyze(corpus, s, f, diff_mode=mode)
    res = E.analyze(corpus, s, f, diff_mode=mode, engine=eng, pulls=pulls)
    assert_same(corpus, res, orc, len(f), check_pulls=pulls)


@pytest.mark.parametrize("seed", range(60))
def test_random_small(eng, seed):
    corpus, _ = random_corpus(seed, max_nodes=16)
    _check(eng, corpus)


@pytest.mark.parametrize("seed", range(20))
def test_random_small_per_run_diff(eng, seed):
    corpus, _ = random_corpus(1000 + seed, n_runs=4, max_nodes=16)
    _check(eng, corpus, mode=DIFF_PER_RUN)


def test_batched_many_graphs(eng):
    # many tiny corpora concatenated into one corpus: one workgroup per graph
    graphs = []
    import random
    from tests.small import random_prov
    rng = random.Random(7)
    for it in range(300):
        st = "success" if it == 0 or rng.random() < 0.8 else "failure"
        graphs.append((it, st, random_prov(rng, "pre", 24, p_next=0.7), random_prov(rng, "post", 24, p_next=0.7)))
    _check(eng, corpus_from_graphs(graphs))


def test_empty_graphs(eng):
    empty = {"goals": [], "rules": [], "edges": []}
    corpus = corpus_from_graphs([(0, "success", empty, empty), (1, "failure", empty, empty)])
    _check(eng, corpus)


def test_load_error_duplicate_and_nonbipartite(eng):
    g = {"goals": [{"id": "goal0", "label": "a(1)", "table": "a", "time": "1"},
                   {"id": "goal1", "label": "b(1)", "table": "b", "time": "1"}],
         "rules": [], "edges": []}
    corpus = corpus_from_graphs([(0, "success", g, g)])
    # inject a goal->goal edge behind the host layer's back: the device load must refuse it
    import numpy as np
    corpus.edge_src = np.array([0], np.uint32)
    corpus.edge_dst = np.array([1], np.uint32)
    corpus.edge_off = np.array([0, 1, 1], np.uint64)
    with pytest.raises(E.NemoError) as ei:
        eng.load(corpus)
    assert "inserted number of edges (0) does not equal number of antecedent provenance edges (1)" in str(ei.value)


def test_cycle_refused(eng):
    g = {"goals": [{"id": "goal0", "label": "a(1)", "table": "a", "time": "1"}],
         "rules": [{"id": "rule0", "label": "a", "table": "a", "type": "next"}],
         "edges": [{"from": "goal0", "to": "rule0"}, {"from": "rule0", "to": "goal0"}]}
    corpus = corpus_from_graphs([(0, "success", g, g)])
    with pytest.raises(E.NemoError) as ei:
        eng.load(corpus)
    assert ei.value.code == 4


def test_load_async_reports_at_mark(eng):
    """Option load_async: nemo_load_corpus returns once its work is queued; the graph checks come from the next
    call that reads the graphs (here nemo_mark_holds), which then leaves no corpus loaded, as a failed load
    does.  A good corpus loaded the same way analyses as the oracle does."""
    g = {"goals": [{"id": "goal0", "label": "a(1)", "table": "a", "time": "1"}],
         "rules": [{"id": "rule0", "label": "a", "table": "a", "type": "next"}],
         "edges": [{"from": "goal0", "to": "rule0"}, {"from": "rule0", "to": "goal0"}]}
    eng.set_option("load_async", 1)
    try:
        eng.load(corpus_from_graphs([(0, "success", g, g)]))
        with pytest.raises(E.NemoError) as ei:
            eng.mark()
        assert ei.value.code == 4 and "not acyclic" in str(ei.value)
        with pytest.raises(E.NemoError) as ei:
            eng.mark()
        assert ei.value.code == 5
        corpus, _ = random_corpus(77, n_runs=6, max_nodes=16)
        _check(eng, corpus)
    finally:
        eng.set_option("load_async", 0)


def test_diff_edge_pulls(eng):
    corpus, _ = random_corpus(4242, n_runs=5, max_nodes=20)
    f = corpus.failed_iters()
    if not f:
        pytest.skip("no failed run")
    E.analyze(corpus, corpus.success_iters(), f, diff_mode=DIFF_PER_RUN, engine=eng, pulls=False)
    eng.pull(2)
    g0 = 2 * corpus.run_index(0) + 1
    e0, e1 = int(corpus.edge_off[g0]), int(corpus.edge_off[g0 + 1])
    src, dst = corpus.edge_src[e0:e1], corpus.edge_dst[e0:e1]
    for e in range(len(f)):
        m = eng.diff_mask(e)
        want = sorted((int(a), int(b)) for a, b in zip(src, dst) if m[a] and m[b])
        s, d = eng.pulled(e)
        assert sorted(zip(s.tolist(), d.tolist())) == want


@pytest.mark.parametrize("lds_max,comp_max", [(-1, -1), (0, -1), (0, 0), (0, 8), (12, 5), (30, -1)])
def test_chain_paths_lds_and_fallback(eng, lds_max, comp_max):
    # exercise the LDS wave path, the workgroup fallback, and mixtures of both
    import random
    from tests.small import random_prov
    rng = random.Random(99)
    graphs = []
    for it in range(40):
        st = "success" if it == 0 or rng.random() < 0.8 else "failure"
        graphs.append((it, st, random_prov(rng, "pre", 40, p_edge=0.2, p_next=0.9),
                       random_prov(rng, "post", 40, p_edge=0.2, p_next=0.9)))
    corpus = corpus_from_graphs(graphs)
    eng.set_option("chains_lds_max", lds_max)
    eng.set_option("chains_comp_max", comp_max)
    try:
        _check(eng, corpus)
    finally:
        eng.set_option("chains_lds_max", -1)
        eng.set_option("chains_comp_max", -1)


@pytest.mark.parametrize("lds_max,comp_max,nval", [(-1, -1, 8), (0, -1, 8), (0, 0, 8), (-1, -1, 2), (0, -1, 2)])
def test_synthetic_corpus(eng, lds_max, comp_max, nval):
    from tools import synth
    corpus, _ = synth.generate(40, target_nodes=3000, nval=nval)
    eng.set_option("chains_lds_max", lds_max)
    eng.set_option("chains_comp_max", comp_max)
    try:
        _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)
    finally:
        eng.set_option("chains_lds_max", -1)
        eng.set_option("chains_comp_max", -1)


def test_large_graphs_global_paths(eng):
    # V >= 8192 takes the global-memory CSR build; |H*| > 2048 takes k_chains_big
    from tools import synth
    corpus, _ = synth.generate(6, target_nodes=14000)
    assert max(corpus.graph_size(g) for g in range(corpus.n_graphs)) >= 8192
    _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)


def test_staged_simplified_views(eng):
    # nemo_stage_simplified: pinned async hand-over of the 2-bit node state and the
    # chain (head, tail) pairs, overlapping later kernels; restaging reuses the buffers
    from tools import synth
    corpus, _ = synth.generate(30, target_nodes=2000)
    s, f = corpus.success_iters(), corpus.failed_iters()
    orc = O.analyze(corpus, s, f, skip_pulls=True)
    eng.load(corpus)
    for _ in range(2):
        eng.rebuild()
        eng.mark()
        eng.simplify()
        eng.stage_simplified()
        eng.prototypes(s)  # launched while the copies are in flight
        eng.diffprov(f, DIFF_PER_RUN)
        state, off, ht = eng.simplified_view()
        from nemo_amd.corpus import F_DELETED, F_HOLDS, F_KEPT
        alive, holds = E.Engine.unpack_state(state, len(orc.flags))
        assert np.array_equal(alive, (orc.flags & (F_KEPT | F_DELETED)) == F_KEPT)
        assert np.array_equal(holds, (orc.flags & F_HOLDS) != 0)
        if f:
            assert np.array_equal(eng.diff_masks_view(), eng.diff_masks(len(f)))
        G = corpus.n_graphs
        assert len(off) == G + 1 and int(off[-1]) == len(ht) == len(orc.chains)
        g = np.repeat(np.arange(G), np.diff(off.astype(np.int64)))
        k = np.arange(len(ht)) - off[g].astype(np.int64)
        got = np.stack([g, k, ht[:, 0].astype(np.int64), ht[:, 1].astype(np.int64)], 1)
        assert np.array_equal(got, orc.chains[:, :4].astype(np.int64))


@pytest.mark.parametrize("build_max", [0, 1500])
def test_build_tiers(eng, build_max):
    # k_build (LDS CSR + Kahn levels) vs the global k_csr/k_topo tier, and a mix
    from tools import synth
    corpus, _ = synth.generate(30, target_nodes=2500)
    eng.set_option("build_lds_max", build_max)
    try:
        _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)
    finally:
        eng.set_option("build_lds_max", -1)


def _long_graph(n, tag):
    """goal0 -> rule0 -> goal1 -> ... (2n Kahn levels) with a side branch per step, as Molly JSON."""
    goals = [{"id": f"goal{i}", "label": f"log(a, {i}, {tag})", "table": "log" if i else "post", "time": str(n - i)}
             for i in range(n + 1)]
    goals += [{"id": f"goals{i}", "label": f"ack(a, {i})", "table": "ack", "time": "1"} for i in range(0, n, 7)]
    rules = [{"id": f"rule{i}", "label": "log", "table": "log", "type": "next" if i % 5 else "single"} for i in range(n)]
    edges = []
    for i in range(n):
        edges += [{"from": f"goal{i}", "to": f"rule{i}"}, {"from": f"rule{i}", "to": f"goal{i + 1}"}]
        if i % 7 == 0:
            edges.append({"from": f"rule{i}", "to": f"goals{i}"})
    return {"goals": goals, "rules": rules, "edges": edges}


@pytest.mark.parametrize("shape", ["synthetic", "long"])
def test_build_tiers_identical_device_arrays(eng, shape):
    # both tiers must produce the same CSR rows, Kahn order and level offsets; the long graphs
    # have more Kahn levels than k_build sweeps (BLD_MAXLV) and are redone by the global tier
    from tools import synth
    if shape == "long":
        runs = [(0, "success", _long_graph(150, 0), _long_graph(400, 0)),
                (1, "failure", _long_graph(90, 1), _long_graph(300, 1)),
                (2, "success", _long_graph(20, 0), _long_graph(600, 0))]
        corpus = corpus_from_graphs(runs)
        _check(eng, corpus, mode=DIFF_REFERENCE, pulls=True)
    else:
        corpus, _ = synth.generate(12, target_nodes=2500)
    V, E, G = int(corpus.node_off[-1]), int(corpus.edge_off[-1]), corpus.n_graphs
    sizes = {"topo": 4 * V, "lvl": 4 * (V + G), "nlev": 4 * G, "fp": 4 * (V + G), "fc": 4 * E,
             "rp": 4 * (V + G), "rc": 4 * E}
    got = {}
    # k_build with its relaxation sweeps (build_relax 1), the global tier, k_build peeling (the default)
    for key, build_max, relax in (("relax", -1, 1), ("global", 0, 0), ("peel", -1, 0)):
        eng.set_option("build_lds_max", build_max)
        eng.set_option("build_relax", relax)
        try:
            eng.load(corpus)
            got[key] = {k: eng.debug_copy(k, 0, n).view(np.uint32) for k, n in sizes.items()}
            got[key]["nlv"] = eng.debug_copy("nlv", 0, 4 * V).view(np.uint32)
        finally:
            eng.set_option("build_lds_max", -1)
            eng.set_option("build_relax", -1)
    for other in ("global", "peel"):
        for k in ("nlev", "fp", "fc", "rp", "rc"):
            assert np.array_equal(got["relax"][k], got[other][k]), (other, k)
        # Kahn order inside a level depends on wave timing: compare level sets
        a, b, lv = got["relax"]["topo"], got[other]["topo"], got["relax"]["lvl"]
        for g in range(G):
            n0, n1 = int(corpus.node_off[g]), int(corpus.node_off[g + 1])
            off = lv[n0 + g: n0 + g + int(got["relax"]["nlev"][g]) + 1]
            assert np.array_equal(off, got[other]["lvl"][n0 + g: n0 + g + len(off)]), (other, g)
            for l0, l1 in zip(off[:-1], off[1:]):
                assert sorted(a[n0 + l0:n0 + l1]) == sorted(b[n0 + l0:n0 + l1])
            assert int(off[-1]) == n1 - n0
    assert np.array_equal(got["relax"]["nlv"], got["peel"]["nlv"])
    if shape == "long":
        assert int(got["relax"]["nlev"].max()) > 256


@pytest.mark.parametrize("lds_max", [0, 1500, 2600])
def test_graph_lds_tier(eng, lds_max):
    # kernels' LDS graph tier (graphs staged as u16 CSR) vs their global tier, and mixtures
    from tools import synth
    corpus, _ = synth.generate(30, target_nodes=2500)
    eng.set_option("graph_lds_max", lds_max)
    try:
        _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)
    finally:
        eng.set_option("graph_lds_max", -1)


@pytest.mark.parametrize("lds_max", [-1, 0])
def test_holds_before_simplify(eng, lds_max):
    # markConditionHolds is deferred for LDS-tier graphs (fused into nemo_simplify);
    # reading the flags in between materialises exactly the holds bits
    from nemo_amd.corpus import F_HOLDS
    from tools import synth
    corpus, _ = synth.generate(12, target_nodes=1500)
    s, f = corpus.success_iters(), corpus.failed_iters()
    orc = O.analyze(corpus, s, f, skip_pulls=True)
    eng.set_option("graph_lds_max", lds_max)
    try:
        eng.load(corpus)
        eng.mark()
        assert np.array_equal(eng.flags(), orc.flags & F_HOLDS)
        eng.simplify()
        assert np.array_equal(eng.flags(), orc.flags)
    finally:
        eng.set_option("graph_lds_max", -1)


def test_build_heavy_indegree_redo(eng):
    # a body goal shared by 300 rules: in-degree beyond k_build's u8 counters,
    # so the graph is flagged and rebuilt by the global tier
    goals = [{"id": "goal_hub", "label": "clock(a, b, 1, 2)", "table": "clock", "time": "1"}]
    rules, edges = [], []
    for i in range(300):
        goals.append({"id": f"goal{i}", "label": f"log(a, {i}, 2)", "table": "log", "time": "2"})
        rules.append({"id": f"rule{i}", "label": "log", "table": "log", "type": "async" if i % 3 else "next"})
        edges += [{"from": f"goal{i}", "to": f"rule{i}"}, {"from": f"rule{i}", "to": "goal_hub"}]
    g = {"goals": goals, "rules": rules, "edges": edges}
    small = {"goals": goals[:3], "rules": rules[:2], "edges": edges[:4]}
    corpus = corpus_from_graphs([(0, "success", g, small), (1, "failure", small, g)])
    _check(eng, corpus)


@pytest.mark.parametrize("prep", [1, 0])
@pytest.mark.parametrize("block", [256, 512])
@pytest.mark.parametrize("kind", ["random", "synthetic", "branchy"])
def test_chains_glob_tier(kind, block, prep):
    # k_chains_glob (deep-graph tier, scratch in HBM) on every graph of small corpora, at both
    # workgroup sizes, with the H* order and adjacency built by the XCD teams of k_glob_prep
    # (identity-rank corpora) and by k_chains_glob's own front phases
    import random as _r
    from tests.small import random_prov
    e = E.Engine(0)
    try:
        e.set_option("chains_glob_min_v", 0)
        e.set_option("chains_glob_block", block)
        e.set_option("chains_glob_prep", prep)
        if kind == "random":
            for seed in range(12):
                corpus, _ = random_corpus(300 + seed, max_nodes=16)
                _check(e, corpus)
        elif kind == "synthetic":
            from tools import synth
            corpus, _ = synth.generate(16, target_nodes=3000)
            _check(e, corpus, mode=DIFF_PER_RUN, pulls=True)
        else:
            rng = _r.Random(5)
            graphs = []
            for it in range(40):
                st = "success" if it == 0 or rng.random() < 0.8 else "failure"
                graphs.append((it, st, random_prov(rng, "pre", 40, p_edge=0.2, p_next=0.9),
                               random_prov(rng, "post", 40, p_edge=0.2, p_next=0.9)))
            _check(e, corpus_from_graphs(graphs))
    finally:
        e.close()


@pytest.mark.parametrize("shape", ["wide_hstar", "many_levels", "long_chains"])
def test_chains_lds_tiers(eng, shape):
    # k_chains<1664, 120> (4 workgroups/CU) hands graphs whose chain subgraph,
    # level count or longest prefix exceed it to k_chains<2048, 512>; both
    # against the oracle on graphs that land in each tier
    from nemo_amd.corpus import corpus_from_graphs
    from tools import synth
    if shape == "wide_hstar":  # H* of ~1.7-2k nodes: past the first tier's 1664
        corpus, _ = synth.generate(8, target_nodes=5600, eot=10)
    elif shape == "many_levels":  # > 120 Kahn levels: the first tier's old front
        corpus, _ = synth.generate(8, target_nodes=3000, eot=60)
    else:  # one @next chain of 80 rules (prefix length 159 > 118): the second tier
        def chain(cond, n):
            goals = [{"id": f"goal{i}", "label": f"log(a, {i})", "table": cond if i == 0 else "log", "time": "1"}
                     for i in range(n + 1)]
            rules = [{"id": f"rule{i}", "label": "log", "table": "log", "type": "next"} for i in range(n)]
            edges = [e for i in range(n) for e in ({"from": f"goal{i}", "to": f"rule{i}"},
                                                   {"from": f"rule{i}", "to": f"goal{i + 1}"})]
            return {"goals": goals, "rules": rules, "edges": edges}
        corpus = corpus_from_graphs([(0, "success", chain("pre", 80), chain("post", 80)),
                                     (1, "failure", chain("pre", 40), chain("post", 70))])
    _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)


@pytest.mark.parametrize("block", [256, 1024])
def test_global_tier_block(eng, block):
    # every graph on the global-memory kernels (k_csr, k_topo, k_mark,
    # k_simplify_flags, k_proto, k_diff, k_pull) at both workgroup sizes; deep
    # corpora select 1024 threads by shape
    from tools import synth
    corpus, _ = synth.generate(24, target_nodes=2500)
    for k, v in (("graph_lds_max", 0), ("build_lds_max", 0), ("global_block", block)):
        eng.set_option(k, v)
    try:
        _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)
        _check(eng, corpus, mode=DIFF_REFERENCE)
        for seed in range(4):
            c2, _ = random_corpus(900 + seed, max_nodes=24)
            _check(eng, c2)
    finally:
        for k in ("graph_lds_max", "build_lds_max", "global_block"):
            eng.set_option(k, -1)


@pytest.mark.parametrize("lds_max", [-1, 0])
def test_dense_graph_edge_reload(eng, lds_max):
    # a dense LDS-tier graph (2000 nodes, > 8192 edges): k_marksimp re-reads
    # its edge list from HBM per pass instead of holding it in registers
    import random
    rng = random.Random(11)
    tabs = ["pre", "post", "log", "ack", "node", "clock"]

    def dense(cond):
        goals, rules, edges = [], [], []
        for t in range(10):
            for i in range(100):
                tb = rng.choice(tabs)
                goals.append({"id": f"goal{t}_{i}", "label": f"{tb}(a, {i}, {t})", "table": tb, "time": str(t)})
                rt = cond if rng.random() < 0.3 else rng.choice(tabs)
                rules.append({"id": f"r{t}_{i}", "label": rt, "table": rt,
                              "type": "next" if rng.random() < 0.5 else rng.choice(["async", "single"])})
        for t in range(10):
            for i in range(100):
                for j in rng.sample(range(100), 5):
                    edges.append({"from": f"goal{t}_{i}", "to": f"r{t}_{j}"})
                if t < 9:
                    for j in rng.sample(range(100), 4):
                        edges.append({"from": f"r{t}_{i}", "to": f"goal{t + 1}_{j}"})
        return {"goals": goals, "rules": rules, "edges": edges}

    graphs = [(0, "success", dense("pre"), dense("post")), (1, "failure", dense("pre"), dense("post"))]
    corpus = corpus_from_graphs(graphs)
    assert max(corpus.edge_off[g + 1] - corpus.edge_off[g] for g in range(corpus.n_graphs)) > 8192
    eng.set_option("graph_lds_max", lds_max)
    try:
        _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)
    finally:
        eng.set_option("graph_lds_max", -1)


@pytest.mark.parametrize("tiers", ["default", "deep"])
def test_dense_c5_shape(eng, tiers):
    # bench.py's C5 generator settings (~4 edges per node, body goals shared
    # across rules) at 15k-node graphs; "deep" forces every kernel onto the
    # tiers the 1M-node C5 graphs take (global CSR/Kahn, k_chains_glob, 1024 threads)
    from tools import synth
    corpus, _ = synth.generate(16, target_nodes=20000, eot=20, body_extra=6, nval=3, nloc=4)
    assert corpus.edge_off[-1] > 3.5 * corpus.node_off[-1] and corpus.failed_iters()
    knobs = (("graph_lds_max", 0), ("build_lds_max", 0), ("chains_glob_min_v", 0), ("global_block", 1024))
    if tiers == "deep":
        for k, v in knobs:
            eng.set_option(k, v)
    try:
        _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)
    finally:
        for k, _ in knobs:
            eng.set_option(k, 65536 if k == "chains_glob_min_v" else -1)  # the library's defaults


def _next_chain(cond, n):
    goals = [{"id": f"goal{i}", "label": f"log(a, {i})", "table": cond if i == 0 else "log", "time": "1"}
             for i in range(n + 1)]
    rules = [{"id": f"rule{i}", "label": "log", "table": "log", "type": "next"} for i in range(n)]
    edges = [e for i in range(n) for e in ({"from": f"goal{i}", "to": f"rule{i}"},
                                           {"from": f"rule{i}", "to": f"goal{i + 1}"})]
    return {"goals": goals, "rules": rules, "edges": edges}


@pytest.mark.parametrize("fallback", [False, True])
def test_fallback_worklists_stride(eng, fallback):
    # The fallback tiers run over worklists with a capped grid (k_chains_list:
    # 1024 workgroups, k_csr/k_topo/k_pull: 2048), so a workgroup takes several
    # listed graphs in turn.  1400 runs, two thirds of them 70-rule @next chains
    # (141 Kahn levels: the first k_chains tier hands them to k_chains_list),
    # the rest 10-rule chains (kept by the first tier): ~1870 listed graphs.
    # With the graph and build LDS tiers off, all 2800 graphs go through the
    # k_csr/k_topo and k_pull lists.
    graphs = []
    for r in range(1400):
        n = 10 if r % 3 == 0 else 70
        st = "failure" if r % 7 == 3 else "success"
        graphs.append((r, st, _next_chain("pre", n), _next_chain("post", n - (r % 5))))
    corpus = corpus_from_graphs(graphs)
    keys = ("graph_lds_max", "build_lds_max")
    if fallback:
        for k in keys:
            eng.set_option(k, 0)
    try:
        _check(eng, corpus, mode=DIFF_PER_RUN, pulls=True)
        # the lists really were longer than their grids (k += gridDim.x taken);
        # sel = [pull list | chains list | load list], G+1 u32 each, count first
        G = corpus.n_graphs
        sel = eng.debug_copy("sel", 0, 4 * 3 * (G + 1)).view(np.uint32)
        n_pull, n_chains, n_load = int(sel[0]), int(sel[G + 1]), int(sel[2 * (G + 1)])
        assert n_chains > 1024, n_chains
        if fallback:
            assert n_load > 2048 and n_pull > 2048, (n_load, n_pull)
    finally:
        for k in keys:
            eng.set_option(k, -1)


def test_diff_label_set_mode(eng):
    # nemo_goal_labels (device label set of failedRuns[0]) -> nemo_diffprov_labels
    # equals the reference mode's in-place substitution (differential-provenance.go:22-43)
    import torch
    from tools import synth
    corpus, _ = synth.generate(30, target_nodes=2000, p_fault=0.5)
    s, f = corpus.success_iters(), corpus.failed_iters()
    assert len(f) >= 2
    orc = O.analyze(corpus, s, f, diff_mode=DIFF_REFERENCE, skip_pulls=True)
    eng.load(corpus)
    eng.mark()
    eng.simplify()
    cap = corpus.graph_size(2 * corpus.run_index(f[0]) + 1) + 1
    d = torch.zeros(cap, dtype=torch.int32, device="cuda:0")
    eng.goal_labels(f[0], 1, d.data_ptr(), cap)
    eng.synchronize()
    g = 2 * corpus.run_index(f[0]) + 1
    n0, n1 = int(corpus.node_off[g]), int(corpus.node_off[g + 1])
    want = corpus.label[n0:n1][(corpus.node_word[n0:n1] & 0x80000000) == 0]
    h = d.cpu().numpy().view(np.uint32)
    assert int(h[0]) == len(want) and sorted(h[1:1 + len(want)].tolist()) == sorted(want.tolist())
    eng.diffprov_labels(f, d.data_ptr(), cap)
    assert np.array_equal(eng.diff_masks(len(f)), orc.diff_mask)
    assert np.array_equal(eng.missing(), orc.missing)
    with pytest.raises(E.NemoError):
        eng.goal_labels(f[0], 1, d.data_ptr(), cap - 1)  # capacity below the graph's nodes + 1


@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0)])
def test_node_context(devices):
    # nemo_ctx_create_node: the corpus LPT-sharded over the node context's
    # shards, run 0 replicated, the prototype vector all-reduced (RCCL for one
    # device, peer copies when shards share the device), the reference diff's
    # failedRuns[0] label set broadcast from its owner; every result in the
    # corpus' global numbering, bit-exact with the oracle
    from tools import synth
    corpus, _ = synth.generate(36, target_nodes=1500, p_fault=0.5)
    e = E.Engine(devices=list(devices))
    try:
        assert e.devices() == list(devices)
        e.set_timing(True)
        for mode in (DIFF_REFERENCE, DIFF_PER_RUN):
            _check(e, corpus, mode=mode, pulls=True)
        s, f = corpus.success_iters(), corpus.failed_iters()
        orc = O.analyze(corpus, s, f, diff_mode=DIFF_REFERENCE, skip_pulls=True)
        e.diffprov(f, DIFF_REFERENCE)
        assert np.array_equal(e.diff_masks_view(), orc.diff_mask)
        # the staged hand-over, reassembled in global node / graph order
        e.stage_simplified()
        state, off, ht = e.simplified_view()
        from nemo_amd.corpus import F_DELETED, F_HOLDS, F_KEPT
        alive, holds = E.Engine.unpack_state(state, len(orc.flags))
        assert np.array_equal(alive, (orc.flags & (F_KEPT | F_DELETED)) == F_KEPT)
        assert np.array_equal(holds, (orc.flags & F_HOLDS) != 0)
        G = corpus.n_graphs
        g = np.repeat(np.arange(G), np.diff(off.astype(np.int64)))
        k = np.arange(len(ht)) - off[g].astype(np.int64)
        got = np.stack([g, k, ht[:, 0].astype(np.int64), ht[:, 1].astype(np.int64)], 1)
        assert np.array_equal(got, orc.chains[:, :4].astype(np.int64))
        # diff-graph pulls by global entry
        e.pull(2)
        g0 = 2 * corpus.run_index(0) + 1
        e0, e1 = int(corpus.edge_off[g0]), int(corpus.edge_off[g0 + 1])
        src, dst = corpus.edge_src[e0:e1], corpus.edge_dst[e0:e1]
        for i in range(len(f)):
            m = orc.diff_mask[i]
            want = sorted((int(a), int(b)) for a, b in zip(src, dst) if m[a] and m[b])
            sp, dp = e.pulled(i)
            assert sorted(zip(sp.tolist(), dp.tolist())) == want
        tim = e.timings()
        assert tim["k_chains"]["launches"] >= len(devices)
        if len(devices) > 1:
            with pytest.raises(E.NemoError):
                e.set_stream(0)
    finally:
        e.close()


def test_pull_on_aux_stream(eng):
    """Option pull_aux 1: the simplified pull runs on the diff stream behind the end of the simplification
    (beside the protos); the pulled edges, the protos and every other output still equal the oracle's."""
    from tools import synth
    corpus, _ = synth.generate(40, p_fault=0.5, prepend_run0=True, **synth.CONFIGS["c3"])
    eng.set_option("pull_aux", 1)
    try:
        _check(eng, corpus)
        _check(eng, corpus, mode=DIFF_PER_RUN)  # twice on one context: the second load joins the first pull
    finally:
        eng.set_option("pull_aux", 0)


@pytest.mark.parametrize("stage_aux,diff_aux", [(1, 1), (0, 1), (1, 0), (0, 0)])
def test_stage_and_diff_streams(eng, stage_aux, diff_aux):
    """Options stage_aux / diff_aux: the hand-over kernels and the diff kernels on the aux stream or on
    the context's stream.  A small corpus is staged first, so the next corpus' stage runs at a short
    pair-count hint and nemo_simplified_view re-stages (on the context's stream) -- every output still
    equals the oracle's."""
    from nemo_amd.corpus import F_DELETED, F_HOLDS, F_KEPT
    from tools import synth
    small, _ = synth.generate(4, target_nodes=300)
    big, _ = synth.generate(30, target_nodes=2500, p_fault=0.4)
    eng.set_option("stage_aux", stage_aux)
    eng.set_option("diff_aux", diff_aux)
    try:
        for corpus in (small, big):
            s, f = corpus.success_iters(), corpus.failed_iters()
            orc = O.analyze(corpus, s, f, diff_mode=DIFF_PER_RUN, skip_pulls=True)
            eng.load(corpus)
            eng.mark()
            eng.simplify()
            eng.stage_simplified()
            eng.prototypes(s)
            eng.diffprov(f, DIFF_PER_RUN)
            state, off, ht = eng.simplified_view()
            alive, holds = E.Engine.unpack_state(state, len(orc.flags))
            assert np.array_equal(alive, (orc.flags & (F_KEPT | F_DELETED)) == F_KEPT)
            assert np.array_equal(holds, (orc.flags & F_HOLDS) != 0)
            G = corpus.n_graphs
            g = np.repeat(np.arange(G), np.diff(off.astype(np.int64)))
            k = np.arange(len(ht)) - off[g].astype(np.int64)
            got = np.stack([g, k, ht[:, 0].astype(np.int64), ht[:, 1].astype(np.int64)], 1)
            assert np.array_equal(got, orc.chains[:, :4].astype(np.int64))
            if f:
                assert np.array_equal(eng.diff_masks(len(f)), orc.diff_mask)
                assert np.array_equal(eng.missing(), orc.missing)
    finally:
        eng.set_option("stage_aux", 1)
        eng.set_option("diff_aux", 1)


@pytest.mark.parametrize("knobs", [(), (("chains_lds_max", 12), ("chains_comp_max", 5), ("graph_lds_max", 30),
                                        ("build_lds_max", 30))])
def test_repeated_passes_tier_cache(eng, knobs):
    """The global tiers' list sizes are captured after the first full pass and an empty tier is not launched
    afterwards (api.hip tier_empty).  Several passes (rebuild, mark, simplify, protos, diff, triggers, pulls) over
    one loaded corpus, with every tier empty (library defaults) and with every tier taking graphs (small LDS caps),
    each pass equal to the oracle; then an option change (which resets the cache) and one more pass."""
    import random
    from tests.small import random_prov
    from tools import synth
    rng = random.Random(3)
    graphs = [(it, "success" if it == 0 or rng.random() < 0.7 else "failure",
               random_prov(rng, "pre", 40, p_edge=0.2, p_next=0.9), random_prov(rng, "post", 40, p_edge=0.2, p_next=0.9))
              for it in range(30)]
    corpus = corpus_from_graphs(graphs) if knobs else synth.generate(30, target_nodes=2000, p_fault=0.4)[0]
    s, f = corpus.success_iters(), corpus.failed_iters()
    orc = O.analyze(corpus, s, f, diff_mode=DIFF_PER_RUN)
    for k, v in knobs:
        eng.set_option(k, v)
    try:
        eng.load(corpus)
        for p in range(4):
            if p == 3:
                eng.set_option("global_block", 256)  # resets the cache: the tiers run again
            eng.rebuild()
            eng.mark()
            eng.simplify()
            achieved, inter, uni = eng.prototypes(s)
            eng.diffprov(f, DIFF_PER_RUN)
            eng.triggers()
            eng.pull(1)
            off, cnt, src, dst = eng.pulled_all(corpus.n_graphs)
            pulled = [(src[int(a):int(a) + int(n)], dst[int(a):int(a) + int(n)]) for a, n in zip(off, cnt)]
            pre, post, asy = eng.trigger_rows()
            res = E.EngineResult(flags=eng.flags(), chains=eng.chains(), proto_bits=eng.run_tables(0),
                                 graph_tables=eng.run_tables(1), achieved=achieved, inter=inter, union=uni,
                                 diff_mask=eng.diff_masks(len(f)), missing=eng.missing(), pre_rows=pre,
                                 post_rows=post, async_rules=asy, pulled=pulled)
            assert_same(corpus, res, orc, len(f))
    finally:
        for k, _ in knobs:
            eng.set_option(k, -1)
        eng.set_option("global_block", -1)


@pytest.mark.parametrize("seq", ["plain", "off", "twice", "option_between", "holds_first", "build_caps"])
def test_build_marksimp_tail(eng, seq):
    """k_build's tail runs the deferred mark + simplification (marksimp.h) of its graphs at load / rebuild and
    nemo_simplify skips them in k_marksimp (api.hip ms_fused).  The result must not depend on the call sequence:
    the tail off (option build_marksimp 0, the default); mark + simplify twice after one rebuild (the second pass recomputes:
    the chain cover has marked the flags); an option change between rebuild and mark (tiers may move); the holds
    flags read before the simplification (k_mark rewrites them); k_build's caps below some graphs (k_marksimp takes
    those beside the tail's).  Flags, chains and protos against the oracle each time."""
    from tools import synth
    from nemo_amd.corpus import F_HOLDS
    corpus, _ = synth.generate(24, target_nodes=1500, p_fault=0.4)
    s, f = corpus.success_iters(), corpus.failed_iters()
    orc = O.analyze(corpus, s, f, skip_pulls=True)
    opts = [("build_marksimp", 0 if seq == "off" else 1)] + ([("build_lds_max", 1200)] if seq == "build_caps" else [])
    for k, v in opts:
        eng.set_option(k, v)
    try:
        eng.load(corpus)
        for p in range(2):
            eng.rebuild()
            if seq == "option_between":
                eng.set_option("chains_lds_max", -1)
            eng.mark()
            if seq == "holds_first":
                assert np.array_equal(eng.flags(), orc.flags & F_HOLDS)
            eng.simplify()
            if seq == "twice":
                eng.mark()
                eng.simplify()
            assert np.array_equal(eng.flags(), orc.flags), (seq, p)
            assert np.array_equal(eng.chains(), orc.chains), (seq, p)
            achieved, inter, uni = eng.prototypes(s)
            assert achieved == orc.achieved and np.array_equal(inter, orc.inter) and np.array_equal(uni, orc.union)
    finally:
        for k, _ in opts:
            eng.set_option(k, -1)
