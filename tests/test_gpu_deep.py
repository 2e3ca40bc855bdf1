"""GPU parity of the deep tier's edge cases (graphs of >= 8192 nodes: the
multi-workgroup CSR build, k_topo_deep and the global-tier sweeps), against
the CPU oracle.

- a Kahn level wider than k_topo_deep's LDS frontier (TD_Q = 2048 nodes), so
  the level's tail is read back from topo[];
- a cycle inside a big graph (loadProv's refusal, NEMO_ERR_CYCLE);
- a hub goal whose out-degree exceeds one batch of child loads (TD_BATCH).
"""
import random

import pytest

from nemo_amd import engine as E
from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE, corpus_from_graphs
from oracle import oracle as O
from tests.compare import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def _check(eng, corpus, mode=DIFF_REFERENCE):
    s, f = corpus.success_iters(), corpus.failed_iters()
    orc = O.analyze(corpus, s, f, diff_mode=mode)
    res = E.analyze(corpus, s, f, diff_mode=mode, engine=eng, pulls=True)
    assert_same(corpus, res, orc, len(f), check_pulls=True)


def wide_prov(cond: str, width: int, seed: int, hub: int = 0, cycle: bool = False) -> dict:
    """Three wide levels (root goals -> rules -> goals) plus a @next chain per
    column and a few cross edges; `hub` extra rule children hang off goal 0."""
    rng = random.Random(seed)
    goals, rules, edges = [], [], []

    def goal(name, table, t):
        goals.append({"id": "goal_" + name, "label": f"{table}({name})", "table": table, "time": str(t)})

    def rule(name, table, typ):
        rules.append({"id": "rule_" + name, "label": table, "table": table, "type": typ})

    goal("c0", cond, 1)
    rule("c1", cond, "single")
    edges += [{"from": "c0", "to": "c1"}]
    for i in range(width):
        t = ["t1", "t2", cond][i % 3]
        goal(f"a{i}", t, 1)
        rule(f"r{i}", t, "next" if i % 2 else "single")
        goal(f"b{i}", t, 2)
        rule(f"n{i}", t, "next")
        goal(f"d{i}", t, 3)
        edges += [{"from": f"a{i}", "to": f"r{i}"}, {"from": f"r{i}", "to": f"b{i}"},
                  {"from": f"b{i}", "to": f"n{i}"}, {"from": f"n{i}", "to": f"d{i}"}]
        if i and rng.random() < 0.3:
            edges.append({"from": f"a{rng.randrange(i)}", "to": f"r{i}"})
    edges.append({"from": "c1", "to": "a0"})
    for k in range(hub):
        rule(f"h{k}", "t1", "single")
        goal(f"hg{k}", "t1", 2)
        edges += [{"from": "a0", "to": f"h{k}"}, {"from": f"h{k}", "to": f"hg{k}"}]
    gset = {g["id"][5:] for g in goals}
    edges = [{"from": ("goal_" if e["from"] in gset else "rule_") + e["from"],
              "to": ("goal_" if e["to"] in gset else "rule_") + e["to"]} for e in edges]
    if cycle:
        edges.append({"from": "goal_d7", "to": "rule_r7"})  # r7 -> b7 -> n7 -> d7 -> r7
    return {"goals": goals, "rules": rules, "edges": edges}


@pytest.fixture(params=["topo_deep", "topo_ell"])
def kahn(request, eng):
    """The big graphs' Kahn levels by k_topo_deep, or by k_topo_ell (child records in the deep-graph
    scratch: every big graph gets one at chains_glob_min_v 0; records of 8 children, longer rows read
    from fc[])."""
    ell = request.param == "topo_ell"
    eng.set_option("topo_ell", 1 if ell else 0)
    eng.set_option("chains_glob_min_v", 0 if ell else 65536)
    yield request.param
    eng.set_option("topo_ell", -1)
    eng.set_option("chains_glob_min_v", 65536)


def test_wide_level_past_lds_frontier(eng, kahn):
    graphs = [(it, "success" if it != 2 else "failure", wide_prov("pre", 5000, it), wide_prov("post", 5000, 10 + it))
              for it in range(3)]
    corpus = corpus_from_graphs(graphs)
    assert min(corpus.graph_size(g) for g in range(corpus.n_graphs)) >= 8192
    _check(eng, corpus)
    _check(eng, corpus, mode=DIFF_PER_RUN)


def test_hub_out_degree(eng, kahn):
    graphs = [(it, "success" if it != 1 else "failure", wide_prov("pre", 2000, it, hub=300),
               wide_prov("post", 2000, 20 + it, hub=37)) for it in range(2)]
    corpus = corpus_from_graphs(graphs)
    assert min(corpus.graph_size(g) for g in range(corpus.n_graphs)) >= 8192
    _check(eng, corpus)


def test_cycle_in_big_graph_refused(eng, kahn):
    graphs = [(0, "success", wide_prov("pre", 3000, 1), wide_prov("post", 3000, 2, cycle=True))]
    corpus = corpus_from_graphs(graphs)
    assert corpus.graph_size(1) >= 8192
    with pytest.raises(E.NemoError) as ei:
        eng.load(corpus)
    assert ei.value.code == 4


def test_topo_ell_same_levels_as_topo_deep(eng):
    """k_topo_ell and k_topo_deep give the same Kahn level offsets and per-level node sets (the order within
    a level depends on timing) on the C5 generator's shape (~4 children per rule, rows past 8 children)."""
    import numpy as np
    from tools import synth
    corpus, _ = synth.generate(3, target_nodes=70000, eot=60, body_extra=6, nval=3, nloc=4, p_fault=0.5)
    V, G = int(corpus.node_off[-1]), corpus.n_graphs
    got = {}
    for ell in (0, 1):
        eng.set_option("topo_ell", ell)
        try:
            eng.load(corpus)
            got[ell] = {k: eng.debug_copy(k, 0, n).view(np.uint32)
                        for k, n in (("topo", 4 * V), ("lvl", 4 * (V + G)), ("nlev", 4 * G), ("nlv", 4 * V))}
        finally:
            eng.set_option("topo_ell", -1)
    a, b = got[0], got[1]
    assert np.array_equal(a["nlev"], b["nlev"]) and np.array_equal(a["lvl"], b["lvl"])
    assert np.array_equal(a["nlv"], b["nlv"])
    for g in range(G):
        n0 = int(corpus.node_off[g])
        off = a["lvl"][n0 + g: n0 + g + int(a["nlev"][g]) + 1]
        for l0, l1 in zip(off[:-1], off[1:]):
            assert sorted(a["topo"][n0 + l0:n0 + l1]) == sorted(b["topo"][n0 + l0:n0 + l1])


def _inject(corpus, g, extra):
    """Append graph-local edges `extra` [(src, dst)] to graph g (behind the host layer's back)."""
    import numpy as np
    eo = corpus.edge_off.astype(np.int64)
    a, b = int(eo[g]), int(eo[g + 1])
    xs = np.array([e[0] for e in extra], np.uint32)
    ys = np.array([e[1] for e in extra], np.uint32)
    corpus.edge_src = np.concatenate([corpus.edge_src[:b], xs, corpus.edge_src[b:]])
    corpus.edge_dst = np.concatenate([corpus.edge_dst[:b], ys, corpus.edge_dst[b:]])
    eo[g + 1:] += len(extra)
    corpus.edge_off = eo.astype(np.uint64)


def _created(corpus, g):
    """pre-post-prov.go:150-210's relationships-created count: distinct edges joining a goal and a rule."""
    import numpy as np
    from nemo_amd.corpus import NODE_RULE
    eo, no = corpus.edge_off.astype(np.int64), corpus.node_off.astype(np.int64)
    rule = (corpus.node_word[no[g]:no[g + 1]] & NODE_RULE) != 0
    pairs = set(zip(corpus.edge_src[eo[g]:eo[g + 1]].tolist(), corpus.edge_dst[eo[g]:eo[g + 1]].tolist()))
    return sum(1 for x, y in pairs if rule[x] != rule[y]), int(eo[g + 1] - eo[g])


@pytest.mark.parametrize("case", ["short_rows", "wide_row", "long_row", "hbm_bucket"])
def test_load_error_counts_in_big_graph(eng, case):
    """The bucketed CSR build's relationships-created count (edge-parallel goal/rule check, duplicates
    taken back out per row) against a direct count, in each of its row-sort paths: rows of <= 16
    entries (register networks), 17..64 (wave sort), > 64 (thread sort), and a bucket past the LDS
    capacity (rows assembled and sorted in HBM)."""
    hub = {"short_rows": 0, "wide_row": 30, "long_row": 300, "hbm_bucket": 15000}[case]
    graphs = [(0, "success", wide_prov("pre", 3000, 1), wide_prov("post", 3000, 2, hub=hub))]
    corpus = corpus_from_graphs(graphs)
    assert corpus.graph_size(1) >= 8192
    eo = corpus.edge_off.astype(int)
    src, dst = corpus.edge_src[eo[1]:eo[2]], corpus.edge_dst[eo[1]:eo[2]]
    # duplicates of a few edges (short rows, and the last edge of a0's row: the hub's), plus a goal -> goal edge
    extra = [(int(src[i]), int(dst[i])) for i in (0, 5, 17, 17)]
    a0 = [i for i in range(len(src)) if int(src[i]) == int(src[1])]  # goal a0's forward row (the hub)
    extra += [(int(src[a0[-1]]), int(dst[a0[-1]]))] * 2
    extra.append((int(src[0]), int(src[1])))
    _inject(corpus, 1, extra)
    want, E_ = _created(corpus, 1)
    assert want != E_
    with pytest.raises(E.NemoError) as ei:
        eng.load(corpus)
    assert f"inserted number of edges ({want}) does not equal number of antecedent provenance edges ({E_})" \
        in str(ei.value)


def test_diff_fallback_past_walk_window(eng):
    """A run-0 post graph with a row of more links than one walk window holds (dx_max_row = 8192): the
    multi-entry diff (k_dx) cannot stage it, and CreateNaiveDiffProv runs on the one-workgroup-per-entry
    kernels of k_diff.hip, the library's fallback tier; both diff modes against the oracle."""
    graphs = [(0, "success", wide_prov("pre", 2500, 1), wide_prov("post", 2500, 2, hub=9000)),
              (1, "failure", wide_prov("pre", 2500, 3), wide_prov("post", 2500, 4)),
              (2, "failure", wide_prov("pre", 2500, 5), wide_prov("post", 2400, 6))]
    corpus = corpus_from_graphs(graphs)
    _check(eng, corpus)
    _check(eng, corpus, mode=DIFF_PER_RUN)
