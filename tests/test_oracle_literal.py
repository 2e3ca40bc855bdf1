"""Pin the C oracle (O(V+E) closed forms) to the literal Cypher evaluator on random tiny corpora.

Neither is the reference engine (Neo4j is absent): parity with
the reference itself is UNPINNED; this test is what the closed forms stand on.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from nemo_amd.corpus import F_DELETED, F_HOLDS, F_KEPT
from oracle import cypher_literal as CL
from oracle import oracle as O
from tests.small import bits_to_tables, diff_missing_sets, literal_view, prefixed_runs, random_corpus


def check_seed(seed: int, max_nodes: int = 12, diff_mode: int = 0):
    corpus, graphs = random_corpus(seed, max_nodes=max_nodes)
    runs = prefixed_runs(graphs)
    success = corpus.success_iters()
    failed = corpus.failed_iters()
    lit = CL.run_reference_pipeline(runs)
    view = literal_view(corpus, lit)
    res = O.analyze(corpus, success, failed, diff_mode=diff_mode)
    for g in range(corpus.n_graphs):
        n0 = int(corpus.node_off[g])
        V = corpus.graph_size(g)
        fl = res.flags[n0:n0 + V]
        assert np.array_equal((fl & F_HOLDS) != 0, view["holds"][g]), f"holds g={g}"
        assert set(np.nonzero(fl & F_KEPT)[0]) == view["kept"][g], f"clean g={g}"
        assert set(np.nonzero(fl & F_DELETED)[0]) == view["deleted"][g], f"deleted g={g}"
        och = [tuple(int(x) for x in row[1:]) for row in res.chains if row[0] == g]
        assert och == view["chains"][g], f"chains g={g}"
        s, d = res.pulled(g)
        assert sorted(zip(s.tolist(), d.tolist())) == view["gprime"][g], f"graph' g={g}"
    for it in success:
        r = corpus.run_index(it)
        assert bits_to_tables(corpus, res.proto_bits[r]) == view["lists"][it], f"proto list run {it}"
    inter = {corpus.tables[t] for t in res.inter}
    union = {corpus.tables[t] for t in res.union}
    assert inter == view["inter"]
    assert union == view["union"]
    for j, f in enumerate(failed):
        have = bits_to_tables(corpus, res.graph_tables[corpus.run_index(f)])
        assert {t for t in inter if t not in have} == view["inter_miss"][j]
        assert {t for t in union if t not in have} == view["union_miss"][j]
    if res.run0 >= 0:
        g0 = 2 * res.run0 + 1
        for e in range(len(failed)):
            mask = res.diff_mask[e]
            assert set(np.nonzero(mask)[0]) == view["diff"][e], f"diff entry {e}"
            rules = [int(r) for en, r in res.missing if en == e]
            assert diff_missing_sets(corpus, mask, rules, g0) == view["missing"][e], f"missing entry {e}"
        assert {tuple(int(x) for x in row) for row in res.pre_rows} == view["pre"]
        assert {tuple(int(x) for x in row) for row in res.post_rows} == view["post"]
        assert {int(x) for x in res.async_rules} == view["async"]
    T = corpus.n_tables
    assert (not (int(res.reduce[2 * T + 2]) < corpus.n_runs)) == view["all_pre"]


@settings(max_examples=400, deadline=None, suppress_health_check=list(HealthCheck))
@given(st.integers(min_value=0, max_value=2**31 - 1))
def test_oracle_matches_literal(seed):
    check_seed(seed)


@settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck))
@given(st.integers(min_value=0, max_value=2**31 - 1))
def test_oracle_matches_literal_bigger(seed):
    check_seed(seed, max_nodes=16)


@pytest.mark.parametrize("seed", range(40))
def test_oracle_matches_literal_fixed(seed):
    check_seed(seed)
