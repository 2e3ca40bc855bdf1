"""Quirk fixtures (tests/golden/, made by tests/golden/make_fixtures.py):
Molly-format inputs through molly.go-equivalent loading, checked against the
expected outputs: the oracle here on CPU, libnemohip in the gpu-marked test."""
import json
import os

import numpy as np
import pytest

from nemo_amd.corpus import load_molly
from oracle import oracle as O
from tests.golden_view import tables, view

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(d for d in os.listdir(HERE) if os.path.isfile(os.path.join(HERE, d, "expected.json")))


def _compare(corpus, res, exp, failed, proto_bits, graph_tables, inter, union):
    got = view(corpus, res, failed)
    assert got["clean"] == exp["clean"]
    assert got["deleted"] == exp["deleted"]
    assert {k: v for k, v in got["holds"].items() if v} == {k: v for k, v in exp["holds"].items() if v}
    for key, chains in exp["chains"].items():
        assert [(c["k"], c["head"], c["tail"], c["len"], c["id"]) for c in got["chains"][key]] == \
               [(c["k"], c["head"], c["tail"], c["len"], c["id"]) for c in chains], key
    for it, lst in exp["lists"].items():
        assert tables(corpus, proto_bits[corpus.run_index(int(it))]) == lst
    if exp["inter"] is not None:
        assert sorted(corpus.tables[t] for t in inter) == exp["inter"]
        assert sorted(corpus.tables[t] for t in union) == exp["union"]
        for j, f in enumerate(failed):
            have = set(tables(corpus, graph_tables[corpus.run_index(f)]))
            assert sorted(t for t in exp["inter"] if t not in have) == sorted(
                x[len("<code>"):-len("</code>")] for x in exp["inter_miss"][j])
            assert sorted(t for t in exp["union"] if t not in have) == sorted(
                x[len("<code>"):-len("</code>")] for x in exp["union_miss"][j])


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_oracle(name):
    d = os.path.join(HERE, name)
    exp = json.load(open(os.path.join(d, "expected.json")))
    corpus = load_molly(d)
    s, f = corpus.success_iters(), corpus.failed_iters()
    res = O.analyze(corpus, s, f)
    _compare(corpus, res, exp, f, res.proto_bits, res.graph_tables, res.inter, res.union)
    ids = corpus.node_ids
    if res.run0 >= 0:
        g0 = 2 * res.run0 + 1
        n0 = int(corpus.node_off[g0])
        for e in range(len(f)):
            assert sorted(ids[n0 + i] for i in np.nonzero(res.diff_mask[e])[0]) == exp["diff"][e]
        np0 = int(corpus.node_off[2 * res.run0])
        assert sorted([ids[np0 + a], ids[np0 + g], ids[np0 + r]] for a, g, r in res.pre_rows.tolist()) == exp["pre_rows"]
        assert sorted([ids[n0 + g], ids[n0 + r]] for g, r in res.post_rows.tolist()) == exp["post_rows"]
        assert sorted(ids[np0 + r] for r in res.async_rules.tolist()) == exp["async"]
    T = corpus.n_tables
    assert (not (int(res.reduce[2 * T + 2]) < corpus.n_runs)) == exp["all_pre"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_gpu(name):
    from nemo_amd import engine as E
    d = os.path.join(HERE, name)
    exp = json.load(open(os.path.join(d, "expected.json")))
    corpus = load_molly(d)
    s, f = corpus.success_iters(), corpus.failed_iters()
    eng = E.Engine(0)
    try:
        res = E.analyze(corpus, s, f, engine=eng, pulls=False)
        _compare(corpus, res, exp, f, res.proto_bits, res.graph_tables, res.inter, res.union)
        ids = corpus.node_ids
        r0 = corpus.run_index(0)
        n0 = int(corpus.node_off[2 * r0 + 1])
        for e in range(len(f)):
            assert sorted(ids[n0 + i] for i in np.nonzero(res.diff_mask[e])[0]) == exp["diff"][e]
        # trigger rows (corrections.go:30-34,121-125), async rules and allAchievedPre (extensions.go:25-67)
        np0 = int(corpus.node_off[2 * r0])
        assert sorted([ids[np0 + a], ids[np0 + g], ids[np0 + r]] for a, g, r in res.pre_rows.tolist()) == exp["pre_rows"]
        assert sorted([ids[n0 + g], ids[n0 + r]] for g, r in res.post_rows.tolist()) == exp["post_rows"]
        assert sorted(ids[np0 + r] for r in res.async_rules.tolist()) == exp["async"]
        if len(s):
            assert (not (eng.protos_finalize(0)["pre_holds"] < corpus.n_runs)) == exp["all_pre"]
    finally:
        eng.close()
