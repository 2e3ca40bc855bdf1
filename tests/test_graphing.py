"""The host side of the drop-in (nemo_amd/graphing.py, nemo_amd/dot.py): the
strings, Missing records and DOT graphs the reference's Go code builds around
its queries (diagrams.go, corrections.go, extensions.go, hazard-analysis.go,
prototype.go:245-251).

CPU tests pin the gographviz serialisation with hand-derived strings and check
the string synthesis against the literal restatement (oracle/host_literal.py);
the gpu test runs the whole `Neo4J` mirror over libnemohip in main.go's call
order against the golden fixtures and random corpora."""
import json
import os
import random

import pytest

from nemo_amd import graphing as GR
from nemo_amd.dot import DotGraph, ProvNode, create_dot, read_dot
from oracle import cypher_literal as CL
from oracle import host_literal as HL
from tests.golden_view import digest, host_expected
from tests.small import prefixed_runs, random_corpus

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(d for d in os.listdir(HERE) if os.path.isfile(os.path.join(HERE, d, "expected.json")))


# ---- gographviz serialisation (write.go:118-154, ast.go), hand-derived -------------
def test_dot_writer_pinned():
    g = DotGraph("dataflow", True)
    g.add_node("dataflow", "graph", {"bgcolor": '"transparent"'})
    g.add_node("dataflow", "b", {"label": '"B"', "shape": "rect"})
    g.add_node("dataflow", "a", {"shape": "ellipse"})
    g.add_node("dataflow", "b", {"color": '"red"'})  # AddNode of an existing node extends its attributes
    g.add_edge("b", "a", True, {"color": '"black"'})
    g.add_edge("a", "b", True, {})
    assert g.string() == ('digraph dataflow {\n'
                          '\tb->a[ color="black" ];\n'
                          '\ta->b;\n'
                          '\ta [ shape=ellipse ];\n'
                          '\tb [ color="red", label="B", shape=rect ];\n'
                          '\tgraph [ bgcolor="transparent" ];\n'
                          '\n}\n')


SPACETIME = """digraph spacetime {
  rankdir=TB; // layout
  node [shape=box];
  /* process a */
  subgraph cluster_a { label="a"; a_1; a_2 [color=red] }
  a_1 -> a_2 -> b_2 [label="m"];
  b_2 [label="b@2"];
}
"""


def test_dot_reader_subgraphs_defaults_chains():
    g = read_dot(SPACETIME)
    assert g.name == "spacetime" and g.directed
    assert [(e.src, e.dst, e.attrs) for e in g.edges] == [("a_1", "a_2", {"label": '"m"'}),
                                                         ("a_2", "b_2", {"label": '"m"'})]
    assert g.nodes["a_2"] == {"color": "red", "shape": "box"}
    assert g.nodes["b_2"] == {"label": '"b@2"', "shape": "box"}
    # analyse.go: edge endpoints join the scope they are used in; subgraphs are
    # written first with their sorted children, then every unwritten node
    assert g.string() == ('digraph spacetime {\n'
                          '\trankdir=TB;\n'
                          '\ta_1->a_2[ label="m" ];\n'
                          '\ta_2->b_2[ label="m" ];\n'
                          '\tsubgraph cluster_a {\n'
                          '\tlabel="a";\n'
                          '\ta_1 [ shape=box ];\n'
                          '\ta_2 [ color=red, shape=box ];\n'
                          '\n}\n;\n'
                          '\tb_2 [ label="b@2", shape=box ];\n'
                          '\n}\n')
    again = read_dot(g.string())
    assert again.nodes == g.nodes and [(e.src, e.dst, e.attrs) for e in again.edges] == \
           [(e.src, e.dst, e.attrs) for e in g.edges]


def test_dot_reader_rejects_garbage():
    from nemo_amd.dot import DotSyntaxError
    for bad in ("digraph {", "foo { a }", "digraph x { a -> }", "digraph x { a } b"):
        with pytest.raises(DotSyntaxError):
            read_dot(bad)


def test_hazard_colouring_pinned(tmp_path):
    """CreateHazardAnalysis (hazard-analysis.go:39-80): pre holds at time 2, post at 1
    (molly.go:38-48 keys the last column of model.tables rows)."""
    run = {"model": {"tables": {"pre": [["n", "2"]], "post": [["n", "1"]]}}}
    g = GR.hazard_colour(read_dot(SPACETIME), GR.time_holds(run, "pre"), GR.time_holds(run, "post"))
    assert g.string() == ('digraph spacetime {\n'
                          '\trankdir=TB;\n'
                          '\ta_1->a_2[ label="m" ];\n'
                          '\ta_2->b_2[ label="m" ];\n'
                          '\tsubgraph cluster_a {\n'
                          '\tlabel="a";\n'
                          '\ta_1 [ color="lightgrey", fillcolor="deepskyblue", shape=box, style="solid, filled" ];\n'
                          '\ta_2 [ color="firebrick", fillcolor="firebrick", shape=box, style="solid, filled" ];\n'
                          '\n}\n;\n'
                          '\tb_2 [ color="firebrick", fillcolor="firebrick", label="b@2", shape=box, '
                          'style="solid, filled" ];\n'
                          '\n}\n')


def test_create_dot_matches_restatement():
    """createDOT: product (dot.py) vs restatement (host_literal.py) on literal-DB edges."""
    for seed in range(20):
        corpus, graphs = random_corpus(seed, max_nodes=14)
        lit = CL.run_reference_pipeline(prefixed_runs(graphs))
        db = lit["db"]
        for it, _, _, _ in graphs:
            for run, cond in ((it, "pre"), (it, "post"), (1000 + it, "pre"), (1000 + it, "post")):
                edges = HL.q24_edges(db, run, cond)
                pn = lambda n: ProvNode(db.prop(n, "id"), db.prop(n, "label"), db.prop(n, "table"),
                                        db.prop(n, "type"), db.prop(n, "condition_holds"),
                                        db.nodes[n].label == "Rule")
                got = create_dot([(pn(a), pn(b)) for a, b in edges], cond)
                assert canon(got) == HL.canon(HL.create_dot(db, edges, cond))


# ---- corrections.go / extensions.go ---------------------------------------------------
def test_receiver_cutset():
    assert GR.receiver("abba(x, 1)", "ab") == "x"          # cutset, not prefix
    assert GR.receiver("ab((y), 2)", "ab") == "y)"         # Trim "()" on both ends only
    assert GR.receiver("log(srv, 2)", "log") == "srv"
    assert GR.receiver("log()", "log") == ""
    assert GR.receiver("clock(a, b, 1, 2)", "clock") == "a"
    rng = random.Random(7)
    alpha = "ab(), x"
    for _ in range(2000):
        lab = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 10)))
        tab = "".join(rng.choice("abx(") for _ in range(rng.randint(0, 3)))
        assert GR.receiver(lab, tab) == HL._receiver(lab, tab)


def _product_rows(db, pre_trig, post_trig):
    """Build graphing.generate_corrections' inputs from literal-DB rows, in the
    product's order (node IDs ascending)."""
    def rule(n):
        p = db.nodes[n].props
        return GR.Rule(p["id"], p["label"], p["table"], p["type"])

    def goal(n):
        p = db.nodes[n].props
        g = GR.Goal(p["id"], p["label"], p["table"], p["time"], bool(p["condition_holds"]))
        g.Receiver = GR.receiver(g.Label, g.Table)
        return g

    pre = sorted(pre_trig, key=lambda t: tuple(db.prop(x, "id") for x in t))
    post = sorted(post_trig, key=lambda t: tuple(db.prop(x, "id") for x in t))
    return ([(rule(a), GR.GoalRulePair(goal(g), rule(r))) for a, g, r in pre],
            [(goal(g), rule(r)) for g, r in post])


@pytest.mark.parametrize("name", FIXTURES)
def test_corrections_fixture_cpu(name):
    """String synthesis of the product over the literal rows is one of the admissible outputs."""
    d = os.path.join(HERE, name)
    exp = json.load(open(os.path.join(d, "expected.json")))
    runs = json.load(open(os.path.join(d, "runs.json")))
    from nemo_amd.corpus import _molly_prefix
    spec = []
    for i, r in enumerate(runs):
        pre = json.load(open(os.path.join(d, f"run_{i}_pre_provenance.json")))
        post = json.load(open(os.path.join(d, f"run_{i}_post_provenance.json")))
        spec.append((r["iteration"], r["status"], _molly_prefix(pre, r["iteration"], "pre"),
                     _molly_prefix(post, r["iteration"], "post")))
    lit = CL.run_reference_pipeline(spec)
    pre, post = _product_rows(lit["db"], lit["pre_trig"], lit["post_trig"])
    got = GR.generate_corrections(pre, post)
    if exp["corrections"] is not None:
        assert got in exp["corrections"]
    tables = [lit["db"].prop(r, "table") for r in sorted(lit["async_rules"])]
    assert sorted(GR.extension_strings(tables)) == HL.extensions(lit["db"], lit["async_rules"])


def test_corrections_random_cpu():
    n_checked = 0
    for seed in range(240):
        corpus, graphs = random_corpus(500 + seed, max_nodes=14)
        lit = CL.run_reference_pipeline(prefixed_runs(graphs))
        adm = HL.corrections_admissible(lit["db"], lit["pre_trig"], lit["post_trig"], max_orders=5000)
        if adm is None:
            continue
        pre, post = _product_rows(lit["db"], lit["pre_trig"], lit["post_trig"])
        assert tuple(GR.generate_corrections(pre, post)) in adm
        n_checked += bool(pre or post)
    assert n_checked >= 12


# ---- the whole mirror on the GPU ---------------------------------------------------------
def canon(g: DotGraph):
    return ({k: dict(sorted(v.items())) for k, v in g.nodes.items()},
            sorted((e.src, e.dst, tuple(sorted(e.attrs.items()))) for e in g.edges))


def canon_json(c):
    return {"nodes": c[0], "edges": [[a, b, dict(at)] for a, b, at in c[1]]}


def run_mirror(corpus, fi_dir=None):
    """main.go:106-177's graphing calls, in order."""
    db = GR.Neo4J()
    db.InitGraphDB("bolt://127.0.0.1:7687", corpus)
    try:
        iters = [int(x) for x in corpus.iteration]
        s, f = corpus.success_iters(), corpus.failed_iters()
        db.LoadRawProvenance()
        db.SimplifyProv(iters)
        hazard = None
        if fi_dir and os.path.exists(os.path.join(fi_dir, "run_0_spacetime.dot")):
            hazard = db.CreateHazardAnalysis(fi_dir)
        protos = db.CreatePrototypes(s, f) if s else None
        pre, post, pre_c, post_c = db.PullPrePostProv()
        diffs, faileds, missing = db.CreateNaiveDiffProv(False, f, post[0])
        corrections = db.GenerateCorrections()
        all_pre, extensions = db.GenerateExtensions()
    finally:
        db.CloseDB()
    return {"protos": protos, "dots": [{"pre": canon_json(canon(a)), "post": canon_json(canon(b)),
                                        "pre_clean": canon_json(canon(c)), "post_clean": canon_json(canon(d))}
                                       for a, b, c, d in zip(pre, post, pre_c, post_c)],
            "diff_dots": [canon_json(canon(x)) for x in diffs], "failed_dots": [canon_json(canon(x)) for x in faileds],
            "missing_events": [sorted(({"rule": m.Rule.to_json(),
                                        "goals": sorted((g.to_json() for g in m.Goals), key=lambda g: g["id"])}
                                       for m in ms), key=lambda m: m["rule"]["id"]) for ms in missing],
            "corrections": corrections, "all_pre": all_pre, "extensions": sorted(extensions), "hazard": hazard,
            "strings": [x.string() for x in pre + post + pre_c + post_c + diffs + faileds]}


def _norm_missing(ms):
    out = []
    for m in ms:
        out.append({"rule": m["rule"], "goals": [{k: v for k, v in g.items() if k != "conditionHolds" or v}
                                                 for g in m["goals"]]})
    return out


def assert_host_equal(got, exp, success):
    for k in ("dots", "diff_dots", "failed_dots"):
        if k in exp:
            assert json.loads(json.dumps(got[k])) == exp[k], k
        else:
            assert digest(got[k]) == exp[k + "_sha256"], k
    assert [_norm_missing(m) for m in got["missing_events"]] == [_norm_missing(m) for m in exp["missing_events"]]
    if exp["corrections"] is not None:
        assert got["corrections"] in exp["corrections"]
    assert got["all_pre"] == exp["all_pre"]
    assert got["extensions"] == exp["extensions"]
    if success and exp.get("inter") is not None:
        inter, inter_miss, union, union_miss = got["protos"]
        strip = lambda xs: sorted(x[len("<code>"):-len("</code>")] for x in xs)
        assert all(x.startswith("<code>") and x.endswith("</code>") for x in inter + union)
        assert strip(inter) == exp["inter"] and strip(union) == exp["union"]
        assert [strip(x) for x in inter_miss] == [sorted(x[len("<code>"):-len("</code>")] for x in y)
                                                  for y in exp["inter_miss"]]
        assert [strip(x) for x in union_miss] == [sorted(x[len("<code>"):-len("</code>")] for x in y)
                                                  for y in exp["union_miss"]]
    for s in got["strings"]:  # every DOT the mirror returns parses (its "graph" node reads back as graph attrs)
        g = read_dot(s)
        assert g.attrs.get("bgcolor") == '"transparent"' or g.attrs.get("style") == '"invis"'


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_mirror_fixture_gpu(name):
    from nemo_amd.corpus import load_molly
    d = os.path.join(HERE, name)
    exp = json.load(open(os.path.join(d, "expected.json")))
    corpus = load_molly(d)
    got = run_mirror(corpus, d)
    assert_host_equal(got, exp, bool(corpus.success_iters()))
    if got["hazard"] is not None:  # hazard-analysis.go:39-80 on the producer's space-time diagrams
        assert len(got["hazard"]) == corpus.n_runs
        for r, g in enumerate(got["hazard"]):
            pre, post = GR.time_holds(corpus.runs[r], "pre"), GR.time_holds(corpus.runs[r], "post")
            for name, attrs in g.nodes.items():
                t = name.split("_")[-1]
                assert attrs["style"] == '"solid, filled"'
                assert attrs["color"] == ('"firebrick"' if t in pre else '"lightgrey"')
                assert attrs["fillcolor"] == ('"deepskyblue"' if t in post else
                                              '"firebrick"' if t in pre else '"lightgrey"')


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_mirror_random_gpu(seed):
    corpus, graphs = random_corpus(700 + seed, max_nodes=14)
    runs = prefixed_runs(graphs)
    lit = CL.run_reference_pipeline(runs)
    exp = host_expected(lit, runs)
    exp["all_pre"] = lit["all_pre"]
    exp["inter"] = sorted(lit["inter"]) if lit["inter"] is not None else None
    exp["union"] = sorted(lit["union"]) if lit["union"] is not None else None
    exp["inter_miss"] = lit["inter_miss"]
    exp["union_miss"] = lit["union_miss"]
    got = run_mirror(corpus)
    assert_host_equal(got, exp, bool(corpus.success_iters()))
