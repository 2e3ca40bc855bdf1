"""The Molly-format producer (nemo_amd/molly): Dedalus
semantics on hand-checked programs, lineage-driven fault injection, and the
output layout faultinjectors/molly.go reads."""
import json
import os

import pytest

from nemo_amd.corpus import load_molly
from nemo_amd.molly import FailureSpec, evaluate, explore, parse, write_output
from nemo_amd.molly.dedalus import DedalusError, WILD, reachable

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = sorted(d for d in os.listdir(HERE) if d.startswith("cs_"))

# A two-node broadcast: `a` sends `msg` to `b` at 1; `b` logs and keeps it.
BCAST = """
// sbt "run-main ... --nodes a,b --EOT 4 --EFF 2 --crashes 0 prog.ded"
msg(B, A, X)@async :- start(A, B, X);
log(B, X) :- msg(B, _, X);
log(B, X)@next :- log(B, X);
pre(X) :- start(_, _, X);
pre(X)@next :- pre(X);
post(X) :- log(_, X);
start("a", "b", 7)@1;
"""


def test_parse_and_options():
    p = parse(BCAST)
    assert p.options == {"nodes": "a,b", "EOT": "4", "EFF": "2", "crashes": "0"}
    assert [(r.head.table, r.kind) for r in p.rules] == [("msg", "async"), ("log", ""), ("log", "next"),
                                                       ("pre", ""), ("pre", "next"), ("post", "")]
    assert p.facts == [("start", ("a", "b", 7), 1)]
    for bad in ("p(X) :- ;", "p(x) :- q(X);", "p(X)@later :- q(X);", "p(X)@1;"):
        with pytest.raises(DedalusError):
            parse(bad)


def test_evaluate_timeline_and_clock_goals():
    p = parse(BCAST)
    run = evaluate(p, FailureSpec(4, 2, 0, ["a", "b"]))
    assert run.tables[1]["pre"] == {(7,)} and "log" not in run.tables[1]
    assert run.tables[2]["log"] == {("b", 7)} and run.tables[4]["post"] == {(7,)}
    assert run.success and run.messages == [("msg", "a", "b", 1, 2)]
    (d,) = run.derivs[("msg", ("b", "a", 7), 2)]
    assert d.rule.kind == "async" and d.body == (("start", ("a", "b", 7), 1), ("clock", ("a", "b", 1, 2), 1))
    (d,) = run.derivs[("log", ("b", 7), 3)]
    assert d.body[-1] == ("clock", ("b", "b", 2, WILD), 2)


def test_omission_and_crash_break_delivery():
    p = parse(BCAST)
    lost = evaluate(p, FailureSpec(4, 2, 0, ["a", "b"], omissions=frozenset({("a", "b", 1)})))
    assert "log" not in lost.tables[4] and not lost.success
    late = evaluate(p, FailureSpec(4, 1, 0, ["a", "b"], omissions=frozenset({("a", "b", 1)})))
    assert late.success  # omissions only before EFF
    crashed = evaluate(p, FailureSpec(4, 2, 1, ["a", "b"], crashes={"b": 3}))
    assert ("b", 7) in crashed.tables[3]["log"] and "log" not in crashed.tables[4]
    assert crashed.tables[4]["crash"] == {("b", "b", 3)}


def test_aggregate_arith_negation():
    p = parse("""
        c(N, K+1)@next :- c(N, K);
        v(N, count<K>) :- c(N, K), notin stop(N);
        big(N) :- v(N, C), C > 1;
        c("a", 0)@1; stop("b")@1; c("b", 5)@1;
    """)
    run = evaluate(p, FailureSpec(3, 0, 0, ["a", "b"]))
    assert run.tables[1]["v"] == {("a", 1)} and run.tables[3]["c"] == {("a", 2), ("b", 7)}
    assert run.tables[3]["v"] == {("a", 1), ("b", 1)} and "big" not in run.tables[3]


def test_ldfi_finds_the_lost_message():
    runs = explore(parse(BCAST), 4, 2, 0, ["a", "b"])
    assert runs[0].success and not runs[0].spec.omissions
    assert any(not r.success and ("a", "b", 1) in r.spec.omissions for r in runs)
    # crashes allowed: a crash of b before delivery is found as well
    runs = explore(parse(BCAST), 4, 2, 1, ["a", "b"])
    assert any(not r.success and r.spec.crashes for r in runs)


def test_output_layout_round_trips_through_the_loader(tmp_path):
    runs = explore(parse(BCAST), 4, 2, 1, ["a", "b"])
    write_output(runs, str(tmp_path))
    meta = json.load(open(tmp_path / "runs.json"))
    assert [r["iteration"] for r in meta] == list(range(len(runs)))
    assert meta[0]["status"] == "success" and meta[0]["model"]["tables"]["pre"][0] == ["7", "1"]
    prov = json.load(open(tmp_path / "run_0_post_provenance.json"))
    assert all("goal" in g["id"] for g in prov["goals"]) and all("goal" not in r["id"] for r in prov["rules"])
    assert any(g["label"] == "clock(a, b, 1, 2)" for g in prov["goals"])
    corpus = load_molly(str(tmp_path))
    assert corpus.n_runs == len(runs) and corpus.failed_iters()
    assert os.path.exists(tmp_path / "run_0_spacetime.dot")


def test_provenance_is_acyclic_and_rooted():
    p = parse(BCAST)
    run = evaluate(p, FailureSpec(4, 2, 0, ["a", "b"]))
    goals, rules = reachable(run, [("post", (7,), 4)])
    pos = {g: i for i, g in enumerate(goals)}
    assert goals[0] == ("post", (7,), 4)
    for head, d in rules:
        assert all(b[2] <= head[2] for b in d.body)
        assert all(b in pos for b in d.body)


@pytest.mark.parametrize("name", CASES)
def test_case_study_outputs_consistent(name):
    """Each committed case-study run's status matches its own model: success iff
    every pre row at EOT has a post row (the invariant Molly checks)."""
    d = os.path.join(HERE, name)
    meta = json.load(open(os.path.join(d, "runs.json")))
    assert meta[0]["status"] == "success" and not meta[0]["failureSpec"]["omissions"]
    assert any(r["status"] != "success" for r in meta)
    for r in meta:
        eot = str(r["failureSpec"]["eot"])
        at = lambda t: {tuple(row[:-1]) for row in r["model"]["tables"].get(t, []) if row[-1] == eot}
        assert (r["status"] == "success") == (at("pre") <= at("post"))
        assert len(r["failureSpec"]["crashes"]) <= r["failureSpec"]["maxCrashes"]
        assert all(o["time"] < r["failureSpec"]["eff"] for o in r["failureSpec"]["omissions"])
    corpus = load_molly(d)
    assert corpus.n_runs == len(meta)
