"""Writes the quirk fixtures of SURVEY.md Appendix C as Molly-format output
directories (runs.json + run_<i>_{pre,post}_provenance.json, the layout
faultinjectors/molly.go:18,59-60 reads) plus expected.json per fixture.

Expected values come from oracle/cypher_literal.py (a literal evaluation of the
reference's Cypher and Go) and each fixture asserts the hand-derived property
it exists for.  No reference outputs exist, so these pin the
restatement, not Neo4j itself.

Run: python tests/golden/make_fixtures.py   (rewrites tests/golden/<name>/)
"""
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from nemo_amd.corpus import _molly_prefix  # noqa: E402
from oracle import cypher_literal as CL  # noqa: E402
from tests.golden_view import host_expected  # noqa: E402


def G(i, table, label=None, time="1"):
    return {"id": f"goal{i}", "label": label or f"{table}(n, {i})", "table": table, "time": time}


def R(i, table, typ="single"):
    return {"id": f"rule{i}", "label": table, "table": table, "type": typ}


def E(a, b):
    return {"from": a, "to": b}


def prov(goals, rules, edges):
    return {"goals": goals, "rules": rules, "edges": edges}


EMPTY = prov([], [], [])


def cond_pattern(C, k=0, body_table="log"):
    """(C goal root) -> (C rule) -> (body goal) -> (rule) -> (leaf): makes body_table qualify."""
    b = 10 * k
    return ([G(b, C, time="3"), G(b + 2, body_table, time="2"), G(b + 4, "leaf", time="1")],
            [R(b + 1, C), R(b + 3, body_table)],
            [E(f"goal{b}", f"rule{b + 1}"), E(f"rule{b + 1}", f"goal{b + 2}"), E(f"goal{b + 2}", f"rule{b + 3}"),
             E(f"rule{b + 3}", f"goal{b + 4}")])


def fixtures():
    fx = {}
    # Q-HOLDS-EMPTY (A.1): the body goal of the pre rule has no rule child, so no
    # goal qualifies, the WITH yields no row and even the "pre" goal stays false.
    fx["q_holds_empty"] = {
        "runs": [(0, "success",
                  prov([G(0, "pre"), G(2, "log")], [R(1, "pre")], [E("goal0", "rule1"), E("rule1", "goal2")]),
                  prov(*cond_pattern("post")))],
        "check": lambda x: not any(x["holds"]["run_0_pre_" + i] for i in ("goal0", "goal2"))
        and x["holds"]["run_0_post_goal0"],
    }
    # Q-CLEAN-DEG (A.2): rules with in=0 or out=0 vanish from the clean copy; every goal stays.
    g, r, e = cond_pattern("pre")
    g += [G(20, "log"), G(22, "ack")]
    r += [R(21, "log"), R(23, "ack")]
    e += [E("rule21", "goal20"), E("goal22", "rule23")]  # rule21: in=0, rule23: out=0
    fx["q_clean_deg"] = {
        "runs": [(0, "success", prov(g, r, e), prov(*cond_pattern("post")))],
        "check": lambda x: "run_0_pre_rule21" not in x["clean"][0] and "run_0_pre_rule23" not in x["clean"][0]
        and "run_0_pre_goal20" in x["clean"][0] and "run_0_pre_goal22" in x["clean"][0],
    }
    # Q-CHAIN-BRANCH (A.3): P1 = r0 g1 r2 g3 r4, P2 = r5 g6 r7 g8 r9, P3 = r0 g1 r7 g8 r9.
    # Canonical order P1 < P3 < P2 accepts all three (3 collapsed rules).
    nx = lambda i: R(i, "log", "next")
    g = [G(1, "log"), G(3, "log"), G(6, "log"), G(8, "log"), G(10, "req"), G(11, "req"), G(12, "out"),
         G(13, "out")]
    r = [nx(0), nx(2), nx(4), nx(5), nx(7), nx(9)]
    e = [E("rule0", "goal1"), E("goal1", "rule2"), E("rule2", "goal3"), E("goal3", "rule4"),
         E("rule5", "goal6"), E("goal6", "rule7"), E("rule7", "goal8"), E("goal8", "rule9"),
         E("goal1", "rule7"), E("goal10", "rule0"), E("goal11", "rule5"), E("rule4", "goal12"),
         E("rule9", "goal13")]
    fx["q_chain_branch"] = {
        "runs": [(0, "success", prov(g, r, e), prov(*cond_pattern("post")))],
        "check": lambda x: [(c["head"], c["tail"]) for c in x["chains"]["run 0 pre"]] == [
            ("run_0_pre_rule0", "run_0_pre_rule4"), ("run_0_pre_rule0", "run_0_pre_rule9"),
            ("run_0_pre_rule5", "run_0_pre_rule9")],
    }
    # Q-PROTO-FIRST (A.5): the first success run has an empty list (its clean pre
    # graph has no holding goal), so inter and union are empty although run 1's is not.
    fx["q_proto_first"] = {
        "runs": [(0, "success", prov([G(0, "x")], [], []), prov(*cond_pattern("post"))),
                 (1, "success", prov(*cond_pattern("pre")), prov(*cond_pattern("post")))],
        "check": lambda x: x["inter"] == [] and x["union"] == [] and x["lists"]["1"] != [],
    }
    # Q-PROTO-POST (A.5): "post" is excluded from inter and union although every list holds it.
    fx["q_proto_post"] = {
        "runs": [(0, "success", prov(*cond_pattern("pre")), prov(*cond_pattern("post"))),
                 (1, "success", prov(*cond_pattern("pre")), prov(*cond_pattern("post")))],
        "check": lambda x: "post" in x["lists"]["0"] and "post" not in x["inter"] and "post" not in x["union"]
        and "log" in x["inter"],
    }
    # Q-DIFF-STALE (A.6): failed runs 1 and 2 miss different post goals; every diff
    # graph is computed with run 1's labels (###RUN### replaced in place on the first pass).
    good = prov([G(0, "post", "post(n, 3)", "3"), G(2, "log", "log(n, 2)", "2"), G(4, "ack", "ack(n, 1)", "1"),
                 G(6, "vote", "vote(n, 1)", "1")],
                [R(1, "post"), R(3, "log", "async"), R(5, "log")],
                [E("goal0", "rule1"), E("rule1", "goal2"), E("goal2", "rule3"), E("rule3", "goal4"),
                 E("goal2", "rule5"), E("rule5", "goal6")])
    f1 = prov([G(0, "post", "post(n, 3)", "3"), G(2, "log", "log(n, 2)", "2"), G(6, "vote", "vote(n, 1)", "1")],
              [R(1, "post"), R(5, "log")], [E("goal0", "rule1"), E("rule1", "goal2"), E("goal2", "rule5"),
                                           E("rule5", "goal6")])
    f2 = prov([G(0, "post", "post(n, 3)", "3"), G(2, "log", "log(n, 2)", "2"), G(4, "ack", "ack(n, 1)", "1")],
              [R(1, "post"), R(3, "log", "async")], [E("goal0", "rule1"), E("rule1", "goal2"), E("goal2", "rule3"),
                                                    E("rule3", "goal4")])
    pre = prov(*cond_pattern("pre"))
    fx["q_diff_stale"] = {
        "runs": [(0, "success", pre, good), (1, "failure", pre, f1), (2, "failure", pre, f2)],
        "check": lambda x: x["diff"][0] == x["diff"][1] == ["run_0_post_goal4"],
    }
    # Q-LEAF-REBIND (A.7): Missing.Goals = ALL D-children of the deepest
    # leaf-parent rules (leaf is rebound after WITH DISTINCT rule); a shallower
    # leaf-parent (rule3) is not reported.
    good = prov([G(0, "post", "post(n, 3)", "3"), G(2, "log", "log(n, 2)", "2"), G(4, "ack", "ack(n, 1)", "1"),
                 G(6, "vote", "vote(n, 1)", "1"), G(8, "commit", "commit(n, 1)", "1")],
                [R(1, "post"), R(3, "log"), R(7, "vote")],
                [E("goal0", "rule1"), E("rule1", "goal2"), E("goal2", "rule3"), E("rule3", "goal4"),
                 E("rule3", "goal6"), E("goal6", "rule7"), E("rule7", "goal8")])
    failed = prov([G(0, "post", "post(n, 3)", "3")], [], [])
    fx["q_leaf_rebind"] = {
        "runs": [(0, "success", pre, good), (1, "failure", pre, failed)],
        "check": lambda x: {"run_0_post_rule7": ["run_0_post_goal8"]} == {m["rule"]: m["goals"] for m in x["missing"][0]},
    }
    # Q-EXT-COUNT (A.9): 2 holding "pre" goals in run 0 and none in run 1 still give
    # count >= len(Runs): all achieved (goals are counted, not runs).
    two = prov([G(0, "pre", time="3"), G(1, "pre", time="4"), G(2, "log"), G(4, "leaf")],
               [R(5, "pre"), R(3, "log")],
               [E("goal0", "rule5"), E("goal1", "rule5"), E("rule5", "goal2"), E("goal2", "rule3"),
                E("rule3", "goal4")])
    fx["q_ext_count"] = {
        "runs": [(0, "success", two, prov(*cond_pattern("post"))),
                 (1, "success", prov([G(0, "x")], [], []), prov(*cond_pattern("post")))],
        "check": lambda x: x["all_pre"] is True,
    }
    # Q-TRIM-CUTSET (A.8): the receiver is strings.TrimLeft(label, table) — a cutset
    # trim — then Trim "()" and the first ", " field.  "abba(x, 1)" with table "ab"
    # gives "x" (a prefix trim would give "ba(x"); "ab((y), 2)" gives "y)".
    pre = prov([G(0, "pre", time="3"), G(2, "log", "log(srv, 2)", "2"), G(4, "ab", "abba(x, 1)"),
                G(6, "ab", "ab((y), 2)"), G(8, "leaf"), G(10, "leaf", "leaf(z, 0)")],
               [R(1, "pre"), R(3, "log"), R(5, "tick", "next"), R(7, "snd")],
               [E("goal0", "rule1"), E("rule1", "goal2"), E("goal2", "rule3"), E("rule3", "goal4"),
                E("rule3", "goal6"), E("goal4", "rule5"), E("rule5", "goal8"), E("goal6", "rule7"),
                E("rule7", "goal10")])
    pg, pr, pe = cond_pattern("post")
    pg[1] = G(2, "log", "log(srv, 2)", "2")
    pg += [G(6, "ack", "ack(n, 0)", "0")]
    pr += [R(5, "ack")]
    pe += [E("goal4", "rule5"), E("rule5", "goal6")]
    fx["q_trim_cutset"] = {
        "runs": [(0, "success", pre, prov(pg, pr, pe))],
        "check": lambda x: x["pre_rows"] and x["post_rows"] and all(
            any("<code>x</code> needs to know that <code>srv</code>" in s for s in out)
            and any("<code>y)</code> needs to know that <code>srv</code>" in s for s in out)
            and any("buffer_snd(y), ...)" in s for s in out) and not any("buffer_tick" in s for s in out)
            for out in x["corrections"]),
    }
    # Q-NS-1000: 1002 runs.  The reference's derived
    # graphs live at run 1000+i (clean copy, preprocessing.go:15) and 2000+f (diff
    # graph, differential-provenance.go:40), so run 0's clean copy lands on raw run
    # 1000 and extensions.go:27's `run < 1000` drops the raw runs >= 1000.  The build
    # keeps every derived graph in its own namespace: the expected values are the
    # literal evaluation with per-run namespaces, and the check shows (a) the
    # reference namespaces give a different answer here, (b) runs 1000/1001 get
    # exactly the results they get as runs 1/2 of a three-run corpus.
    pre = prov(*cond_pattern("pre"))
    good = prov([G(0, "post", "post(n, 3)", "3"), G(2, "log", "log(n, 2)", "2"), G(4, "ack", "ack(n, 1)", "1"),
                 G(6, "vote", "vote(n, 1)", "1"), G(8, "commit", "commit(n, 1)", "1")],
                [R(1, "post"), R(3, "log", "async"), R(7, "vote")],
                [E("goal0", "rule1"), E("rule1", "goal2"), E("goal2", "rule3"), E("rule3", "goal4"),
                 E("rule3", "goal6"), E("goal6", "rule7"), E("rule7", "goal8")])
    f1 = prov([G(0, "post", "post(n, 3)", "3"), G(2, "log", "log(n, 2)", "2"), G(4, "ack", "ack(n, 1)", "1")],
              [R(1, "post"), R(3, "log", "async")],
              [E("goal0", "rule1"), E("rule1", "goal2"), E("goal2", "rule3"), E("rule3", "goal4")])
    f2 = prov([G(0, "post", "post(n, 3)", "3")], [], [])
    ns_runs = [(0, "success", pre, good)] + [(i, "success", EMPTY, EMPTY) for i in range(1, 1000)] + \
              [(1000, "failure", pre, f1), (1001, "failure", pre, f2)]
    fx["q_ns_1000"] = {"runs": ns_runs, "ns": CL.PER_RUN, "digests": True, "check": _check_ns(ns_runs)}
    return fx


def _check_ns(runs):
    def strip(ids):
        return sorted("_".join(x.split("_")[2:]) for x in ids)

    def check(x):
        # the reference's own namespaces: cleanCopyProv of run 1000 also copies run 0's clean copy (run 1000)
        ref = CL.run_reference_pipeline([(it, st, _molly_prefix(pre, it, "pre"), _molly_prefix(post, it, "post"))
                                         for it, st, pre, post in runs])
        raw1000 = set(ref["raw"][(1000, "post")].values())
        differs = any(n not in raw1000 for n in ref["clean"][(1000, "post")])
        small = expected([runs[0], (1,) + runs[1000][1:], (2,) + runs[1001][1:]], digests=True, ns=CL.PER_RUN)
        same = (x["diff"] == small["diff"] and x["missing"] == small["missing"] and x["inter"] == small["inter"]
                and strip(x["clean"][1000]) == strip(small["clean"][1]) and strip(x["clean"][1001]) ==
                strip(small["clean"][2]) and x["lists"]["0"] == small["lists"]["0"] and x["pre_rows"] ==
                small["pre_rows"] and x["post_rows"] == small["post_rows"])
        return differs and same and len(x["clean"]) == 1002
    return check


def expected(runs, digests=False, ns=CL.REFERENCE):
    pruns = [(it, st, _molly_prefix(pre, it, "pre"), _molly_prefix(post, it, "post")) for it, st, pre, post in runs]
    lit = CL.run_reference_pipeline(pruns, ns=ns)
    db = lit["db"]
    out = {"holds": {}, "clean": [], "deleted": [], "chains": {}, "lists": {}}
    for it, _, _, _ in runs:
        for cond in ("pre", "post"):
            for mid, nid in lit["raw"][(it, cond)].items():
                out["holds"][mid] = bool(lit["holds"][(it, cond)][mid])
    for it, _, _, _ in runs:
        kept, dele = [], []
        for cond in ("pre", "post"):
            cm = lit["clean"][(it, cond)]
            inv = {v: k for k, v in lit["raw"][(it, cond)].items()}
            kept += sorted(inv[n] for n in cm)
            dele += sorted(inv[n] for n, c in cm.items() if c not in db.nodes)
            out["chains"][f"run {it} {cond}"] = [
                {"k": c["k"], "head": db.prop(c["nid"], "id") and inv[_orig(cm, c["head"])],
                 "tail": inv[_orig(cm, c["tail"])], "len": c["len"], "id": db.prop(c["nid"], "id")}
                for c in lit["chains"][(it, cond)]]
        out["clean"].append(sorted(kept))
        out["deleted"].append(sorted(dele))
    for j, it in enumerate(lit["success"]):
        out["lists"][str(it)] = sorted(lit["lists"][j])
    out["inter"] = sorted(lit["inter"]) if lit["inter"] is not None else None
    out["union"] = sorted(lit["union"]) if lit["union"] is not None else None
    out["inter_miss"] = [sorted(x) for x in lit["inter_miss"]] if lit["inter_miss"] is not None else None
    out["union_miss"] = [sorted(x) for x in lit["union_miss"]] if lit["union_miss"] is not None else None
    out["diff"], out["missing"] = [], []
    for d in lit["diffs"]:
        inv0 = {v: k for k, v in lit["raw"][(0, "post")].items()}
        out["diff"].append(sorted(inv0[n] for n in d["nodes"]))
        out["missing"].append([{"rule": inv0[d["inv"][m["rule"]]], "goals": sorted(inv0[d["inv"][x]] for x in m["goals"])}
                               for m in d["missing"]])
    if (0, "pre") in lit["raw"]:
        invp = {v: k for k, v in lit["raw"][(0, "pre")].items()}
        invq = {v: k for k, v in lit["raw"][(0, "post")].items()}
        out["pre_rows"] = sorted([invp[a], invp[g], invp[r]] for a, g, r in lit["pre_trig"])
        out["post_rows"] = sorted([invq[g], invq[r]] for g, r in lit["post_trig"])
        out["async"] = sorted(invp[r] for r in lit["async_rules"])
    out["all_pre"] = lit["all_pre"]
    out.update(host_expected(lit, runs, digests))
    if ns is not CL.REFERENCE:
        out["namespaces"] = "per_run"
    return out


def _orig(cm, clean_nid):
    for raw, c in cm.items():
        if c == clean_nid:
            return raw
    raise KeyError(clean_nid)


def write(name, spec):
    d = os.path.join(HERE, name)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    runs_json = []
    for i, (it, st, pre, post) in enumerate(spec["runs"]):
        runs_json.append({"iteration": it, "status": st,
                          "failureSpec": {"eot": 4, "eff": 2, "maxCrashes": 0, "nodes": ["n"], "crashes": [],
                                          "omissions": []},
                          "model": {"tables": {"pre": [["n", "3"]], "post": [["n", "3"]]}}, "messages": []})
        ind = None if len(spec["runs"]) > 100 else 1
        with open(os.path.join(d, f"run_{i}_pre_provenance.json"), "w") as fh:
            json.dump(pre, fh, indent=ind)
        with open(os.path.join(d, f"run_{i}_post_provenance.json"), "w") as fh:
            json.dump(post, fh, indent=ind)
    with open(os.path.join(d, "runs.json"), "w") as fh:
        json.dump(runs_json, fh, indent=1 if len(spec["runs"]) <= 100 else None)
    exp = expected(spec["runs"], spec.get("digests", False), spec.get("ns", CL.REFERENCE))
    assert spec["check"](exp), f"{name}: hand-derived property does not hold: {json.dumps(exp)[:400]}"
    with open(os.path.join(d, "expected.json"), "w") as fh:
        json.dump(exp, fh, indent=1, sort_keys=True)
    return exp


if __name__ == "__main__":
    only = sys.argv[1:]
    for name, spec in fixtures().items():
        if only and name not in only:
            continue
        write(name, spec)
        print("wrote", name)
