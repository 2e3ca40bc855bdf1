"""TEST INFRASTRUCTURE ONLY: the host (Go) side of the reference's graphing
package, restated over the literal evaluator's property graph
(oracle/cypher_literal.py).  It is the checker for nemo_amd/graphing.py and
nemo_amd/dot.py; nothing in the product imports it.

Outputs are canonical, order-free views:
* a DOT graph = ({node name: attrs}, sorted [(src, dst, attrs)]) — gographviz's
  node set and edge multiset; its serialisation order is pinned separately by
  hand-written strings in tests/test_graphing.py;
* corrections = the set of outputs over every iteration order of the
  reference's Go maps (permutation-enumerated, bounded by `max_orders`).
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Sequence, Tuple

from .cypher_literal import DB

Canon = Tuple[Dict[str, Dict[str, str]], List[tuple]]


def _q(s) -> str:
    return f'"{s}"'


def node_attrs(db: DB, n: int, graph_type: str) -> Dict[str, str]:
    """diagrams.go:44-103 for one endpoint."""
    p = db.nodes[n].props
    a = {"label": _q(p["label"]), "style": _q("filled, solid"), "color": _q("black"), "fontcolor": _q("black"),
         "fillcolor": _q("white")}
    if p.get("type") == "async":
        a["style"], a["color"] = _q("filled, bold"), _q("lawngreen")
    elif p.get("type") == "next":
        a["fontcolor"] = _q("gold")
    if p.get("condition_holds") is True:
        if graph_type == "pre":
            a["color"] = a["fillcolor"] = _q("firebrick")
        elif graph_type == "post":
            a["color"] = a["fillcolor"] = _q("deepskyblue")
    a["shape"] = "rect" if db.nodes[n].label == "Rule" else "ellipse"
    return a


def q24_edges(db: DB, run: int, cond: str) -> List[Tuple[int, int]]:
    """MATCH path = ({run, condition})-[:DUETO*1]->({run, condition}) RETURN path
    (pre-post-prov.go:297-300, differential-provenance.go:151-154)."""
    return [(a, b) for a in db.match(None, run=run, condition=cond) for b in sorted(db.out[a])
            if db.is_(b, None, run=run, condition=cond)]


def create_dot(db: DB, edges: Sequence[Tuple[int, int]], graph_type: str) -> Canon:
    """createDOT (diagrams.go:15-130)."""
    nodes = {"graph": {"bgcolor": _q("transparent")}}
    out = []
    for a, b in edges:
        ia, ib = db.prop(a, "id"), db.prop(b, "id")
        nodes.setdefault(ia, {}).update(node_attrs(db, a, graph_type))
        nodes.setdefault(ib, {}).update(node_attrs(db, b, graph_type))
        out.append((ia, ib, {"color": _q("black")}))
    return nodes, out


def pull_pre_post(db: DB, iters: Sequence[int], ns=None) -> List[Dict[str, Canon]]:
    """PullPrePostProv (pre-post-prov.go:288-459); clean copies in `ns` (cypher_literal.Namespaces)."""
    clean = ns.clean if ns is not None else (lambda it: 1000 + it)
    res = []
    for it in iters:
        res.append({"pre": create_dot(db, q24_edges(db, it, "pre"), "pre"),
                    "post": create_dot(db, q24_edges(db, it, "post"), "post"),
                    "pre_clean": create_dot(db, q24_edges(db, clean(it), "pre"), "pre"),
                    "post_clean": create_dot(db, q24_edges(db, clean(it), "post"), "post")})
    return res


def missing_records(db: DB, d: dict) -> List[dict]:
    """fi.Missing records of one diff graph (differential-provenance.go:115-142)."""
    out = []
    for m in d["missing"]:
        r = db.nodes[m["rule"]].props
        goals = []
        for x in m["goals"]:
            gp = db.nodes[x].props
            goals.append({"id": gp["id"], "label": gp["label"], "table": gp["table"], "time": gp["time"],
                          "conditionHolds": bool(gp["condition_holds"])})
        out.append({"rule": {"id": r["id"], "label": r["label"], "table": r["table"], "type": r["type"]},
                    "goals": sorted(goals, key=lambda g: g["id"])})
    return sorted(out, key=lambda m: m["rule"]["id"])


def create_diff_dot(db: DB, d: dict, failed_run: int, success_post: Canon) -> Tuple[Canon, Canon]:
    """createDiffDot (diagrams.go:133-291) over the literal diff graph `d`."""
    diff_run = d["run"]
    missing = set()
    for m in d["missing"]:
        missing.add(db.prop(m["rule"], "id"))
        missing.update(db.prop(x, "id") for x in m["goals"])
    rn = lambda s: s.replace("run_0", f"run_{d['id_run']}")
    views = []
    for _ in range(2):
        nodes = {rn(k): dict(v, style=_q("invis")) for k, v in success_post[0].items()}
        edges = [[rn(a), rn(b), dict(at, style=_q("invis"))] for a, b, at in success_post[1]]
        views.append((nodes, edges))
    (dn, de), (fn, fe) = views
    for a, b in q24_edges(db, diff_run, "post"):
        ia, ib = db.prop(a, "id"), db.prop(b, "id")
        dn[ia]["style"] = dn[ib]["style"] = _q("filled, solid")
        for e in de:
            if e[0] == ia and e[1] == ib:
                e[2]["style"] = _q("filled, solid")
        for x in (ia, ib):
            if x in missing:
                dn[x]["style"], dn[x]["color"] = _q("filled, dashed, bold"), _q("mediumvioletred")
    for a, b in q24_edges(db, failed_run, "post"):
        la, lb = _q(db.prop(a, "label")), _q(db.prop(b, "label"))
        for attrs in fn.values():
            if attrs.get("label") in (la, lb):
                attrs["style"] = _q("filled, solid")
    for e in fe:
        if fn[e[0]].get("style") == _q("filled, solid") and fn[e[1]].get("style") == _q("filled, solid"):
            e[2]["style"] = _q("filled, solid")
    return (dn, [tuple(e) for e in de]), (fn, [tuple(e) for e in fe])


def canon(c: Canon) -> Tuple[dict, list]:
    """Order-free form: node dict + sorted edge list with sorted attribute items."""
    nodes, edges = c
    return ({k: dict(sorted(v.items())) for k, v in nodes.items()},
            sorted((a, b, tuple(sorted(at.items()))) for a, b, at in edges))


# ---- corrections.go ----------------------------------------------------------------
def _receiver(label: str, table: str) -> str:
    # strings.TrimLeft is a cutset trim; then Trim "()" and Split ", " (corrections.go:65-67)
    i = 0
    cut = set(table)
    while i < len(label) and label[i] in cut:
        i += 1
    s = label[i:]
    a, b = 0, len(s)
    while a < b and s[a] in "()":
        a += 1
    while b > a and s[b - 1] in "()":
        b -= 1
    return s[a:b].split(", ")[0]


def _synth(pre: List[dict], post: List[dict], inner_order) -> List[str]:
    """corrections.go:219-324 for one map-iteration order."""
    recs, pre_rules, diff = [], {}, {}
    for row in pre:
        diff[row["agg_table"]] = {}
        t = row["agg_table"]
        if not pre_rules.get(t):
            pre_rules[t] = f"{t}({row['recv']}, ...) :- {row['rule_table']}({row['recv']}, ...)"
        else:
            pre_rules[t] += f", {row['rule_table']}({row['recv']}, ...)"
    for row in pre:
        t = row["agg_table"]
        for pg in post:
            if row["recv"] != pg["recv"]:
                diff[t].setdefault(row["recv"], []).append(pg)
        new = pre_rules[t]
        if len(diff[t]) == 0:
            for pg in post:
                new += f", {pg['table']}({pg['recv']}, ...)"
        else:
            for pre_node in inner_order(list(diff[t])):
                for pg in diff[t][pre_node]:
                    recs.append(f"<code>{pre_node}</code> needs to know that <code>{pg['recv']}</code> has executed "
                                f"<code>{pg['table']}</code>. Add:<br /> &nbsp; &nbsp; &nbsp; &nbsp; <code>ack_"
                                f"{pg['table']}({pre_node}, ...)@async :- {pg['table']}({pg['recv']}, ...), ...;</code>")
                    new += f", ack_{pg['table']}({pre_node}, sender={pg['recv']}, ...)"
            if row["rule_type"] != "next":
                ru, nd = row["rule_table"], row["recv"]
                recs.append("Antecedent depends on timing of an onetime event. Make it persistent. Add:<br /> &nbsp; "
                            f"&nbsp; &nbsp; &nbsp; <code>buffer_{ru}({nd}, ...) :- {ru}({nd}, ...), ...;</code><br /> "
                            f"&nbsp; &nbsp; &nbsp; &nbsp; <code>buffer_{ru}({nd}, ...)@next :- buffer_{ru}({nd}, ...), "
                            "...;")
                new = new.replace(f"{ru}({nd}, ...)", f"buffer_{ru}({nd}, ...)")
        recs.append(f"Change: <code>{pre_rules[t]};</code> &nbsp; <i class = \"fas fa-long-arrow-alt-right\"></i> "
                    f"&nbsp; <code>{new};</code>")
    return recs


def trigger_rows(db: DB, pre_trig, post_trig) -> Tuple[List[dict], List[dict]]:
    pre = []
    for a, g, r in pre_trig:
        gp = db.nodes[g].props
        pre.append({"agg_table": db.prop(a, "table"), "recv": _receiver(gp["label"], gp["table"]),
                    "rule_table": db.prop(r, "table"), "rule_type": db.prop(r, "type"),
                    "key": (db.prop(a, "id"), gp["id"], db.prop(r, "id"))})
    post = []
    for g, r in post_trig:
        gp = db.nodes[g].props
        post.append({"table": gp["table"], "recv": _receiver(gp["label"], gp["table"]),
                     "key": (gp["id"], db.prop(r, "id"))})
    return pre, post


def corrections_admissible(db: DB, pre_trig, post_trig, max_orders: int = 20000) -> Optional[set]:
    """Every output GenerateCorrections can produce over the iteration orders of
    its maps (rows of preTriggers / postTriggers, the receivers of
    differentNodes[table]); None if there are more than `max_orders` orders."""
    pre, post = trigger_rows(db, pre_trig, post_trig)
    n_orders = 1
    for k in (len(pre), len(post)):
        for i in range(2, k + 1):
            n_orders *= i
    recvs = sorted({r["recv"] for r in pre})
    inner = list(itertools.permutations(recvs)) if len(recvs) <= 4 else [tuple(recvs)]
    if n_orders * len(inner) > max_orders:
        return None
    out = set()
    for pp in itertools.permutations(pre):
        for qq in itertools.permutations(post):
            for io in inner:
                rank = {r: i for i, r in enumerate(io)}
                out.add(tuple(_synth(list(pp), list(qq), lambda ks: sorted(ks, key=lambda k: rank[k]))))
    return out


def extensions(db: DB, async_rules) -> List[str]:
    """extensions.go:76-90 as a sorted set."""
    return sorted({f"<code>{db.prop(r, 'table')}(node, ...)@async :- ...;</code>" for r in async_rules})
