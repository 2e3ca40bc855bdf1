"""TEST INFRASTRUCTURE ONLY: a literal evaluator of the reference's Cypher.

Each function below re-executes one statement the reference sends to Neo4j
(graphing/*.go) the way Cypher defines it — by enumerating the matching
paths over a tiny in-memory property graph — plus the Go post-processing
around it.  It is exponential in graph size and meant for graphs of a few
dozen nodes: it pins the O(V+E) closed forms in oracle/nemo_oracle.c, which in
turn check the HIP kernels.  Parity against Neo4j itself remains UNPINNED
(no reference outputs exist).

Cypher semantics used (Neo4j 3.3): variable-length patterns match paths with
relationship isomorphism (no relationship repeated in one path); `[*0..]`
includes the zero-length path; WITH/aggregation over zero rows yields zero
rows unless the aggregate has no grouping key; ORDER BY ties are unspecified
(resolved here by `tie_key`, default: the lexicographic sequence of node IDs).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, Dict, List, Optional, Sequence, Tuple


class Node:
    __slots__ = ("nid", "label", "props")

    def __init__(self, nid: int, label: str, props: dict):
        self.nid = nid
        self.label = label
        self.props = props


class DB:
    """Minimal property graph with Neo4j-style internal IDs."""

    def __init__(self) -> None:
        self.nodes: Dict[int, Node] = {}
        self.out: Dict[int, set] = defaultdict(set)
        self.inn: Dict[int, set] = defaultdict(set)
        self._next = 0

    def create(self, label: str, props: dict) -> int:
        nid = self._next
        self._next += 1
        self.nodes[nid] = Node(nid, label, dict(props))
        return nid

    def merge(self, a: int, b: int) -> int:
        if b in self.out[a]:
            return 0
        self.out[a].add(b)
        self.inn[b].add(a)
        return 1

    def detach_delete(self, nid: int) -> None:
        for b in list(self.out[nid]):
            self.inn[b].discard(nid)
        for a in list(self.inn[nid]):
            self.out[a].discard(nid)
        self.out.pop(nid, None)
        self.inn.pop(nid, None)
        self.nodes.pop(nid, None)

    def match(self, label: Optional[str] = None, **props) -> List[int]:
        res = []
        for nid, n in self.nodes.items():
            if label is not None and n.label != label:
                continue
            if all(n.props.get(k) == v for k, v in props.items()):
                res.append(nid)
        return sorted(res)

    def is_(self, nid: int, label: Optional[str] = None, **props) -> bool:
        n = self.nodes.get(nid)
        if n is None or (label is not None and n.label != label):
            return False
        return all(n.props.get(k) == v for k, v in props.items())

    def paths_from(self, start: int, lo: int, hi: Optional[int] = None,
                   ok: Callable[[int], bool] = lambda n: True) -> List[List[int]]:
        """All paths start-[*lo..hi]->x (relationship-unique; node predicate on every node)."""
        res: List[List[int]] = []
        if not ok(start):
            return res

        def rec(path: List[int], used: set) -> None:
            if len(path) - 1 >= lo:
                res.append(list(path))
            if hi is not None and len(path) - 1 >= hi:
                return
            for b in sorted(self.out[path[-1]]):
                rel = (path[-1], b)
                if rel in used or not ok(b):
                    continue
                used.add(rel)
                path.append(b)
                rec(path, used)
                path.pop()
                used.discard(rel)

        rec([start], set())
        return res

    def prop(self, nid: int, k: str, default=None):
        return self.nodes[nid].props.get(k, default)


def load(db: DB, iteration: int, cond: str, prov: dict) -> Dict[str, int]:
    """loadProv (graphing/pre-post-prov.go:25-213) with Molly-prefixed prov."""
    ids: Dict[Tuple[str, str], int] = {}
    for g in prov["goals"]:
        ids[("Goal", g["id"])] = db.create("Goal", {"id": g["id"], "run": iteration, "condition": cond,
                                                     "label": g["label"], "table": g["table"],
                                                     "time": g.get("time", ""), "condition_holds": False})
    for r in prov["rules"]:
        ids[("Rule", r["id"])] = db.create("Rule", {"id": r["id"], "run": iteration, "condition": cond,
                                                     "label": r["label"], "table": r["table"],
                                                     "type": r.get("type", "")})
    created = 0
    for e in prov["edges"]:
        if "goal" in e["from"]:
            a, b = ids.get(("Goal", e["from"])), ids.get(("Rule", e["to"]))
        else:
            a, b = ids.get(("Rule", e["from"])), ids.get(("Goal", e["to"]))
        if a is not None and b is not None:
            created += db.merge(a, b)
    if created != len(prov["edges"]):
        raise RuntimeError(f"Run {iteration}: inserted number of edges ({created}) does not equal number "
                           f"of antecedent provenance edges ({len(prov['edges'])})")
    return {k[1]: v for k, v in ids.items()}


def mark_condition_holds(db: DB, run: int, C: str) -> None:
    """pre-post-prov.go:220-228, literally."""
    rows = []
    for g in db.match("Goal", run=run, condition=C):
        for r in sorted(db.out[g]):
            if not db.is_(r, "Rule", run=run, condition=C):
                continue
            pos = any(db.is_(t, "Goal", run=run, condition=C, table=C) and db.is_(rc, "Rule", run=run, condition=C, table=C)
                      for rc in db.inn[g] for t in db.inn[rc])
            neg = any(db.is_(t, "Goal", run=run, condition=C, table=C) and db.is_(rc, "Rule", run=run, condition=C, table=C)
                      and len(db.inn[t]) > 0 for rc in db.inn[g] for t in db.inn[rc])
            if pos and not neg:
                rows.append(db.prop(g, "table"))
    for rule in rows:
        for n in db.match("Goal", run=run, condition=C):
            if db.prop(n, "table") == C or db.prop(n, "table") == rule:
                db.nodes[n].props["condition_holds"] = True


class Namespaces:
    """The `run` property values of the derived graphs and the numbers their IDs are printed with.

    REFERENCE is the reference verbatim: the clean copy of run i is run 1000+i
    (preprocessing.go:15,33,45), the diff graph of failed run f is run 2000+f
    (differential-provenance.go:40) and the raw runs are those with run < 1000
    (extensions.go:27); with >= 1000 runs these collide.
    PER_RUN keeps every derived graph in a namespace of its own (the `run`
    property is a (kind, iteration) pair) while IDs are still printed as
    run_<1000+i> / run_<2000+f>: the semantics libnemohip implements."""

    def __init__(self, tagged: bool):
        self.tagged = tagged

    def clean(self, it: int):
        return ("clean", it) if self.tagged else 1000 + it

    def diff(self, f: int):
        return ("diff", f) if self.tagged else 2000 + f

    def is_raw(self, run) -> bool:
        return isinstance(run, int) if self.tagged else run < 1000


REFERENCE = Namespaces(False)
PER_RUN = Namespaces(True)


def _rewrite_id(s: str, old: int, new: int) -> str:
    pfx = f"run_{old}"
    return f"run_{new}" + s[len(pfx):] if s.startswith(pfx) else s


def clean_copy_prov(db: DB, it: int, C: str, ns: Namespaces = REFERENCE) -> Dict[int, int]:
    """preprocessing.go:13-63: export every (g1:Goal)-[*0..]->(g2:Goal) path, sed run/id, re-import."""
    nodes, rels = set(), set()
    for g1 in db.match("Goal", run=it, condition=C):
        for p in db.paths_from(g1, 0):
            if db.is_(p[-1], "Goal", run=it, condition=C):
                nodes.update(p)
                rels.update(zip(p, p[1:]))
    copy: Dict[int, int] = {}
    for n in sorted(nodes):
        props = dict(db.nodes[n].props)
        props["run"] = ns.clean(it)
        props["id"] = _rewrite_id(props["id"], it, 1000 + it)
        copy[n] = db.create(db.nodes[n].label, props)
    for a, b in sorted(rels):
        db.merge(copy[a], copy[b])
    return copy


def collapse_next_chains(db: DB, it: int, C: str,
                         tie_key: Optional[Callable[[List[int]], object]] = None,
                         ns: Namespaces = REFERENCE) -> List[dict]:
    """preprocessing.go:66-348, literally (tie order of ORDER BY len DESC via tie_key)."""
    run = ns.clean(it)
    okn = lambda n: db.nodes[n].props.get("type") == "next" or "type" not in db.nodes[n].props
    groups: Dict[Tuple[int, ...], List[int]] = {}
    for r1 in db.match("Rule", run=run, condition=C, type="next"):
        for p in db.paths_from(r1, 2, ok=okn):
            if not db.is_(p[-1], "Rule", run=run, condition=C, type="next"):
                continue
            for i in range(1, len(p) - 1):  # one row per binding of (g:Goal)
                if db.is_(p[i], "Goal", run=run, condition=C):
                    groups.setdefault(tuple(p), []).extend(p)  # UNWIND + collect grouped by path
    if tie_key is None:
        tie_key = lambda p: [db.prop(n, "id") for n in p]
    rows = sorted(groups.items(), key=lambda kv: tie_key(list(kv[0])))
    rows.sort(key=lambda kv: -(len(kv[0]) - 1))  # stable: ORDER BY len DESC
    chains, seen = [], set()
    for path, ids in rows:
        if any(n not in seen for n in ids):
            chains.append(list(path))
            seen.update(ids)
    preds = [sorted(a for a in db.inn[ch[0]] if db.is_(a, "Goal", run=run, condition=C)) for ch in chains]
    succs = [sorted(b for b in db.out[ch[-1]] if db.is_(b, "Goal", run=run, condition=C)) for ch in chains]
    created = []
    for i, ch in enumerate(chains):
        table = db.prop(ch[0], "table")
        label = f"{table}_collapsed"
        cid = f"run_{1000 + it}_{C}_{label}_{i}"
        c = db.create("Rule", {"run": run, "condition": C, "id": cid, "label": label, "table": table,
                               "type": "collapsed"})
        if not preds[i] or not succs[i]:
            raise RuntimeError("Cypher syntax error: ID(pred) IN ] (preprocessing.go:254-263)")
        for p in preds[i]:
            for s in succs[i]:
                db.merge(p, c)
                db.merge(c, s)
        created.append({"nid": c, "k": i, "head": ch[0], "tail": ch[-1], "len": len(ch) - 1,
                        "preds": preds[i], "succs": succs[i], "path": ch})
    dele = set()
    for r in db.match("Rule", run=run, condition=C, type="next"):
        if r not in seen:
            continue
        for p in db.paths_from(r, 2, ok=lambda n: n in seen):
            if db.is_(p[-1], "Rule", run=run, condition=C, type="next") and any(
                    db.is_(x, "Goal", run=run, condition=C) for x in p[1:-1]):
                dele.update(p)
    for n in dele:
        db.detach_delete(n)
    return created


def extract_protos_lists(db: DB, iters: Sequence[int], C: str, ns: Namespaces = REFERENCE) -> List[List[str]]:
    """prototype.go:11-76: per success run, the list of distinct rule tables."""
    lists = []
    for it in iters:
        run = ns.clean(it)
        gate = len(db.match("Goal", run=run, condition="pre", condition_holds=True)) > 0
        paths = []
        for root in db.match("Goal", run=run, condition=C):
            if db.inn[root]:
                continue
            for r1 in sorted(db.out[root]):
                if not db.is_(r1, "Rule", run=run, condition=C):
                    continue
                for p in db.paths_from(r1, 1):
                    if db.is_(p[-1], "Rule", run=run, condition=C):
                        paths.append([root] + p)
        out: List[str] = []
        if gate:
            paths.sort(key=lambda p: -(len(p) - 1))
            for p in paths:
                for n in p:
                    if "type" in db.nodes[n].props:
                        t = db.prop(n, "table")
                        if t not in out:
                            out.append(t)
        lists.append(out)
    return lists


def protos_from_lists(iter_prov: List[List[str]], condition: str) -> Tuple[List[str], List[str]]:
    """prototype.go:79-130, the Go loops verbatim (index out of range if no success run)."""
    achvd = sum(1 for x in iter_prov if len(x) > 0)
    inter, union = [], []
    longest = len(iter_prov[0])
    for i in range(len(iter_prov[0])):
        found = 1
        for j in range(1, len(iter_prov)):
            if len(iter_prov[j]) > 0:
                for k in range(len(iter_prov[j])):
                    if iter_prov[0][i] == iter_prov[j][k]:
                        found += 1
            if len(iter_prov[j]) > longest:
                longest = len(iter_prov[j])
        if found == achvd and iter_prov[0][i] != condition:
            inter.append(iter_prov[0][i])
    seen = set()
    for i in range(longest):
        for j in range(len(iter_prov)):
            if i < len(iter_prov[j]):
                if iter_prov[j][i] not in seen and iter_prov[j][i] != condition:
                    union.append(iter_prov[j][i])
                    seen.add(iter_prov[j][i])
    return inter, union


def missing_from(db: DB, proto: List[str], failed_iter: int, C: str, ns: Namespaces = REFERENCE) -> List[str]:
    """prototype.go:141-206."""
    tabs = {db.prop(r, "table") for r in db.match("Rule", run=ns.clean(failed_iter), condition=C)}
    return [f"<code>{p}</code>" for p in proto if p not in tabs]


def naive_diff_prov(db: DB, failed_runs: Sequence[int], ns: Namespaces = REFERENCE) -> List[dict]:
    """differential-provenance.go:18-146, including the in-place ###RUN### substitution (:43)."""
    res = []
    source = failed_runs[0] if failed_runs else None  # stale substitution: every export uses failedRuns[0]
    for f in failed_runs:
        diff_run = ns.diff(f)
        fail_goals = [db.prop(n, "label") for n in db.match("Goal", run=source, condition="post")]
        nodes, rels = set(), set()
        for root in db.match("Goal", run=0, condition="post"):
            if db.prop(root, "label") in fail_goals:
                continue
            for p in db.paths_from(root, 0):
                if db.is_(p[-1], "Goal", run=0, condition="post") and db.prop(p[-1], "label") not in fail_goals:
                    nodes.update(p)
                    rels.update(zip(p, p[1:]))
        copy = {}
        for n in sorted(nodes):
            props = dict(db.nodes[n].props)
            props["run"] = diff_run
            props["id"] = _rewrite_id(props["id"], 0, 2000 + f)
            copy[n] = db.create(db.nodes[n].label, props)
        for a, b in sorted(rels):
            db.merge(copy[a], copy[b])
        # leaves query (:82-98)
        rows = []
        for root in db.match("Goal", run=diff_run, condition="post"):
            if db.inn[root]:
                continue
            for p in db.paths_from(root, 0):
                rule = p[-1]
                if not db.is_(rule, "Rule", run=diff_run, condition="post"):
                    continue
                for leaf in sorted(db.out[rule]):
                    if db.is_(leaf, "Goal", run=diff_run, condition="post") and not db.out[leaf]:
                        rows.append((len(p), rule))
        missing = []
        if rows:
            max_len = max(r[0] for r in rows)
            rules = sorted({r for (ln, r) in rows if ln == max_len})
            for r in rules:
                leaves = sorted(x for x in db.out[r] if db.is_(x, "Goal", run=diff_run, condition="post"))
                missing.append({"rule": r, "goals": leaves})
        inv = {v: k for k, v in copy.items()}
        res.append({"run": diff_run, "id_run": 2000 + f, "nodes": set(nodes), "copy": copy, "inv": inv, "missing": missing,
                    "edges": {(a, b) for a in copy.values() for b in db.out[a]}})
    return res


def find_pre_triggers(db: DB, run: int) -> List[Tuple[int, int, int]]:
    """corrections.go:30-34."""
    rows = []
    for a in db.match("Rule", run=run, condition="pre"):
        for g in sorted(db.out[a]):
            if not db.is_(g, "Goal", run=run, condition="pre", condition_holds=False):
                continue
            for r in sorted(db.out[g]):
                if not db.is_(r, "Rule", run=run, condition="pre"):
                    continue
                if any(db.is_(h, "Goal", run=run, condition="pre", condition_holds=True) for h in db.inn[a]):
                    rows.append((a, g, r))
    return rows


def find_post_triggers(db: DB, run: int) -> List[Tuple[int, int]]:
    """corrections.go:121-125."""
    rows = []
    for g in db.match("Goal", run=run, condition="post", condition_holds=True):
        for r in sorted(db.out[g]):
            if not db.is_(r, "Rule", run=run, condition="post"):
                continue
            left = any(db.is_(x, "Rule", run=run, condition="post") for x in db.inn[g])
            right = any(db.is_(x, "Goal", run=run, condition="post", condition_holds=False)
                        and any(db.is_(y, "Rule", run=run, condition="post") for y in db.out[x]) for x in db.out[r])
            if left and right:
                rows.append((g, r))
    return rows


def extensions(db: DB, n_runs: int, ns: Namespaces = REFERENCE) -> Tuple[bool, List[int]]:
    """extensions.go:25-90 (rule list only; strings are built by the host)."""
    pres = [n for n in db.match("Goal", condition="pre", table="pre", condition_holds=True)
            if ns.is_raw(db.prop(n, "run"))]
    all_achieved = not (len(pres) < n_runs)
    rules = []
    for r in db.match("Rule", run=0, condition="pre", type="async"):
        a = any(db.is_(h, "Goal", run=0, condition="pre", condition_holds=True) for h in db.inn[r]) and any(
            db.is_(x, "Goal", run=0, condition="pre", condition_holds=False)
            and any(db.is_(y, "Rule", run=0, condition="pre") for y in db.out[x]) for x in db.out[r])
        b = any(db.is_(h, "Goal", run=0, condition="pre", condition_holds=False) for h in db.inn[r])
        if a or b:
            rules.append(r)
    return all_achieved, rules


def run_reference_pipeline(runs: Sequence[Tuple[int, str, dict, dict]], tie_key=None,
                           ns: Namespaces = REFERENCE) -> dict:
    """main.go:106-177's call order over the literal evaluator.

    `runs`: [(iteration, status, pre_prov, post_prov)] with Molly-prefixed IDs.
    `ns`: the derived graphs' namespaces (REFERENCE, or PER_RUN for >= 1000 runs)."""
    db = DB()
    raw: Dict[Tuple[int, str], Dict[str, int]] = {}
    for it, _, pre, post in runs:
        raw[(it, "pre")] = load(db, it, "pre", pre)
        mark_condition_holds(db, it, "pre")
        raw[(it, "post")] = load(db, it, "post", post)
        mark_condition_holds(db, it, "post")
    holds = {k: {i: db.prop(n, "condition_holds") for i, n in v.items()} for k, v in raw.items()}
    clean, chains = {}, {}
    for it, _, _, _ in runs:
        clean[(it, "pre")] = clean_copy_prov(db, it, "pre", ns)
        clean[(it, "post")] = clean_copy_prov(db, it, "post", ns)
        chains[(it, "pre")] = collapse_next_chains(db, it, "pre", tie_key, ns)
        chains[(it, "post")] = collapse_next_chains(db, it, "post", tie_key, ns)
    success = [it for it, st, _, _ in runs if st == "success"]
    failed = [it for it, st, _, _ in runs if st != "success"]
    lists = extract_protos_lists(db, success, "post", ns)
    inter, union = protos_from_lists(lists, "post") if success else (None, None)
    inter_miss = [missing_from(db, inter, f, "post", ns) for f in failed] if success else None
    union_miss = [missing_from(db, union, f, "post", ns) for f in failed] if success else None
    diffs = naive_diff_prov(db, failed, ns)
    pre_trig = find_pre_triggers(db, 0)
    post_trig = find_post_triggers(db, 0)
    all_pre, async_rules = extensions(db, len(runs), ns)
    return {"db": db, "ns": ns, "raw": raw, "holds": holds, "clean": clean, "chains": chains, "lists": lists,
            "success": success, "failed": failed, "inter": inter, "union": union, "inter_miss": inter_miss,
            "union_miss": union_miss, "diffs": diffs, "pre_trig": pre_trig, "post_trig": post_trig,
            "all_pre": all_pre, "async_rules": async_rules}
