"""Lineage-driven exploration of the failure space and Molly-format output.

Molly (the fault injector behind faultinjectors/molly.go) starts from the
failure-free run, reads the lineage of the good outcome (the `post` tuples at
EOT) and injects the smallest fault sets that break every derivation of one of
them; runs that still succeed add their own lineage, and the search goes on.
This module restates that loop over `dedalus.evaluate`:

* a clock goal clock(f, d, t, t+1) with f != d and t < EFF can be omitted; a
  node n with a clock goal at time t can be crashed at t (at most `crashes`
  distinct nodes);
* the support of a goal is the set of minimal fault-event sets that appear in
  one of its derivation trees (a DNF, capped);
* candidates are the minimal hitting sets of one post tuple's support, added to
  the current run's faults; every distinct fault set runs once, breadth first,
  up to `max_runs`.

Output (faultinjectors/data-types.go:43-98, molly.go:18,59-60, hazard-analysis.go:25):
runs.json, run_<i>_{pre,post}_provenance.json (goal/rule/edge lists, IDs
`goal<N>`/`rule<N>`, labels `table(v1, v2, ...)`, clock labels
`clock(f, d, t, t+1)` / `clock(n, n, t, __WILDCARD__)`) and
run_<iteration>_spacetime.dot.
"""
from __future__ import annotations

import json
import os
from collections import deque
from typing import Dict, FrozenSet, List, Optional, Sequence, Set, Tuple

from .dedalus import WILD, FailureSpec, Key, Program, Run, evaluate, goals_of, label, reachable

Event = Tuple[str, object, object, int]  # ("omit", from, to, t) | ("crash", node, None, t)


def _events(key: Key, spec: FailureSpec) -> List[FrozenSet[Event]]:
    """Fault alternatives that remove one clock goal: any one of them suffices."""
    tab, tup, _ = key
    if tab != "clock":
        return []
    f, d, t, r = tup
    alts = []
    if r != WILD and f != d and t < spec.eff:
        alts.append(frozenset([("omit", f, d, t)]))
    alts.append(frozenset([("crash", f, None, t)]))
    if r != WILD and d != f:
        alts.append(frozenset([("crash", d, None, t + 1)]))
    return alts


def supports(run: Run, root: Key, cap: int = 128, max_term: int = 96) -> List[FrozenSet[Key]]:
    """Minimal sets of clock goals that some derivation tree of `root` needs (DNF)."""
    memo: Dict[Key, List[FrozenSet[Key]]] = {}
    order: List[Key] = []  # post-order: body goals before their heads
    seen: Set[Key] = {root}
    stack = [(root, iter([b for d in run.derivs.get(root, []) for b in d.body]))]
    while stack:
        k, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            stack.pop()
            order.append(k)
        elif nxt not in seen:
            seen.add(nxt)
            stack.append((nxt, iter([b for d in run.derivs.get(nxt, []) for b in d.body])))
    for k in order:
        if k[0] == "clock":
            memo[k] = [frozenset([k])]
            continue
        ds = run.derivs.get(k, [])
        if not ds:
            memo[k] = [frozenset()]
            continue
        terms: Set[FrozenSet[Key]] = set()
        for d in ds:
            acc = [frozenset()]
            for b in d.body:
                sub = memo.get(b, [frozenset()])
                acc = list({a | s for a in acc for s in sub if len(a | s) <= max_term})[:cap]
                if not acc:
                    break
            terms.update(acc)
        mins = sorted(terms, key=len)
        keep: List[FrozenSet[Key]] = []
        for s in mins:
            if not any(k2 <= s for k2 in keep):
                keep.append(s)
            if len(keep) >= cap:
                break
        memo[k] = keep
    return memo[root]


def hitting_sets(terms: List[FrozenSet[Key]], spec: FailureSpec, limit: int = 64,
                 max_faults: int = 4) -> List[FrozenSet[Event]]:
    """Minimal fault sets that remove at least one clock goal of every term."""
    out: List[FrozenSet[Event]] = []

    def crashes_ok(fs):
        nodes = {e[1] for e in fs if e[0] == "crash"} | set(spec.crashes)
        return len(nodes) <= spec.max_crashes

    def kills(fs, key):
        f, d, t, r = key[1]
        for e in fs:
            if e[0] == "omit" and (e[1], e[2], e[3]) == (f, d, t):
                return True
            if e[0] == "crash" and ((e[1] == f and t >= e[3]) or (r != WILD and e[1] == d and t + 1 >= e[3])):
                return True
        return False

    def rec(fs: FrozenSet[Event]):
        if len(out) >= limit:
            return
        for term in terms:
            if not any(kills(fs, k) for k in term):
                break
        else:
            if not any(o <= fs for o in out):
                out.append(fs)
            return
        if len(fs) >= max_faults:
            return
        for k in sorted(term, key=repr):
            for alt in _events(k, spec):
                nf = fs | alt
                if crashes_ok(nf):
                    rec(nf)

    rec(frozenset())
    return out


def apply(spec: FailureSpec, faults: FrozenSet[Event]) -> FailureSpec:
    crashes = dict(spec.crashes)
    omissions = set(spec.omissions)
    for e in faults:
        if e[0] == "omit":
            omissions.add((e[1], e[2], e[3]))
        else:
            crashes[e[1]] = min(crashes.get(e[1], e[3]), e[3])
    return FailureSpec(spec.eot, spec.eff, spec.max_crashes, spec.nodes, crashes, frozenset(omissions))


def explore(prog: Program, eot: int, eff: int, crashes: int, nodes: Sequence[str], max_runs: int = 32) -> List[Run]:
    """The LDFI loop: failure-free run first, then breadth-first fault injection."""
    base = FailureSpec(eot, eff, crashes, list(nodes))
    queue = deque([base])
    seen = {base.key()}
    runs: List[Run] = []
    while queue and len(runs) < max_runs:
        spec = queue.popleft()
        run = evaluate(prog, spec)
        runs.append(run)
        if not run.success:
            continue
        for root in [k for k in goals_of(run, "post") if k[2] == eot]:
            for hs in hitting_sets(supports(run, root), spec):
                nxt = apply(spec, hs)
                if nxt.key() not in seen:
                    seen.add(nxt.key())
                    queue.append(nxt)
    return runs


# ---- Molly-format output ------------------------------------------------------------
def provenance(run: Run, table: str) -> dict:
    """ProvData (data-types.go:67-72) of every `table` tuple of the run."""
    goals, rules = reachable(run, goals_of(run, table))
    gid = {k: f"goal{i}" for i, k in enumerate(goals)}
    out = {"goals": [], "rules": [], "edges": []}
    for k in goals:
        out["goals"].append({"id": gid[k], "label": label(k), "table": k[0], "time": str(k[2])})
    for i, (head, d) in enumerate(rules):
        rid = f"rule{i}"
        typ = d.rule.kind or "single"
        out["rules"].append({"id": rid, "label": d.rule.head.table, "table": d.rule.head.table, "type": typ})
        out["edges"].append({"from": gid[head], "to": rid})
        for b in dict.fromkeys(d.body):
            out["edges"].append({"from": rid, "to": gid[b]})
    return out


def spacetime_dot(run: Run) -> str:
    """A space-time diagram whose node names end in _<time> (hazard-analysis.go:48-54)."""
    spec = run.spec
    lines = ["digraph spacetime {", "\trankdir=TB;", "\tnode [shape=point];"]
    for n in spec.nodes:
        lines.append(f'\tsubgraph cluster_{n} {{ label="{n}";')
        for t in range(1, spec.eot + 1):
            lab = f"{n}@{t}" + (" (crashed)" if not spec.alive(n, t) else "")
            lines.append(f'\t\t{n}_{t} [xlabel="{lab}"];')
        lines.append("\t}")
    for n in spec.nodes:
        for t in range(1, spec.eot):
            style = "solid" if spec.alive(n, t) else "dotted"
            lines.append(f"\t{n}_{t} -> {n}_{t + 1} [style={style}, arrowhead=none];")
    for tab, f, d, s, r in run.messages:
        if f != d and f in spec.nodes and d in spec.nodes:
            lines.append(f'\t{f}_{s} -> {d}_{r} [label="{tab}"];')
    for (f, d, s) in sorted(spec.omissions):
        if f in spec.nodes and d in spec.nodes and s + 1 <= spec.eot:
            lines.append(f'\t{f}_{s} -> {d}_{s + 1} [style=dashed, color="red", label="lost"];')
    lines.append("}")
    return "\n".join(lines) + "\n"


def run_record(i: int, run: Run) -> dict:
    """fi.Run (data-types.go:81-98) as runs.json holds it."""
    spec = run.spec
    tables: Dict[str, List[List[str]]] = {}
    for t in sorted(run.tables):
        for tab, tups in sorted(run.tables[t].items()):
            if tab == "crash":
                continue
            for tup in sorted(tups, key=repr):
                tables.setdefault(tab, []).append([str(v) for v in tup] + [str(t)])
    return {
        "iteration": i,
        "status": "success" if run.success else "fail",
        "failureSpec": {"eot": spec.eot, "eff": spec.eff, "maxCrashes": spec.max_crashes, "nodes": list(spec.nodes),
                        "crashes": [{"node": n, "time": t} for n, t in sorted(spec.crashes.items())],
                        "omissions": [{"from": f, "to": d, "time": t} for f, d, t in sorted(spec.omissions)]},
        "model": {"tables": tables},
        "messages": [{"table": tab, "from": f, "to": d, "sendTime": s, "receiveTime": r}
                     for tab, f, d, s, r in run.messages if f != d],
    }


def write_output(runs: List[Run], out_dir: str, indent: Optional[int] = 1) -> None:
    """The directory faultinjectors/molly.go:15-163 loads."""
    os.makedirs(out_dir, exist_ok=True)
    sep = (",", ":") if indent is None else None
    recs = []
    for i, run in enumerate(runs):
        recs.append(run_record(i, run))
        for cond in ("pre", "post"):
            with open(os.path.join(out_dir, f"run_{i}_{cond}_provenance.json"), "w") as fh:
                json.dump(provenance(run, cond), fh, indent=indent, separators=sep)
        with open(os.path.join(out_dir, f"run_{i}_spacetime.dot"), "w") as fh:
            fh.write(spacetime_dot(run))
    with open(os.path.join(out_dir, "runs.json"), "w") as fh:
        json.dump(recs, fh, indent=indent, separators=sep)
