"""Host mirror of the reference's `graphing.Neo4J` plugin (the `GraphDatabase`
implementation main.go:33-44,95 drives) over libnemohip.

Every method keeps the reference's name, argument meaning, result layout and
call order (main.go:106-177).  The graph work happens in the gfx950 kernels
behind the C ABI (nemo_amd/engine.py -> include/nemohip.h); this module only
turns the integer results back into the strings, `fi.Missing` records and DOT
graphs the reference returns — the part the Go side of the drop-in keeps
(INTEGRATION.md).  Errors raise (`NemoError` from the engine, `ValueError` /
`OSError` here) where the reference returns a Go `error` that main.go turns
into `log.Fatalf`.

Orders the reference leaves unspecified (Neo4j row order, Go map iteration,
SURVEY.md Appendix C) are fixed here so results are reproducible: edges of a
pulled graph in (source, target) node order, trigger rows in node-index order,
maps in first-insertion order; prototype lists are in table-interning order
(the reference's list order comes from Neo4j path order and is compared as a
set).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import engine as E
from .corpus import DIFF_REFERENCE, F_HOLDS, NODE_RULE, TABLE_MASK, Corpus
from .dot import DotGraph, ProvNode, create_diff_dot, create_dot, read_dot


# ---- faultinjectors/data-types.go:43-78 -------------------------------------------
@dataclass
class Goal:
    ID: str
    Label: str
    Table: str
    Time: str
    CondHolds: bool = False
    Sender: str = ""
    Receiver: str = ""

    def to_json(self) -> dict:
        d = {"id": self.ID, "label": self.Label, "table": self.Table, "time": self.Time}
        if self.CondHolds:
            d["conditionHolds"] = True
        if self.Sender:
            d["sender"] = self.Sender
        if self.Receiver:
            d["receiver"] = self.Receiver
        return d


@dataclass
class Rule:
    ID: str
    Label: str
    Table: str
    Type: str

    def to_json(self) -> dict:
        return {"id": self.ID, "label": self.Label, "table": self.Table, "type": self.Type}


@dataclass
class Missing:
    Rule: Rule
    Goals: List[Goal] = field(default_factory=list)

    def to_json(self) -> dict:  # no json tags on fi.Missing: Go uses the field names
        return {"Rule": self.Rule.to_json(), "Goals": [g.to_json() for g in self.Goals]}


@dataclass
class GoalRulePair:
    """corrections.go:15-18."""
    Goal: Goal
    Rule: Rule


def receiver(label: str, table: str) -> str:
    """Receiver of a trigger goal (corrections.go:65-67,155-157):
    strings.TrimLeft(label, table) — a *cutset* trim — then Trim "()" and the
    first ", "-separated field."""
    return label.lstrip(table).strip("()").split(", ")[0]


def generate_corrections(pre_triggers: Sequence[Tuple[Rule, GoalRulePair]],
                         post_triggers: Sequence[Tuple[Goal, Rule]]) -> List[str]:
    """GenerateCorrections' string synthesis (corrections.go:219-324).

    `pre_triggers` are the rows of findPreTriggers as (aggregation, pair) and
    `post_triggers` the rows of findPostTriggers as (goal, rule), each in the
    order the reference's map iteration would visit them: both maps are keyed
    by a fresh pointer per row (:76,168), so every row is its own key."""
    recs: List[str] = []
    pre_rules: Dict[str, str] = {}
    different: Dict[str, Dict[str, List[Goal]]] = {}
    for agg, pair in pre_triggers:
        different[agg.Table] = {}
        recv = pair.Goal.Receiver
        if pre_rules.get(agg.Table, "") == "":
            pre_rules[agg.Table] = f"{agg.Table}({recv}, ...) :- {pair.Rule.Table}({recv}, ...)"
        else:
            pre_rules[agg.Table] = f"{pre_rules[agg.Table]}, {pair.Rule.Table}({recv}, ...)"
    for agg, pair in pre_triggers:
        nodes = different[agg.Table]
        recv = pair.Goal.Receiver
        for post_goal, _ in post_triggers:
            if recv != post_goal.Receiver:
                nodes.setdefault(recv, []).append(post_goal)
        agg_new = pre_rules[agg.Table]
        if not nodes:
            for post_goal, _ in post_triggers:
                agg_new = f"{agg_new}, {post_goal.Table}({post_goal.Receiver}, ...)"
        else:
            for pre_node, posts in nodes.items():
                for post in posts:
                    post_node, post_rule = post.Receiver, post.Table
                    recs.append(f"<code>{pre_node}</code> needs to know that <code>{post_node}</code> has executed "
                                f"<code>{post_rule}</code>. Add:<br /> &nbsp; &nbsp; &nbsp; &nbsp; "
                                f"<code>ack_{post_rule}({pre_node}, ...)@async :- {post_rule}({post_node}, ...), "
                                f"...;</code>")
                    agg_new = f"{agg_new}, ack_{post_rule}({pre_node}, sender={post_node}, ...)"
            if pair.Rule.Type != "next":
                rule, node = pair.Rule.Table, recv
                recs.append(f"Antecedent depends on timing of an onetime event. Make it persistent. Add:<br /> "
                            f"&nbsp; &nbsp; &nbsp; &nbsp; <code>buffer_{rule}({node}, ...) :- {rule}({node}, ...), "
                            f"...;</code><br /> &nbsp; &nbsp; &nbsp; &nbsp; <code>buffer_{rule}({node}, ...)@next "
                            f":- buffer_{rule}({node}, ...), ...;")
                agg_new = agg_new.replace(f"{rule}({node}, ...)", f"buffer_{rule}({node}, ...)")
        recs.append(f"Change: <code>{pre_rules[agg.Table]};</code> &nbsp; <i class = \"fas fa-long-arrow-alt-right\">"
                    f"</i> &nbsp; <code>{agg_new};</code>")
    return recs


def extension_strings(async_tables: Sequence[str]) -> List[str]:
    """extensions.go:76-90: one suggestion per distinct table (map order: first seen)."""
    state: Dict[str, str] = {}
    for t in async_tables:
        state[t] = f"<code>{t}(node, ...)@async :- ...;</code>"
    return list(state.values())


def hazard_colour(dot: DotGraph, time_pre_holds: Dict[str, bool], time_post_holds: Dict[str, bool]) -> DotGraph:
    """CreateHazardAnalysis' colouring of one space-time graph (hazard-analysis.go:39-80)."""
    for name, attrs in dot.nodes.items():
        attrs.update({"style": '"solid, filled"', "color": '"lightgrey"', "fillcolor": '"lightgrey"'})
        t = name.split("_")[-1]
        if t in time_pre_holds:
            attrs.update({"color": '"firebrick"', "fillcolor": '"firebrick"'})
        if t in time_post_holds:
            attrs["fillcolor"] = '"deepskyblue"'
    return dot


def time_holds(run: dict, cond: str) -> Dict[str, bool]:
    """Run.TimePreHolds / TimePostHolds (faultinjectors/molly.go:38-48): the last
    column of every row of model.tables[cond]."""
    rows = ((run or {}).get("model") or {}).get("tables", {}).get(cond) or []
    return {row[-1]: True for row in rows}


def _rewrite(id_: str, old: int, new: int) -> str:
    """The `id`:"run_<old> -> run_<new> prefix rewrite of the exports
    (preprocessing.go:33-45, differential-provenance.go:46-55)."""
    pfx = f"run_{old}"
    return f"run_{new}" + id_[len(pfx):] if id_.startswith(pfx) else id_


class Neo4J:
    """graphing.Neo4J (pre-post-prov.go:16-20): `Runs` is the loaded corpus."""

    def __init__(self) -> None:
        self.Runs: Optional[Corpus] = None
        self.eng: Optional[E.Engine] = None
        self._flags: Optional[np.ndarray] = None
        self._chains: Dict[int, List[Tuple[int, int]]] = {}
        self._protos: Optional[dict] = None
        self.diff_mode = DIFF_REFERENCE

    # ---- helpers.go -------------------------------------------------------------
    def InitGraphDB(self, boltURI: str, runs: Corpus, device: int = 0) -> None:
        """helpers.go:17-55: binds a HIP device instead of starting Neo4j; boltURI is unused."""
        if runs is None or runs.node_ids is None:
            raise ValueError("InitGraphDB needs a corpus with its string tables (corpus.load_molly)")
        self.Runs = runs
        self.eng = E.Engine(device)

    def CloseDB(self) -> None:
        """helpers.go:58-86."""
        if self.eng is not None:
            self.eng.close()
            self.eng = None

    # ---- node properties --------------------------------------------------------
    def _g(self, it: int, cond: str) -> int:
        return 2 * self.Runs.run_index(it) + (0 if cond == "pre" else 1)

    def _flag_arr(self) -> np.ndarray:
        if self._flags is None:
            self._flags = self.eng.flags()
        return self._flags

    def _node(self, g: int, i: int, run: Optional[int] = None) -> ProvNode:
        """Properties of local node i of graph g as the reference stores them
        (loadProv :28,91 + markConditionHolds); `run` re-prefixes the ID like
        the clean (1000+i) and diff (2000+f) copies."""
        c = self.Runs
        V = c.graph_size(g)
        it = int(c.iteration[g // 2])
        cond = "pre" if g % 2 == 0 else "post"
        if i >= V:  # collapsed rule k of a simplified graph (preprocessing.go:249-252)
            k = i - V
            head = self._chains[g][k][0]
            table = c.tables[int(c.node_word[int(c.node_off[g]) + head]) & TABLE_MASK]
            lab = f"{table}_collapsed"
            return ProvNode(f"run_{1000 + it}_{cond}_{lab}_{k}", lab, table, "collapsed", None, True)
        n = int(c.node_off[g]) + i
        w = int(c.node_word[n])
        is_rule = bool(w & NODE_RULE)
        id_ = c.node_ids[n] if run is None else _rewrite(c.node_ids[n], it, run)
        holds = None if is_rule else bool(self._flag_arr()[n] & F_HOLDS)
        return ProvNode(id_, c.labels[int(c.label[n])], c.tables[w & TABLE_MASK], c.node_types[n] if is_rule else None,
                        holds, is_rule, "" if is_rule else c.node_times[n])

    def _goal(self, p: ProvNode) -> Goal:
        return Goal(p.id, p.label, p.table, p.time, bool(p.holds))

    def _rule(self, p: ProvNode) -> Rule:
        return Rule(p.id, p.label, p.table, p.type or "")

    def _edges(self, slot: Optional[int], g: int, run: Optional[int] = None) -> List[Tuple[ProvNode, ProvNode]]:
        """Edge rows of a pulled slot, or (slot None) of raw graph g: the raw graph's relationships
        are exactly the loaded edges, which the host holds, so no device pull is made for them."""
        if slot is None:
            e0, e1 = int(self.Runs.edge_off[g]), int(self.Runs.edge_off[g + 1])
            s, d = self.Runs.edge_src[e0:e1], self.Runs.edge_dst[e0:e1]
        else:
            s, d = self.eng.pulled(slot)
        order = np.lexsort((d, s))
        cache: Dict[int, ProvNode] = {}

        def node(i: int) -> ProvNode:
            if i not in cache:
                cache[i] = self._node(g, i, run)
            return cache[i]

        return [(node(int(s[j])), node(int(d[j]))) for j in order]

    # ---- pre-post-prov.go -------------------------------------------------------
    def LoadRawProvenance(self) -> None:
        """pre-post-prov.go:247-285: load every run, then markConditionHolds."""
        self.eng.load(self.Runs)
        self.eng.mark()
        self._flags = None

    def SimplifyProv(self, iters: Sequence[int]) -> None:
        """preprocessing.go:351-387 (every loaded run is simplified; `iters` must name loaded runs)."""
        for it in iters:
            self.Runs.run_index(it)
        self.eng.simplify()
        self._flags = None
        self._chains = {}
        for g, k, head, tail, _ in self.eng.chains().tolist():
            lst = self._chains.setdefault(g, [])
            assert k == len(lst)
            lst.append((head, tail))

    def PullPrePostProv(self) -> Tuple[List[DotGraph], List[DotGraph], List[DotGraph], List[DotGraph]]:
        """pre-post-prov.go:288-459: raw (run i) and simplified (run 1000+i) DOT per run."""
        c = self.Runs
        n = c.n_runs
        pre, post, pre_c, post_c = [None] * n, [None] * n, [None] * n, [None] * n
        for r in range(n):  # raw graphs: the loaded edges (host-held), no device pull
            pre[r] = create_dot(self._edges(None, 2 * r), "pre")
            post[r] = create_dot(self._edges(None, 2 * r + 1), "post")
        self.eng.pull(1)
        for r in range(n):
            it = int(c.iteration[r])
            pre_c[r] = create_dot(self._edges(2 * r, 2 * r, 1000 + it), "pre")
            post_c[r] = create_dot(self._edges(2 * r + 1, 2 * r + 1, 1000 + it), "post")
        return pre, post, pre_c, post_c

    # ---- hazard-analysis.go -----------------------------------------------------
    def CreateHazardAnalysis(self, faultInjOut: str) -> List[DotGraph]:
        """hazard-analysis.go:16-88: read run_<iteration>_spacetime.dot and colour it."""
        c = self.Runs
        dots = []
        for r in range(c.n_runs):
            it = int(c.iteration[r])
            with open(os.path.join(faultInjOut, f"run_{it}_spacetime.dot")) as fh:
                dot = read_dot(fh.read())
            run = c.runs[r] if c.runs else {}
            dots.append(hazard_colour(dot, time_holds(run, "pre"), time_holds(run, "post")))
        return dots

    # ---- prototype.go -----------------------------------------------------------
    def _reduce(self, success: Sequence[int]) -> dict:
        self.eng.protos_partial(success, 0)
        self._protos = self.eng.protos_finalize(0)
        return self._protos

    def CreatePrototypes(self, iters: Sequence[int], failedIters: Sequence[int]):
        """prototype.go:209-256 -> (interProto, interProtoMiss, unionProto, unionProtoMiss)."""
        if len(iters) == 0:
            raise ValueError("no successful runs: extractProtos indexes iterProv[0] (prototype.go:80)")
        c = self.Runs
        red = self._reduce(iters)
        inter, union = red["inter"], red["union"]
        code = lambda ts: [f"<code>{c.tables[t]}</code>" for t in ts]
        inter_miss = [code(self.eng.missing_from(f, inter)) for f in failedIters]
        union_miss = [code(self.eng.missing_from(f, union)) for f in failedIters]
        return code(inter), inter_miss, code(union), union_miss

    # ---- differential-provenance.go ---------------------------------------------
    def CreateNaiveDiffProv(self, symmetric: bool, failedRuns: Sequence[int], successPostProv: DotGraph):
        """differential-provenance.go:18-243 -> (diffDots, failedDots, missingEvents).
        `symmetric` is unused, as in the reference."""
        c = self.Runs
        r0 = c.run_index(0)
        g0 = 2 * r0 + 1
        self.eng.diffprov(failedRuns, self.diff_mode)
        missing_rows = self.eng.missing()
        # D-children of every missing rule (the `leaf` rebinding of :93-95 collects all of them)
        e0, e1 = int(c.edge_off[g0]), int(c.edge_off[g0 + 1])
        src, dst = c.edge_src[e0:e1], c.edge_dst[e0:e1]
        children: Dict[int, List[int]] = {}
        for rule in set(int(x) for x in missing_rows[:, 1]):
            children[rule] = sorted(int(x) for x in dst[src == rule])
        missing: List[List[Missing]] = [[] for _ in failedRuns]
        masks = [self.eng.diff_mask(e) for e in range(len(failedRuns))] if len(failedRuns) else []
        for entry, rule in missing_rows.tolist():
            run = 2000 + int(failedRuns[entry])
            m = Missing(self._rule(self._node(g0, rule, run)))
            for ch in children[rule]:
                if masks[entry][ch]:
                    m.Goals.append(self._goal(self._node(g0, ch, run)))
            missing[entry].append(m)
        self.eng.pull(2)
        diff_edges = [self._edges(e, g0, 2000 + int(f)) for e, f in enumerate(failedRuns)]
        diffs, faileds = [], []
        for e, f in enumerate(failedRuns):
            gf = self._g(int(f), "post")
            failed_edges = self._edges(None, gf)
            ids = set()
            for m in missing[e]:
                ids.add(m.Rule.ID)
                ids.update(gl.ID for gl in m.Goals)
            d, fd = create_diff_dot(2000 + int(f), diff_edges[e], failed_edges, 0, successPostProv, ids)
            diffs.append(d)
            faileds.append(fd)
        return diffs, faileds, missing

    # ---- corrections.go / extensions.go -----------------------------------------
    def _trigger_rows(self):
        self.eng.triggers()
        pre, post, asy = self.eng.trigger_rows()
        pre = pre[np.lexsort((pre[:, 2], pre[:, 1], pre[:, 0]))] if len(pre) else pre
        post = post[np.lexsort((post[:, 1], post[:, 0]))] if len(post) else post
        return pre, post, np.sort(asy)

    def GenerateCorrections(self) -> List[str]:
        """corrections.go:202-328 on run 0."""
        r0 = self.Runs.run_index(0)
        pre, post, _ = self._trigger_rows()
        gp, gq = 2 * r0, 2 * r0 + 1
        pre_t = []
        for a, g, r in pre.tolist():
            goal = self._goal(self._node(gp, g))
            goal.Receiver = receiver(goal.Label, goal.Table)
            pre_t.append((self._rule(self._node(gp, a)), GoalRulePair(goal, self._rule(self._node(gp, r)))))
        post_t = []
        for g, r in post.tolist():
            goal = self._goal(self._node(gq, g))
            goal.Receiver = receiver(goal.Label, goal.Table)
            post_t.append((goal, self._rule(self._node(gq, r))))
        return generate_corrections(pre_t, post_t)

    def GenerateExtensions(self) -> Tuple[bool, List[str]]:
        """extensions.go:13-99 -> (allAchievedPre, extensions)."""
        red = self._protos if self._protos is not None else self._reduce([])
        all_achieved = not (red["pre_holds"] < self.Runs.n_runs)
        if all_achieved:
            return True, []
        _, _, asy = self._trigger_rows()
        gp = 2 * self.Runs.run_index(0)
        return False, extension_strings([self._node(gp, int(r)).table for r in asy])
