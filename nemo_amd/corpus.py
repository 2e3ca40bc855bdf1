"""Host-side corpus model: Molly output -> interned integer arrays.

This is the work the Go side of the drop-in does above the C ABI
(INTEGRATION.md): `faultinjectors/molly.go:15-163` (LoadOutput: ID prefixing,
clock-goal times, success/failed iteration lists) followed by the interning
that replaces `loadProv`'s per-element CREATE/MERGE round trips
(`graphing/pre-post-prov.go:25-213`).  Strings never cross the boundary: the
arrays below index into the string tables kept here.

Graph g of a corpus is run r's pre graph (g = 2r) or post graph (g = 2r+1).
"""
from __future__ import annotations

import ctypes
import json
import os
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

NODE_RULE = 0x80000000
TYPE_SHIFT = 28
TYPE_OTHER, TYPE_NEXT, TYPE_ASYNC = 0, 1, 2
TABLE_MASK = 0x00FFFFFF
NONE32 = 0xFFFFFFFF

F_HOLDS, F_KEPT, F_DELETED, F_HEAD, F_TAIL = 0x01, 0x02, 0x04, 0x08, 0x10

DIFF_REFERENCE, DIFF_PER_RUN = 0, 1


class LoadError(RuntimeError):
    """A loadProv-style validation failure (graphing/pre-post-prov.go:84-86,144-146,208-210)."""


def type_class(t: str) -> int:
    return TYPE_NEXT if t == "next" else TYPE_ASYNC if t == "async" else TYPE_OTHER


def word(is_rule: bool, type_cls: int, table: int) -> int:
    return (NODE_RULE if is_rule else 0) | (type_cls << TYPE_SHIFT) | (table & TABLE_MASK)


class CCorpus(ctypes.Structure):
    """ctypes mirror of `nemo_corpus` (include/nemohip.h)."""

    _fields_ = [
        ("n_runs", ctypes.c_uint32),
        ("n_tables", ctypes.c_uint32),
        ("table_pre", ctypes.c_uint32),
        ("table_post", ctypes.c_uint32),
        ("iteration", ctypes.c_void_p),
        ("owned", ctypes.c_void_p),
        ("node_off", ctypes.c_void_p),
        ("edge_off", ctypes.c_void_p),
        ("node_word", ctypes.c_void_p),
        ("label", ctypes.c_void_p),
        ("id_rank", ctypes.c_void_p),
        ("edge_src", ctypes.c_void_p),
        ("edge_dst", ctypes.c_void_p),
    ]


class CChain(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("graph", "k", "head", "tail", "len")]


class CMissing(ctypes.Structure):
    _fields_ = [("entry", ctypes.c_uint32), ("rule", ctypes.c_uint32)]


def _ptr(a: Optional[np.ndarray]) -> Optional[int]:
    return None if a is None else a.ctypes.data


@dataclass
class Corpus:
    """Interned, concatenated corpus (all arrays C-contiguous numpy)."""

    iteration: np.ndarray
    node_off: np.ndarray
    edge_off: np.ndarray
    node_word: np.ndarray
    label: np.ndarray
    edge_src: np.ndarray
    edge_dst: np.ndarray
    n_tables: int
    table_pre: int
    table_post: int
    id_rank: Optional[np.ndarray] = None
    owned: Optional[np.ndarray] = None
    status: Optional[List[str]] = None
    # host-side string tables (absent for large synthetic corpora)
    tables: Optional[List[str]] = None
    labels: Optional[List[str]] = None
    node_ids: Optional[List[str]] = None      # Molly IDs after molly.go prefixing
    node_types: Optional[List[str]] = None    # rule type strings ("" for goals)
    node_times: Optional[List[str]] = None    # goal time strings ("" for rules)
    runs: Optional[list] = None               # parsed runs.json entries
    _keep: list = field(default_factory=list, repr=False)

    @property
    def n_runs(self) -> int:
        return len(self.iteration)

    @property
    def n_graphs(self) -> int:
        return 2 * self.n_runs

    def graph_nodes(self, g: int) -> range:
        return range(int(self.node_off[g]), int(self.node_off[g + 1]))

    def graph_size(self, g: int) -> int:
        return int(self.node_off[g + 1] - self.node_off[g])

    def run_index(self, iteration: int) -> int:
        idx = getattr(self, "_run_index", None)
        if idx is None or len(idx) != len(self.iteration):
            idx = {}
            for i, it in enumerate(self.iteration.tolist()):
                idx.setdefault(int(it), i)
            self._run_index = idx
        try:
            return idx[int(iteration)]
        except KeyError:
            raise KeyError(f"unknown run iteration {iteration}") from None

    def success_iters(self) -> List[int]:
        return [int(self.iteration[r]) for r in range(self.n_runs) if self.status[r] == "success"]

    def failed_iters(self) -> List[int]:
        return [int(self.iteration[r]) for r in range(self.n_runs) if self.status[r] != "success"]

    def subset(self, runs: Sequence[int], owned: Optional[Sequence[int]] = None) -> "Corpus":
        """The corpus of runs `runs` (run indices, in that order) with their two graphs each;
        `owned` marks which of them count in cross-run reductions (None: all).  Numeric
        arrays only: the host string tables stay with the parent corpus."""
        runs = np.asarray(runs, np.int64)
        gs = np.stack([2 * runs, 2 * runs + 1], 1).reshape(-1)
        n0, n1 = self.node_off[gs].astype(np.int64), self.node_off[gs + 1].astype(np.int64)
        e0, e1 = self.edge_off[gs].astype(np.int64), self.edge_off[gs + 1].astype(np.int64)
        nv, ne = n1 - n0, e1 - e0
        node_off = np.concatenate([[0], np.cumsum(nv)]).astype(np.uint64)
        edge_off = np.concatenate([[0], np.cumsum(ne)]).astype(np.uint64)
        vi = np.repeat(n0 - node_off[:-1].astype(np.int64), nv) + np.arange(int(node_off[-1]), dtype=np.int64)
        ei = np.repeat(e0 - edge_off[:-1].astype(np.int64), ne) + np.arange(int(edge_off[-1]), dtype=np.int64)
        own = None
        if owned is not None:
            own = np.ascontiguousarray(owned, dtype=np.uint8)
            if own.all():
                own = None
        return Corpus(iteration=np.ascontiguousarray(self.iteration[runs]), node_off=node_off, edge_off=edge_off,
                      node_word=self.node_word[vi], label=self.label[vi], edge_src=self.edge_src[ei],
                      edge_dst=self.edge_dst[ei], n_tables=self.n_tables, table_pre=self.table_pre,
                      table_post=self.table_post, id_rank=None if self.id_rank is None else self.id_rank[vi],
                      owned=own, status=None if self.status is None else [self.status[int(r)] for r in runs],
                      tables=self.tables)

    def c_struct(self) -> CCorpus:
        arrs = [self.iteration, self.node_off, self.edge_off, self.node_word, self.label, self.edge_src,
                self.edge_dst, self.id_rank, self.owned]
        for a in arrs:
            if a is not None:
                assert a.flags.c_contiguous
        c = CCorpus()
        c.n_runs = self.n_runs
        c.n_tables = self.n_tables
        c.table_pre = self.table_pre
        c.table_post = self.table_post
        c.iteration = _ptr(self.iteration)
        c.owned = _ptr(self.owned)
        c.node_off = _ptr(self.node_off)
        c.edge_off = _ptr(self.edge_off)
        c.node_word = _ptr(self.node_word)
        c.label = _ptr(self.label)
        c.id_rank = _ptr(self.id_rank)
        c.edge_src = _ptr(self.edge_src)
        c.edge_dst = _ptr(self.edge_dst)
        return c


class CorpusBuilder:
    """Interns Molly provenance (ProvData, faultinjectors/data-types.go:67-72) run by run."""

    def __init__(self) -> None:
        self.tables: Dict[str, int] = {}
        self.table_names: List[str] = []
        self.labels: Dict[str, int] = {}
        self.label_names: List[str] = []
        self.iteration: List[int] = []
        self.status: List[str] = []
        self.runs: List[dict] = []
        self.node_off = [0]
        self.edge_off = [0]
        self.words: List[int] = []
        self.lab: List[int] = []
        self.rank: List[int] = []
        self.src: List[int] = []
        self.dst: List[int] = []
        self.ids: List[str] = []
        self.types: List[str] = []
        self.times: List[str] = []

    def _table(self, t: str) -> int:
        if t not in self.tables:
            self.tables[t] = len(self.table_names)
            self.table_names.append(t)
        return self.tables[t]

    def _label(self, s: str) -> int:
        if s not in self.labels:
            self.labels[s] = len(self.label_names)
            self.label_names.append(s)
        return self.labels[s]

    def add_graph(self, iteration: int, prov: dict) -> None:
        """loadProv (graphing/pre-post-prov.go:25-213) for one graph, as interning."""
        goals = prov.get("goals") or []
        rules = prov.get("rules") or []
        edges = prov.get("edges") or []
        gidx: Dict[str, int] = {}
        ridx: Dict[str, int] = {}
        ids: List[str] = []
        for g in goals:
            if g["id"] in gidx:
                raise LoadError(f"Run {iteration}: duplicate goal id {g['id']} (Goal.id IS UNIQUE, pre-post-prov.go:68)")
            gidx[g["id"]] = len(ids)
            ids.append(g["id"])
            self.words.append(word(False, 0, self._table(g["table"])))
            self.lab.append(self._label(g["label"]))
            self.types.append("")
            self.times.append(g.get("time", ""))
        if len(gidx) != len(goals):
            raise LoadError(f"Run {iteration}: inserted number of goals")
        for r in rules:
            if r["id"] in ridx:
                raise LoadError(f"Run {iteration}: duplicate rule id {r['id']} (Rule.id IS UNIQUE, pre-post-prov.go:129)")
            ridx[r["id"]] = len(ids)
            ids.append(r["id"])
            self.words.append(word(True, type_class(r.get("type", "")), self._table(r["table"])))
            self.lab.append(self._label(r["label"]))
            self.types.append(r.get("type", ""))
            self.times.append("")
        # rank of each node's ID string inside this graph (collapse tie-break)
        order = sorted(range(len(ids)), key=lambda i: ids[i])
        rank = [0] * len(ids)
        for pos, i in enumerate(order):
            rank[i] = pos
        self.rank.extend(rank)
        self.ids.extend(ids)
        created = 0
        seen = set()
        for e in edges:
            f, t = e["from"], e["to"]
            # direction by strings.Contains(From, "goal") (pre-post-prov.go:173)
            if "goal" in f:
                u, v = gidx.get(f), ridx.get(t)
            else:
                u, v = ridx.get(f), gidx.get(t)
            if u is None or v is None or (u, v) in seen:
                continue  # MATCH fails / MERGE finds the edge: relationships-created += 0
            seen.add((u, v))
            self.src.append(u)
            self.dst.append(v)
            created += 1
        if created != len(edges):
            raise LoadError(
                f"Run {iteration}: inserted number of edges ({created}) does not equal number of "
                f"antecedent provenance edges ({len(edges)})")
        self.node_off.append(len(self.words))
        self.edge_off.append(len(self.src))

    def add_run(self, iteration: int, status: str, pre: dict, post: dict, run: Optional[dict] = None) -> None:
        self.iteration.append(iteration)
        self.status.append(status)
        self.runs.append(run or {"iteration": iteration, "status": status})
        self.add_graph(iteration, pre)
        self.add_graph(iteration, post)

    def build(self) -> Corpus:
        self._table("pre")
        self._table("post")
        return Corpus(
            iteration=np.asarray(self.iteration, dtype=np.uint32),
            node_off=np.asarray(self.node_off, dtype=np.uint64),
            edge_off=np.asarray(self.edge_off, dtype=np.uint64),
            node_word=np.asarray(self.words, dtype=np.uint32),
            label=np.asarray(self.lab, dtype=np.uint32),
            edge_src=np.asarray(self.src, dtype=np.uint32),
            edge_dst=np.asarray(self.dst, dtype=np.uint32),
            id_rank=np.asarray(self.rank, dtype=np.uint32),
            n_tables=len(self.table_names),
            table_pre=self.tables["pre"],
            table_post=self.tables["post"],
            status=list(self.status),
            tables=list(self.table_names),
            labels=list(self.label_names),
            node_ids=list(self.ids),
            node_types=list(self.types),
            node_times=list(self.times),
            runs=list(self.runs),
        )


_CLK_WILD = re.compile(r", ([\d]+), __WILDCARD__\)")
_CLK_TWO = re.compile(r", ([\d]+), ([\d]+)\)")


def _molly_prefix(prov: dict, iteration: int, cond: str) -> dict:
    """ID prefixing and clock-time rewrite of Molly.LoadOutput (faultinjectors/molly.go:71-116,119-164)."""
    out = {"goals": [], "rules": [], "edges": []}
    pfx = f"run_{iteration}_{cond}_"
    for g in prov.get("goals") or []:
        g = dict(g)
        if g.get("table") == "clock":
            m = _CLK_WILD.search(g["label"])
            if m:
                g["time"] = m.group(1)
            m = _CLK_TWO.search(g["label"])
            if m:
                g["time"] = m.group(1)
        g["id"] = pfx + g["id"]
        out["goals"].append(g)
    for r in prov.get("rules") or []:
        r = dict(r)
        r["id"] = pfx + r["id"]
        out["rules"].append(r)
    for e in prov.get("edges") or []:
        out["edges"].append({"from": pfx + e["from"], "to": pfx + e["to"]})
    return out


def load_molly(out_dir: str) -> Corpus:
    """Molly.LoadOutput (faultinjectors/molly.go:15-163) + interning.

    The provenance file name uses the run's *index* and the ID prefix its
    *iteration* (molly.go:59-60 vs :92), exactly as the reference does."""
    with open(os.path.join(out_dir, "runs.json")) as fh:
        runs = json.load(fh)
    b = CorpusBuilder()
    for i, run in enumerate(runs):
        it = int(run["iteration"])
        with open(os.path.join(out_dir, f"run_{i}_pre_provenance.json")) as fh:
            pre = _molly_prefix(json.load(fh), it, "pre")
        with open(os.path.join(out_dir, f"run_{i}_post_provenance.json")) as fh:
            post = _molly_prefix(json.load(fh), it, "post")
        b.add_run(it, run.get("status", ""), pre, post, run)
    return b.build()


def corpus_from_graphs(graphs: Sequence[tuple]) -> Corpus:
    """Build from [(iteration, status, pre_prov, post_prov), ...] with Molly-style
    unprefixed IDs; applies molly.go's prefixing."""
    b = CorpusBuilder()
    for it, status, pre, post in graphs:
        b.add_run(it, status, _molly_prefix(pre, it, "pre"), _molly_prefix(post, it, "post"))
    return b.build()
