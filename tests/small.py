"""Tiny random Molly-shaped corpora and the literal-evaluator <-> index-space mapping (test helpers)."""
from __future__ import annotations

import random
from typing import Dict, List, Tuple

import numpy as np

from nemo_amd.corpus import F_DELETED, F_HOLDS, F_KEPT, Corpus, _molly_prefix, corpus_from_graphs


def random_prov(rng: random.Random, cond: str, max_nodes: int = 12, label_pool: int = 4,
                p_edge: float = 0.35, p_next: float = 0.5) -> dict:
    """A random bipartite DAG (edges follow a random topological order)."""
    n = rng.randint(2, max_nodes)
    is_rule = [rng.random() < 0.5 for _ in range(n)]
    tables = [cond, "t1", "t2", "pre" if cond == "post" else "post"]
    forced: Dict[int, str] = {}
    plant = []
    if n >= 4 and rng.random() < 0.8:
        # plant the condition pattern markConditionHolds looks for: (C goal)->(C rule)->(goal)->(rule)
        base = rng.randrange(0, 2) if n > 5 else 0
        i, j = base, base + 1
        is_rule[i], is_rule[j] = False, True
        forced[i] = cond
        forced[j] = cond
        plant.append((i, j))
        if base == 1 and rng.random() < 0.5:
            is_rule[0] = True
            plant.append((0, i))
    goals, rules, names = [], [], []
    for i in range(n):
        if is_rule[i]:
            name = f"rule{i}"
            u = rng.random()
            typ = "next" if u < p_next else ("async" if u < p_next + 0.2 else "single")
            t = forced.get(i) or rng.choice(tables)
            if i in forced:
                typ = "single"
            rules.append({"id": name, "label": t, "table": t, "type": typ})
        else:
            name = f"goal{i}"
            t = forced.get(i) or rng.choice(tables)
            goals.append({"id": name, "label": f"{t}(a, {rng.randrange(label_pool)})", "table": t,
                          "time": str(rng.randint(1, 4))})
        names.append(name)
    edges = []
    planted = set(plant)
    for a, b in plant:
        edges.append({"from": names[a], "to": names[b]})
    for i in range(n):
        for j in range(i + 1, n):
            if (i, j) not in planted and is_rule[i] != is_rule[j] and rng.random() < p_edge:
                edges.append({"from": names[i], "to": names[j]})
    return {"goals": goals, "rules": rules, "edges": edges}


def random_corpus(seed: int, n_runs: int = None, max_nodes: int = 12) -> Tuple[Corpus, list]:
    rng = random.Random(seed)
    if n_runs is None:
        n_runs = rng.randint(1, 3)
    p_next = rng.choice([0.3, 0.6, 0.9])
    p_edge = rng.choice([0.25, 0.4, 0.6])
    graphs = []
    for it in range(n_runs):
        status = "success" if it == 0 or rng.random() < 0.5 else "failure"
        graphs.append((it, status, random_prov(rng, "pre", max_nodes, p_edge=p_edge, p_next=p_next),
                       random_prov(rng, "post", max_nodes, p_edge=p_edge, p_next=p_next)))
    return corpus_from_graphs(graphs), graphs


def prefixed_runs(graphs) -> list:
    return [(it, st, _molly_prefix(pre, it, "pre"), _molly_prefix(post, it, "post")) for it, st, pre, post in graphs]


def literal_view(corpus: Corpus, lit: dict) -> dict:
    """Express the literal evaluator's results in the corpus' (graph, local index) space."""
    db = lit["db"]
    view = {"holds": [], "kept": [], "deleted": [], "chains": [], "gprime": [], "lists": {}, "diff": [],
            "missing": [], "pre": set(), "post": set(), "async": set()}
    loc: Dict[Tuple[int, str], Dict[int, int]] = {}
    for r in range(corpus.n_runs):
        it = int(corpus.iteration[r])
        for ci, cond in enumerate(("pre", "post")):
            g = 2 * r + ci
            n0 = int(corpus.node_off[g])
            V = corpus.graph_size(g)
            ids = corpus.node_ids[n0:n0 + V]
            rawmap = lit["raw"][(it, cond)]
            nid2loc = {rawmap[ids[i]]: i for i in range(V)}
            loc[(it, cond)] = nid2loc
            view["holds"].append(np.array([bool(lit["holds"][(it, cond)][ids[i]]) for i in range(V)]))
            cm = lit["clean"][(it, cond)]
            view["kept"].append({nid2loc[n] for n in cm})
            c2l = {c: nid2loc[n] for n, c in cm.items()}
            view["deleted"].append({c2l[c] for c in cm.values() if c not in db.nodes})
            chains = lit["chains"][(it, cond)]
            view["chains"].append([(c["k"], c2l[c["head"]], c2l[c["tail"]], c["len"]) for c in chains])
            coll = {c["nid"]: V + c["k"] for c in chains}
            m = dict(c2l)
            m.update(coll)
            edges = []
            for a in m:
                if a in db.nodes:
                    for b in db.out[a]:
                        edges.append((m[a], m[b]))
            view["gprime"].append(sorted(edges))
    tabs = lambda lst: set(lst)
    for j, it in enumerate(lit["success"]):
        view["lists"][it] = tabs(lit["lists"][j])
    view["inter"] = None if lit["inter"] is None else set(lit["inter"])
    view["union"] = None if lit["union"] is None else set(lit["union"])
    strip = lambda xs: {x[len("<code>"):-len("</code>")] for x in xs}
    view["inter_miss"] = None if lit["inter_miss"] is None else [strip(x) for x in lit["inter_miss"]]
    view["union_miss"] = None if lit["union_miss"] is None else [strip(x) for x in lit["union_miss"]]
    if (0, "post") in loc:
        l0 = loc[(0, "post")]
        for d in lit["diffs"]:
            view["diff"].append({l0[n] for n in d["nodes"]})
            view["missing"].append({(l0[d["inv"][m["rule"]]], frozenset(l0[d["inv"][x]] for x in m["goals"]))
                                    for m in d["missing"]})
        lp = loc[(0, "pre")]
        view["pre"] = {(lp[a], lp[g], lp[r]) for a, g, r in lit["pre_trig"]}
        view["post"] = {(l0[g], l0[r]) for g, r in lit["post_trig"]}
        view["async"] = {lp[r] for r in lit["async_rules"]}
    view["all_pre"] = lit["all_pre"]
    return view


def bits_to_tables(corpus: Corpus, bits: np.ndarray) -> set:
    out = set()
    for t in range(corpus.n_tables):
        if (int(bits[t >> 5]) >> (t & 31)) & 1:
            out.add(corpus.tables[t])
    return out


def diff_missing_sets(corpus: Corpus, mask: np.ndarray, rules: List[int], g0: int) -> set:
    """(rule, frozenset(D children)) for the given missing rules of run 0's post graph."""
    n0 = int(corpus.node_off[g0])
    V = corpus.graph_size(g0)
    src = corpus.edge_src[int(corpus.edge_off[g0]):int(corpus.edge_off[g0 + 1])]
    dst = corpus.edge_dst[int(corpus.edge_off[g0]):int(corpus.edge_off[g0 + 1])]
    ch = {}
    for a, b in zip(src, dst):
        if mask[b]:
            ch.setdefault(int(a), set()).add(int(b))
    return {(r, frozenset(ch.get(r, set()))) for r in rules}
