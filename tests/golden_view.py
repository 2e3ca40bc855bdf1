"""Express oracle / engine results in the ID-keyed layout of tests/golden/*/expected.json."""
import hashlib
import json

import numpy as np

from oracle import host_literal as HL

from nemo_amd.corpus import F_DELETED, F_HOLDS, F_KEPT


def view(corpus, res, failed):
    ids = corpus.node_ids
    out = {"holds": {}, "clean": [], "deleted": [], "chains": {}, "lists": {}}
    for g in range(corpus.n_graphs):
        n0 = int(corpus.node_off[g])
        for i in range(corpus.graph_size(g)):
            if not (corpus.node_word[n0 + i] >> 31):
                out["holds"][ids[n0 + i]] = bool(res.flags[n0 + i] & F_HOLDS)
            else:
                out["holds"].setdefault(ids[n0 + i], False)
    for r in range(corpus.n_runs):
        kept, dele = [], []
        for ci in range(2):
            g = 2 * r + ci
            n0 = int(corpus.node_off[g])
            for i in range(corpus.graph_size(g)):
                if res.flags[n0 + i] & F_KEPT:
                    kept.append(ids[n0 + i])
                if res.flags[n0 + i] & F_DELETED:
                    dele.append(ids[n0 + i])
            it = int(corpus.iteration[r])
            cond = "pre" if ci == 0 else "post"
            rows = [row for row in res.chains if int(row[0]) == g]
            out["chains"][f"run {it} {cond}"] = [
                {"k": int(row[1]), "head": ids[n0 + int(row[2])], "tail": ids[n0 + int(row[3])], "len": int(row[4]),
                 "id": f"run_{1000 + it}_{cond}_{corpus.tables[corpus.node_word[n0 + int(row[2])] & 0xFFFFFF]}"
                       f"_collapsed_{int(row[1])}"} for row in rows]
        out["clean"].append(sorted(kept))
        out["deleted"].append(sorted(dele))
    return out


def tables(corpus, bits):
    return sorted(corpus.tables[t] for t in range(corpus.n_tables) if (int(bits[t >> 5]) >> (t & 31)) & 1)


def _canon_json(c):
    nodes, edges = HL.canon(c)
    return {"nodes": nodes, "edges": [[a, b, dict(at)] for a, b, at in edges]}


def digest(obj) -> str:
    """sha256 of the canonical JSON of `obj` (large DOT views are pinned by digest)."""
    txt = json.dumps(json.loads(json.dumps(obj)), sort_keys=True, separators=(",", ":"))
    return hashlib.sha256(txt.encode()).hexdigest()


def host_expected(lit, runs, digests: bool = False):
    """The host side (Go) outputs: DOT graphs, missing events, corrections, extensions.
    With `digests`, the DOT views are stored as `<key>_sha256` digests."""
    db = lit["db"]
    iters = [it for it, _, _, _ in runs]
    dots = HL.pull_pre_post(db, iters, lit.get("ns"))
    out = {"dots": [{k: _canon_json(v) for k, v in d.items()} for d in dots]}
    out["diff_dots"], out["failed_dots"], out["missing_events"] = [], [], []
    for f, d in zip(lit["failed"], lit["diffs"]):
        dd, fd = HL.create_diff_dot(db, d, f, dots[0]["post"])
        out["diff_dots"].append(_canon_json(dd))
        out["failed_dots"].append(_canon_json(fd))
        out["missing_events"].append(HL.missing_records(db, d))
    adm = HL.corrections_admissible(db, lit["pre_trig"], lit["post_trig"])
    out["corrections"] = sorted(list(x) for x in adm) if adm is not None else None
    out["extensions"] = HL.extensions(db, lit["async_rules"]) if not lit["all_pre"] else []
    if digests:
        for k in ("dots", "diff_dots", "failed_dots"):
            out[k + "_sha256"] = digest(out.pop(k))
    return out
