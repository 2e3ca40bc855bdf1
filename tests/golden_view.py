"""Express oracle / engine results in the ID-keyed layout of tests/golden/*/expected.json."""
import numpy as np

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
