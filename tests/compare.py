"""Field-by-field comparison of an engine (GPU) result with the oracle's (test helper)."""
import numpy as np


def assert_same(corpus, eng, orc, n_failed: int, check_pulls: bool = True):
    assert np.array_equal(eng.flags, orc.flags), _first_diff("flags", eng.flags, orc.flags)
    assert np.array_equal(eng.chains, orc.chains), f"chains differ: gpu {len(eng.chains)} vs oracle {len(orc.chains)}"
    if eng.proto_bits is not None:
        assert np.array_equal(eng.proto_bits, orc.proto_bits), "proto lists differ"
        assert np.array_equal(eng.graph_tables, orc.graph_tables), "simplified-graph table sets differ"
        assert eng.achieved == orc.achieved
        assert eng.inter == [int(x) for x in orc.inter]
        assert eng.union == [int(x) for x in orc.union]
    if orc.run0 >= 0 and n_failed:
        assert np.array_equal(eng.diff_mask, orc.diff_mask), "diff masks differ"
        assert np.array_equal(eng.missing, orc.missing), "missing events differ"
    if orc.run0 >= 0:
        assert np.array_equal(eng.pre_rows, orc.pre_rows), "pre trigger rows differ"
        assert np.array_equal(eng.post_rows, orc.post_rows), "post trigger rows differ"
        assert np.array_equal(np.sort(eng.async_rules), np.sort(orc.async_rules)), "async rules differ"
    if check_pulls and eng.pulled is not None:
        G = corpus.n_graphs
        gi = np.repeat(np.arange(G, dtype=np.int64), [len(s) for s, _ in eng.pulled])
        es = np.concatenate([s for s, _ in eng.pulled] + [np.zeros(0, np.uint32)])
        ed = np.concatenate([d for _, d in eng.pulled] + [np.zeros(0, np.uint32)])
        po = orc.pulled_off.astype(np.int64)
        og = np.repeat(np.arange(G, dtype=np.int64), np.diff(po))
        a, b = _edge_multiset(gi, es, ed), _edge_multiset(og, orc.pulled_src, orc.pulled_dst)
        if not (len(a) == len(b) and np.array_equal(a, b)):
            bad = next((g for g in range(G) if not np.array_equal(a[a[:, 0] == g], b[b[:, 0] == g])), None)
            raise AssertionError(f"pulled edge multisets differ (gpu {len(a)} vs oracle {len(b)} edges), first graph {bad}")


def _edge_multiset(g, s, d):
    """(graph, src, dst) rows in a canonical order: the multiset of pulled edges, vectorised."""
    g, s, d = (np.asarray(x, np.int64) for x in (g, s, d))
    order = np.lexsort((d, s, g))
    return np.stack([g[order], s[order], d[order]], 1)


def _first_diff(name, a, b):
    if a.shape != b.shape:
        return f"{name}: shape {a.shape} vs {b.shape}"
    idx = np.nonzero(a != b)[0]
    return f"{name}: {len(idx)} differ, first at {idx[:5].tolist()}: gpu {a[idx[:5]].tolist()} oracle {b[idx[:5]].tolist()}"
