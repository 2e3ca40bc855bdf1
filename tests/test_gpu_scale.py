"""GPU parity at BASELINE.json's configuration sizes.

The small cases in test_gpu_parity.py cover every tier and quirk; these run
the bench workloads themselves (or their deep-graph shape) through the C ABI
and compare with the CPU oracle, bit-exact:

  C3  the whole 10k-run corpus bench.py times (E ~ 1.5 V), every field incl.
      edge pulls, both diff modes
  C5  graphs of 100k-1M nodes at the library's default thresholds: they take
      the deep tiers (k_chains_glob at V >= 65536, global CSR/Kahn, the
      u32 wide_pairs hand-over of nemo_stage_simplified)
  C4  the 100k-run corpus on one context: the run-sharded partial reduction
      vectors (nemo_partition_runs' LPT shards, run 0 replicated) sum to the
      single-context vector, and a random sample of runs (flags, chains, table
      sets, diff masks) equals the oracle on those runs

Reference semantics: preprocessing.go:13-348, prototype.go:9-206,
differential-provenance.go:18-146 (the oracle's citations).
"""
import os

import numpy as np
import pytest

from nemo_amd import engine as E
from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE, F_DELETED, F_HOLDS, F_KEPT
from oracle import oracle as O
from tests.compare import assert_same
from tools import synth

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def _say(*a):
    print("[scale]", *a, flush=True)  # progress for long cases (run with -s)


@pytest.fixture(scope="module")
def eng():
    e = E.Engine(0)
    yield e
    e.close()


def _check_staged(eng, corpus, orc):
    """nemo_stage_simplified / nemo_simplified_view against the oracle (2-bit state + chain pairs)."""
    eng.stage_simplified()
    state, off, ht = eng.simplified_view()
    alive, holds = E.Engine.unpack_state(state, len(orc.flags))
    assert np.array_equal(alive, (orc.flags & (F_KEPT | F_DELETED)) == F_KEPT)
    assert np.array_equal(holds, (orc.flags & F_HOLDS) != 0)
    G = corpus.n_graphs
    assert len(off) == G + 1 and int(off[-1]) == len(ht) == len(orc.chains)
    g = np.repeat(np.arange(G), np.diff(off.astype(np.int64)))
    k = np.arange(len(ht)) - off[g].astype(np.int64)
    got = np.stack([g, k, ht[:, 0].astype(np.int64), ht[:, 1].astype(np.int64)], 1)
    assert np.array_equal(got, orc.chains[:, :4].astype(np.int64))


@pytest.mark.timeout(600)
def test_c3_full_corpus(eng):
    corpus, _ = synth.generate(10000, threads=THREADS, **synth.CONFIGS["c3"])
    V, Ed = int(corpus.node_off[-1]), int(corpus.edge_off[-1])
    assert V > 45_000_000 and 1.4 < Ed / V < 1.6
    s, f = corpus.success_iters(), corpus.failed_iters()
    assert len(f) > 100
    _say("c3 generated", V, Ed)
    res = E.analyze(corpus, s, f, diff_mode=DIFF_REFERENCE, engine=eng, pulls=True)
    _say("c3 gpu done")
    orc = O.analyze(corpus, s, f, diff_mode=DIFF_REFERENCE, threads=THREADS)
    _say("c3 oracle done")
    assert_same(corpus, res, orc, len(f))
    _say("c3 compared")
    del res
    _check_staged(eng, corpus, orc)
    # raw pulls (run i: the loaded edges, pre-post-prov.go:298-301) and diff-graph pulls (Q24, run 2000+f:
    # D's induced edges, differential-provenance.go:159-222) of every graph / entry
    _check_raw_pulls(eng, corpus)
    eng.diffprov(f, DIFF_REFERENCE)
    _check_diff_pulls(eng, corpus, orc.diff_mask)
    del orc
    # the bench's per-run diff mode on the same resident corpus
    eng.diffprov(f, DIFF_PER_RUN)
    orc = O.analyze(corpus, s, f, diff_mode=DIFF_PER_RUN, threads=THREADS, skip_pulls=True)
    assert np.array_equal(eng.diff_masks(len(f)), orc.diff_mask)
    assert np.array_equal(eng.missing(), orc.missing)


def _edge_keys(g, s, d):
    """The multiset of (graph, src, dst) rows as sorted packed u64 keys (one sort instead of a lexsort)."""
    g, s, d = (np.asarray(x, np.uint64) for x in (g, s, d))
    bs = max(int(s.max()).bit_length() if len(s) else 1, int(d.max()).bit_length() if len(d) else 1)
    bg = int(g.max()).bit_length() if len(g) else 1
    assert bg + 2 * bs <= 64
    k = (g << np.uint64(2 * bs)) | (s << np.uint64(bs)) | d
    k.sort()
    return k


def _pulled_rows(eng, slots):
    off, cnt, src, dst = eng.pulled_all(slots)
    gi = np.repeat(np.arange(slots, dtype=np.int64), np.asarray(cnt, np.int64))
    idx = np.concatenate([np.arange(int(o), int(o) + int(n), dtype=np.int64) for o, n in zip(off, cnt)]
                         + [np.zeros(0, np.int64)])
    return _edge_keys(gi, src[idx], dst[idx])


def _check_raw_pulls(eng, corpus):
    """nemo_pull_edges(0) == every graph's loaded edges, as a multiset per graph."""
    eng.pull(0)
    G = corpus.n_graphs
    got = _pulled_rows(eng, G)
    eg = np.repeat(np.arange(G, dtype=np.int64), np.diff(corpus.edge_off.astype(np.int64)))
    want = _edge_keys(eg, corpus.edge_src, corpus.edge_dst)
    assert np.array_equal(got, want), "raw pulls differ from the loaded edges"


def _check_diff_pulls(eng, corpus, masks):
    """nemo_pull_edges(2) == for every diff entry, run 0's post edges with both endpoints in the oracle's D."""
    eng.pull(2)
    n = len(masks)
    got = _pulled_rows(eng, n)
    g0 = 2 * corpus.run_index(0) + 1
    e0, e1 = int(corpus.edge_off[g0]), int(corpus.edge_off[g0 + 1])
    src, dst = corpus.edge_src[e0:e1].astype(np.int64), corpus.edge_dst[e0:e1].astype(np.int64)
    keep = (masks[:, src] != 0) & (masks[:, dst] != 0)  # [entries, E0]
    ent, j = np.nonzero(keep)
    want = _edge_keys(ent, src[j], dst[j])
    assert np.array_equal(got, want), f"diff pulls differ ({len(got)} vs {len(want)} edges)"


# (runs, nodes per graph, EOT, generator extras): Molly-density deep graphs and C5's ~4 edges per node
DEEP = {
    "molly_200k": (4, 200_000, 400, {}),
    "dense_100k": (3, 100_000, 200, {"body_extra": 6, "nval": 3, "nloc": 4}),
    "molly_1m": (2, 1_000_000, 2000, {}),
}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("shape", sorted(DEEP))
def test_c5_deep_graphs_default_tiers(eng, shape):
    n, nodes, eot, gen = DEEP[shape]
    corpus, _ = synth.generate(n, target_nodes=nodes, eot=eot, p_fault=1.0, threads=THREADS, **gen)
    sizes = [corpus.graph_size(g) for g in range(corpus.n_graphs)]
    # run 0 and at least one more run on the deep tiers (>= 65536 nodes); dropped messages in failed runs
    # leave smaller or empty graphs beside them, so the deep and LDS tiers share the launches
    assert min(sizes[:2]) >= 65536 and sum(v >= 65536 for v in sizes) >= 3 and corpus.failed_iters()
    for mode in (DIFF_REFERENCE, DIFF_PER_RUN):
        s, f = corpus.success_iters(), corpus.failed_iters()
        res = E.analyze(corpus, s, f, diff_mode=mode, engine=eng, pulls=mode == DIFF_REFERENCE)
        orc = O.analyze(corpus, s, f, diff_mode=mode, threads=THREADS, skip_pulls=mode != DIFF_REFERENCE)
        assert_same(corpus, res, orc, len(f), check_pulls=mode == DIFF_REFERENCE)
        _say(shape, "mode", mode, "ok")
    _check_staged(eng, corpus, orc)  # u32 (head, tail) pairs: graphs of >= 65536 nodes


def _reduce_vector(eng, success):
    eng.protos_partial(success, 0)  # the context's own vector
    return eng.reduce_vector().astype(np.int64)


@pytest.fixture(scope="module")
def c4():
    corpus, _ = synth.generate(100_000, threads=THREADS, **synth.CONFIGS["c3"])
    _say("c4 generated", int(corpus.node_off[-1]))
    return corpus


@pytest.mark.timeout(900)
def test_c4_sharded_partials_and_sample(eng, c4):
    from nemo_amd.shard import shard_layout
    R, parts = 100_000, 8
    corpus = c4
    s, f = corpus.success_iters(), corpus.failed_iters()
    eng.load(corpus)
    eng.mark()
    eng.simplify()
    full = _reduce_vector(eng, s)
    _say("c4 full pass")
    T = corpus.n_tables
    assert full[2 * T + 3] == R and full[2 * T] > 0
    rng = np.random.default_rng(0x4E454D4F)
    sample = np.unique(np.concatenate([[0], rng.choice(R, 48, replace=False),
                                       rng.choice([corpus.run_index(x) for x in f], 16, replace=False)]))
    # per-run results of the sampled runs from the full context
    flags = {int(r): (eng.flags(2 * int(r), 2 * int(r) + 1), eng.flags(2 * int(r) + 1, 2 * int(r) + 2)) for r in sample}
    chains = eng.chains()
    tabs = (eng.run_tables(0)[sample], eng.run_tables(1)[sample])
    f_sample = [int(corpus.iteration[r]) for r in sample if corpus.status[int(r)] != "success"]
    eng.diffprov(f_sample, DIFF_PER_RUN)
    masks = eng.diff_masks(len(f_sample))
    # the sample against the oracle on a corpus of just those runs
    sub = corpus.subset(sample)
    orc = O.analyze(sub, sub.success_iters(), f_sample, diff_mode=DIFF_PER_RUN, threads=THREADS, skip_pulls=True)
    _say("c4 sample oracle")
    for i, r in enumerate(sample):
        a, b = int(sub.node_off[2 * i]), int(sub.node_off[2 * i + 1])
        c = int(sub.node_off[2 * i + 2])
        assert np.array_equal(flags[int(r)][0], orc.flags[a:b]), f"pre flags of run {r}"
        assert np.array_equal(flags[int(r)][1], orc.flags[b:c]), f"post flags of run {r}"
    gmap = {2 * int(r) + k: 2 * i + k for i, r in enumerate(sample) for k in (0, 1)}
    mine = chains[np.isin(chains[:, 0], list(gmap))].copy()
    mine[:, 0] = [gmap[int(g)] for g in mine[:, 0]]
    assert np.array_equal(mine[np.lexsort((mine[:, 1], mine[:, 0]))], orc.chains)
    assert np.array_equal(tabs[1], orc.graph_tables)
    # proto lists depend on the run alone (prototype.go:11-24); rows of failed runs are not computed
    ok = np.array([corpus.status[int(r)] == "success" for r in sample])
    assert np.array_equal(tabs[0][ok], orc.proto_bits[ok])
    assert np.array_equal(masks, orc.diff_mask)
    # run-sharded partial vectors (bench.py / nemo_ctx_create_node layout) sum to the full one
    total = np.zeros_like(full)
    for rank in range(parts):
        runs, owned = shard_layout(corpus, rank, parts)
        shard = corpus.subset(runs, owned)
        eng.load(shard)
        eng.mark()
        eng.simplify()
        own = shard.owned if shard.owned is not None else np.ones(shard.n_runs, np.uint8)
        succ = [0] + [int(it) for it, o, st in zip(shard.iteration, own, shard.status)
                      if o and st == "success" and it != 0]
        total += _reduce_vector(eng, succ)
        _say("c4 shard", rank)
    assert np.array_equal(total, full)


def _results(e, corpus, s, f):
    """Every host-facing result of one analysis (main.go:106-177's calls), pulls of the diff graphs
    and the staged simplification included."""
    res = E.analyze(corpus, s, f, diff_mode=DIFF_REFERENCE, engine=e, pulls=False)
    e.stage_simplified()
    state, off, ht = e.simplified_view()
    res.staged = (np.array(state, copy=True), np.array(off, copy=True), np.array(ht, copy=True))
    e.pull(2)
    res.diff_pulls = _pulled_rows(e, len(f))
    res.run0 = corpus.run_index(0)
    return res


@pytest.mark.timeout(900)
def test_c4_node_context_8_shards(eng, c4):
    """nemo_ctx_create_node with 8 shards (all on device 0: the one-GPU layout of an 8-GPU node) over the
    100k-run C4 corpus equals one single-device context on every field: flags, chains, proto lists,
    table sets, inter/union, D masks, missing events, trigger rows, diff pulls, the staged view.  The
    shards' calls run on one host thread each (main.go:95's single Neo4J value drives the whole node)."""
    corpus = c4
    s, f = corpus.success_iters(), corpus.failed_iters()
    one = _results(eng, corpus, s, f)
    _say("c4 single context")
    eng.load(synth.generate(2, target_nodes=100)[0])  # release the single context's corpus
    node = E.Engine(devices=[0] * 8)
    try:
        got = _results(node, corpus, s, f)
        _say("c4 node context")
    finally:
        node.close()
    assert_same(corpus, got, one, len(f), check_pulls=False)
    assert np.array_equal(got.diff_pulls, one.diff_pulls), "diff pulls differ"
    for a, b, name in zip(got.staged, one.staged, ("state", "chain_off", "chain_ht")):
        assert np.array_equal(a, b), f"staged {name} differs"
