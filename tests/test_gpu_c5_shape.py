"""GPU parity on the bench's own C5 workload: the first 128 runs of bench.py --config c5's corpus (~1M-node
/ ~4.2M-edge graphs at EOT 2000; the bench keeps 320 runs resident, and each run's graphs depend only on
its own seed), against the oracle digest tests/golden/c5_shape/digest.json that
tests/golden/make_c5_shape.py computed once in the build container (the oracle's greedy chain cover
takes ~15 min per 1M-node graph, too long for a GPU test).

The whole 128-run corpus goes through libnemohip at its default tiers (deep CSR / Kahn, k_chains_glob,
the k_pg_* protos, the global diff tier, the multi-workgroup pulls), exactly as the bench runs it; the
digest's four runs (run 0, a success run, the first two failed runs) are then compared field by field:
node flags, accepted chains, simplified-graph edges, proto bits, table sets; the per-run D masks and
missing rules of all 16 failed runs (the digest's diff_per_run_all, from the oracle's diff-only mode);
and the reference mode, whose entries all equal failedRuns[0]'s per-run entry
(differential-provenance.go:22-43).  Reference: preprocessing.go:13-348, prototype.go:9-206,
differential-provenance.go:18-146, pre-post-prov.go:288-459.
"""
import json
import os

import numpy as np
import pytest

from nemo_amd import engine as E
from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE
from tests.golden.make_c5_shape import BENCH_RUNS, bench_corpus, chain_digest, edge_digest, pick_runs, sha

pytestmark = pytest.mark.gpu
DIGEST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c5_shape", "digest.json")


@pytest.mark.timeout(900)
def test_c5_bench_corpus_matches_oracle_digest():
    dig = json.load(open(DIGEST))
    assert dig["bench_runs"] == BENCH_RUNS
    corpus = bench_corpus(threads=min(16, os.cpu_count() or 1))
    runs, f_its = pick_runs(corpus)
    assert [e["run"] for e in dig["runs"]] == runs and f_its == dig["failed_iters"]
    s = [0] + [x for x in corpus.success_iters() if x != 0]
    f = corpus.failed_iters()
    assert f[:2] == f_its  # failedRuns[0] of the whole corpus is in the digest
    eng = E.Engine(0)
    try:
        eng.load(corpus)
        eng.mark()
        eng.simplify()
        eng.protos_partial(s, 0)
        proto = eng.run_tables(0)
        tabs = eng.run_tables(1)
        chains = eng.chains()
        eng.pull(1)
        modes = {}
        for mode in (DIFF_PER_RUN, DIFF_REFERENCE):
            eng.diffprov(f, mode)
            modes[mode] = (eng.diff_masks(len(f)), eng.missing())
        for ent in dig["runs"]:
            r = ent["run"]
            assert int(corpus.iteration[r]) == ent["iteration"] and corpus.status[r] == ent["status"]
            for k, gd in enumerate(ent["graphs"]):
                g = 2 * r + k
                assert corpus.graph_size(g) == gd["nodes"]
                assert sha(eng.flags(g, g + 1)) == gd["flags_sha256"], f"flags of graph {g}"
                ch = chains[chains[:, 0] == g]
                ch = ch[np.argsort(ch[:, 1], kind="stable")][:, 1:5]
                assert chain_digest(ch) == gd["chains"], f"chains of graph {g}"
                src, dst = eng.pulled(g)
                assert edge_digest(src, dst) == gd["pulled"], f"simplified edges of graph {g}"
            assert [int(x) for x in tabs[r]] == ent["graph_tables"]
            if "proto_bits" in ent:
                assert [int(x) for x in proto[r]] == ent["proto_bits"], f"proto list of run {r}"
            if "diff_per_run" in ent:
                d = ent["diff_per_run"]
                e = f.index(ent["iteration"])
                masks, miss = modes[DIFF_PER_RUN]
                assert sha(masks[e]) == d["mask_sha256"] and int(np.count_nonzero(masks[e])) == d["mask_popcount"]
                assert sorted(int(x) for x in miss[miss[:, 0] == e][:, 1]) == d["missing"]
        # per-run mode: every failed run of the corpus (diff_per_run_all)
        alld = dig["diff_per_run_all"]
        assert alld["failed_iters"] == f
        masks, miss = modes[DIFF_PER_RUN]
        for e, it in enumerate(f):
            d = alld["entries"][str(it)]
            assert sha(masks[e]) == d["mask_sha256"], f"per-run D mask of failed run {it}"
            assert int(np.count_nonzero(masks[e])) == d["mask_popcount"]
            assert sorted(int(x) for x in miss[miss[:, 0] == e][:, 1]) == d["missing"], f"missing of {it}"
        # reference mode: every entry is failedRuns[0]'s per-run entry
        d0 = next(e["diff_per_run"] for e in dig["runs"] if e["iteration"] == f_its[0])
        masks, miss = modes[DIFF_REFERENCE]
        for e in range(len(f)):
            assert sha(masks[e]) == d0["mask_sha256"], f"reference-mode D mask of entry {e}"
            assert sorted(int(x) for x in miss[miss[:, 0] == e][:, 1]) == d0["missing"]
    finally:
        eng.close()
