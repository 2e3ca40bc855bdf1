"""GPU parity of the batched passes (nemo_amd/batched.py) that bench.py's C5 1k-run line times
(BASELINE.json configs[4]: a corpus larger than one GPU's HBM, in batches over two contexts).

Each pass loads batch i+1 on one context from a second host thread while batch i is analysed on the other,
reuses the cached (not zero-filled) device allocations of earlier batches of other sizes, uploads from
page-locked host arrays (nemo_host_register) and sums the batches' proto vectors on the host.  Checked
against the oracle (oracle/nemo_oracle.c):
  - the summed reduction vector and inter / union / achvdCond == the oracle's on the whole corpus
    (prototype.go:79-130);
  - every batch's node state (alive, holds), accepted chains, clean-post table sets (missingFrom,
    prototype.go:141-206), D masks and missing rows == the oracle's on that batch, in the per-run diff mode
    and in the reference mode (failedRuns[0]'s label set for every entry, differential-provenance.go:22-43).
Deep-graph shape (~4 edges per node, long-span parents) on the deep tiers (global CSR / Kahn, k_chains_glob,
1024-thread global kernels), and the library's default tiers.
"""
import numpy as np
import pytest

from nemo_amd.batched import BatchedPasses
from nemo_amd.corpus import DIFF_PER_RUN, DIFF_REFERENCE, F_DELETED, F_HOLDS, F_KEPT, NODE_RULE
from oracle import oracle as O
from tools import synth

pytestmark = pytest.mark.gpu

DEEP = (("graph_lds_max", 0), ("build_lds_max", 0), ("chains_glob_min_v", 0), ("global_block", 1024))
SHAPE = dict(target_nodes=12000, eot=16, body_extra=6, nval=3, nloc=4, p_fault=0.4)


def _batches(sizes, **gen):
    out, a = [], 0
    for n in sizes:
        c, _ = synth.generate(n, run_base=a, prepend_run0=True, **gen)
        out.append(c)
        a += n
    whole, _ = synth.generate(a, **gen)
    return out, whole


def _rows(m):
    m = np.asarray(m, np.int64).reshape(-1, 2)
    return m[np.lexsort((m[:, 1], m[:, 0]))]


def _check_passes(sizes, mode, options=(), prefetch=False, passes=2, load_async=None):
    batches, whole = _batches(sizes, **SHAPE)
    s_all, f_all = whole.success_iters(), whole.failed_iters()
    assert f_all and len(batches) >= 3
    orc_all = O.analyze(whole, s_all, f_all, diff_mode=mode, threads=8, skip_pulls=True)
    f0_labels = None
    if mode == DIFF_REFERENCE:
        g = 2 * whole.run_index(min(f_all)) + 1
        a, b = int(whole.node_off[g]), int(whole.node_off[g + 1])
        f0_labels = whole.label[a:b][(whole.node_word[a:b] & NODE_RULE) == 0]
    bp = BatchedPasses(batches, mode=mode, options=options, prefetch=prefetch, load_async=load_async)
    try:
        assert bp.pin_failed == 0
        assert bp.success[0] == 0 and sorted(bp.success) == sorted(s_all) and sorted(bp.failed) == sorted(f_all)
        for p in range(passes):  # a later pass reloads every batch into the other context's cached blocks
            res = bp.run_pass(collect=True)
            assert np.array_equal(res.vec.astype(np.uint32), orc_all.reduce), f"pass {p}: reduction vectors differ"
            assert res.achieved == orc_all.achieved
            assert res.inter == [int(x) for x in orc_all.inter] and res.union == [int(x) for x in orc_all.union]
            for c, r in zip(batches, res.batches):
                own = c.owned if c.owned is not None else np.ones(c.n_runs, np.uint8)
                bs = [int(x) for x, o in zip(c.iteration, own) if o and int(x) in set(s_all)]
                assert r.failed == [int(x) for x, o in zip(c.iteration, own) if o and int(x) in set(f_all)]
                orc = O.analyze(c, bs if 0 in bs else [0] + bs, r.failed, diff_mode=DIFF_PER_RUN, threads=8,
                                skip_pulls=True, diff_labels=f0_labels)
                assert np.array_equal(r.alive, (orc.flags & (F_KEPT | F_DELETED)) == F_KEPT), "alive differs"
                assert np.array_equal(r.holds, (orc.flags & F_HOLDS) != 0), "holds differs"
                G = c.n_graphs
                g = np.repeat(np.arange(G), np.diff(r.chain_off.astype(np.int64)))
                k = np.arange(len(r.chain_ht)) - r.chain_off[g].astype(np.int64)
                got = np.stack([g, k, r.chain_ht[:, 0].astype(np.int64), r.chain_ht[:, 1].astype(np.int64)], 1)
                assert np.array_equal(got, orc.chains[:, :4].astype(np.int64)), "chains differ"
                assert np.array_equal(r.tables, orc.graph_tables), "clean-post table sets differ"
                if r.failed:
                    assert np.array_equal(r.masks, orc.diff_mask), "D masks differ"
                    assert np.array_equal(_rows(r.missing), _rows(orc.missing)), "missing rows differ"
    finally:
        bp.close()


@pytest.mark.parametrize("tiers", ["deep", "default"])
@pytest.mark.parametrize("mode", [DIFF_PER_RUN, DIFF_REFERENCE])
def test_batched_passes_match_oracle(tiers, mode):
    # unequal: the second load shrinks, the third and fourth grow again
    _check_passes([9, 4, 7, 9], mode, options=DEEP if tiers == "deep" else ())


@pytest.mark.parametrize("parts,load_async", [(4, True), (1, True), (4, False)])
def test_batched_passes_prefetch(parts, load_async):
    """bench.py's C5 1k line: the next pass's first batch loaded beside the last analysis (three batches, so the
    batch ordinals alternate the contexts across passes), edge uploads in parts with each part's CSR build
    behind its own copy (option load_parts) and in one piece, loads that return before their kernels finish
    (option load_async) and loads that wait; three passes against the oracle."""
    _check_passes([9, 4, 7], DIFF_PER_RUN, options=(("load_parts", parts),), prefetch=True, passes=3,
                  load_async=load_async)
