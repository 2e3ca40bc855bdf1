"""Run sharding (nemo_partition_runs): host-only, no GPU."""
import numpy as np

from nemo_amd.shard import partition_runs, shard_layout
from tools import synth


def test_lpt_partition_balanced_and_deterministic():
    corpus, _ = synth.generate(300, target_nodes=900, threads=2)
    w = np.diff(corpus.node_off.astype(np.int64)).reshape(-1, 2).sum(1) + \
        np.diff(corpus.edge_off.astype(np.int64)).reshape(-1, 2).sum(1)
    for parts in (1, 2, 3, 8):
        p = partition_runs(corpus, parts)
        assert p.shape == (corpus.n_runs,) and p.max() < parts
        assert np.array_equal(p, partition_runs(corpus, parts))
        load = np.bincount(p, weights=w, minlength=parts)
        # LPT: the heaviest part exceeds the mean by at most one run's weight
        assert load.max() - load.mean() <= w.max()
        # the same greedy restated here: longest first, least-loaded part, ties by index
        ref, acc = np.zeros(corpus.n_runs, np.int64), np.zeros(parts, np.int64)
        for r in sorted(range(corpus.n_runs), key=lambda r: (-w[r], r)):
            k = int(np.argmin(acc))
            ref[r] = k
            acc[k] += w[r]
        assert np.array_equal(p, ref)


def test_shard_layout_replicates_run0():
    corpus, _ = synth.generate(40, target_nodes=500, threads=2)
    parts = partition_runs(corpus, 4)
    owned_total = 0
    for rank in range(4):
        runs, owned = shard_layout(corpus, rank, 4, parts)
        assert 0 in runs.tolist()
        assert int(owned[runs.tolist().index(0)]) == int(parts[0] == rank)
        assert np.all(np.diff(runs) > 0)
        owned_total += int(owned.sum())
        sub = corpus.subset(runs, owned)
        for i, r in enumerate(runs):
            for k in (0, 1):
                a, b = int(corpus.node_off[2 * r + k]), int(corpus.node_off[2 * r + k + 1])
                c, d = int(sub.node_off[2 * i + k]), int(sub.node_off[2 * i + k + 1])
                assert np.array_equal(corpus.label[a:b], sub.label[c:d])
                e0, e1 = int(corpus.edge_off[2 * r + k]), int(corpus.edge_off[2 * r + k + 1])
                f0, f1 = int(sub.edge_off[2 * i + k]), int(sub.edge_off[2 * i + k + 1])
                assert np.array_equal(corpus.edge_src[e0:e1], sub.edge_src[f0:f1])
    assert owned_total == corpus.n_runs
