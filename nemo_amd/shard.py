"""Run sharding of a corpus over ranks / devices.

Runs are independent except for four cross-run steps (protos, extensions, the
diff's good run 0 and its failedRuns[0] label set), so a corpus is split by
run: nemo_partition_runs (libnemohip, host-only) assigns runs longest-first by
Σ(V+E) to the least-loaded part, and run 0 — the good run of every diff
(differential-provenance.go:26) and the subject of the corrections
(corrections.go:210) — is replicated on every part, owned (counted in the
reductions) by its own part only.
"""
from __future__ import annotations

import ctypes
from typing import Tuple

import numpy as np

from .corpus import Corpus


def partition_runs(corpus: Corpus, n_parts: int) -> np.ndarray:
    """part_of_run[r] for every run (nemo_partition_runs)."""
    from .engine import lib
    L = lib()
    out = np.zeros(max(corpus.n_runs, 1), np.uint32)
    cs = corpus.c_struct()
    rc = L.nemo_partition_runs(ctypes.byref(cs), n_parts, out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"nemo_partition_runs failed ({rc})")
    return out[:corpus.n_runs]


def shard_layout(corpus: Corpus, rank: int, world: int, parts: np.ndarray = None) -> Tuple[np.ndarray, np.ndarray]:
    """(run indices, owned flags) of part `rank`: its runs in corpus order, plus run 0 (not owned) if
    another part owns it."""
    if parts is None:
        parts = partition_runs(corpus, world)
    runs = np.nonzero(parts == rank)[0]
    owned = np.ones(len(runs), np.uint8)
    its = corpus.iteration
    if 0 in set(its.tolist()):
        r0 = corpus.run_index(0)
        if parts[r0] != rank:
            runs = np.concatenate([[r0], runs])
            owned = np.concatenate([[0], owned]).astype(np.uint8)
            order = np.argsort(runs, kind="stable")
            runs, owned = runs[order], owned[order]
    return runs.astype(np.int64), owned
