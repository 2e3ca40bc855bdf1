"""Corpora larger than one GPU's HBM: batched passes over two libnemohip contexts.

BASELINE.json configs[4] (C5: 1k runs x 1M-node graphs, ~740 GB with every step buffer) does not fit one
MI355X's 288 GB.  The runs are split into batches, each a corpus of its own with run 0 replicated (not
owned) after the first, as the reference's own calls would see them: main.go:106-177 runs every graphing
method over all runs, and the only cross-run results are the prototype reduction (prototype.go:79-130,
a sum of per-run count vectors here) and failedRuns[0]'s label set of the reference diff mode
(differential-provenance.go:22-43, taken from the batch that holds it).

A pass loads batch i+1 (nemo_load_corpus: H2D + CSR + Kahn levels) on one context, from a second host
thread, while batch i is analysed on the other: mark, diff, simplify, protos partial, hand-over, pulls,
every D2H.  Batches are page-locked once (nemo_host_register), so each upload runs at the DMA rate.
With prefetch=True the last batch's analysis also overlaps the load of the next pass's first batch (the
batch ordinals run on across passes, so that load goes to the context the last batch is not on); every
pass then does one load per batch inside it (its own batches 1.. and the next pass's batch 0), and
close() waits for a load no pass used.  With load_async a load returns once its work is queued: the deep
graphs' Kahn levels (~74 ms of per-graph latency at C5) finish behind the host, and the batch's mark
reports the load's checks (nemo_set_option "load_async"; at C5 1k no faster, 418.6 vs 427.3 runs/s: the
pass is then bound by the analyses, slowed from 0.25 to 0.30 s by the loads' kernels beside them).
bench.py's C5 1k-run line (`--runs-total`) and tests/test_gpu_batched.py run this same code.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import engine as E
from .corpus import DIFF_PER_RUN, DIFF_REFERENCE, NODE_RULE, Corpus


@dataclass
class BatchResult:
    """One batch's host-facing results (collect=True): copies of the staged views and fetches."""

    iterations: np.ndarray          # the batch's runs (run 0 replicated after the first batch)
    owned: np.ndarray               # u8 per run
    alive: np.ndarray               # per node: kept in the simplified graph
    holds: np.ndarray               # per node: condition_holds
    chain_off: np.ndarray           # u64[G + 1]
    chain_ht: np.ndarray            # (n, 2) head, tail of every accepted chain
    tables: np.ndarray              # run_tables(1): per-run clean-post table bitsets (missingFrom)
    failed: List[int]               # the batch's diff entries (owned failed runs)
    masks: Optional[np.ndarray]     # (len(failed), V0) D masks
    missing: np.ndarray             # (entry, rule) rows
    vec: np.ndarray                 # the batch's reduction vector


@dataclass
class PassResult:
    achieved: int
    inter: List[int]
    union: List[int]
    vec: np.ndarray                                   # summed reduction vector
    phases: Dict[str, list] = field(default_factory=dict)
    batches: Optional[List[BatchResult]] = None       # collect=True


def split_even(n: int, batch: int) -> List[int]:
    """Batch sizes of near-equal size (1000 at 160: seven of 143, not six of 160 and one of 40), so that each
    reload reuses the previous batch's device allocations (nemo_ctx's cache takes blocks at most 1/8 larger
    than asked)."""
    nb = -(-n // max(1, min(batch, n)))
    b = -(-n // nb)
    return [min(b, n - a) for a in range(0, n, b)]


def _owned(c: Corpus) -> np.ndarray:
    return c.owned if c.owned is not None else np.ones(c.n_runs, np.uint8)


class BatchedPasses:
    """Two contexts on one device; pass() analyses every batch once, uploads included."""

    def __init__(self, batches: Sequence[Corpus], mode: int = DIFF_REFERENCE, device: int = 0,
                 options: Sequence[tuple] = (), pin: bool = True, prefetch: bool = False,
                 load_async: bool = False):
        self.batches = list(batches)
        self.mode = mode
        self.prefetch = prefetch
        # option load_async: a load returns once queued (its Kahn levels still running); the batch's
        # analysis (mark) then reports the load's checks
        self.load_async = load_async
        self._ord = 0                      # batch ordinal across passes: batch k of the pass is on engine (_ord + k) % 2
        self._pending = None               # (thread, errors, times) of a started load of the next pass's batch 0
        succ, fail = [], []
        for c in self.batches:
            for it, st, o in zip(c.iteration, c.status, _owned(c)):
                if o:
                    (succ if st == "success" else fail).append(int(it))
        self.success = [0] + [x for x in succ if x != 0]  # GetSuccessRunsIters(): run 0 leads
        self.failed = fail
        self.fset = set(fail)
        # reference mode: failedRuns[0]'s post-goal labels for every entry, from the batch holding it
        self.f0_labels = None
        if fail and mode == DIFF_REFERENCE:
            f0 = min(fail)
            for c in self.batches:
                if f0 in set(int(x) for x in c.iteration):
                    g = 2 * c.run_index(f0) + 1
                    a, b = int(c.node_off[g]), int(c.node_off[g + 1])
                    self.f0_labels = c.label[a:b][(c.node_word[a:b] & NODE_RULE) == 0].copy()
                    break
        self.engines = []
        for _ in range(2):
            e = E.Engine(device)
            for k, v in options:
                e.set_option(k, int(v))
            if self.load_async:
                e.set_option("load_async", 1)
            self.engines.append(e)
        self.T = self.batches[0].n_tables
        self.table_post = self.batches[0].table_post
        self.pinned: List[list] = []
        self.pin_s = 0.0
        self.pin_failed = 0
        if pin:  # page-locked once, up front; the cost and any refusals are reported (bench pass_phases)
            t = time.perf_counter()
            for c in self.batches:
                p = E.pin_corpus(c)
                tried = [a for a in (getattr(c, k, None) for k in E.PIN_FIELDS)
                         if a is not None and a.size > 0 and a.flags["C_CONTIGUOUS"]]
                self.pin_failed += len(tried) - len(p)
                self.pinned.append(p)
            self.pin_s = time.perf_counter() - t

    def drain(self) -> None:
        """Wait for a started load of the next pass's batch 0 (the next pass still uses it)."""
        if self._pending is not None:
            self._pending[0].join()

    def close(self) -> None:
        if self._pending is not None:
            self._pending[0].join()
            self._pending = None
        for e in self.engines:
            e.close()
        self.engines = []
        for p in self.pinned:
            E.unpin_corpus(p)
        self.pinned = []

    def _analyse(self, eng: E.Engine, c: Corpus, collect: bool):
        its = [int(x) for x, o in zip(c.iteration, _owned(c)) if o]
        bf = [it for it in its if it in self.fset]
        eng.mark()
        if bf:
            if self.f0_labels is not None:
                eng.diffprov_host_labels(bf, self.f0_labels)
            else:
                eng.diffprov(bf, DIFF_PER_RUN)
        eng.simplify()
        eng.protos_partial(self.success, 0)
        eng.stage_simplified()
        has0 = 0 in its
        if has0:
            eng.triggers()
        eng.pull(1)
        if bf:
            eng.pull(2)
        vec = eng.reduce_vector().astype(np.int64)
        tabs = eng.run_tables(1)
        if has0:
            eng.trigger_rows()
        masks = eng.diff_masks_view() if bf else None
        miss = eng.missing()
        state, off, ht = eng.simplified_view()
        if not collect:
            return vec, None
        alive, holds = E.Engine.unpack_state(state, int(c.node_off[-1]))
        return vec, BatchResult(iterations=c.iteration.copy(), owned=_owned(c).copy(), alive=alive, holds=holds,
                                chain_off=off.copy(), chain_ht=ht.copy(), tables=tabs.copy(), failed=bf,
                                masks=None if masks is None else masks.copy(), missing=miss.copy(), vec=vec)

    def run_pass(self, collect: bool = False) -> PassResult:
        phases = {"load_s": [], "analyse_s": [], "join_wait_s": []}
        errs: List[BaseException] = []

        def timed_load(eng, c):
            try:
                t = time.perf_counter()
                eng.load(c)
                if not self.load_async:
                    eng.synchronize()
                phases["load_s"].append(round(time.perf_counter() - t, 3))
            except BaseException as ex:  # re-raised on the calling thread
                errs.append(ex)

        vec = np.zeros(2 * self.T + 4, np.int64)
        out = [] if collect else None
        nb, o = len(self.batches), self._ord
        eng = lambda k: self.engines[(o + k) % 2]  # noqa: E731
        if self._pending is not None:  # batch 0's load, started beside the previous pass's last analysis
            th0, errs0, times0 = self._pending
            self._pending = None
            tj = time.perf_counter()
            th0.join()
            phases["join_wait_s"].append(round(time.perf_counter() - tj, 3))
            phases["load_s"] += times0
            if errs0:
                raise errs0[0]
        else:
            timed_load(eng(0), self.batches[0])
            if errs:
                raise errs[0]
        for i, c in enumerate(self.batches):
            th = None
            if i + 1 < nb:
                th = threading.Thread(target=timed_load, args=(eng(i + 1), self.batches[i + 1]))
                th.start()
            elif self.prefetch:  # the next pass's batch 0, on the other engine
                errs1: List[BaseException] = []
                times1: List[float] = []

                def load_next(e=eng(nb), c0=self.batches[0]):
                    try:
                        t1 = time.perf_counter()
                        e.load(c0)
                        if not self.load_async:
                            e.synchronize()
                        times1.append(round(time.perf_counter() - t1, 3))
                    except BaseException as ex:  # re-raised by the pass that uses it
                        errs1.append(ex)

                th1 = threading.Thread(target=load_next)
                th1.start()
                self._pending = (th1, errs1, times1)
            t = time.perf_counter()
            try:
                v, res = self._analyse(eng(i), c, collect)
                phases["analyse_s"].append(round(time.perf_counter() - t, 3))
            finally:
                if th is not None:
                    tj = time.perf_counter()
                    th.join()
                    phases["join_wait_s"].append(round(time.perf_counter() - tj, 3))
            if errs:
                raise errs[0]
            vec += v
            if collect:
                out.append(res)
        self._ord = (o + nb) % 2
        for e in self.engines:
            e.synchronize()
        a, inter, uni = E.reduce_interpret(vec.astype(np.uint32), self.T, self.table_post)
        return PassResult(achieved=a, inter=inter, union=uni, vec=vec, phases=phases, batches=out)
