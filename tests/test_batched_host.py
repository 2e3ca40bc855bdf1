"""Host logic of nemo_amd/batched.py (no GPU): the order of loads and analyses over the two contexts.

A recording stand-in for engine.Engine checks, for passes with and without prefetch, odd and even batch
counts: every batch is loaded once per pass and analysed on the context that loaded it, a context never
loads while it analyses, the load of the next pass's first batch goes to the context the last batch is
not on, and drain() / close() wait for it.  The device results are the GPU tests' (test_gpu_batched.py).
"""
import threading
import time

import numpy as np
import pytest

import nemo_amd.batched as B
from tools import synth


class _Recorder:
    def __init__(self):
        self.lock = threading.Lock()
        self.events = []   # (engine id, "load" | "analyse", batch first iteration, start, end)
        self.busy = {}     # engine id -> what it is doing now

    def enter(self, eid, what):
        with self.lock:
            assert eid not in self.busy, f"engine {eid}: {what} while {self.busy[eid]}"
            self.busy[eid] = what

    def leave(self, eid):
        with self.lock:
            del self.busy[eid]


def _fake_engine_cls(rec, T):
    class FakeEngine:
        n = 0

        def __init__(self, device=0):
            self.id = FakeEngine.n
            FakeEngine.n += 1
            self.loaded = None
            self.options = {}

        def set_option(self, k, v):
            self.options[k] = v

        def load(self, c):
            rec.enter(self.id, "load")
            t = time.perf_counter()
            time.sleep(0.01)
            self.loaded = int(c.iteration[-1])
            rec.events.append((self.id, "load", self.loaded, t, time.perf_counter()))
            rec.leave(self.id)

        def synchronize(self):
            pass

        def mark(self):
            rec.enter(self.id, "analyse")
            self._t = time.perf_counter()

        def diffprov(self, *a):
            pass

        diffprov_host_labels = diffprov

        def simplify(self):
            pass

        def protos_partial(self, *a):
            pass

        def stage_simplified(self):
            pass

        def triggers(self):
            pass

        def pull(self, which):
            pass

        def reduce_vector(self):
            return np.zeros(2 * T + 4, np.uint32)

        def run_tables(self, which):
            return np.zeros((1, 1), np.uint32)

        def trigger_rows(self):
            return None

        def diff_masks_view(self):
            return None

        def missing(self):
            return np.zeros((0, 2), np.uint32)

        def simplified_view(self):
            rec.events.append((self.id, "analyse", self.loaded, self._t, time.perf_counter()))
            rec.leave(self.id)
            return None, None, None

        def close(self):
            pass

    return FakeEngine


@pytest.mark.parametrize("n_batches", [3, 4])
@pytest.mark.parametrize("prefetch", [True, False])
def test_batched_pass_order(monkeypatch, n_batches, prefetch):
    batches, a = [], 0
    for n in [3] * n_batches:
        c, _ = synth.generate(n, run_base=a, prepend_run0=True, target_nodes=200, eot=6)
        batches.append(c)
        a += n
    rec = _Recorder()
    monkeypatch.setattr(B.E, "Engine", _fake_engine_cls(rec, batches[0].n_tables))
    bp = B.BatchedPasses(batches, pin=False, prefetch=prefetch)
    last = [int(c.iteration[-1]) for c in batches]
    try:
        for p in range(3):
            n0 = len(rec.events)
            res = bp.run_pass()
            ev = rec.events[n0:]
            analysed = [e for e in ev if e[1] == "analyse"]
            assert [e[2] for e in analysed] == last, "every batch analysed once, in order"
            assert len(res.phases["analyse_s"]) == n_batches
            # the context that analysed batch k is the one that loaded it last
            for e in analysed:
                loads = [x for x in rec.events if x[0] == e[0] and x[1] == "load" and x[4] <= e[3]]
                assert loads and loads[-1][2] == e[2]
            # the two contexts alternate, across passes too with prefetch
            ids = [e[0] for e in analysed]
            assert all(x != y for x, y in zip(ids, ids[1:]))
            if prefetch and p:
                assert ids[0] != prev_last
            prev_last = ids[-1]
        bp.drain()
        if prefetch:  # the next pass's first batch is loaded on the other context
            assert rec.events[-1][1] == "load" and rec.events[-1][2] == last[0] and rec.events[-1][0] != prev_last
    finally:
        bp.close()
    assert not rec.busy
