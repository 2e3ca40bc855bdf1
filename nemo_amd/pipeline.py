"""End-to-end path (SURVEY.md §8d metric 1 second half, §8f-4): a Molly output
directory -> streaming native ingest -> libnemohip -> host results, with the
JSON decode of chunk i+1 overlapping the upload and device analysis of chunk i.

`faultinjectors/molly.go:15-163` (LoadOutput) and the per-element interning of
`loadProv` (graphing/pre-post-prov.go:25-213) are what nemo_ingest_next
replaces; the chunks share one interning (include/nemohip.h), so label and
table ids agree across them.  Cross-chunk steps are the same as across
devices (nemo_amd/shard.py): the prototype vectors are summed on the host, run 0
is replicated (not owned) into every chunk after the first, and the reference
diff mode's failedRuns[0] label set, taken from the chunk that holds that run,
is passed to the later chunks (nemo_diffprov_host_labels).
"""
from __future__ import annotations

import ctypes
import json
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import engine as E
from .corpus import CCorpus, Corpus, DIFF_PER_RUN, DIFF_REFERENCE, LoadError, NODE_RULE
from .ingest import STR_LABEL, STR_TABLE

NOTFOUND = 7


def _lib():
    L = E.lib()
    if not getattr(L, "_stream_sigs", False):
        vp, P = ctypes.c_void_p, ctypes.POINTER
        L.nemo_ingest_open.argtypes = [ctypes.c_char_p, vp, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int, P(vp)]
        L.nemo_ingest_open.restype = ctypes.c_int
        L.nemo_ingest_next.argtypes = [vp, ctypes.c_uint32, ctypes.c_int, P(CCorpus), ctypes.c_char_p, ctypes.c_size_t]
        L.nemo_ingest_next.restype = ctypes.c_int
        L.nemo_ingest_stream_count.argtypes = [vp, ctypes.c_int]
        L.nemo_ingest_stream_count.restype = ctypes.c_uint64
        L.nemo_ingest_stream_string.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, P(ctypes.c_char_p),
                                                P(ctypes.c_size_t)]
        L.nemo_ingest_stream_string.restype = ctypes.c_int
        L.nemo_ingest_close.argtypes = [vp]
        L.nemo_ingest_close.restype = None
        L._stream_sigs = True
    return L


class IngestStream:
    """nemo_ingest_open / nemo_ingest_next: the directory's runs as chunk corpora."""

    def __init__(self, out_dir: str, threads: int = 0):
        with open(os.path.join(out_dir, "runs.json")) as fh:
            self.runs = json.load(fh)
        self.iteration = np.asarray([int(r["iteration"]) for r in self.runs], dtype=np.uint32)
        self.status = {int(r["iteration"]): r.get("status", "") for r in self.runs}
        # failedRuns[0] (GetFailedRunsIters order, molly.go:53) is parsed right after run 0
        first_failed = next((i for i, r in enumerate(self.runs) if r.get("status", "") != "success"), -1)
        self.L = _lib()
        self.h = ctypes.c_void_p()
        rc = self.L.nemo_ingest_open(out_dir.encode(), self.iteration.ctypes.data if len(self.iteration) else None,
                                     len(self.iteration), first_failed, threads, ctypes.byref(self.h))
        if rc != 0:
            raise LoadError(f"nemo_ingest_open failed ({rc})")

    def next(self, chunk: int, with_run0: bool = True) -> Optional[Corpus]:
        """The next chunk's corpus (its arrays stay valid through the following call), or None."""
        cs = CCorpus()
        err = ctypes.create_string_buffer(1024)
        rc = self.L.nemo_ingest_next(self.h, chunk, int(with_run0), ctypes.byref(cs), err, len(err))
        if rc == NOTFOUND:
            return None
        if rc != 0:
            raise LoadError(err.value.decode() or f"nemo_ingest_next failed ({rc})")
        R = cs.n_runs
        G = 2 * R

        def arr(ptr, n, ct, dt):
            if n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(n,))

        node_off = arr(cs.node_off, G + 1, ctypes.c_uint64, np.uint64)
        edge_off = arr(cs.edge_off, G + 1, ctypes.c_uint64, np.uint64)
        V, Ecount = int(node_off[-1]), int(edge_off[-1])
        u32 = lambda p, n: arr(p, n, ctypes.c_uint32, np.uint32)  # noqa: E731
        it = u32(cs.iteration, R)
        owned = arr(cs.owned, R, ctypes.c_uint8, np.uint8)
        return Corpus(iteration=it, node_off=node_off, edge_off=edge_off, node_word=u32(cs.node_word, V),
                      label=u32(cs.label, V), edge_src=u32(cs.edge_src, Ecount), edge_dst=u32(cs.edge_dst, Ecount),
                      id_rank=u32(cs.id_rank, V), n_tables=cs.n_tables, table_pre=cs.table_pre,
                      table_post=cs.table_post, owned=owned if not owned.all() else None,
                      status=[self.status[int(x)] for x in it])

    def strings(self, kind: int) -> List[str]:
        n = int(self.L.nemo_ingest_stream_count(self.h, kind))
        out = []
        for i in range(n):
            p, m = ctypes.c_char_p(), ctypes.c_size_t()
            self.L.nemo_ingest_stream_string(self.h, kind, i, ctypes.byref(p), ctypes.byref(m))
            out.append(ctypes.string_at(p, m.value).decode() if m.value else "")
        return out

    def close(self) -> None:
        if self.h:
            self.L.nemo_ingest_close(self.h)
            self.h = None

    def __del__(self):
        self.close()


@dataclass
class PipelineResult:
    """Per-run results in the directory's run order (run index r -> graphs 2r, 2r+1)."""

    n_runs: int = 0
    achieved: int = 0
    inter: List[int] = field(default_factory=list)
    union: List[int] = field(default_factory=list)
    reduce: Optional[np.ndarray] = None
    flags: Dict[int, np.ndarray] = field(default_factory=dict)        # graph -> per-node flags
    chains: List[np.ndarray] = field(default_factory=list)            # rows (graph, k, head, tail, len)
    run_tables: Dict[int, tuple] = field(default_factory=dict)        # run -> (proto bits, table set)
    diff_mask: Dict[int, np.ndarray] = field(default_factory=dict)    # failed iteration -> D mask
    missing: Dict[int, np.ndarray] = field(default_factory=dict)      # failed iteration -> rules
    triggers: Optional[tuple] = None
    tables: List[str] = field(default_factory=list)                   # table id -> name (stream interning)
    timings: Dict[str, float] = field(default_factory=dict)


def run(out_dir: str, engine: "E.Engine", chunk: int = 500, threads: int = 0, diff_mode: int = DIFF_REFERENCE,
        keep: bool = True) -> PipelineResult:
    """main.go:106-177's graph calls over a Molly directory, chunk by chunk, with the next chunk's
    JSON decode running beside the current chunk's device work.  keep=False fetches every result
    (the hand-over bench.py times) but does not keep the per-node arrays."""
    t0 = time.perf_counter()
    st = IngestStream(out_dir, threads)
    its = [int(x) for x in st.iteration]
    ok = {it: st.status[it] == "success" for it in its}
    # GetSuccessRunsIters / GetFailedRunsIters (molly.go:53), run 0 first among the successes
    success = [it for it in its if ok[it]]
    if 0 in success:
        success = [0] + [x for x in success if x != 0]
    failed = [it for it in its if not ok[it]]
    if failed and diff_mode == DIFF_REFERENCE and chunk < 2:
        raise ValueError("the reference diff mode needs chunk >= 2: run 0 and failedRuns[0] share the first chunk")
    # no run of iteration 0: CreateNaiveDiffProv's MATCH on run 0 finds nothing (differential-provenance.go:
    # 22-28) and every diff is empty, which the library reports as zero entries
    has_good = 0 in ok
    f0 = failed[0] if failed else None
    f0_labels = None
    run_of = {it: r for r, it in enumerate(its)}  # results are kept in runs.json order
    res = PipelineResult(n_runs=len(its))
    acc = np.zeros(0, np.int64)  # summed [cnt[T], first[T], achvd, first_nonempty, prehold, nruns]
    T_seen = 0
    nxt: Dict[str, object] = {}

    def parse():
        try:
            nxt["c"] = st.next(chunk)
        except Exception as e:  # surfaced in the main thread
            nxt["e"] = e

    th = threading.Thread(target=parse)
    th.start()
    t_dev = 0.0
    while True:
        th.join()
        if "e" in nxt:
            raise nxt["e"]
        c = nxt.pop("c")
        if c is None:
            break
        th = threading.Thread(target=parse)  # decode the next chunk while this one is on the device
        th.start()
        td = time.perf_counter()
        own = c.owned if c.owned is not None else np.ones(c.n_runs, np.uint8)
        engine.load(c)
        engine.mark()
        engine.simplify()
        engine.stage_simplified()
        engine.protos_partial(success, 0)
        vec = engine.reduce_vector().astype(np.int64)
        T = c.n_tables
        if T > T_seen:  # tables interned by this chunk extend the layout
            grown = np.zeros(2 * T + 4, np.int64)
            if T_seen:
                grown[:T_seen] = acc[:T_seen]
                grown[T:T + T_seen] = acc[T_seen:2 * T_seen]
                grown[2 * T:] = acc[2 * T_seen:]
            acc, T_seen = grown, T
        acc += vec
        chunk_its = [int(x) for x, o in zip(c.iteration, own) if o]
        cf = [f for f in failed if f in set(chunk_its)]
        if cf and diff_mode == DIFF_REFERENCE:
            if f0_labels is None:  # the stream parses run 0 and failedRuns[0] first: both are in the first chunk
                g = 2 * c.run_index(f0) + 1
                n0, n1 = int(c.node_off[g]), int(c.node_off[g + 1])
                f0_labels = c.label[n0:n1][(c.node_word[n0:n1] & NODE_RULE) == 0].copy()
            engine.diffprov_host_labels(cf, f0_labels)
        else:
            engine.diffprov(cf, DIFF_PER_RUN)
        has0 = 0 in set(chunk_its)
        if has0:
            engine.triggers()
        engine.pull(1)
        # host hand-over, as bench.py retrieves it
        state, chain_off, chain_ht = engine.simplified_view()
        tabs = (engine.run_tables(0), engine.run_tables(1))
        masks = engine.diff_masks_view() if cf and has_good else None
        miss = engine.missing()
        trig = engine.trigger_rows() if has0 else None
        if keep:
            flags = engine.flags()
            ch = engine.chains()
            for lr, it in enumerate(int(x) for x in c.iteration):
                if not own[lr]:
                    continue
                r = run_of[it]
                for k in (0, 1):
                    g = 2 * lr + k
                    res.flags[2 * r + k] = flags[int(c.node_off[g]) - int(c.node_off[0]):
                                                 int(c.node_off[g + 1]) - int(c.node_off[0])].copy()
                    rows = ch[ch[:, 0] == g].copy()
                    rows[:, 0] = 2 * r + k
                    res.chains.append(rows)
                res.run_tables[r] = (tabs[0][lr].copy(), tabs[1][lr].copy())
            for e, f in enumerate(cf if has_good else []):
                res.diff_mask[f] = np.asarray(masks[e]).copy()
                res.missing[f] = np.sort(miss[miss[:, 0] == e][:, 1])
            if trig is not None:
                res.triggers = tuple(np.asarray(x).copy() for x in trig)
        t_dev += time.perf_counter() - td
    st_tables = st.strings(STR_TABLE)
    st.close()
    T = T_seen
    table_post = st_tables.index("post") if "post" in st_tables else 0xFFFFFFFF
    res.achieved, res.inter, res.union = E.reduce_interpret(acc.astype(np.uint32), T, table_post)
    res.reduce = acc
    res.tables = st_tables
    res.timings = {"total_s": time.perf_counter() - t0, "device_s": t_dev}
    return res
