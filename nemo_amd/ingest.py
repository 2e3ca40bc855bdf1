"""Native Molly ingest (nemo_ingest_molly, include/nemohip.h): the multi-threaded
C++ replacement of `corpus.load_molly` (faultinjectors/molly.go:15-163 +
loadProv's interning).  Same Corpus, same arrays; per-node strings stay in
native memory and are decoded on access."""
from __future__ import annotations

import ctypes
import json
import os
from typing import Optional

import numpy as np

from . import engine as E
from .corpus import CCorpus, Corpus, LoadError

STR_TABLE, STR_LABEL, STR_NODE_ID, STR_NODE_TYPE, STR_NODE_TIME = range(5)


def _lib():
    L = E.lib()
    if not getattr(L, "_ingest_sigs", False):
        vp, P = ctypes.c_void_p, ctypes.POINTER
        L.nemo_ingest_molly.argtypes = [ctypes.c_char_p, vp, ctypes.c_uint32, ctypes.c_int, P(vp), ctypes.c_char_p,
                                        ctypes.c_size_t]
        L.nemo_ingest_molly.restype = ctypes.c_int
        L.nemo_ingest_corpus.argtypes = [vp, P(CCorpus)]
        L.nemo_ingest_corpus.restype = ctypes.c_int
        L.nemo_ingest_count.argtypes = [vp, ctypes.c_int]
        L.nemo_ingest_count.restype = ctypes.c_uint64
        L.nemo_ingest_string.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, P(ctypes.c_char_p), P(ctypes.c_size_t)]
        L.nemo_ingest_string.restype = ctypes.c_int
        L.nemo_ingest_free.argtypes = [vp]
        L.nemo_ingest_free.restype = None
        L._ingest_sigs = True
    return L


class _Handle:
    def __init__(self, h):
        self.h = h

    def __del__(self):
        if self.h:
            _lib().nemo_ingest_free(self.h)
            self.h = None

    def string(self, kind: int, i: int) -> str:
        p, n = ctypes.c_char_p(), ctypes.c_size_t()
        rc = _lib().nemo_ingest_string(self.h, kind, int(i), ctypes.byref(p), ctypes.byref(n))
        if rc != 0:
            raise IndexError(i)
        return ctypes.string_at(p, n.value).decode() if n.value else ""

    def strings(self, kind: int, n: int) -> list:
        """Strings 0..n-1 of a kind (the lookup bound once, its out-arguments reused)."""
        f = _lib().nemo_ingest_string
        p, ln = ctypes.c_char_p(), ctypes.c_size_t()
        bp, bn, h, at = ctypes.byref(p), ctypes.byref(ln), self.h, ctypes.string_at
        out = []
        for i in range(n):
            if f(h, kind, i, bp, bn) != 0:
                raise IndexError(i)
            out.append(at(p, ln.value).decode() if ln.value else "")
        return out


class NodeStrings:
    """Lazy per-node string column (node IDs are re-prefixed like molly.go:92)."""

    def __init__(self, handle: _Handle, kind: int, corpus: "Corpus", prefixed: bool = False):
        self.h, self.kind, self.c, self.prefixed = handle, kind, corpus, prefixed
        self.n = int(corpus.node_off[-1])

    def __len__(self) -> int:
        return self.n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self.n))]
        if i < 0:
            i += self.n
        s = self.h.string(self.kind, i)
        if self.prefixed:
            g = int(np.searchsorted(self.c.node_off, i, side="right")) - 1
            s = f"run_{int(self.c.iteration[g // 2])}_{'pre' if g % 2 == 0 else 'post'}_{s}"
        return s


def load_molly_native(out_dir: str, threads: int = 0) -> Corpus:
    """Corpus of a Molly output directory via the native ingest."""
    with open(os.path.join(out_dir, "runs.json")) as fh:
        runs = json.load(fh)
    it = np.asarray([int(r["iteration"]) for r in runs], dtype=np.uint32)
    L = _lib()
    h = ctypes.c_void_p()
    err = ctypes.create_string_buffer(1024)
    rc = L.nemo_ingest_molly(out_dir.encode(), it.ctypes.data if len(it) else None, len(it), threads,
                             ctypes.byref(h), err, len(err))
    if rc != 0:
        raise LoadError(err.value.decode() or f"nemo_ingest_molly failed ({rc})")
    handle = _Handle(h)
    cs = CCorpus()
    L.nemo_ingest_corpus(h, ctypes.byref(cs))
    G, n = 2 * len(it), len(it)
    node_off = np.ctypeslib.as_array(ctypes.cast(cs.node_off, ctypes.POINTER(ctypes.c_uint64)), shape=(G + 1,))
    edge_off = np.ctypeslib.as_array(ctypes.cast(cs.edge_off, ctypes.POINTER(ctypes.c_uint64)), shape=(G + 1,))
    V, Ecount = int(node_off[-1]), int(edge_off[-1])

    def arr(ptr, count):
        if count == 0:
            return np.zeros(0, np.uint32)
        return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint32)), shape=(count,))

    c = Corpus(iteration=it, node_off=node_off, edge_off=edge_off, node_word=arr(cs.node_word, V),
               label=arr(cs.label, V), edge_src=arr(cs.edge_src, Ecount), edge_dst=arr(cs.edge_dst, Ecount),
               id_rank=arr(cs.id_rank, V), n_tables=cs.n_tables, table_pre=cs.table_pre, table_post=cs.table_post,
               status=[r.get("status", "") for r in runs],
               tables=handle.strings(STR_TABLE, int(L.nemo_ingest_count(h, STR_TABLE))),
               labels=handle.strings(STR_LABEL, int(L.nemo_ingest_count(h, STR_LABEL))),
               runs=runs)
    c.node_ids = NodeStrings(handle, STR_NODE_ID, c, prefixed=True)
    c.node_types = NodeStrings(handle, STR_NODE_TYPE, c)
    c.node_times = NodeStrings(handle, STR_NODE_TIME, c)
    c._keep.append(handle)  # the arrays above are views into the ingest's memory
    return c
