"""ctypes wrapper of tools/libnemosynth.so: deterministic synthetic Molly-shaped corpora.

Default shape: seed 0x4E454D4F, 32 regular tables (Zipf 1.1)
plus clock/pre/post, @next/@async/deductive rules 55/15/30 %, 1-2 derivations
per goal, 1-3 body atoms, message omissions on runs other than 0.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass
from typing import Optional

import numpy as np

from nemo_amd.corpus import Corpus

_HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x4E454D4F
TABLE_NAMES = ["log", "ack", "bcast", "rbcast", "node", "member", "vote", "commit", "prepare", "leader", "term",
               "append", "replica", "request", "response", "timer", "elect", "heartbeat", "lease", "lock", "write",
               "read", "sync", "chunk", "block", "meta", "queue", "offset", "session", "watch", "znode",
               "missing_log", "clock", "pre", "post"]


# Generator settings of BASELINE.json's synthetic configurations, shared by bench.py
# and the parity tests at those sizes.
#   c3: ~5k-node graphs, E ~ 1.5 V (Molly-like bodies of 1-3 atoms give 1.18; body_extra 4 adds 0-8
#       shared body atoms per rule, which lands at E/V ~ 1.48), EOT 10
#   c5: deep provenance, ~1M nodes / ~4M edges per graph at EOT 2000 (body goals shared over a small
#       key space so that 0-12 extra atoms per rule give ~4 edges per node)
CONFIGS = {
    "c3": {"target_nodes": 5000, "eot": 10, "body_extra": 4},
    "c3_molly": {"target_nodes": 5000, "eot": 10, "body_extra": 0},
    "c5": {"target_nodes": 1_000_000, "eot": 2000, "body_extra": 6, "nval": 3, "nloc": 4},
}


class CParams(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("n_runs", ctypes.c_uint32), ("run_base", ctypes.c_uint32),
                ("eot", ctypes.c_uint32), ("nloc", ctypes.c_uint32), ("nval", ctypes.c_uint32),
                ("target_nodes", ctypes.c_uint32), ("p_fault", ctypes.c_double), ("max_drops", ctypes.c_uint32),
                ("prepend_run0", ctypes.c_int), ("threads", ctypes.c_int), ("body_extra", ctypes.c_uint32)]


class COut(ctypes.Structure):
    _fields_ = [("n_runs", ctypes.c_uint32), ("n_tables", ctypes.c_uint32), ("table_pre", ctypes.c_uint32),
                ("table_post", ctypes.c_uint32), ("table_clock", ctypes.c_uint32), ("eot", ctypes.c_uint32),
                ("nloc", ctypes.c_uint32), ("nval", ctypes.c_uint32),
                ("iteration", ctypes.POINTER(ctypes.c_uint32)), ("status_ok", ctypes.POINTER(ctypes.c_uint8)),
                ("owned", ctypes.POINTER(ctypes.c_uint8)), ("node_off", ctypes.POINTER(ctypes.c_uint64)),
                ("edge_off", ctypes.POINTER(ctypes.c_uint64)), ("node_word", ctypes.POINTER(ctypes.c_uint32)),
                ("label", ctypes.POINTER(ctypes.c_uint32)), ("edge_src", ctypes.POINTER(ctypes.c_uint32)),
                ("edge_dst", ctypes.POINTER(ctypes.c_uint32)), ("base_id", ctypes.POINTER(ctypes.c_uint32))]


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libnemosynth.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        _LIB = ctypes.CDLL(path)
        _LIB.synth_generate.argtypes = [ctypes.POINTER(CParams), ctypes.POINTER(COut)]
        _LIB.synth_generate.restype = ctypes.c_int
        _LIB.synth_free.argtypes = [ctypes.POINTER(COut)]
    return _LIB


def _np(p, n, dt):
    if n == 0:
        return np.zeros(0, dt)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True)


@dataclass
class SynthInfo:
    eot: int
    nloc: int
    nval: int
    base_id: np.ndarray


def generate(n_runs: int, target_nodes: int = 5000, eot: int = 10, nloc: int = 5, nval: int = 8,
             p_fault: float = 0.15, max_drops: int = 2, seed: int = SEED, run_base: int = 0,
             prepend_run0: bool = False, threads: Optional[int] = None, body_extra: int = 0):
    """Returns (Corpus, SynthInfo).  Runs are iterations run_base .. run_base+n_runs-1
    (plus a replicated, not-owned run 0 first when prepend_run0 and run_base > 0)."""
    L = lib()
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    p = CParams(seed, n_runs, run_base, eot, nloc, nval, target_nodes, p_fault, max_drops, int(prepend_run0),
                threads, body_extra)
    o = COut()
    rc = L.synth_generate(ctypes.byref(p), ctypes.byref(o))
    if rc != 0:
        raise RuntimeError(f"synth_generate failed ({rc})")
    try:
        R = o.n_runs
        node_off = _np(o.node_off, 2 * R + 1, np.uint64)
        edge_off = _np(o.edge_off, 2 * R + 1, np.uint64)
        V, E = int(node_off[-1]), int(edge_off[-1])
        status_ok = _np(o.status_ok, R, np.uint8)
        owned = _np(o.owned, R, np.uint8)
        corpus = Corpus(iteration=_np(o.iteration, R, np.uint32), node_off=node_off, edge_off=edge_off,
                        node_word=_np(o.node_word, V, np.uint32), label=_np(o.label, V, np.uint32),
                        edge_src=_np(o.edge_src, E, np.uint32), edge_dst=_np(o.edge_dst, E, np.uint32),
                        n_tables=o.n_tables, table_pre=o.table_pre, table_post=o.table_post, id_rank=None,
                        owned=owned if not owned.all() else None,
                        status=["success" if s else "failure" for s in status_ok], tables=list(TABLE_NAMES))
        info = SynthInfo(o.eot, o.nloc, o.nval, _np(o.base_id, V, np.uint32))
        return corpus, info
    finally:
        L.synth_free(ctypes.byref(o))


def label_string(lab: int, info: SynthInfo) -> str:
    if lab >= 0xF0000000:
        return TABLE_NAMES[lab - 0xF0000000]
    t = lab % (info.eot + 2)
    rest = lab // (info.eot + 2)
    val = rest % info.nval
    rest //= info.nval
    loc = rest % info.nloc
    tab = rest // info.nloc
    name = TABLE_NAMES[tab]
    if name == "clock":
        return f"clock(n{loc}, n{val}, {t - 1}, {t})"
    if name in ("pre", "post"):
        return f"{name}(n{loc}, {t})"
    return f"{name}(n{loc}, v{val}, {t})"


def write_molly(corpus: Corpus, info: SynthInfo, out_dir: str, threads: Optional[int] = None) -> None:
    """to_molly in C (libnemosynth synth_write_molly): the same files, byte for byte, one file per
    OpenMP task -- fast enough to stage the bench's end-to-end input."""
    L = lib()
    if not getattr(L, "_wm", False):
        vp = ctypes.c_void_p
        L.synth_write_molly.argtypes = [ctypes.c_char_p, ctypes.c_uint32] + [vp] * 9 + \
                                       [ctypes.c_uint32] * 3 + [vp, ctypes.c_int]
        L.synth_write_molly.restype = ctypes.c_int
        L._wm = True
    os.makedirs(out_dir, exist_ok=True)
    ok = np.ascontiguousarray([s == "success" for s in corpus.status], dtype=np.uint8)
    names = (ctypes.c_char_p * len(TABLE_NAMES))(*[n.encode() for n in TABLE_NAMES])
    arrs = [corpus.iteration, ok, corpus.node_off, corpus.edge_off, corpus.node_word, corpus.label,
            corpus.edge_src, corpus.edge_dst, np.ascontiguousarray(info.base_id)]
    rc = L.synth_write_molly(out_dir.encode(), corpus.n_runs, *[a.ctypes.data for a in arrs], info.eot, info.nloc,
                             info.nval, ctypes.cast(names, ctypes.c_void_p), int(threads or min(16, os.cpu_count() or 1)))
    if rc != 0:
        raise OSError(f"synth_write_molly failed writing {out_dir}")


def to_molly(corpus: Corpus, info: SynthInfo, out_dir: str) -> None:
    """Write a Molly-format output directory (runs.json + run_<i>_{pre,post}_provenance.json),
    the layout faultinjectors/molly.go:18,59-60 reads."""
    import json
    os.makedirs(out_dir, exist_ok=True)
    types = {0: "single", 1: "next", 2: "async"}
    runs = []
    for r in range(corpus.n_runs):
        it = int(corpus.iteration[r])
        runs.append({"iteration": it, "status": corpus.status[r],
                     "failureSpec": {"eot": info.eot, "eff": max(1, info.eot - 2), "maxCrashes": 0,
                                     "nodes": [f"n{i}" for i in range(info.nloc)], "crashes": [], "omissions": []},
                     "model": {"tables": {"pre": [["n0", str(info.eot)]], "post": [["n0", str(info.eot)]]}},
                     "messages": []})
        for ci, cond in enumerate(("pre", "post")):
            g = 2 * r + ci
            n0, n1 = int(corpus.node_off[g]), int(corpus.node_off[g + 1])
            e0, e1 = int(corpus.edge_off[g]), int(corpus.edge_off[g + 1])
            ids, goals, rules = [], [], []
            for v in range(n0, n1):
                w = int(corpus.node_word[v])
                tab = TABLE_NAMES[w & 0xFFFFFF]
                lab = label_string(int(corpus.label[v]), info)
                if w & 0x80000000:
                    ids.append(f"rule{int(info.base_id[v]):08d}")
                    rules.append({"id": ids[-1], "label": lab, "table": tab, "type": types[(w >> 28) & 7]})
                else:
                    ids.append(f"goal{int(info.base_id[v]):08d}")
                    t = lab.rsplit(", ", 1)[-1].rstrip(")")
                    goals.append({"id": ids[-1], "label": lab, "table": tab, "time": t})
            edges = [{"from": ids[int(corpus.edge_src[e])], "to": ids[int(corpus.edge_dst[e])]} for e in range(e0, e1)]
            with open(os.path.join(out_dir, f"run_{r}_{cond}_provenance.json"), "w") as fh:
                json.dump({"goals": goals, "rules": rules, "edges": edges}, fh)
    with open(os.path.join(out_dir, "runs.json"), "w") as fh:
        json.dump(runs, fh)
