"""TEST INFRASTRUCTURE ONLY: ctypes binding of the C oracle (liboracle.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  Parity status against the reference engine: UNPINNED (see
nemo_oracle.h); the restatement is pinned to oracle/cypher_literal.py.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from nemo_amd.corpus import CChain, CMissing, Corpus

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


class COut(ctypes.Structure):
    _fields_ = [
        ("status", ctypes.c_int),
        ("err", ctypes.c_char * 256),
        ("V", ctypes.c_uint64),
        ("E", ctypes.c_uint64),
        ("n_graphs", ctypes.c_uint32),
        ("words", ctypes.c_uint32),
        ("n_tables", ctypes.c_uint32),
        ("flags", ctypes.POINTER(ctypes.c_uint8)),
        ("chains", ctypes.POINTER(CChain)),
        ("n_chains", ctypes.c_uint64),
        ("proto_bits", ctypes.POINTER(ctypes.c_uint32)),
        ("graph_tables", ctypes.POINTER(ctypes.c_uint32)),
        ("reduce", ctypes.POINTER(ctypes.c_uint32)),
        ("achieved", ctypes.c_uint32),
        ("inter", ctypes.POINTER(ctypes.c_uint32)),
        ("n_inter", ctypes.c_uint32),
        ("uni", ctypes.POINTER(ctypes.c_uint32)),
        ("n_union", ctypes.c_uint32),
        ("run0", ctypes.c_int32),
        ("v0", ctypes.c_uint32),
        ("n_entries", ctypes.c_uint32),
        ("diff_mask", ctypes.POINTER(ctypes.c_uint8)),
        ("missing", ctypes.POINTER(CMissing)),
        ("n_missing", ctypes.c_uint64),
        ("pre_rows", ctypes.POINTER(ctypes.c_uint32)),
        ("n_pre", ctypes.c_uint64),
        ("post_rows", ctypes.POINTER(ctypes.c_uint32)),
        ("n_post", ctypes.c_uint64),
        ("async_rules", ctypes.POINTER(ctypes.c_uint32)),
        ("n_async", ctypes.c_uint64),
        ("pulled_off", ctypes.POINTER(ctypes.c_uint64)),
        ("pulled_src", ctypes.POINTER(ctypes.c_uint32)),
        ("pulled_dst", ctypes.POINTER(ctypes.c_uint32)),
    ]


class COpts(ctypes.Structure):
    _fields_ = [
        ("threads", ctypes.c_int),
        ("success_iters", ctypes.c_void_p),
        ("n_success", ctypes.c_size_t),
        ("failed_iters", ctypes.c_void_p),
        ("n_failed", ctypes.c_size_t),
        ("diff_mode", ctypes.c_int),
        ("skip_pulls", ctypes.c_int),
        ("diff_labels", ctypes.c_void_p),
        ("n_diff_labels", ctypes.c_size_t),
        ("diff_only", ctypes.c_int),
    ]


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        _LIB = ctypes.CDLL(path)
        _LIB.oracle_analyze.argtypes = [ctypes.c_void_p, ctypes.POINTER(COpts), ctypes.POINTER(COut)]
        _LIB.oracle_analyze.restype = ctypes.c_int
        _LIB.oracle_free.argtypes = [ctypes.POINTER(COut)]
    return _LIB


class OracleError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code
        self.msg = msg


def _arr(p, n, dtype):
    if n == 0 or not p:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dtype, copy=True)


@dataclass
class OracleResult:
    flags: np.ndarray
    chains: np.ndarray          # [n, 5] graph, k, head, tail, len
    proto_bits: np.ndarray      # [n_runs, words]
    graph_tables: np.ndarray    # [n_runs, words]
    reduce: np.ndarray
    achieved: int
    inter: List[int]
    union: List[int]
    run0: int
    v0: int
    diff_mask: np.ndarray       # [n_entries, v0]
    missing: np.ndarray         # [n, 2] entry, rule
    pre_rows: np.ndarray        # [n, 3]
    post_rows: np.ndarray       # [n, 2]
    async_rules: np.ndarray
    pulled_off: Optional[np.ndarray]
    pulled_src: Optional[np.ndarray]
    pulled_dst: Optional[np.ndarray]

    def pulled(self, g: int):
        a, b = int(self.pulled_off[g]), int(self.pulled_off[g + 1])
        return self.pulled_src[a:b], self.pulled_dst[a:b]


def analyze(corpus: Corpus, success: Sequence[int], failed: Sequence[int], diff_mode: int = 0,
            threads: int = 1, skip_pulls: bool = False, diff_labels: Optional[Sequence[int]] = None,
            diff_only: bool = False) -> OracleResult:
    """diff_labels: failGoals label set of every diff entry (the sharded reference mode's broadcast set).
    diff_only: only CreateNaiveDiffProv (run 0's post graph and the label sources are loaded; flags,
    chains, prototypes, pulls and triggers come back empty)."""
    skip_pulls = skip_pulls or diff_only
    L = lib()
    cs = corpus.c_struct()
    s = np.asarray(success, dtype=np.uint32)
    f = np.asarray(failed, dtype=np.uint32)
    dl = None if diff_labels is None else np.ascontiguousarray(diff_labels, dtype=np.uint32)
    dbuf = None if dl is None else (dl if len(dl) else np.zeros(1, np.uint32))  # non-NULL even when empty
    o = COpts(threads, s.ctypes.data if len(s) else None, len(s), f.ctypes.data if len(f) else None, len(f),
              diff_mode, int(skip_pulls), None if dbuf is None else dbuf.ctypes.data, 0 if dl is None else len(dl),
              int(diff_only))
    out = COut()
    rc = L.oracle_analyze(ctypes.byref(cs), ctypes.byref(o), ctypes.byref(out))
    try:
        if rc != 0:
            raise OracleError(rc, out.err.decode())
        W = out.words
        R = corpus.n_runs
        ch = _arr(ctypes.cast(out.chains, ctypes.POINTER(ctypes.c_uint32)), 5 * out.n_chains, np.uint32)
        res = OracleResult(
            flags=_arr(out.flags, out.V, np.uint8),
            chains=ch.reshape(-1, 5),
            proto_bits=_arr(out.proto_bits, R * W, np.uint32).reshape(-1, W),
            graph_tables=_arr(out.graph_tables, R * W, np.uint32).reshape(-1, W),
            reduce=_arr(out.reduce, 2 * out.n_tables + 4, np.uint32),
            achieved=out.achieved,
            inter=list(_arr(out.inter, out.n_inter, np.uint32)),
            union=list(_arr(out.uni, out.n_union, np.uint32)),
            run0=out.run0,
            v0=out.v0,
            diff_mask=_arr(out.diff_mask, out.n_entries * out.v0, np.uint8).reshape(out.n_entries, out.v0),
            missing=_arr(ctypes.cast(out.missing, ctypes.POINTER(ctypes.c_uint32)), 2 * out.n_missing,
                         np.uint32).reshape(-1, 2),
            pre_rows=_arr(out.pre_rows, 3 * out.n_pre, np.uint32).reshape(-1, 3),
            post_rows=_arr(out.post_rows, 2 * out.n_post, np.uint32).reshape(-1, 2),
            async_rules=_arr(out.async_rules, out.n_async, np.uint32),
            pulled_off=None if skip_pulls else _arr(out.pulled_off, out.n_graphs + 1, np.uint64),
            pulled_src=None,
            pulled_dst=None,
        )
        if not skip_pulls:
            n = int(res.pulled_off[-1])
            res.pulled_src = _arr(out.pulled_src, n, np.uint32)
            res.pulled_dst = _arr(out.pulled_dst, n, np.uint32)
        return res
    finally:
        L.oracle_free(ctypes.byref(out))
