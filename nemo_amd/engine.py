"""ctypes binding of libnemohip (include/nemohip.h) and a phase-level engine.

This is the Python equivalent of the cgo stub in INTEGRATION.md: it only moves
interned arrays across the C ABI and calls the gfx950 kernels.  There is no
fallback: if libnemohip.so is missing or no HIP device is present, every entry
point raises.
"""
from __future__ import annotations

import ctypes
import os
import re
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from .corpus import CChain, CMissing, Corpus

_HERE = os.path.dirname(os.path.abspath(__file__))
# NEMO_LIB: a variant build of the same library (A/B kernel experiments: tools/variants.sh)
LIB_PATH = os.environ.get("NEMO_LIB") or os.path.join(_HERE, "libnemohip.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "nemohip.h")
_LIB = None


class NemoError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[nemo {code}] {msg}")
        self.code = code
        self.msg = msg


class CTiming(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_uint64), ("ms", ctypes.c_double),
                ("bytes", ctypes.c_double), ("edges", ctypes.c_double)]


def header_symbols() -> List[str]:
    """Every function the C ABI header declares."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nemo_[a-z0-9_]+)\s*\(", txt)))


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libnemohip.so not built ({LIB_PATH}); run `make` or __graft_entry__.build()")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 under another file name,
        # so loading libnemohip (which resolves /opt/rocm's libamdhip64.so.7) before torch would leave
        # torch with a second runtime that cannot open the device ("No HIP GPUs are available").
        # Loading torch first makes libnemohip bind to the runtime torch already holds (same soname).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, sz, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int
        P = ctypes.POINTER
        sig = {
            "nemo_abi_version": ([], i32),
            "nemo_partition_runs": ([vp, u32, vp], i32),
            "nemo_ctx_create": ([i32, P(vp)], i32),
            "nemo_ctx_create_node": ([i32, vp, P(vp)], i32),
            "nemo_node_devices": ([vp, vp, i32], i32),
            "nemo_ctx_destroy": ([vp], None),
            "nemo_last_error": ([vp], ctypes.c_char_p),
            "nemo_set_stream": ([vp, vp], i32),
            "nemo_set_timing": ([vp, i32], i32),
            "nemo_set_timing_groups": ([vp, ctypes.c_char_p], i32),
            "nemo_set_option": ([vp, ctypes.c_char_p, ctypes.c_int64], i32),
            "nemo_load_corpus": ([vp, vp], i32),
            "nemo_host_register": ([vp, u64], i32),
            "nemo_host_unregister": ([vp], i32),
            "nemo_rebuild": ([vp], i32),
            "nemo_num_nodes": ([vp], u64),
            "nemo_num_edges": ([vp], u64),
            "nemo_mark_holds": ([vp], i32),
            "nemo_simplify": ([vp], i32),
            "nemo_reduce_len": ([vp], sz),
            "nemo_protos_partial": ([vp, vp, sz, vp], i32),
            "nemo_protos_stage": ([vp, vp], i32),
            "nemo_protos_finalize": ([vp, vp, P(u32), vp, P(u32), vp, P(u32), P(u64), P(u32)], i32),
            "nemo_fetch_reduce": ([vp, vp, u64], i32),
            "nemo_prototypes": ([vp, vp, sz, P(u32), vp, P(u32), vp, P(u32)], i32),
            "nemo_missing_from": ([vp, u32, vp, u32, vp, P(u32)], i32),
            "nemo_diffprov": ([vp, vp, sz, i32], i32),
            "nemo_diffprov_labels": ([vp, vp, sz, vp, u64], i32),
            "nemo_diffprov_host_labels": ([vp, vp, sz, vp, u64], i32),
            "nemo_goal_labels": ([vp, u32, i32, vp, u64], i32),
            "nemo_fetch_diff_mask": ([vp, u32, vp, u64], i32),
            "nemo_fetch_missing": ([vp, vp, u64, P(u64)], i32),
            "nemo_fetch_diff_masks": ([vp, vp, u64], i32),
            "nemo_diff_masks_view": ([vp, vp, vp, vp], i32),
            "nemo_triggers": ([vp], i32),
            "nemo_fetch_triggers": ([vp, vp, u64, P(u64), vp, u64, P(u64), vp, u64, P(u64)], i32),
            "nemo_fetch_node_flags": ([vp, u32, u32, vp, u64], i32),
            "nemo_fetch_chains": ([vp, vp, u64, P(u64)], i32),
            "nemo_stage_simplified": ([vp], i32),
            "nemo_simplified_view": ([vp, P(vp), P(vp), P(vp), P(u64)], i32),
            "nemo_fetch_run_tables": ([vp, i32, vp, u64], i32),
            "nemo_pull_edges": ([vp, i32], i32),
            "nemo_reduce_interpret": ([vp, u32, u32, P(u32), vp, P(u32), vp, P(u32)], i32),
            "nemo_pulled_count": ([vp, u32], u64),
            "nemo_fetch_pulled": ([vp, u32, vp, vp, u64, P(u64)], i32),
            "nemo_fetch_pulled_all": ([vp, vp, vp, vp, vp, u64, P(u64)], i32),
            "nemo_timings": ([vp, vp, u32, P(u32)], i32),
            "nemo_reset_timings": ([vp], i32),
            "nemo_synchronize": ([vp], i32),
            "nemo_debug_copy": ([vp, ctypes.c_char_p, vp, u64, u64], i32),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _LIB = L
    return _LIB


def _p(a: Optional[np.ndarray]):
    return None if a is None or a.size == 0 else a.ctypes.data


PIN_FIELDS = ("node_word", "label", "edge_src", "edge_dst", "id_rank")


def pin_corpus(corpus: Corpus) -> list:
    """Page-lock a corpus' large host arrays (nemo_host_register) so that every nemo_load_corpus of it
    uploads by DMA; returns the registered arrays for unpin_corpus."""
    L = lib()
    pinned = []
    for k in PIN_FIELDS:
        a = getattr(corpus, k, None)
        if a is None or a.size == 0 or not a.flags["C_CONTIGUOUS"]:
            continue
        if L.nemo_host_register(a.ctypes.data, a.nbytes) == 0:
            pinned.append(a)
    return pinned


def unpin_corpus(pinned: list) -> None:
    L = lib()
    for a in pinned:
        L.nemo_host_unregister(a.ctypes.data)


class Engine:
    """One libnemohip context bound to one HIP device."""

    def __init__(self, device: int = 0, devices: Optional[Sequence[int]] = None):
        """devices: a node context over these devices (nemo_ctx_create_node; repeats allowed)."""
        self.L = lib()
        h = ctypes.c_void_p()
        if devices is None:
            rc = self.L.nemo_ctx_create(device, ctypes.byref(h))
        else:
            d = np.ascontiguousarray(devices, dtype=np.int32)
            rc = self.L.nemo_ctx_create_node(len(d), d.ctypes.data, ctypes.byref(h))
        if rc != 0:
            raise NemoError(rc, "context creation failed (no HIP device?)")
        self.h = h
        self.corpus: Optional[Corpus] = None

    def devices(self) -> List[int]:
        out = np.zeros(64, np.int32)
        n = self.L.nemo_node_devices(self.h, out.ctypes.data, 64)
        return out[:n].tolist()

    def close(self) -> None:
        if self.h:
            self.L.nemo_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int) -> None:
        if rc != 0:
            raise NemoError(rc, self.L.nemo_last_error(self.h).decode())

    # ---- phases -------------------------------------------------------------------
    def set_stream(self, stream_handle: int) -> None:
        self._chk(self.L.nemo_set_stream(self.h, ctypes.c_void_p(stream_handle)))

    def set_option(self, name: str, value: int) -> None:
        self._chk(self.L.nemo_set_option(self.h, name.encode(), int(value)))

    def set_timing(self, on: bool = True) -> None:
        self._chk(self.L.nemo_set_timing(self.h, int(on)))

    def set_timing_groups(self, groups: Sequence[str] = ()) -> None:
        """Time only these groups (empty: every group)."""
        self._chk(self.L.nemo_set_timing_groups(self.h, ",".join(groups).encode()))

    def load(self, corpus: Corpus) -> None:
        cs = corpus.c_struct()
        self._chk(self.L.nemo_load_corpus(self.h, ctypes.byref(cs)))
        self.corpus = corpus

    def rebuild(self) -> None:
        self._chk(self.L.nemo_rebuild(self.h))

    def mark(self) -> None:
        self._chk(self.L.nemo_mark_holds(self.h))

    def simplify(self) -> None:
        self._chk(self.L.nemo_simplify(self.h))

    def reduce_len(self) -> int:
        return int(self.L.nemo_reduce_len(self.h))

    def protos_partial(self, success: Sequence[int], d_reduce_ptr: int) -> None:
        s = np.ascontiguousarray(success, dtype=np.uint32)
        self._chk(self.L.nemo_protos_partial(self.h, _p(s), len(s), ctypes.c_void_p(d_reduce_ptr)))

    def reduce_vector(self) -> np.ndarray:
        """nemo_fetch_reduce: the context's own reduction vector (after protos_partial(.., 0))."""
        n = self.reduce_len()
        out = np.zeros(n, np.uint32)
        self._chk(self.L.nemo_fetch_reduce(self.h, _p(out), n))
        return out

    def protos_stage(self, d_reduce_ptr: int) -> None:
        """nemo_protos_stage: queue the (reduced) vector's D2H now; protos_finalize then only waits."""
        self._chk(self.L.nemo_protos_stage(self.h, ctypes.c_void_p(d_reduce_ptr)))

    def protos_finalize(self, d_reduce_ptr: int):
        T = self.corpus.n_tables
        inter = np.zeros(T + 1, np.uint32)
        uni = np.zeros(T + 1, np.uint32)
        a, ni, nu, nr = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        ph = ctypes.c_uint64()
        self._chk(self.L.nemo_protos_finalize(self.h, ctypes.c_void_p(d_reduce_ptr), ctypes.byref(a), _p(inter),
                                              ctypes.byref(ni), _p(uni), ctypes.byref(nu), ctypes.byref(ph),
                                              ctypes.byref(nr)))
        return {"achieved": a.value, "inter": inter[:ni.value].tolist(), "union": uni[:nu.value].tolist(),
                "pre_holds": ph.value, "n_runs": nr.value}

    def prototypes(self, success: Sequence[int]):
        s = np.ascontiguousarray(success, dtype=np.uint32)
        T = self.corpus.n_tables
        inter = np.zeros(T + 1, np.uint32)
        uni = np.zeros(T + 1, np.uint32)
        a, ni, nu = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._chk(self.L.nemo_prototypes(self.h, _p(s), len(s), ctypes.byref(a), _p(inter), ctypes.byref(ni),
                                         _p(uni), ctypes.byref(nu)))
        return a.value, inter[:ni.value].tolist(), uni[:nu.value].tolist()

    def missing_from(self, failed_iter: int, proto: Sequence[int]) -> List[int]:
        p = np.ascontiguousarray(proto, dtype=np.uint32)
        out = np.zeros(len(p) + 1, np.uint32)
        n = ctypes.c_uint32()
        self._chk(self.L.nemo_missing_from(self.h, failed_iter, _p(p), len(p), _p(out), ctypes.byref(n)))
        return out[:n.value].tolist()

    def diffprov(self, failed: Sequence[int], mode: int = 0) -> None:
        f = np.ascontiguousarray(failed, dtype=np.uint32)
        self._chk(self.L.nemo_diffprov(self.h, _p(f), len(f), mode))

    def goal_labels(self, iteration: int, cond: int, d_out_ptr: int, cap: int) -> None:
        """nemo_goal_labels: [n, label...] of a run's goal labels into device memory."""
        self._chk(self.L.nemo_goal_labels(self.h, iteration, cond, ctypes.c_void_p(d_out_ptr), cap))

    def diffprov_labels(self, failed: Sequence[int], d_labels_ptr: int, cap: int) -> None:
        """nemo_diffprov_labels: reference-mode diff with a (broadcast) device label set."""
        f = np.ascontiguousarray(failed, dtype=np.uint32)
        self._chk(self.L.nemo_diffprov_labels(self.h, _p(f), len(f), ctypes.c_void_p(d_labels_ptr), cap))

    def diffprov_host_labels(self, failed: Sequence[int], labels: Sequence[int]) -> None:
        """nemo_diffprov_host_labels: reference-mode diff with a host label set."""
        f = np.ascontiguousarray(failed, dtype=np.uint32)
        lab = np.ascontiguousarray(labels, dtype=np.uint32)
        self._chk(self.L.nemo_diffprov_host_labels(self.h, _p(f), len(f), _p(lab), len(lab)))

    def triggers(self) -> None:
        self._chk(self.L.nemo_triggers(self.h))

    def pull(self, which: int) -> None:
        self._chk(self.L.nemo_pull_edges(self.h, which))

    def synchronize(self) -> None:
        self._chk(self.L.nemo_synchronize(self.h))

    # ---- fetches ------------------------------------------------------------------
    def flags(self, g_lo: int = 0, g_hi: Optional[int] = None) -> np.ndarray:
        c = self.corpus
        g_hi = c.n_graphs if g_hi is None else g_hi
        n = int(c.node_off[g_hi] - c.node_off[g_lo])
        out = np.zeros(max(n, 1), np.uint8)
        self._chk(self.L.nemo_fetch_node_flags(self.h, g_lo, g_hi, _p(out), n))
        return out[:n]

    def stage_simplified(self) -> None:
        """nemo_stage_simplified: async D2H of flags + chain (head, tail) pairs."""
        self._chk(self.L.nemo_stage_simplified(self.h))

    def simplified_view(self):
        """Zero-copy views of the staged results: (state[ceil(V/4)] u8 with 2 bits
        per node (NEMO_STATE_ALIVE | NEMO_STATE_HOLDS << 1), chain_off[G+1] u64,
        chain_ht[n, 2] u16 (or u32 when a graph has >= 65536 nodes)), valid until
        the next stage_simplified()."""
        vp = ctypes.c_void_p
        f, o, h, n, w = vp(), vp(), vp(), ctypes.c_uint64(), ctypes.c_int32()
        self._chk(self.L.nemo_simplified_view(self.h, ctypes.byref(f), ctypes.byref(o), ctypes.byref(h),
                                              ctypes.byref(n), ctypes.byref(w)))
        c = self.corpus
        V, G = int(c.node_off[-1]), c.n_graphs

        def view(ptr, ctype, count, dtype):
            if count == 0 or not ptr.value:
                return np.zeros(0, dtype)
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctype)), shape=(count,))

        state = view(f, ctypes.c_uint8, (V + 3) // 4, np.uint8)
        off = view(o, ctypes.c_uint64, G + 1, np.uint64)
        if w.value:
            ht = view(h, ctypes.c_uint32, 2 * n.value, np.uint32).reshape(-1, 2)
        else:
            ht = view(h, ctypes.c_uint16, 2 * n.value, np.uint16).reshape(-1, 2)
        return state, off, ht

    @staticmethod
    def unpack_state(state: np.ndarray, V: int):
        """(alive, holds) bool arrays of length V from the 2-bit staged node state."""
        bits = np.unpackbits(state, bitorder="little")[:2 * V].reshape(V, 2)
        return bits[:, 0].astype(bool), bits[:, 1].astype(bool)

    def chains(self) -> np.ndarray:
        n = ctypes.c_uint64()
        self._chk(self.L.nemo_fetch_chains(self.h, None, 0, ctypes.byref(n)))
        buf = (CChain * max(n.value, 1))()
        self._chk(self.L.nemo_fetch_chains(self.h, buf, n.value, ctypes.byref(n)))
        arr = np.frombuffer(buf, dtype=np.uint32).reshape(-1, 5)
        return arr[:n.value].copy()

    def run_tables(self, which: int) -> np.ndarray:
        c = self.corpus
        W = (c.n_tables + 31) // 32
        out = np.zeros(c.n_runs * W + 1, np.uint32)
        self._chk(self.L.nemo_fetch_run_tables(self.h, which, _p(out), c.n_runs * W))
        return out[:c.n_runs * W].reshape(c.n_runs, W)

    def diff_mask(self, entry: int) -> np.ndarray:
        c = self.corpus
        r0 = c.run_index(0)
        V0 = c.graph_size(2 * r0 + 1)
        out = np.zeros(max(V0, 1), np.uint8)
        self._chk(self.L.nemo_fetch_diff_mask(self.h, entry, _p(out), V0))
        return out[:V0]

    def diff_masks(self, n_entries: int) -> np.ndarray:
        c = self.corpus
        V0 = c.graph_size(2 * c.run_index(0) + 1)
        out = np.zeros(max(n_entries * V0, 1), np.uint8)
        self._chk(self.L.nemo_fetch_diff_masks(self.h, _p(out), n_entries * V0))
        return out[:n_entries * V0].reshape(n_entries, V0)

    def diff_masks_view(self) -> np.ndarray:
        """Zero-copy (n_entries, V0) view of the D masks in library-owned pinned memory
        (valid until the next diffprov)."""
        p, ne, v0 = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self.L.nemo_diff_masks_view(self.h, ctypes.byref(p), ctypes.byref(ne), ctypes.byref(v0)))
        n = ne.value * v0.value
        if n == 0 or not p.value:
            return np.zeros((ne.value, v0.value), np.uint8)
        buf = (ctypes.c_uint8 * n).from_address(p.value)
        return np.frombuffer(buf, np.uint8).reshape(ne.value, v0.value)

    def missing(self) -> np.ndarray:
        n = ctypes.c_uint64()
        self._chk(self.L.nemo_fetch_missing(self.h, None, 0, ctypes.byref(n)))
        buf = (CMissing * max(n.value, 1))()
        self._chk(self.L.nemo_fetch_missing(self.h, buf, n.value, ctypes.byref(n)))
        return np.frombuffer(buf, dtype=np.uint32).reshape(-1, 2)[:n.value].copy()

    def trigger_rows(self):
        npre, npost, nasync = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(self.L.nemo_fetch_triggers(self.h, None, 0, ctypes.byref(npre), None, 0, ctypes.byref(npost), None,
                                             0, ctypes.byref(nasync)))
        pre = np.zeros(3 * npre.value + 1, np.uint32)
        post = np.zeros(2 * npost.value + 1, np.uint32)
        asy = np.zeros(nasync.value + 1, np.uint32)
        self._chk(self.L.nemo_fetch_triggers(self.h, _p(pre), npre.value, ctypes.byref(npre), _p(post), npost.value,
                                             ctypes.byref(npost), _p(asy), nasync.value, ctypes.byref(nasync)))
        return (pre[:3 * npre.value].reshape(-1, 3), post[:2 * npost.value].reshape(-1, 2), asy[:nasync.value])

    def pulled(self, slot: int):
        n = ctypes.c_uint64()
        self._chk(self.L.nemo_fetch_pulled(self.h, slot, None, None, 0, ctypes.byref(n)))
        s = np.zeros(n.value + 1, np.uint32)
        d = np.zeros(n.value + 1, np.uint32)
        self._chk(self.L.nemo_fetch_pulled(self.h, slot, _p(s), _p(d), n.value, ctypes.byref(n)))
        return s[:n.value], d[:n.value]

    def pulled_all(self, n_slots: int):
        """(off[n_slots], cnt[n_slots], src, dst) of the last pull in one call (nemo_fetch_pulled_all)."""
        off = np.zeros(max(n_slots, 1), np.uint64)
        cnt = np.zeros(max(n_slots, 1), np.uint32)
        n = ctypes.c_uint64()
        self._chk(self.L.nemo_fetch_pulled_all(self.h, _p(off), _p(cnt), None, None, 0, ctypes.byref(n)))
        src = np.zeros(max(n.value, 1), np.uint32)
        dst = np.zeros(max(n.value, 1), np.uint32)
        self._chk(self.L.nemo_fetch_pulled_all(self.h, None, None, _p(src), _p(dst), n.value, ctypes.byref(n)))
        return off[:n_slots], cnt[:n_slots], src[:n.value], dst[:n.value]

    def debug_copy(self, name: str, offset: int, nbytes: int) -> np.ndarray:
        out = np.zeros(max(nbytes, 1), np.uint8)
        self._chk(self.L.nemo_debug_copy(self.h, name.encode(), _p(out), offset, nbytes))
        return out[:nbytes]

    def timings(self) -> Dict[str, dict]:
        n = ctypes.c_uint32()
        self._chk(self.L.nemo_timings(self.h, None, 0, ctypes.byref(n)))
        buf = (CTiming * max(n.value, 1))()
        self._chk(self.L.nemo_timings(self.h, buf, n.value, ctypes.byref(n)))
        return {buf[i].name.decode(): {"launches": buf[i].launches, "ms": buf[i].ms, "bytes": buf[i].bytes,
                                       "edges": buf[i].edges} for i in range(n.value)}

    def reset_timings(self) -> None:
        self._chk(self.L.nemo_reset_timings(self.h))


def reduce_interpret(vec: np.ndarray, n_tables: int, table_post: int):
    """nemo_reduce_interpret: inter/union/achvdCond from a (reduced) host vector; no device needed."""
    v = np.ascontiguousarray(vec, dtype=np.uint32)
    inter = np.zeros(n_tables + 1, np.uint32)
    uni = np.zeros(n_tables + 1, np.uint32)
    a, ni, nu = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    rc = lib().nemo_reduce_interpret(v.ctypes.data, n_tables, table_post, ctypes.byref(a), inter.ctypes.data,
                                     ctypes.byref(ni), uni.ctypes.data, ctypes.byref(nu))
    if rc != 0:
        raise NemoError(rc, "nemo_reduce_interpret")
    return a.value, inter[:ni.value].tolist(), uni[:nu.value].tolist()


@dataclass
class EngineResult:
    """The engine's results in the oracle's result layout (tests compare the two)."""

    flags: np.ndarray
    chains: np.ndarray
    proto_bits: np.ndarray
    graph_tables: np.ndarray
    achieved: int
    inter: List[int]
    union: List[int]
    diff_mask: np.ndarray
    missing: np.ndarray
    pre_rows: np.ndarray
    post_rows: np.ndarray
    async_rules: np.ndarray
    pulled: Optional[List[tuple]]


def analyze(corpus: Corpus, success: Sequence[int], failed: Sequence[int], diff_mode: int = 0,
            engine: Optional[Engine] = None, pulls: bool = True) -> EngineResult:
    """main.go:106-177's graph calls, in order, on the GPU."""
    eng = engine or Engine(0)
    eng.load(corpus)
    eng.mark()
    eng.simplify()
    achieved, inter, uni = eng.prototypes(success) if len(success) else (0, [], [])
    eng.diffprov(failed, diff_mode)
    eng.triggers()
    pulled = None
    if pulls:
        eng.pull(1)
        off, cnt, src, dst = eng.pulled_all(corpus.n_graphs)
        pulled = [(src[int(a):int(a) + int(n)], dst[int(a):int(a) + int(n)]) for a, n in zip(off, cnt)]
    has0 = 0 in set(int(x) for x in corpus.iteration)
    masks = np.stack([eng.diff_mask(e) for e in range(len(failed))]) if (has0 and len(failed)) else np.zeros((0, 0))
    pre, post, asy = eng.trigger_rows()
    res = EngineResult(flags=eng.flags(), chains=eng.chains(),
                       proto_bits=eng.run_tables(0) if len(success) else None,
                       graph_tables=eng.run_tables(1) if len(success) else None,
                       achieved=achieved, inter=inter, union=uni, diff_mask=masks, missing=eng.missing(),
                       pre_rows=pre, post_rows=post, async_rules=asy, pulled=pulled)
    return res
