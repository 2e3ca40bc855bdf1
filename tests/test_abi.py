"""CPU-side checks of the drop-in boundary: the library builds for gfx950, loads, and exports
every entry point include/nemohip.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import subprocess

import pytest

from nemo_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_declares_entry_points():
    syms = E.header_symbols()
    for s in ("nemo_ctx_create", "nemo_load_corpus", "nemo_mark_holds", "nemo_simplify", "nemo_protos_partial",
              "nemo_protos_finalize", "nemo_diffprov", "nemo_triggers", "nemo_pull_edges", "nemo_timings"):
        assert s in syms


def test_library_exports_every_header_symbol():
    if not os.path.exists(E.LIB_PATH):
        subprocess.run(["make", "-s", "-C", ROOT, "nemo_amd/libnemohip.so"], check=True)
    L = ctypes.CDLL(E.LIB_PATH)
    missing = [s for s in E.header_symbols() if not hasattr(L, s)]
    assert not missing, f"symbols declared in nemohip.h but not exported: {missing}"
    assert L.nemo_abi_version() == 1


def test_library_is_gfx950_code_object():
    blob = open(E.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob, "libnemohip.so carries no gfx950 code object"


def test_no_cpu_fallback_when_no_gpu():
    # the product path must fail loudly, never compute on the host
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(E.NemoError):
        E.Engine(0)
