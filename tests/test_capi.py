"""CPU: the C-ABI library loads and exports every symbol include/ssbls.h declares (no GPU calls)."""
import ctypes
import os

from safestakeoperator_amd import _lib
from safestakeoperator_amd.build import build


def test_library_exports_header_symbols():
    build(verbose=False)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = _lib.header_symbols()
    assert "ssb_threshold_aggregate_batch" in syms and len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/ssbls.h"


def test_create_without_gpu_fails_cleanly():
    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.ssb_create(ctypes.byref(h), 0)
    if rc == 0:  # a GPU is present (running on the box): fine, close it
        lib.ssb_destroy(h)
    else:
        assert rc in (-1, -2)
