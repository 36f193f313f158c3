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


def test_pipeline_config_guard():
    """ssb_check_pipeline_config (the rule ssb_set_pipeline_depth / ssb_set_slot_streams enforce):
    24 one-stream slots and 5 three-stream slots are accepted, 8 x 3 (which exhausted the per-queue
    scratch reservations on an MI355X) and out-of-range values are refused."""
    lib = _lib.load()
    ok = lambda d, s: lib.ssb_check_pipeline_config(d, s) == 0
    assert ok(1, 1) and ok(14, 1) and ok(20, 1) and ok(24, 1) and ok(1, 3) and ok(5, 3)
    assert not ok(8, 3) and not ok(6, 3) and not ok(25, 1) and not ok(0, 1) and not ok(4, 2)
    # a null context is refused before any HIP call
    assert lib.ssb_set_pipeline_depth(None, 4) == -1 and lib.ssb_set_slot_streams(None, 3) == -1
