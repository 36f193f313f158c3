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
    20 one-stream slots and 5 three-stream slots are accepted; 8 x 3 and 24 x 1 (which exhausted the
    per-queue scratch reservations on an MI355X) and out-of-range values are refused."""
    lib = _lib.load()
    ok = lambda d, s: lib.ssb_check_pipeline_config(d, s) == 0
    assert ok(1, 1) and ok(14, 1) and ok(20, 1) and ok(1, 3) and ok(5, 3)
    assert not ok(8, 3) and not ok(6, 3) and not ok(21, 1) and not ok(24, 1) and not ok(25, 1) and not ok(0, 1) and not ok(4, 2)
    # a null context is refused before any HIP call
    assert lib.ssb_set_pipeline_depth(None, 4) == -1 and lib.ssb_set_slot_streams(None, 3) == -1


def _capi_input(cases):
    roots = []
    for c in cases:
        if c["root"] not in roots:
            roots.append(c["root"])
    lines = ["%d %d" % (len(cases), len(roots))] + roots
    for c in cases:
        lines.append("%d %d %d" % (c["t"], len(c["sigs"]), roots.index(c["root"])))
        lines += ["%s %s %d" % (s, p, i) for s, p, i in zip(c["sigs"], c["pks"], c["ids"])]
    return "\n".join(lines) + "\n"


def test_plain_c_caller_builds_and_rejects_bad_input():
    """tests/native/capi_golden.c: gcc against include/ssbls.h alone, linked to libssbls.so; on a
    malformed input it stops before touching the device."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "native"))
    from build_capi import build_capi
    build(verbose=False)
    exe = build_capi()
    r = subprocess.run([exe], input="0 0\n", capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "bad header" in r.stderr


import pytest  # noqa: E402


@pytest.mark.gpu
def test_plain_c_caller_golden_cases():
    """The drop-in boundary from plain C (no Python in the call path): every golden threshold case
    in one ssb_threshold_aggregate_batch call, statuses / error fields / combined signatures / share
    verdicts == tests/golden/threshold_cases.json, and ssb_verify_batch's verdicts == the same."""
    import json
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "native"))
    from build_capi import BIN, build_capi
    exe = BIN if os.path.exists(BIN) else build_capi()
    with open(os.path.join(os.path.dirname(__file__), "golden", "threshold_cases.json")) as f:
        cases = json.load(f)["cases"]
    r = subprocess.run([exe], input=_capi_input(cases), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = r.stdout.split("\n")
    want_ver = ""
    for j, c in enumerate(cases):
        f = out[j].split()
        assert f[0] == "job" and int(f[1]) == j
        assert int(f[2]) == c["expected_status"], c["name"]
        if c["expected_status"] == 0:
            assert f[5] == c["expected_sig"] == c["master_sig"], c["name"]
        elif c["expected_status"] in (2, 4):
            assert [int(f[3]), int(f[4])] == c["expected_payload"], c["name"]
        want_ver += "".join("1" if v else "0" for v in c["share_verdicts"])
    assert out[len(cases)] == "verdicts " + want_ver
    assert out[len(cases) + 1] == "verify " + want_ver


def test_batch_kernels_fit_the_queue_primer():
    """Build guard (safestakeoperator_amd/build.py check_private_segments): every kernel the batch
    path can launch on a slot queue has a private segment <= k_scratch_prime's per-lane array, so a
    slot queue never has to grow its scratch while other queues run (HSA_STATUS_ERROR_OUT_OF_RESOURCES,
    round 2); the larger ones are only launched by synchronous entry points."""
    import glob
    from safestakeoperator_amd import build as b
    build(verbose=False)
    objs = sorted(glob.glob(os.path.join(b.OBJDIR, "*.o")))
    res = b.check_private_segments(objs)
    limit = b._prime_bytes()
    for k in ("k_decode_count", "k_subgroup_map", "k_msm_bucket2", "k_msm_window2", "k_miller_pairs", "k_miller_final",
              "k_fp12_prod8", "k_final_lane", "k_fb_rlc", "k_fb_excl", "k_fb_root", "k_fb_single", "k_fb_level", "k_select_combine", "k_combine_terms_gls",
              "k_combine_sum", "k_share_map"):
        assert k in res and res[k]["private"] <= limit, (k, res.get(k))
