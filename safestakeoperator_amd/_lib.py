"""ctypes binding of libssbls.so (include/ssbls.h).  There is no CPU fallback: if the library or
a GPU is missing, every entry point raises."""
import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
# SSB_LIB_VARIANT=name loads the experiment build libssbls_<name>.so (safestakeoperator_amd/build.py)
_VARIANT = os.environ.get("SSB_LIB_VARIANT", "")
LIB_PATH = os.path.join(HERE, "libssbls%s.so" % ("_" + _VARIANT if _VARIANT else ""))
HEADER = os.path.join(HERE, "..", "include", "ssbls.h")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_sz = ctypes.c_size_t
_ctx = ctypes.c_void_p

SIGNATURES = {
    "ssb_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int]),
    "ssb_destroy": (None, [_ctx]),
    "ssb_last_error": (ctypes.c_char_p, [_ctx]),
    "ssb_check_pipeline_config": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "ssb_hw_queue_budget": (ctypes.c_int, []),
    "ssb_set_pipeline_depth": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "ssb_set_slot_streams": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "ssb_slot_stream": (ctypes.c_void_p, [_ctx, ctypes.c_int]),
    "ssb_debug_hold": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "ssb_set_rlc_deterministic": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "ssb_last_kernel_ms": (ctypes.c_int, [_ctx, ctypes.c_char_p, ctypes.POINTER(ctypes.c_float)]),
    "ssb_kernel_timing": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "ssb_kernel_time": (ctypes.c_int, [_ctx, ctypes.c_char_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)]),
    "ssb_hash_to_g2": (ctypes.c_int, [_ctx, _sz, _u8p, _u8p, _sz, _u8p]),
    "ssb_hash_to_g2_msgs": (ctypes.c_int, [_ctx, _sz, _u8p, _u8p, _u8p, _sz, _u8p]),
    "ssb_verify_batch": (ctypes.c_int, [_ctx, _sz, _u8p, _u8p, _u32p, _sz, _u8p, _u8p, _sz, ctypes.c_uint64, _u8p]),
    "ssb_threshold_aggregate_batch": (ctypes.c_int, [_ctx, _sz, _u32p, _u32p, _u8p, _u8p, _u64p, _u32p, _sz, _u8p,
                                                     _u8p, _sz, ctypes.c_uint64, _u8p, _i32p, _u64p, _u8p]),
    "ssb_threshold_aggregate_batch_dev": (ctypes.c_int, [_ctx, _sz, _sz, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p, _sz, ctypes.c_void_p, _u8p, _sz,
                                                         ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_threshold_aggregate_batch_submit": (ctypes.c_int, [_ctx, _sz, _u32p, _u32p, _u8p, _u8p, _u64p, _u32p, _sz,
                                                            _u8p, _u8p, _sz, ctypes.c_uint64, _u8p, _i32p, _u64p, _u8p,
                                                            ctypes.POINTER(ctypes.c_uint64)]),
    "ssb_threshold_aggregate_batch_cached_submit": (ctypes.c_int, [_ctx, _sz, _u32p, _u32p, _u8p, _u32p, _u64p, _u32p,
                                                                   _sz, _u8p, _u8p, _sz, ctypes.c_uint64, _u8p, _i32p,
                                                                   _u64p, _u8p, ctypes.POINTER(ctypes.c_uint64)]),
    "ssb_batch_wait": (ctypes.c_int, [_ctx, ctypes.c_uint64]),
    "ssb_pk_cache_set": (ctypes.c_int, [_ctx, _sz, _u8p]),
    "ssb_pk_cache_add": (ctypes.c_int, [_ctx, _sz, _u8p, _u32p]),
    "ssb_collector_create": (ctypes.c_int, [_ctx, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "ssb_collector_create2": (ctypes.c_int, [_ctx, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                             ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "ssb_collector_destroy": (None, [ctypes.c_void_p]),
    "ssb_collector_submit_wire": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_collector_register_keys": (ctypes.c_int, [ctypes.c_void_p, _sz, _u8p, _u32p]),
    "ssb_collector_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_collector_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_collector_flush": (ctypes.c_int, [ctypes.c_void_p]),
    "ssb_collector_stats": (ctypes.c_int, [ctypes.c_void_p, _u64p, _u64p, _u64p]),
    "ssb_collector_profile": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), _u64p]),
    "ssb_signer_create": (ctypes.c_int, [_ctx, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "ssb_signer_destroy": (None, [ctypes.c_void_p]),
    "ssb_signer_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_signer_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_signer_flush": (ctypes.c_int, [ctypes.c_void_p]),
    "ssb_signer_stats": (ctypes.c_int, [ctypes.c_void_p, _u64p, _u64p]),
    "ssb_verify_batch_dev": (ctypes.c_int, [_ctx, _sz, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _sz,
                                            ctypes.c_void_p, _u8p, _sz, ctypes.c_uint64, ctypes.c_void_p,
                                            ctypes.c_void_p]),
    "ssb_verify_batch_cached_dev": (ctypes.c_int, [_ctx, _sz, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, _sz,
                                                   ctypes.c_void_p, _u8p, _sz, ctypes.c_uint64, ctypes.c_void_p,
                                                   ctypes.c_void_p]),
    "ssb_threshold_aggregate_batch_cached_dev": (ctypes.c_int, [_ctx, _sz, _sz, ctypes.c_void_p, ctypes.c_void_p,
                                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                                ctypes.c_void_p, _sz, ctypes.c_void_p, _u8p, _sz,
                                                                ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_threshold_aggregate_batch_wire_cached_dev": (ctypes.c_int, [_ctx, _sz, _sz, ctypes.c_void_p, ctypes.c_void_p,
                                                                     ctypes.c_void_p, _sz, ctypes.c_void_p,
                                                                     ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_void_p,
                                                                     _u8p, _sz, ctypes.c_uint64, ctypes.c_void_p,
                                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                                     ctypes.c_void_p, ctypes.c_void_p]),
    "ssb_unsafe_aggregate_batch": (ctypes.c_int, [_ctx, _sz, _u32p, _u8p, _u64p, _u8p, _i32p]),
    "ssb_sign_batch": (ctypes.c_int, [_ctx, _sz, _u8p, _u32p, _sz, _u8p, _u8p, _sz, _u8p]),
    "ssb_sk_to_pk_batch": (ctypes.c_int, [_ctx, _sz, _u8p, _u8p]),
    "ssb_pk_validate_batch": (ctypes.c_int, [_ctx, _sz, _u8p, _u8p, _u8p]),
    "ssb_lagrange_coeffs": (ctypes.c_int, [_ctx, _sz, _u64p, _u8p]),
    "ssb_feldman_verify_batch": (ctypes.c_int, [_ctx, _sz, _sz, _u8p, _u64p, _u8p, _u8p, _u8p]),
    "ssb_dleq_verify_batch": (ctypes.c_int, [_ctx, _sz, _u8p, _u8p, _u8p, _u8p]),
    "ssb_decode_wire_sigs": (ctypes.c_int, [_ctx, _sz, _u8p, _sz, _u8p, _i32p]),
    "ssb_decode_wire_sigs_dev": (ctypes.c_int, [_ctx, _sz, ctypes.c_void_p, _sz, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_void_p]),
}


class JobResult(ctypes.Structure):
    """ssb_job_result (include/ssbls.h): one collector job's outcome."""
    _fields_ = [("sig96", ctypes.c_uint8 * 96), ("err", ctypes.c_uint64 * 2), ("verdicts", ctypes.c_uint64),
                ("status", ctypes.c_int32), ("rc", ctypes.c_int32), ("n_shares", ctypes.c_uint32),
                ("done", ctypes.c_uint32), ("absent", ctypes.c_uint64)]


# ssb_job_done_fn: void (*)(void* user, const ssb_job_result* result)
JOB_DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(JobResult))


class SignResult(ctypes.Structure):
    """ssb_sign_result (include/ssbls.h): one local signature from the signing window."""
    _fields_ = [("sig96", ctypes.c_uint8 * 96), ("rc", ctypes.c_int32), ("done", ctypes.c_uint32)]


# ssb_sign_done_fn: void (*)(void* user, const ssb_sign_result* result)
SIGN_DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(SignResult))


def header_symbols():
    """Every function declared in include/ssbls.h."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void\*?|const char\*)\s+(ssb_\w+)\s*\(", txt, re.M)))


_LIB = None


def load():
    global _LIB
    if _LIB is not None:
        return _LIB
    # One HIP runtime per process: PyTorch (device memory, streams, RCCL for the callers) ships its
    # own libamdhip64; load it first so libssbls.so binds to the same runtime.  (With the library
    # loaded first, a later torch.cuda init in the same process finds "No HIP GPUs".)  A C-ABI-only
    # caller that never uses torch sets SSB_NO_TORCH=1 and skips the import; a broken torch install
    # is logged, not fatal -- the library itself does not need torch.
    if os.environ.get("SSB_NO_TORCH", "") not in ("1", "true"):
        try:
            import torch  # noqa: F401
        except Exception as e:  # ImportError, or OSError / RuntimeError from a broken ROCm install
            import logging
            logging.getLogger(__name__).warning("torch not loaded before libssbls.so (%s); a later torch.cuda "
                                                "init in this process may not see the GPU", e)
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("libssbls.so is not built (run `python -m safestakeoperator_amd.build`); "
                           "there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def buf(b):
    """bytes/bytearray/numpy -> ctypes uint8 pointer (kept alive by the caller's object)."""
    import numpy as np
    a = np.ascontiguousarray(np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else b)
    return a, a.ctypes.data_as(_u8p)
