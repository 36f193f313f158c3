"""ctypes loader of the plain-C oracle (oracle/bls_c.c -> oracle/_build/libblsoracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/ and by bench.py's cpu_baseline leg (multi-threaded CPU
baseline), never by the product path.  Build: `make -C oracle` (also run by
__graft_entry__.build())."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libblsoracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i32p = ctypes.POINTER(ctypes.c_int32)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        lib.bls_oracle_verify.argtypes = [_u8p, _u8p, _u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t]
        lib.bls_oracle_hash_to_g2.argtypes = [_u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p]
        lib.bls_oracle_hash_to_g2.restype = None
        lib.bls_oracle_threshold_aggregate.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _u8p, _u8p, _u64p, _u8p,
                                                       ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p, _u64p]
        lib.bls_oracle_threshold_batch.argtypes = [ctypes.c_size_t, _u32p, _u32p, _u8p, _u8p, _u64p, _u32p,
                                                   ctypes.c_size_t, _u8p, _u8p, ctypes.c_size_t, _u8p, _i32p, _u64p,
                                                   _u8p, ctypes.c_int, ctypes.c_int]
        lib.bls_oracle_threshold_batch_rlc.argtypes = [ctypes.c_size_t, _u32p, _u32p, _u8p, _u8p, _u64p, _u32p,
                                                       ctypes.c_size_t, _u8p, _u8p, ctypes.c_size_t, _u8p, _i32p, _u64p,
                                                       _u8p, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        lib.bls_oracle_sk_to_pk.argtypes = [_u8p, _u8p]
        lib.bls_oracle_pk_validate.argtypes = [_u8p, _u8p]
        lib.bls_oracle_sign.argtypes = [_u8p, _u8p, ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p]
        lib.bls_oracle_init()
        _lib = lib
    return _lib


def _b(x):
    a = (ctypes.c_uint8 * max(1, len(x))).from_buffer_copy(bytes(x) if len(x) else b"\0")
    return ctypes.cast(a, _u8p), a


DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"


def verify(pk48, sig96, msg, dst=DST_POP):
    lib = load()
    (p, _a), (s, _b2), (m, _c), (d, _d) = _b(pk48), _b(sig96), _b(msg), _b(dst)
    return bool(lib.bls_oracle_verify(p, s, m, len(msg), d, len(dst)))


def hash_to_g2(msg, dst=DST_POP):
    lib = load()
    out = (ctypes.c_uint8 * 192)()
    (m, _a), (d, _b2) = _b(msg), _b(dst)
    lib.bls_oracle_hash_to_g2(m, len(msg), d, len(dst), ctypes.cast(out, _u8p))
    return bytes(out)


def threshold_aggregate(t, sigs96, pks48, ids, msg, dst=DST_POP):
    """(status, out96 or err fields) as oracle/bls12_381.py:threshold_aggregate (packed inputs)."""
    lib = load()
    n = len(sigs96)
    ids_a = (ctypes.c_uint64 * max(1, n))(*ids)
    out = (ctypes.c_uint8 * 96)()
    err = (ctypes.c_uint64 * 2)()
    (s, _a), (p, _b2), (m, _c), (d, _d) = _b(b"".join(sigs96)), _b(b"".join(pks48)), _b(msg), _b(dst)
    st = lib.bls_oracle_threshold_aggregate(t, n, s, p, ctypes.cast(ids_a, _u64p), m, len(msg), d, len(dst),
                                            ctypes.cast(out, _u8p), ctypes.cast(err, _u64p))
    return st, (bytes(out) if st == 0 else tuple(err))


def threshold_batch(share_off, t, sigs96, pks48, ids, job_root, roots, threads, dst=DST_POP, verify_all=False):
    """All jobs of a packed batch on `threads` POSIX threads; returns (out96, status, err, verdicts).
    verify_all=False: the reference's scan (stops at the t-th valid share); True: every share is
    verified (the device engine's work), the combined signature is the same."""
    import numpy as np
    lib = load()
    J = len(t)
    off = np.ascontiguousarray(np.asarray(share_off, dtype=np.uint32))
    tt = np.ascontiguousarray(np.asarray(t, dtype=np.uint32))
    jr = np.ascontiguousarray(np.asarray(job_root, dtype=np.uint32))
    idv = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64))
    sg = np.frombuffer(sigs96, dtype=np.uint8)
    pk = np.frombuffer(pks48, dtype=np.uint8)
    rt = np.frombuffer(b"".join(roots), dtype=np.uint8)
    out = np.zeros((J, 96), dtype=np.uint8)
    st = np.zeros(J, dtype=np.int32)
    err = np.zeros((J, 2), dtype=np.uint64)
    ver = np.zeros(max(1, int(off[-1]) if J else 0), dtype=np.uint8)
    d, _keep = _b(dst)
    lib.bls_oracle_threshold_batch(J, off.ctypes.data_as(_u32p), tt.ctypes.data_as(_u32p), sg.ctypes.data_as(_u8p),
                                   pk.ctypes.data_as(_u8p), idv.ctypes.data_as(_u64p), jr.ctypes.data_as(_u32p),
                                   len(roots), rt.ctypes.data_as(_u8p), d, len(dst), out.ctypes.data_as(_u8p),
                                   st.ctypes.data_as(_i32p), err.ctypes.data_as(_u64p), ver.ctypes.data_as(_u8p),
                                   1 if verify_all else 0, int(threads))
    return out, st, err, ver


def threshold_batch_rlc(share_off, t, sigs96, pks48, ids, job_root, roots, threads, dst=DST_POP, seed=0x5AFE57A4E):
    """The RLC-batched CPU path (bls_oracle_threshold_batch_rlc): one multi-pairing and one final
    exponentiation for the whole batch, per-share verification only if it fails.  Returns
    (out96, status, err, verdicts, batch_ok)."""
    import numpy as np
    lib = load()
    J = len(t)
    off = np.ascontiguousarray(np.asarray(share_off, dtype=np.uint32))
    tt = np.ascontiguousarray(np.asarray(t, dtype=np.uint32))
    jr = np.ascontiguousarray(np.asarray(job_root, dtype=np.uint32))
    idv = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64))
    sg = np.frombuffer(sigs96, dtype=np.uint8)
    pk = np.frombuffer(pks48, dtype=np.uint8)
    rt = np.frombuffer(b"".join(roots), dtype=np.uint8)
    out = np.zeros((J, 96), dtype=np.uint8)
    st = np.zeros(J, dtype=np.int32)
    err = np.zeros((J, 2), dtype=np.uint64)
    ver = np.zeros(max(1, int(off[-1]) if J else 0), dtype=np.uint8)
    ok = ctypes.c_int(0)
    d, _keep = _b(dst)
    rc = lib.bls_oracle_threshold_batch_rlc(J, off.ctypes.data_as(_u32p), tt.ctypes.data_as(_u32p), sg.ctypes.data_as(_u8p),
                                            pk.ctypes.data_as(_u8p), idv.ctypes.data_as(_u64p), jr.ctypes.data_as(_u32p),
                                            len(roots), rt.ctypes.data_as(_u8p), d, len(dst), out.ctypes.data_as(_u8p),
                                            st.ctypes.data_as(_i32p), err.ctypes.data_as(_u64p), ver.ctypes.data_as(_u8p),
                                            seed & (2**64 - 1), int(threads), ctypes.byref(ok))
    if rc != 0:
        raise RuntimeError("bls_oracle_threshold_batch_rlc: %d" % rc)
    return out, st, err, ver, bool(ok.value)


def sk_to_pk(sk32be):
    """bls::SecretKey::deserialize(32 B big-endian) -> public_key().serialize() (48 B), or None
    for a key outside (0, r)."""
    lib = load()
    out = (ctypes.c_uint8 * 48)()
    s, _a = _b(sk32be)
    return bytes(out) if lib.bls_oracle_sk_to_pk(s, ctypes.cast(out, _u8p)) else None


def pk_validate(pk48):
    """bls::PublicKey::deserialize: (valid, recompressed 48 B)."""
    lib = load()
    out = (ctypes.c_uint8 * 48)()
    p, _a = _b(pk48)
    ok = bool(lib.bls_oracle_pk_validate(p, ctypes.cast(out, _u8p)))
    return ok, bytes(out)


def sign(sk32be, msg, dst=DST_POP):
    """bls::SecretKey::sign (src/node/dvfcore.rs:241-243): [sk] hash_to_G2(msg) compressed (96 B),
    or None for a key outside (0, r)."""
    lib = load()
    out = (ctypes.c_uint8 * 96)()
    s, _a = _b(sk32be)
    m, _m = _b(msg)
    d, _d = _b(dst)
    return bytes(out) if lib.bls_oracle_sign(s, m, len(msg), d, len(dst), ctypes.cast(out, _u8p)) else None
