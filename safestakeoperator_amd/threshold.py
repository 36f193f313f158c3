"""Host-side mirror of SafeStake's threshold-signature API, backed by the MI355X engine.

Reference interface (paths in the SafeStakeOperator repository):
  * trait TThresholdSignature            src/crypto/generic_threshold.rs:15-23
  * GenericThresholdSignature<T>         src/crypto/generic_threshold.rs:25-180
      - new / infinity / threshold       :30-45
      - threshold_aggregate              :132-175  (selection + error order reproduced exactly)
      - unsafe_aggregate                 :177-179 -> src/crypto/impls/blst.rs:67-87
  * DvfError                             src/utils/error.rs:12-60
  * backend selection define_mod!        src/crypto/mod.rs:7-22  (here: the HIP engine)

Added, as SURVEY.md §8b proposes: `threshold_aggregate_batch(jobs)`, the batched entry point a
per-slot collector calls once for every (validator, signing-root) job of a slot.

Every compute call goes through libssbls.so on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import secrets
from dataclasses import dataclass
from typing import List, Optional, Sequence, Union, Tuple

import numpy as np

from . import _lib

WIRE_SIG_BYTES = 202   # bincode(bls::Signature): u64 length 194 + "0x" + 192 hex digits
DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"  # src/crypto/impls/blst.rs:11
INFINITY_SIGNATURE = bytes([0xC0]) + bytes(95)          # bls::INFINITY_SIGNATURE

SSB_OK = 0
DVF_OK, DVF_DIFFERENT_LENGTH, DVF_INSUFFICIENT_SIGNATURES, DVF_INVALID_OPERATOR_ID, \
    DVF_INSUFFICIENT_VALID_SIGNATURES, DVF_BAD_SIGNATURE_ENCODING, DVF_INVALID_JOB, DVF_ENGINE_ERROR = range(8)
MAX_T = 64


def _rlc_seed(seed: Optional[int]) -> int:
    """The rlc_seed argument: a fresh random value unless the caller passes one.  The library
    draws its own 256-bit key per call from getrandom() and only XORs this in (include/ssbls.h),
    so the scalars stay secret either way; a fixed seed matters only on an engine switched to
    set_rlc_deterministic(True) (tests, reproducible profiling)."""
    return (secrets.randbits(64) if seed is None else int(seed)) & (2**64 - 1)


# ------------------------------------------------------------------------------------------
# DvfError (src/utils/error.rs:12-60), the variants the threshold path can return
# ------------------------------------------------------------------------------------------
class DvfError(Exception):
    tag = -1

    def __eq__(self, other):
        return type(self) is type(other) and self.args == other.args

    def __hash__(self):
        return hash((type(self).__name__, self.args))


class DifferentLength(DvfError):
    tag = DVF_DIFFERENT_LENGTH

    def __init__(self, x, y):
        super().__init__(int(x), int(y))
        self.x, self.y = int(x), int(y)


class InsufficientSignatures(DvfError):
    tag = DVF_INSUFFICIENT_SIGNATURES

    def __init__(self, got, expected):
        super().__init__(int(got), int(expected))
        self.got, self.expected = int(got), int(expected)


class InvalidOperatorId(DvfError):
    tag = DVF_INVALID_OPERATOR_ID

    def __init__(self, id):  # noqa: A002 (reference field name)
        super().__init__(int(id))
        self.id = int(id)


class InsufficientValidSignatures(DvfError):
    tag = DVF_INSUFFICIENT_VALID_SIGNATURES

    def __init__(self, got, expected):
        super().__init__(int(got), int(expected))
        self.got, self.expected = int(got), int(expected)


class BadSignatureEncoding(DvfError):
    """unsafe_aggregate on bytes that do not decode (the reference would panic in unwrap())."""
    tag = DVF_BAD_SIGNATURE_ENCODING


def _error_from(status: int, e0: int, e1: int) -> Optional[DvfError]:
    if status == DVF_OK:
        return None
    if status == DVF_INSUFFICIENT_SIGNATURES:
        return InsufficientSignatures(e0, e1)
    if status == DVF_INVALID_OPERATOR_ID:
        return InvalidOperatorId(e0)
    if status == DVF_INSUFFICIENT_VALID_SIGNATURES:
        return InsufficientValidSignatures(e0, e1)
    if status == DVF_BAD_SIGNATURE_ENCODING:
        return BadSignatureEncoding()
    if status == DVF_DIFFERENT_LENGTH:
        return DifferentLength(e0, e1)
    if status == DVF_INVALID_JOB:      # _dev callers only (t or share range outside the limits)
        return ValueError("job outside the engine's limits: t = %d, %d shares" % (e0, e1))
    if status == DVF_ENGINE_ERROR:     # the job's batch did not complete: never a reference result
        return RuntimeError("engine error: the batch did not complete (code %d)" % (e0 - (1 << 64) if e0 >= 1 << 63 else e0))
    raise RuntimeError("unknown status %d" % status)


# ------------------------------------------------------------------------------------------
# Engine: one ssb_ctx (device, stream, workspace)
# ------------------------------------------------------------------------------------------
class Engine:
    def __init__(self, device: int = 0):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        rc = self._lib.ssb_create(ctypes.byref(h), int(device))
        if rc != SSB_OK:
            raise RuntimeError("ssb_create(device=%d) failed with %d (no usable GPU?)" % (device, rc))
        self._h = h
        self.device = device
        # host-buffer batches not yet waited for, by ticket: the library writes their outputs into
        # the PendingBatch's arrays when the batch is delivered -- possibly inside a later call that
        # reuses the slot (include/ssbls.h, ssb_batch_wait LIFETIME) -- so they stay alive here
        self._pending = {}

    def close(self):
        if getattr(self, "_h", None):
            self._lib.ssb_destroy(self._h)   # (delivers every pending batch first)
            self._h = None
            self._pending = {}

    def _delivered_all(self):
        """Every pending host batch has been delivered by the library (set_pipeline_depth,
        set_slot_streams, pk_cache_set / pk_cache_add, kernel_timing deliver them all)."""
        self._pending.clear()

    def set_pipeline_depth(self, depth: int):
        self._check(self._lib.ssb_set_pipeline_depth(self._h, int(depth)), "ssb_set_pipeline_depth")
        self._delivered_all()

    def set_slot_streams(self, streams: int):
        self._check(self._lib.ssb_set_slot_streams(self._h, int(streams)), "ssb_set_slot_streams")
        self._delivered_all()

    def pk_cache_set(self, pks) -> None:
        """ssb_pk_cache_set: the decoded-key table = these keys, row i = key i."""
        buf = np.frombuffer(b"".join(pks) if not isinstance(pks, (bytes, bytearray, np.ndarray)) else pks, dtype=np.uint8)
        if buf.size % 48:
            raise ValueError("public keys are 48 bytes")
        self._check(self._lib.ssb_pk_cache_set(self._h, buf.size // 48, buf.ctypes.data_as(_lib._u8p)), "ssb_pk_cache_set")
        self._delivered_all()

    def pk_cache_add(self, pks) -> np.ndarray:
        """ssb_pk_cache_add: register keys (a committee's operator keys), return their stable rows."""
        buf = np.frombuffer(b"".join(pks) if not isinstance(pks, (bytes, bytearray, np.ndarray)) else pks, dtype=np.uint8)
        if buf.size % 48:
            raise ValueError("public keys are 48 bytes")
        n = buf.size // 48
        idx = np.zeros(max(n, 1), dtype=np.uint32)
        if n:
            self._check(self._lib.ssb_pk_cache_add(self._h, n, buf.ctypes.data_as(_lib._u8p), idx.ctypes.data_as(_lib._u32p)),
                        "ssb_pk_cache_add")
        return idx[:n]

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def _check(self, rc, what):
        if rc != SSB_OK:
            msg = self._lib.ssb_last_error(self._h)
            raise RuntimeError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))

    def set_rlc_deterministic(self, on: bool):
        """TESTS ONLY: derive the RLC scalars from the caller's seed alone (ssb_set_rlc_deterministic).
        Scalars that are a public function of the seed let two colluding senders cancel errors in
        the batch sums; the default (off) draws a secret key from the OS for every call."""
        self._check(self._lib.ssb_set_rlc_deterministic(self._h, 1 if on else 0), "ssb_set_rlc_deterministic")

    def last_kernel_ms(self, name: str) -> float:
        ms = ctypes.c_float()
        self._check(self._lib.ssb_last_kernel_ms(self._h, name.encode(), ctypes.byref(ms)), "ssb_last_kernel_ms")
        return float(ms.value)

    def kernel_timing(self, on, last_only: bool = False):
        """Start (accumulate every launch, or with last_only the last launch of each stage for
        last_kernel_ms) or stop the engine's event timing; off by default."""
        self._check(self._lib.ssb_kernel_timing(self._h, (2 if last_only else 1) if on else 0), "ssb_kernel_timing")
        self._delivered_all()

    def kernel_time(self, name: str):
        """(total ms, launches) accumulated since kernel_timing(True)."""
        ms, n = ctypes.c_float(), ctypes.c_int()
        self._check(self._lib.ssb_kernel_time(self._h, name.encode(), ctypes.byref(ms), ctypes.byref(n)),
                    "ssb_kernel_time")
        return float(ms.value), int(n.value)

    # --- primitives -------------------------------------------------------------------------
    def hash_to_g2(self, msgs: Sequence[bytes], dst: bytes = DST) -> List[bytes]:
        """hash_to_G2 (RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_) of messages of at most 32 bytes
        (signing roots are 32): 192-byte uncompressed points."""
        n = len(msgs)
        if n == 0:
            return []
        if any(len(x) > 32 for x in msgs):
            raise ValueError("messages are at most 32 bytes")
        out = np.zeros(192 * n, dtype=np.uint8)
        d, dp = _lib.buf(dst)
        if all(len(x) == 32 for x in msgs):
            m = np.frombuffer(b"".join(msgs), dtype=np.uint8)
            rc = self._lib.ssb_hash_to_g2(self._h, n, m.ctypes.data_as(_lib._u8p), dp, len(dst), out.ctypes.data_as(_lib._u8p))
        else:
            m = np.frombuffer(b"".join(bytes(x).ljust(32, b"\0") for x in msgs), dtype=np.uint8)
            ln = np.asarray([len(x) for x in msgs], dtype=np.uint8)
            rc = self._lib.ssb_hash_to_g2_msgs(self._h, n, m.ctypes.data_as(_lib._u8p), ln.ctypes.data_as(_lib._u8p), dp,
                                               len(dst), out.ctypes.data_as(_lib._u8p))
        self._check(rc, "ssb_hash_to_g2")
        return [out[192 * i:192 * (i + 1)].tobytes() for i in range(n)]

    def feldman_verify_batch(self, commitments: Sequence[Sequence[bytes]], ids: Sequence[int],
                             shares: Sequence[int], h48: bytes) -> List[bool]:
        """DKG share_verification (src/crypto/dkg.rs:433-450) for n received shares: check i has
        its dealer's t compressed commitments, this party's id and the decrypted share scalar."""
        n = len(ids)
        if n == 0:
            return []
        t = len(commitments[0])
        if len(commitments) != n or len(shares) != n or any(len(c) != t for c in commitments):
            raise ValueError("one commitment vector (all of length t) and one share per check")
        cm = np.frombuffer(b"".join(b"".join(c) for c in commitments), dtype=np.uint8)
        x = np.asarray(ids, dtype=np.uint64)
        sv = np.frombuffer(b"".join(int(s).to_bytes(32, "little") for s in shares), dtype=np.uint8)
        hp = np.frombuffer(bytes(h48), dtype=np.uint8)
        v = np.zeros(n, dtype=np.uint8)
        self._check(self._lib.ssb_feldman_verify_batch(self._h, n, t, cm.ctypes.data_as(_lib._u8p),
                                                       x.ctypes.data_as(_lib._u64p), sv.ctypes.data_as(_lib._u8p),
                                                       hp.ctypes.data_as(_lib._u8p), v.ctypes.data_as(_lib._u8p)),
                    "ssb_feldman_verify_batch")
        return [bool(b) for b in v]

    def dleq_verify_batch(self, proofs: Sequence[Tuple[bytes, bytes, bytes, bytes, bytes, bytes]]) -> List[bool]:
        """DKG::dleq_verify (src/crypto/dkg.rs:674-692) per proof (x1, y1, x2, y2 compressed G1; c, r
        32-byte little-endian scalars)."""
        n = len(proofs)
        if n == 0:
            return []
        for pr in proofs:
            if [len(x) for x in pr] != [48, 48, 48, 48, 32, 32]:
                raise ValueError("proof = (x1, y1, x2, y2: 48 bytes, c, r: 32 bytes)")
        pts = np.frombuffer(b"".join(b"".join(pr[:4]) for pr in proofs), dtype=np.uint8)
        cs = np.frombuffer(b"".join(pr[4] for pr in proofs), dtype=np.uint8)
        rs = np.frombuffer(b"".join(pr[5] for pr in proofs), dtype=np.uint8)
        v = np.zeros(n, dtype=np.uint8)
        self._check(self._lib.ssb_dleq_verify_batch(self._h, n, pts.ctypes.data_as(_lib._u8p), cs.ctypes.data_as(_lib._u8p),
                                                    rs.ctypes.data_as(_lib._u8p), v.ctypes.data_as(_lib._u8p)),
                    "ssb_dleq_verify_batch")
        return [bool(b) for b in v]

    def decode_wire_sigs(self, records: Sequence[bytes]) -> List[Optional[bytes]]:
        """bincode(bls::Signature) records (202 bytes each, src/node/dvfcore.rs:245-251) -> the
        96-byte compressed signatures, None where the record does not parse or its point does not
        decompress (the reference's "Deserialize failed" at src/validation/operator.rs:113 drops
        that share)."""
        n = len(records)
        if n == 0:
            return []
        if any(len(r) != WIRE_SIG_BYTES for r in records):
            raise ValueError("wire records are %d bytes" % WIRE_SIG_BYTES)
        w = np.frombuffer(b"".join(records), dtype=np.uint8)
        out = np.zeros(96 * n, dtype=np.uint8)
        st = np.zeros(n, dtype=np.int32)
        self._check(self._lib.ssb_decode_wire_sigs(self._h, n, w.ctypes.data_as(_lib._u8p), WIRE_SIG_BYTES,
                                                   out.ctypes.data_as(_lib._u8p), st.ctypes.data_as(_lib._i32p)),
                    "ssb_decode_wire_sigs")
        return [out[96 * i:96 * (i + 1)].tobytes() if st[i] == 0 else None for i in range(n)]

    def verify_batch(self, pks: Sequence[bytes], sigs: Sequence[bytes], root_idx: Sequence[int],
                     roots: Sequence[bytes], seed: Optional[int] = None, dst: bytes = DST) -> np.ndarray:
        n = len(sigs)
        out = np.zeros(n, dtype=np.uint8)
        if n == 0:
            return out
        pk = np.frombuffer(b"".join(pks), dtype=np.uint8)
        sg = np.frombuffer(b"".join(sigs), dtype=np.uint8)
        ri = np.ascontiguousarray(np.asarray(root_idx, dtype=np.uint32))
        rt = np.frombuffer(b"".join(roots), dtype=np.uint8)
        d, dp = _lib.buf(dst)
        self._check(self._lib.ssb_verify_batch(
            self._h, n, pk.ctypes.data_as(_lib._u8p), sg.ctypes.data_as(_lib._u8p), ri.ctypes.data_as(_lib._u32p),
            len(roots), rt.ctypes.data_as(_lib._u8p), dp, len(dst), _rlc_seed(seed),
            out.ctypes.data_as(_lib._u8p)), "ssb_verify_batch")
        return out

    def sign_batch(self, sks: Sequence[int], root_idx: Sequence[int], roots: Sequence[bytes],
                   dst: bytes = DST) -> List[bytes]:
        n = len(sks)
        if n == 0:
            return []
        sk = np.frombuffer(b"".join(int(k).to_bytes(32, "little") for k in sks), dtype=np.uint8)
        ri = np.ascontiguousarray(np.asarray(root_idx, dtype=np.uint32))
        rt = np.frombuffer(b"".join(roots), dtype=np.uint8)
        out = np.zeros(96 * n, dtype=np.uint8)
        d, dp = _lib.buf(dst)
        self._check(self._lib.ssb_sign_batch(self._h, n, sk.ctypes.data_as(_lib._u8p), ri.ctypes.data_as(_lib._u32p),
                                             len(roots), rt.ctypes.data_as(_lib._u8p), dp, len(dst),
                                             out.ctypes.data_as(_lib._u8p)), "ssb_sign_batch")
        return [out[96 * i:96 * (i + 1)].tobytes() for i in range(n)]

    def sk_to_pk_batch(self, sks: Sequence[int]) -> List[bytes]:
        n = len(sks)
        if n == 0:
            return []
        sk = np.frombuffer(b"".join(int(k).to_bytes(32, "little") for k in sks), dtype=np.uint8)
        out = np.zeros(48 * n, dtype=np.uint8)
        self._check(self._lib.ssb_sk_to_pk_batch(self._h, n, sk.ctypes.data_as(_lib._u8p),
                                                 out.ctypes.data_as(_lib._u8p)), "ssb_sk_to_pk_batch")
        return [out[48 * i:48 * (i + 1)].tobytes() for i in range(n)]

    def pk_validate_batch(self, pks: Sequence[bytes]) -> List[Optional[bytes]]:
        """bls::PublicKey::deserialize + serialize per key: the recompressed key, or None for a key
        that does not decode, is infinity or lies outside G1 (ssb_pk_validate_batch)."""
        n = len(pks)
        if n == 0:
            return []
        if any(len(p) != 48 for p in pks):
            raise ValueError("public keys are 48 bytes")
        inp = np.frombuffer(b"".join(pks), dtype=np.uint8)
        ok = np.zeros(n, dtype=np.uint8)
        out = np.zeros(48 * n, dtype=np.uint8)
        self._check(self._lib.ssb_pk_validate_batch(self._h, n, inp.ctypes.data_as(_lib._u8p), ok.ctypes.data_as(_lib._u8p),
                                                    out.ctypes.data_as(_lib._u8p)), "ssb_pk_validate_batch")
        return [out[48 * i:48 * (i + 1)].tobytes() if ok[i] else None for i in range(n)]

    def lagrange_coeffs(self, ids: Sequence[int]) -> List[int]:
        t = len(ids)
        if t == 0:
            return []
        x = np.ascontiguousarray(np.asarray([int(i) for i in ids], dtype=np.uint64))
        out = np.zeros(32 * t, dtype=np.uint8)
        self._check(self._lib.ssb_lagrange_coeffs(self._h, t, x.ctypes.data_as(_lib._u64p),
                                                  out.ctypes.data_as(_lib._u8p)), "ssb_lagrange_coeffs")
        return [int.from_bytes(out[32 * i:32 * (i + 1)].tobytes(), "little") for i in range(t)]

    def threshold_aggregate_batch_raw(self, t: Sequence[int], share_off: Sequence[int], sigs: bytes, pks: bytes,
                                      ids: Sequence[int], job_root: Sequence[int], roots: Sequence[bytes],
                                      seed: Optional[int] = None, dst: bytes = DST):
        """Packed form: returns (out_sig96[J,96], status[J], err[J,2], share_verdicts[N])."""
        J = len(t)
        off = np.ascontiguousarray(np.asarray(share_off, dtype=np.uint32))
        N = int(off[-1]) if J else 0
        tt = np.ascontiguousarray(np.asarray(t, dtype=np.uint32))
        sg = np.frombuffer(sigs, dtype=np.uint8) if N else np.zeros(1, np.uint8)
        pk = np.frombuffer(pks, dtype=np.uint8) if N else np.zeros(1, np.uint8)
        idv = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64)) if N else np.zeros(1, np.uint64)
        jr = np.ascontiguousarray(np.asarray(job_root, dtype=np.uint32))
        rt = np.frombuffer(b"".join(roots), dtype=np.uint8)
        out = np.zeros((max(J, 1), 96), dtype=np.uint8)
        st = np.zeros(max(J, 1), dtype=np.int32)
        err = np.zeros((max(J, 1), 2), dtype=np.uint64)
        ver = np.zeros(max(N, 1), dtype=np.uint8)
        d, dp = _lib.buf(dst)
        self._check(self._lib.ssb_threshold_aggregate_batch(
            self._h, J, off.ctypes.data_as(_lib._u32p), tt.ctypes.data_as(_lib._u32p), sg.ctypes.data_as(_lib._u8p),
            pk.ctypes.data_as(_lib._u8p), idv.ctypes.data_as(_lib._u64p), jr.ctypes.data_as(_lib._u32p), len(roots),
            rt.ctypes.data_as(_lib._u8p), dp, len(dst), _rlc_seed(seed), out.ctypes.data_as(_lib._u8p),
            st.ctypes.data_as(_lib._i32p), err.ctypes.data_as(_lib._u64p), ver.ctypes.data_as(_lib._u8p)),
            "ssb_threshold_aggregate_batch")
        return out[:J], st[:J], err[:J], ver[:N]

    def submit_batch_raw(self, t, share_off, sigs, pks, ids, job_root, roots, seed: Optional[int] = None,
                         dst: bytes = DST, pk_index=None) -> "PendingBatch":
        """Asynchronous packed form (ssb_threshold_aggregate_batch_submit): the inputs are staged and
        the batch enqueued on the next pipeline slot; PendingBatch.wait() returns (out_sig96[J,96],
        status[J], err[J,2], share_verdicts[N]).  Inputs may be numpy arrays (uint32 offsets / t /
        job roots, uint64 ids, uint8 signatures / keys / roots) or Python sequences / bytes."""
        J = len(t)
        off = np.ascontiguousarray(np.asarray(share_off, dtype=np.uint32))
        N = int(off[-1]) if J else 0
        tt = np.ascontiguousarray(np.asarray(t, dtype=np.uint32))
        sg = np.frombuffer(sigs, dtype=np.uint8) if isinstance(sigs, (bytes, bytearray)) else np.ascontiguousarray(sigs)
        if pk_index is not None:
            pk = np.ascontiguousarray(np.asarray(pk_index, dtype=np.uint32))
        else:
            pk = np.frombuffer(pks, dtype=np.uint8) if isinstance(pks, (bytes, bytearray)) else np.ascontiguousarray(pks)
        idv = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64)) if N else np.zeros(1, np.uint64)
        jr = np.ascontiguousarray(np.asarray(job_root, dtype=np.uint32))
        rt = (np.frombuffer(b"".join(roots), dtype=np.uint8) if not isinstance(roots, np.ndarray)
              else np.ascontiguousarray(roots))
        n_roots = len(roots) if not isinstance(roots, np.ndarray) else rt.size // 32
        pb = PendingBatch(self, J, N)
        d, dp = _lib.buf(dst)
        tk = ctypes.c_uint64(0)
        fn = (self._lib.ssb_threshold_aggregate_batch_cached_submit if pk_index is not None
              else self._lib.ssb_threshold_aggregate_batch_submit)
        pkp = pk.ctypes.data_as(_lib._u32p) if pk_index is not None else pk.ctypes.data_as(_lib._u8p)
        self._check(fn(
            self._h, J, off.ctypes.data_as(_lib._u32p), tt.ctypes.data_as(_lib._u32p), sg.ctypes.data_as(_lib._u8p),
            pkp, idv.ctypes.data_as(_lib._u64p), jr.ctypes.data_as(_lib._u32p), n_roots,
            rt.ctypes.data_as(_lib._u8p), dp, len(dst), _rlc_seed(seed), pb.out.ctypes.data_as(_lib._u8p),
            pb.st.ctypes.data_as(_lib._i32p), pb.err.ctypes.data_as(_lib._u64p), pb.ver.ctypes.data_as(_lib._u8p),
            ctypes.byref(tk)), "ssb_threshold_aggregate_batch_submit")
        pb.ticket = tk.value
        # this submit delivered the slot's previous batch (same slot = the ticket's low byte)
        slot = pb.ticket & 0xFF
        for t in [t for t in self._pending if t & 0xFF == slot]:
            del self._pending[t]
        self._pending[pb.ticket] = pb
        return pb

    def unsafe_aggregate_batch_raw(self, share_off: Sequence[int], sigs: bytes, ids: Sequence[int]):
        J = len(share_off) - 1
        off = np.ascontiguousarray(np.asarray(share_off, dtype=np.uint32))
        N = int(off[-1])
        sg = np.frombuffer(sigs, dtype=np.uint8) if N else np.zeros(1, np.uint8)
        idv = np.ascontiguousarray(np.asarray(ids, dtype=np.uint64)) if N else np.zeros(1, np.uint64)
        out = np.zeros((max(J, 1), 96), dtype=np.uint8)
        st = np.zeros(max(J, 1), dtype=np.int32)
        self._check(self._lib.ssb_unsafe_aggregate_batch(
            self._h, J, off.ctypes.data_as(_lib._u32p), sg.ctypes.data_as(_lib._u8p), idv.ctypes.data_as(_lib._u64p),
            out.ctypes.data_as(_lib._u8p), st.ctypes.data_as(_lib._i32p)), "ssb_unsafe_aggregate_batch")
        return out[:J], st[:J]


_DEFAULT_ENGINE: Optional[Engine] = None


class PendingBatch:
    """A submitted host-buffer batch (Engine.submit_batch_raw): its output arrays stay alive here
    until the library has delivered into them."""

    def __init__(self, engine: Engine, J: int, N: int):
        self.engine, self.J, self.N, self.ticket = engine, J, N, 0
        self.out = np.zeros((max(J, 1), 96), dtype=np.uint8)
        self.st = np.zeros(max(J, 1), dtype=np.int32)
        self.err = np.zeros((max(J, 1), 2), dtype=np.uint64)
        self.ver = np.zeros(max(N, 1), dtype=np.uint8)

    def wait(self):
        try:
            self.engine._check(self.engine._lib.ssb_batch_wait(self.engine._h, self.ticket), "ssb_batch_wait")
        finally:
            self.engine._pending.pop(self.ticket, None)
        return self.out[:self.J], self.st[:self.J], self.err[:self.J], self.ver[:self.N]


def default_engine() -> Engine:
    global _DEFAULT_ENGINE
    if _DEFAULT_ENGINE is None:
        _DEFAULT_ENGINE = Engine(int(os.environ.get("SSB_DEVICE", "0")))
    return _DEFAULT_ENGINE


# ------------------------------------------------------------------------------------------
# The reference API
# ------------------------------------------------------------------------------------------
@dataclass
class ThresholdJob:
    """One call's worth of threshold_aggregate arguments (SURVEY.md §8b batched entry point)."""
    sigs: Sequence[bytes]
    pks: Sequence[bytes]
    ids: Sequence[int]
    msg: bytes


def job_shape_error(job: ThresholdJob) -> Optional[str]:
    """Why a job's arguments could not come from the reference's types, or None: msg is a Hash256
    (32 bytes), a Signature serialises to 96 bytes, a PublicKey to 48, an id is a u64."""
    if len(job.msg) != 32:
        return "msg must be a 32-byte Hash256"
    if any(len(s) != 96 for s in job.sigs) or any(len(p) != 48 for p in job.pks):
        return "signatures are 96 bytes, public keys 48 bytes"
    if any(not 0 <= int(i) < 2**64 for i in job.ids):
        return "operator ids are u64"
    return None


class ThresholdSignature:
    """GenericThresholdSignature<HipThresholdSignature> (src/crypto/generic_threshold.rs:25-180)."""

    def __init__(self, threshold: int, engine: Optional[Engine] = None):
        self._t = int(threshold)
        self._engine = engine

    @classmethod
    def new(cls, threshold: int, engine: Optional[Engine] = None) -> "ThresholdSignature":
        return cls.infinity(threshold, engine)

    @classmethod
    def infinity(cls, threshold: int, engine: Optional[Engine] = None) -> "ThresholdSignature":
        return cls(threshold, engine)

    def threshold(self) -> int:
        return self._t

    @property
    def engine(self) -> Engine:
        return self._engine or default_engine()

    def threshold_aggregate(self, sigs: Sequence[bytes], pks: Sequence[bytes], ids: Sequence[int],
                            msg: bytes) -> bytes:
        """Returns the 96-byte combined signature or raises the DvfError the reference returns."""
        r = self.threshold_aggregate_batch([ThresholdJob(sigs, pks, ids, msg)])[0]
        if isinstance(r, (DvfError, ValueError)):
            raise r
        return r

    def threshold_aggregate_batch(self, jobs: Sequence[ThresholdJob], seed: Optional[int] = None
                                  ) -> List[Union[bytes, DvfError, ValueError]]:
        """One result per job: the combined signature, the DvfError the reference returns, or a
        ValueError for a job whose arguments the reference's types could not hold (a message that
        is not a 32-byte Hash256, a signature / public key of the wrong length).  A malformed job
        fails alone; the rest of the batch is aggregated."""
        results: List[Union[bytes, DvfError, ValueError, None]] = [None] * len(jobs)
        t = self._t
        if t < 1 or t > MAX_T:
            raise ValueError("threshold must be in [1, %d]" % MAX_T)
        roots: dict = {}
        dev_jobs = []
        for j, job in enumerate(jobs):
            # length checks, in the reference's order (generic_threshold.rs:133-141)
            if len(job.sigs) != len(job.pks):
                results[j] = DifferentLength(len(job.sigs), len(job.pks))
                continue
            if len(job.sigs) != len(job.ids):
                results[j] = DifferentLength(len(job.sigs), len(job.ids))
                continue
            bad = job_shape_error(job)
            if bad:
                results[j] = ValueError(bad)
                continue
            dev_jobs.append(j)
            roots.setdefault(bytes(job.msg), len(roots))
        if dev_jobs:
            offs = [0]
            sigs, pks, ids, jr = [], [], [], []
            for j in dev_jobs:
                job = jobs[j]
                for s, p, i in zip(job.sigs, job.pks, job.ids):
                    sigs.append(bytes(s)); pks.append(bytes(p)); ids.append(int(i))
                offs.append(len(sigs))
                jr.append(roots[bytes(job.msg)])
            root_list = sorted(roots, key=roots.get)
            out, st, err, _ = self.engine.threshold_aggregate_batch_raw(
                [t] * len(dev_jobs), offs, b"".join(sigs), b"".join(pks), ids, jr, root_list, seed)
            for k, j in enumerate(dev_jobs):
                e = _error_from(int(st[k]), int(err[k, 0]), int(err[k, 1]))
                results[j] = e if e is not None else out[k].tobytes()
        return results  # type: ignore[return-value]

    def unsafe_aggregate(self, sigs: Sequence[bytes], ids: Sequence[int]) -> bytes:
        """src/crypto/impls/blst.rs:67-87: combine the first t shares with Lagrange coefficients of
        `ids` (which must have exactly t entries: require(...) panics otherwise)."""
        t = self._t
        if len(ids) != t:
            raise ValueError("Different length")   # require() panic, src/utils/error.rs:4-8
        if len(sigs) < t:
            raise IndexError("index out of bounds")  # sigs[i] for i < t
        out, st = self.engine.unsafe_aggregate_batch_raw([0, t], b"".join(bytes(s) for s in sigs[:t]), list(ids))
        e = _error_from(int(st[0]), 0, 0)
        if e is not None:
            raise e
        return out[0].tobytes()
