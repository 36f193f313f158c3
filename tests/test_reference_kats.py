"""Known answers held by the REFERENCE's own sources (tests/golden/reference_kats.json, written by
tests/golden/make_reference_kats.py): the deposit test's sk -> pk (src/deposit/mod.rs:75-77) and
the compressed G1 keys SafeStake deserializes into lighthouse's validated PublicKey
(src/exit/mod.rs:173, src/validation/operator_committee_definitions.rs:184-210, ...).

CPU: the Python oracle and the C oracle against the fixture.  GPU: ssb_sk_to_pk_batch,
ssb_pk_validate_batch (PublicKey::deserialize + serialize), and the public-key cache used by the
batch path (a share signed with the deposit KAT's key verifies against the reference's pk bytes)."""
import json
import os

import pytest

from oracle import bls12_381 as B
from oracle import bls_c

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")


def _kats():
    with open(GOLD) as f:
        return json.load(f)


def test_fixture_cites_reference_lines():
    k = _kats()
    assert k["sk_to_pk"][0]["source"] == "src/deposit/mod.rs:75-77"
    assert k["sk_to_pk"][0]["pk"].startswith("9200c374")
    srcs = {c["source"].split(":")[0] for c in k["public_keys"] if c["valid"]}
    assert {"src/exit/mod.rs", "src/validation/operator_committee_definitions.rs"} <= srcs
    assert sum(c["valid"] for c in k["public_keys"]) >= 15
    assert sum(not c["valid"] for c in k["public_keys"]) >= 4


def test_python_oracle_sk_to_pk():
    for c in _kats()["sk_to_pk"]:
        sk = int(c["sk_be"], 16)
        if c["valid"]:
            assert B.g1_compress(B.sk_to_pk(sk)).hex() == c["pk"], c["source"]


def test_c_oracle_sk_to_pk():
    for c in _kats()["sk_to_pk"]:
        got = bls_c.sk_to_pk(bytes.fromhex(c["sk_be"]))
        assert (got.hex() if got else None) == c["pk"], c["source"]


def test_python_oracle_public_keys():
    for c in _kats()["public_keys"]:
        b = bytes.fromhex(c["pk"])
        try:
            p = B.g1_decompress(b)
            ok = p is not None and B.g1_in_subgroup_slow(p)
        except B.DecodeError:
            ok = False
        assert ok == c["valid"], c["source"]
        if ok:
            assert B.g1_compress(p).hex() == c["recompressed"] == c["pk"], c["source"]


def test_c_oracle_public_keys():
    for c in _kats()["public_keys"]:
        ok, rec = bls_c.pk_validate(bytes.fromhex(c["pk"]))
        assert ok == c["valid"], c["source"]
        assert (rec.hex() if ok else None) == c["recompressed"], c["source"]


@pytest.mark.gpu
def test_gpu_sk_to_pk_deposit_kat(engine):
    c = _kats()["sk_to_pk"][0]
    assert engine.sk_to_pk_batch([int(c["sk_be"], 16)])[0].hex() == c["pk"]


@pytest.mark.gpu
def test_gpu_pk_validate_reference_keys(engine):
    cases = _kats()["public_keys"]
    got = engine.pk_validate_batch([bytes.fromhex(c["pk"]) for c in cases])
    for c, g in zip(cases, got):
        assert (g is not None) == c["valid"], c["source"]
        assert (g.hex() if g else None) == c["recompressed"], c["source"]
    # a larger batch (every key 300 times, interleaved) gives the same answers
    big = engine.pk_validate_batch([bytes.fromhex(c["pk"]) for c in cases] * 300)
    assert big == got * 300


@pytest.mark.gpu
def test_gpu_pk_cache_with_reference_key(engine):
    """The batch path's decoded-key table on the reference's own key bytes: shares signed with the
    deposit KAT's secret key verify against its pk bytes (0x9200c374..) taken from the cache, and a
    share whose index points at another reference key does not."""
    import ctypes
    import numpy as np
    import torch
    from safestakeoperator_amd import DST
    from safestakeoperator_amd import _lib
    kat = _kats()
    sk = int(kat["sk_to_pk"][0]["sk_be"], 16)
    pk = bytes.fromhex(kat["sk_to_pk"][0]["pk"])
    other = bytes.fromhex(kat["public_keys"][0]["pk"])
    roots = [bytes([i]) * 32 for i in range(4)]
    sigs = engine.sign_batch([sk] * 4, [0, 1, 2, 3], roots)
    lib = engine._lib
    table = np.frombuffer(pk + other, dtype=np.uint8)
    assert lib.ssb_pk_cache_set(engine.handle, 2, table.ctypes.data_as(_lib._u8p)) == 0
    dev = torch.device("cuda", 0)
    d_sig = torch.tensor(list(b"".join(sigs)), dtype=torch.uint8, device=dev)
    d_idx = torch.tensor([0, 0, 1, 0], dtype=torch.int32, device=dev)
    d_ri = torch.tensor([0, 1, 2, 3], dtype=torch.int32, device=dev)
    d_roots = torch.tensor(list(b"".join(roots)), dtype=torch.uint8, device=dev)
    d_v = torch.zeros(4, dtype=torch.uint8, device=dev)
    dst = (ctypes.c_uint8 * len(DST)).from_buffer_copy(DST)
    rc = lib.ssb_verify_batch_cached_dev(engine.handle, 4, d_idx.data_ptr(), d_sig.data_ptr(), d_ri.data_ptr(), 4,
                                         d_roots.data_ptr(), ctypes.cast(dst, _lib._u8p), len(DST), 1, d_v.data_ptr(),
                                         None)
    assert rc == 0
    torch.cuda.synchronize()
    assert d_v.cpu().tolist() == [1, 1, 0, 1]
    assert lib.ssb_pk_cache_set(engine.handle, 0, None) == 0
