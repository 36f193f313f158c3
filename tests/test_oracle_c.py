"""The plain-C oracle (oracle/bls_c.c) against the published known answers and the committed
golden threshold cases -- a second, independent CPU restatement beside oracle/bls12_381.py (both
pinned to the same vectors), and the multi-threaded CPU baseline of bench.py."""
import hashlib
import json
import os

import pytest

from oracle import bls_c

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_selftests():
    lib = bls_c.load()
    assert lib.bls_oracle_selftest() == 0                 # g1 on curve, [r]g1 == O
    assert lib.bls_oracle_selftest_final_exp() == 0       # x-chain == cube of the textbook exponent


def test_rfc9380_hash_to_g2_vector():
    v = _load("known_answers.json")["rfc9380_g2"][0]
    h = bls_c.hash_to_g2(v["msg"].encode(), v["dst"].encode())
    assert [h[48:96].hex(), h[0:48].hex()] == v["P_x"]
    assert [h[144:192].hex(), h[96:144].hex()] == v["P_y"]


def test_eth_sign_vector_verifies():
    v = _load("known_answers.json")["eth_sign"][0]
    pk, sig, msg = bytes.fromhex(v["pubkey"]), bytes.fromhex(v["signature"]), bytes.fromhex(v["message"])
    assert bls_c.verify(pk, sig, msg)
    assert not bls_c.verify(pk, sig, hashlib.sha256(b"other").digest())
    bad = bytearray(sig)
    bad[5] ^= 1
    assert not bls_c.verify(pk, bytes(bad), msg)


def test_eth_sign_vector_signs():
    """bls_c.sign (the signer tests' oracle) reproduces the Ethereum consensus-spec `sign` vector
    (POP DST, src/crypto/impls/blst.rs:11) byte for byte, and refuses keys outside (0, r)."""
    v = _load("known_answers.json")["eth_sign"][0]
    sk, msg = bytes.fromhex(v["privkey"]), bytes.fromhex(v["message"])
    assert bls_c.sign(sk, msg).hex() == v["signature"]
    assert bls_c.sign(b"\0" * 32, msg) is None
    r = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    assert bls_c.sign(r.to_bytes(32, "big"), msg) is None


@pytest.mark.parametrize("case", _load("threshold_cases.json")["cases"], ids=lambda c: c["name"])
def test_threshold_golden_cases(case):
    sigs = [bytes.fromhex(s) for s in case["sigs"]]
    pks = [bytes.fromhex(p) for p in case["pks"]]
    root = bytes.fromhex(case["root"])
    st, payload = bls_c.threshold_aggregate(case["t"], sigs, pks, case["ids"], root)
    assert st == case["expected_status"]
    if st == 0:
        assert payload.hex() == case["expected_sig"]
    else:
        assert list(payload)[:len(case["expected_payload"])] == case["expected_payload"]
    for i, want in enumerate(case["share_verdicts"]):
        assert bls_c.verify(pks[i], sigs[i], root) == want


def test_threshold_batch_threads_agree():
    cases = [c for c in _load("threshold_cases.json")["cases"] if c["name"] in
             ("hello_world_3of4", "c3_5of7", "two_invalid_insufficient", "dup_id_first_invalid")]
    off, t, sigs, pks, ids, jr, roots = [0], [], [], [], [], [], []
    for j, c in enumerate(cases):
        sigs += [bytes.fromhex(s) for s in c["sigs"]]
        pks += [bytes.fromhex(p) for p in c["pks"]]
        ids += c["ids"]
        off.append(len(sigs))
        t.append(c["t"])
        jr.append(j)
        roots.append(bytes.fromhex(c["root"]))
    res = [bls_c.threshold_batch(off, t, b"".join(sigs), b"".join(pks), ids, jr, roots, threads=k, verify_all=va)
           for k, va in ((1, False), (4, False), (4, True))]
    want = [v for c in cases for v in c["share_verdicts"] + [None] * (len(c["sigs"]) - len(c["share_verdicts"]))]
    ver_all = res[2][3]
    for i, w in enumerate(want):
        if w is not None:
            assert bool(ver_all[i]) == w
    for out, st, _, _ in res:
        for j, c in enumerate(cases):
            assert st[j] == c["expected_status"]
            if st[j] == 0:
                assert out[j].tobytes().hex() == c["expected_sig"]


def test_rlc_batch_path_matches_per_share():
    """The RLC-batched CPU baseline (bls_oracle_threshold_batch_rlc) == the per-share path: on the
    all-valid golden jobs the batch check passes and the combines agree (integer and 255-bit
    Lagrange); on every golden job (invalid / undecodable / duplicate / zero-id shares) it fails and
    the per-share verdicts take over."""
    import json
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "threshold_cases.json")))["cases"]

    def pack(cs):
        roots, t, off, sigs, pks, ids, jr = [], [], [0], [], [], [], []
        for c in cs:
            r = bytes.fromhex(c["root"])
            if r not in roots:
                roots.append(r)
            jr.append(roots.index(r)); t.append(c["t"])
            sigs += [bytes.fromhex(s) for s in c["sigs"]]; pks += [bytes.fromhex(p) for p in c["pks"]]
            ids += c["ids"]; off.append(len(sigs))
        return off, t, b"".join(sigs), b"".join(pks), ids, jr, roots

    good = [c for c in cases if all(c["share_verdicts"]) and c["expected_status"] == 0]
    assert len(good) >= 3
    for cs, want_ok in ((good, True), (cases, False)):
        off, t, sg, pk, ids, jr, roots = pack(cs)
        o1, s1, e1, v1 = bls_c.threshold_batch(off, t, sg, pk, ids, jr, roots, 4, verify_all=True)
        o2, s2, e2, v2, ok = bls_c.threshold_batch_rlc(off, t, sg, pk, ids, jr, roots, 4)
        assert ok == want_ok
        assert (s1 == s2).all() and (e1 == e2).all() and (v1 == v2).all()
        assert (o1[s1 == 0] == o2[s2 == 0]).all()
