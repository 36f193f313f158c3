"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

Run from the repo root:  python tests/golden/make_golden.py
The reference (Rust + blst, not vendored) cannot be built or imported here, so
the fixtures come from the oracle, which is itself pinned by tests/golden/known_answers.json.

Deterministic key derivation (documented, not the reference's StdRng):
  master sk_v      = int(SHA-256(b"ssbls/sk" || seed || v_le64)) mod r
  Shamir coeff k   = int(SHA-256(b"ssbls/coef" || seed || v_le64 || k_le32)) mod r
  share for id     = poly(id) mod r  (Horner; src/math/polynomial.rs:39-51)
"""
import hashlib
import json
import os
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import bls12_381 as B  # noqa: E402

SEED = (0x5AFE57A4E).to_bytes(8, "little")
HELLO_ROOT = hashlib.sha256(b"hello world").digest()  # tests/test_generic_threshold.rs:15-18


def master_sk(v):
    return int.from_bytes(hashlib.sha256(b"ssbls/sk" + SEED + v.to_bytes(8, "little")).digest(), "big") % B.R


def coeff(v, k):
    return int.from_bytes(hashlib.sha256(b"ssbls/coef" + SEED + v.to_bytes(8, "little")
                                         + k.to_bytes(4, "little")).digest(), "big") % B.R


def root_of(tag):
    return hashlib.sha256(b"ssbls/root" + tag.encode()).digest()


def _sign_job(args):
    sk, root = args
    return B.g2_compress(B.sign(sk, root))


def _verify_job(args):
    pk48, sig96, root = args
    return B.verify(pk48, sig96, root)


def non_subgroup_sig(seed_int):
    """A valid compressed E2 point that is NOT in G2 (fails the sig_groupcheck)."""
    x0 = seed_int
    while True:
        x = (x0 % B.P, 7)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(x), x), B.B2))
        if y is not None and not B.g2_in_subgroup((x, y)):
            return B.g2_compress((x, y))
        x0 += 1


def make_committee(v, t, n, ids=None):
    ids = ids or list(range(1, n + 1))
    sk = master_sk(v)
    coeffs = [coeff(v, k) for k in range(1, t)]
    shares = B.key_split(sk, coeffs, ids)
    return sk, ids, shares


def build_cases(pool):
    cases = []
    # (name, validator, t, n, ids, root, tamper) ; tamper: dict index -> kind
    specs = [
        ("hello_world_3of4", 1, 3, 4, None, HELLO_ROOT, {}),
        ("hello_world_5of10", 2, 5, 10, None, HELLO_ROOT, {}),
        ("c3_5of7", 3, 5, 7, None, root_of("c3"), {}),
        ("c5_10of13", 4, 10, 13, None, root_of("c5"), {}),
        ("first_share_wrong_root", 5, 3, 4, None, HELLO_ROOT, {0: "wrong_root"}),
        ("two_invalid_insufficient", 6, 3, 4, None, HELLO_ROOT, {1: "wrong_root", 2: "wrong_key"}),
        ("id_zero_reached", 7, 3, 4, [1, 0, 2, 3], HELLO_ROOT, {}),
        ("id_zero_after_break", 8, 3, 4, [1, 2, 3, 0], HELLO_ROOT, {}),
        ("dup_id_first_valid", 9, 3, 5, [1, 1, 2, 3, 4], HELLO_ROOT, {}),
        ("dup_id_first_invalid", 10, 3, 5, [1, 1, 2, 3, 4], HELLO_ROOT, {0: "wrong_root"}),
        ("infinity_share", 11, 3, 4, None, HELLO_ROOT, {2: "infinity"}),
        ("bad_encoding_shares", 12, 2, 5, None, root_of("enc"), {0: "no_cflag", 1: "x_ge_p", 2: "not_on_curve"}),
        ("non_subgroup_share", 13, 3, 4, None, root_of("sub"), {0: "non_subgroup"}),
        ("invalid_last_share", 14, 3, 4, None, root_of("last"), {3: "wrong_root"}),
        ("t1_single", 15, 1, 1, None, root_of("t1"), {}),
        ("insufficient_signatures", 16, 3, 2, None, HELLO_ROOT, {}),
    ]
    sign_jobs, meta = [], []
    for name, v, t, n, ids, root, tamper in specs:
        sk, ids_, shares = make_committee(v, t, max(n, 1), ids)
        # share i signs with the share key of ids_[i] (a duplicate id repeats that key)
        job_sigs = []
        for i, ident in enumerate(ids_):
            kind = tamper.get(i)
            if ident == 0:
                share_sk = master_sk(999)  # any key; id 0 is rejected before use
            else:
                share_sk = shares[ident]
            if kind == "wrong_root":
                sign_jobs.append((share_sk, root_of("other")))
            elif kind == "wrong_key":
                sign_jobs.append((master_sk(12345), root))
            else:
                sign_jobs.append((share_sk, root))
            job_sigs.append(len(sign_jobs) - 1)
        meta.append((name, v, t, ids_, root, tamper, sk, shares, job_sigs))
    signed = pool.map(_sign_job, sign_jobs)
    masters = pool.map(_sign_job, [(m[6], m[4]) for m in meta])

    verify_jobs = []
    built = []
    for (name, v, t, ids_, root, tamper, sk, shares, job_sigs), msig in zip(meta, masters):
        sigs, pks = [], []
        for i, ident in enumerate(ids_):
            s = signed[job_sigs[i]]
            kind = tamper.get(i)
            if kind == "infinity":
                s = bytes([0xC0]) + bytes(95)
            elif kind == "no_cflag":
                s = bytes([s[0] & 0x7F]) + s[1:]
            elif kind == "x_ge_p":
                s = bytes([0x80 | 0x1F]) + b"\xff" * 95
            elif kind == "not_on_curve":
                x = 5
                while B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr((x, 1)), (x, 1)), B.B2)) is not None:
                    x += 1
                s = B.g2_compress(((x, 1), (0, 0)))  # y ignored on compress; x off-curve
            elif kind == "non_subgroup":
                s = non_subgroup_sig(123456789)
            sigs.append(s)
            pk_sk = shares[ident] if ident != 0 else master_sk(999)
            pks.append(B.g1_compress(B.sk_to_pk(pk_sk)))
        for i in range(len(sigs)):
            verify_jobs.append((pks[i], sigs[i], root))
        built.append(dict(name=name, t=t, root=root.hex(), ids=ids_, pks=[p.hex() for p in pks],
                          sigs=[s.hex() for s in sigs], master_pk=B.g1_compress(B.sk_to_pk(sk)).hex(),
                          master_sig=msig.hex()))
    verdicts = pool.map(_verify_job, verify_jobs)
    k = 0
    for c in built:
        n = len(c["sigs"])
        c["share_verdicts"] = verdicts[k:k + n]
        k += n
        sig_b = [bytes.fromhex(s) for s in c["sigs"]]
        pk_b = [bytes.fromhex(s) for s in c["pks"]]
        vmap = c["share_verdicts"]
        status, payload = B.threshold_aggregate(c["t"], sig_b, pk_b, c["ids"], bytes.fromhex(c["root"]),
                                                verify_fn=lambda i, vmap=vmap: vmap[i])
        c["expected_status"] = status
        if status == B.OK:
            c["expected_sig"] = payload.hex()
            c["expected_payload"] = []
            assert payload.hex() == c["master_sig"], c["name"]  # combine == master sign
        else:
            c["expected_sig"] = None
            c["expected_payload"] = list(payload)
        cases.append(c)
    return cases


def _h2g2_job(msg):
    h = B.hash_to_g2(msg)
    return B.g2_serialize_uncompressed(h).hex()


def build_hash_cases(pool):
    msgs = [HELLO_ROOT, bytes(32), b"\xff" * 32] + [root_of("h%d" % i) for i in range(13)]
    outs = pool.map(_h2g2_job, msgs)
    return [dict(msg=m.hex(), out192=o) for m, o in zip(msgs, outs)]


def build_point_cases(pool):
    """G1/G2 decompression round trips, including the generators and infinity."""
    g1 = [B.G1_GEN, None] + [B.g1_mul(B.G1_GEN, master_sk(100 + i)) for i in range(6)]
    g2 = [B.G2_GEN, None] + [B.g2_mul(B.G2_GEN, master_sk(200 + i)) for i in range(6)]
    out = {"g1": [], "g2": []}
    for p in g1:
        out["g1"].append(dict(compressed=B.g1_compress(p).hex(),
                              x=None if p is None else "%096x" % p[0], y=None if p is None else "%096x" % p[1]))
    for p in g2:
        out["g2"].append(dict(compressed=B.g2_compress(p).hex(), uncompressed=B.g2_serialize_uncompressed(p).hex()))
    return out


def build_lagrange_cases():
    sets = [[1, 2, 3], [1, 2, 4], [2, 3, 4], [1, 3, 4], [1, 2, 3, 4, 5], list(range(1, 11)),
            [3, 7, 11, 12, 13], [5, 5, 6], [1, 0, 2], [2**64 - 1, 2**63, 17]]
    out = []
    for ids in sets:
        lam = B.lagrange_coeffs(ids)
        out.append(dict(ids=[str(i) for i in ids], lambdas_le=[x.to_bytes(32, "little").hex() for x in lam]))
    return out


def main():
    with Pool(min(8, os.cpu_count() or 1)) as pool:
        cases = build_cases(pool)
        hashes = build_hash_cases(pool)
        points = build_point_cases(pool)
    doc = dict(dst=B.DST_POP.decode(), seed="0x5AFE57A4E", cases=cases)
    with open(os.path.join(HERE, "threshold_cases.json"), "w") as f:
        json.dump(doc, f, indent=1)
    with open(os.path.join(HERE, "hash_to_g2.json"), "w") as f:
        json.dump(dict(dst=B.DST_POP.decode(), cases=hashes), f, indent=1)
    with open(os.path.join(HERE, "points.json"), "w") as f:
        json.dump(points, f, indent=1)
    with open(os.path.join(HERE, "lagrange.json"), "w") as f:
        json.dump(build_lagrange_cases(), f, indent=1)
    print("wrote", len(cases), "threshold cases,", len(hashes), "hash cases")


if __name__ == "__main__":
    main()
