"""Writes tests/golden/reference_kats.json: known answers held by the REFERENCE's own sources (data
only: hex strings and where they sit), so the oracle and the device are pinned by SafeStake's own
vectors and not only by the published standards.

  * sk -> pk: src/deposit/mod.rs:75-77 (`get_deposit_test`): SecretKey::deserialize(12a660e5..)
    .public_key().as_hex_string() == 0x9200c374..  -- blst sk_to_pk + compression.
  * compressed G1 public keys that the reference deserializes into the validated `PublicKey` type
    (lighthouse -> blst key_validate: decodes, not infinity, in G1) with unwrap():
      src/exit/mod.rs:173, src/validation/operator_committee_definitions.rs:184-186 and :208-210
      (`OperatorCommitteeDefinition.{validator,operator}_public_key(s)`: `types::PublicKey`),
      src/validation/account_utils/validator_definitions.rs:698 (`voting_public_key: PublicKey`);
    plus keys it holds as `PublicKeyBytes` (graffiti_file.rs:114-116, node/utils.rs:196), which
    must decode the same way on every implementation.
  * negative controls derived from them (a flipped x bit, the infinity encoding, a missing
    compression flag, sk = 0 and sk = r), whose verdicts come from the oracle.

Run from the repo root with the reference mounted:  python tests/golden/make_reference_kats.py
The reference is read as text only (regex over the cited lines); it never runs."""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
REF = "/root/reference"
R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

PK_SOURCES = [  # (file, line range, how the reference types it)
    ("src/exit/mod.rs", (173, 173), "PublicKey::deserialize(..).unwrap()"),
    ("src/validation/operator_committee_definitions.rs", (184, 186), "types::PublicKey (serde_yaml)"),
    ("src/validation/operator_committee_definitions.rs", (208, 210), "types::PublicKey (serde_yaml, commented-out test)"),
    ("src/validation/account_utils/validator_definitions.rs", (698, 698), "voting_public_key: PublicKey"),
    ("src/validation/graffiti_file.rs", (114, 116), "PublicKeyBytes"),
    ("src/node/utils.rs", (196, 196), "String (validator_pk)"),
]


def scan(path, lo, hi):
    with open(os.path.join(REF, path)) as f:
        lines = f.read().split("\n")
    out = []
    for ln in range(lo, hi + 1):
        for m in re.finditer(r"(?<![0-9a-fA-F])([0-9a-f]{96})(?![0-9a-fA-F])", lines[ln - 1]):
            out.append((m.group(1), ln))
    return out


def main():
    from oracle import bls12_381 as B
    dep = open(os.path.join(REF, "src/deposit/mod.rs")).read().split("\n")
    sk_hex = re.search(r'hex::decode\("([0-9a-f]{64})"\)', dep[74]).group(1)
    pk_hex = re.search(r'"0x([0-9a-f]{96})"', dep[76]).group(1)
    sk = int(sk_hex, 16)
    assert B.g1_compress(B.sk_to_pk(sk)).hex() == pk_hex, "oracle disagrees with the reference's deposit KAT"
    sk_cases = [dict(sk_be=sk_hex, pk=pk_hex, valid=True, source="src/deposit/mod.rs:75-77")]
    for v, why in ((0, "sk = 0 (blst_sk_check fails)"), (R_ORDER, "sk = r (not < r)")):
        sk_cases.append(dict(sk_be="%064x" % v, pk=None, valid=False, source="negative control: " + why))

    seen, pk_cases = set(), []
    for path, (lo, hi), typ in PK_SOURCES:
        for h, ln in scan(path, lo, hi):
            if h in seen:
                continue
            seen.add(h)
            p = B.g1_decompress(bytes.fromhex(h))
            ok = p is not None and B.g1_in_subgroup_slow(p)
            pk_cases.append(dict(pk=h, valid=bool(ok), recompressed=B.g1_compress(p).hex() if ok else None,
                                 source="%s:%d" % (path, ln), reference_type=typ))
    base = bytes.fromhex(pk_cases[0]["pk"])
    negs = [
        (bytes([base[0]]) + base[1:47] + bytes([base[47] ^ 1]), "x low bit flipped"),
        (bytes([0xc0]) + bytes(47), "infinity encoding (PublicKey rejects infinity)"),
        (bytes([base[0] & 0x7f]) + base[1:], "compression flag cleared"),
        (bytes([0xff]) + base[1:], "x >= p (top bits set)"),
    ]
    for b, why in negs:
        try:
            p = B.g1_decompress(b)
            ok = p is not None and B.g1_in_subgroup_slow(p)
        except Exception:
            ok = False
        pk_cases.append(dict(pk=b.hex(), valid=bool(ok), recompressed=B.g1_compress(p).hex() if ok else None,
                             source="negative control derived from %s: %s" % (pk_cases[0]["source"], why),
                             reference_type="PublicKey"))
    out = dict(note="Known answers held by the reference's own sources; see make_reference_kats.py",
               sk_to_pk=sk_cases, public_keys=pk_cases)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("%d sk cases, %d public keys (%d valid)" % (len(sk_cases), len(pk_cases), sum(c["valid"] for c in pk_cases)))


if __name__ == "__main__":
    main()
