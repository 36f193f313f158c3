"""The reference-side Rust binding against the reference tree.

No cargo in this image, so the Rust files are type-checked by inspection; what CAN be checked here
is that the patches apply, in order, to the reference files they name (`git apply --check` on a
scratch copy -- the reference itself is read-only), and that the files the patches declare as
modules exist in `rust/`.  Skipped where the reference is absent (the GPU box).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCHES = sorted(os.path.join(ROOT, "rust", "patches", p) for p in os.listdir(os.path.join(ROOT, "rust", "patches"))
                 if p.endswith(".patch"))


def _touched(patch):
    return re.findall(r"^\+\+\+ b/(\S+)", open(patch).read(), re.M)


@pytest.mark.skipif(not os.path.isdir(REF) or shutil.which("git") is None, reason="reference tree absent")
def test_patches_apply_in_order(tmp_path):
    files = sorted({f for p in PATCHES for f in _touched(p)})
    assert files, "no patch hunks found"
    for f in files:
        dst = tmp_path / f
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(os.path.join(REF, f), dst)
    for p in PATCHES:
        r = subprocess.run(["git", "apply", "--check", p], cwd=tmp_path, capture_output=True, text=True)
        assert r.returncode == 0, f"{os.path.basename(p)}: {r.stderr}"
        subprocess.run(["git", "apply", p], cwd=tmp_path, check=True, capture_output=True)
    hot = (tmp_path / "src/validation/impls/hotstuff.rs").read_text()
    assert "slot_collector::threshold_aggregate_wire" in hot and 'cfg(not(feature = "hip"))' in hot
    assert "operator.sign_wire(msg)" in hot   # the shares stay wire records on the receive path
    op = (tmp_path / "src/validation/operator.rs").read_text()
    assert "async fn sign_wire" in op and "pub struct WireSignature" in op and "fn wire_record_ok" in op
    # without the feature the reference's own deserializing sign() is untouched
    assert "bincode::deserialize::<Signature>(&data)" in op
    oc = (tmp_path / "src/validation/operator_committees.rs").read_text()
    assert "register_committee_keys(&def.operator_public_keys)" in oc
    dc = (tmp_path / "src/node/dvfcore.rs").read_text()   # f-3: every duty's local signature batched
    assert "slot_signer::sign(&self.local_keypair.sk, message).await" in dc and "let sig = self.local_sign(message);" in dc
    gt = (tmp_path / "src/crypto/generic_threshold.rs").read_text()
    assert "fn threshold_aggregate_batch" in gt and "pub struct ThresholdJob" in gt


def test_declared_modules_are_shipped():
    """Every `pub mod` a patch adds under `feature = "hip"` has its file in rust/src."""
    mods = {
        "src/crypto/impls/mod.rs": "src/crypto/impls/{}.rs",
        "src/validation/impls/mod.rs": "src/validation/impls/{}.rs",
    }
    for p in PATCHES:
        txt = open(p).read()
        for sect in re.split(r"^diff -ru ", txt, flags=re.M)[1:]:
            target = re.search(r"^\+\+\+ b/(\S+)", sect, re.M).group(1)
            if target not in mods:
                continue
            for name in re.findall(r"^\+\s*pub mod (\w+);", sect, re.M):
                assert os.path.exists(os.path.join(ROOT, "rust", mods[target].format(name))), (p, name)
