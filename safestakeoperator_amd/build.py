"""Build libssbls.so (gfx950) in-tree.  Used by __graft_entry__.build() and the tests.

    python -m safestakeoperator_amd.build [--force]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libssbls.so")
SOURCES = ["ssbls.hip"]
HEADERS = ["ssb_field.h", "ssb_curve.h", "ssb_pairing.h", "ssb_h2c.h", "ssb_consts.h", "ssb_units.h", "ssb_wave.h", "ssb_wave_tables.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SSB_OFFLOAD_ARCH", "gfx950")


STAMP = LIB + ".srchash"


def _source_hash():
    """Content hash of every input (mtimes do not survive the copy to a GPU box)."""
    import hashlib
    h = hashlib.sha256()
    paths = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(HERE, "..", "include", "ssbls.h")]
    for p in paths:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    h.update(" ".join([HIPCC, ARCH]).encode())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = True) -> str:
    want = _source_hash()
    if not force and os.path.exists(LIB) and os.path.exists(STAMP) and open(STAMP).read().strip() == want:
        return LIB
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-shared", "-fPIC",
           "-Wno-unused-result", "-o", LIB + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES]
    if verbose:
        print("[ssbls] building:", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(STAMP, "w") as f:
        f.write(want + "\n")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
