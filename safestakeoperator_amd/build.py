"""Build libssbls.so (gfx950) in-tree.  Used by __graft_entry__.build() and the tests.

Every translation unit in csrc/ is compiled in parallel (hipcc -c), then linked into one shared
library.  A content hash of every source and header decides whether to rebuild (mtimes do not
survive the copy to a GPU box).

    python -m safestakeoperator_amd.build [--force]
"""
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# SSB_VARIANT=name builds an experiment variant (extra -D flags from SSB_VARIANT_DEFS) into
# libssbls_<name>.so with its own object directory; the product library is libssbls.so.
VARIANT = os.environ.get("SSB_VARIANT", "")
LIB = os.path.join(HERE, "libssbls%s.so" % ("_" + VARIANT if VARIANT else ""))
SOURCES = ["ssbls.hip", "ssb_k_lane.hip", "ssb_k_verify.hip", "ssb_k_pair.hip", "ssb_k_hash.hip",
           "ssb_k_combine.hip", "ssb_k_msm.hip", "ssb_k_bisect.hip", "ssb_k_wire.hip", "ssb_k_dkg.hip",
           "ssb_k_fused.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SSB_OFFLOAD_ARCH", "gfx950")
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-Wno-unused-value"]
if VARIANT:
    FLAGS += os.environ.get("SSB_VARIANT_DEFS", "").split()
STAMP = LIB + ".srchash"
OBJDIR = os.path.join(HERE, "build" + ("_" + VARIANT if VARIANT else ""))


def _inputs():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(CSRC, s) for s in SOURCES] +
                  [os.path.join(HERE, "..", "include", "ssbls.h")])


def _hash(paths, extra=""):
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    h.update((" ".join([HIPCC] + FLAGS) + extra).encode())
    return h.hexdigest()


def _source_hash():
    return _hash(_inputs())


def build(force: bool = False, verbose: bool = True) -> str:
    want = _source_hash()
    if not force and os.path.exists(LIB) and os.path.exists(STAMP) and open(STAMP).read().strip() == want:
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(HERE, "..", "include", "ssbls.h")]
    procs, objs = [], []
    for s in SOURCES:
        obj = os.path.join(OBJDIR, s.replace(".hip", ".o"))
        objs.append(obj)
        stamp = obj + ".srchash"
        # per-object cache: the TU and every header (headers are shared)
        h = _hash(headers + [os.path.join(CSRC, s)])
        if not force and os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read().strip() == h:
            continue
        cmd = [HIPCC] + FLAGS + ["-c", "-o", obj + ".tmp", os.path.join(CSRC, s)]
        if verbose:
            print("[ssbls] compiling:", " ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), obj, stamp, h))
    for p, obj, stamp, h in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed for %s" % obj)
        os.replace(obj + ".tmp", obj)
        with open(stamp, "w") as f:
            f.write(h + "\n")
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB + ".tmp"] + objs
    if verbose:
        print("[ssbls] linking:", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(STAMP, "w") as f:
        f.write(want + "\n")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
