"""Compiles tests/native/capi_golden.c with gcc against include/ssbls.h, linked to libssbls.so
(rpath into the tree, so it runs from any working directory).  Called by __graft_entry__.build()
and tests/test_capi.py; the binary is git-ignored and travels to the GPU box with the tree."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SRC = os.path.join(HERE, "capi_golden.c")
BIN = os.path.join(HERE, "capi_golden")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def build_capi(force=False):
    lib_dir = os.path.join(ROOT, "safestakeoperator_amd")
    lib = os.path.join(lib_dir, "libssbls.so")
    if not force and os.path.exists(BIN) and os.path.getmtime(BIN) >= max(os.path.getmtime(SRC), os.path.getmtime(lib)):
        return BIN
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
           "-o", BIN + ".tmp", "-L", lib_dir, "-lssbls", "-L", os.path.join(ROCM, "lib"),
           "-Wl,-rpath,$ORIGIN/../../safestakeoperator_amd", "-Wl,-rpath," + os.path.join(ROCM, "lib")]
    subprocess.run(cmd, check=True)
    os.replace(BIN + ".tmp", BIN)
    return BIN


if __name__ == "__main__":
    print(build_capi(force=True))
