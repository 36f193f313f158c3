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
           "ssb_k_fused.hip", "ssb_collector.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SSB_OFFLOAD_ARCH", "gfx950")
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result", "-Wno-unused-value"]
if VARIANT:
    FLAGS += os.environ.get("SSB_VARIANT_DEFS", "").split()
STAMP = LIB + ".srchash"
OBJDIR = os.path.join(HERE, "build" + ("_" + VARIANT if VARIANT else ""))
LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")

# Kernels that may hold a private segment larger than the queue primer (k_scratch_prime): each runs
# only inside a SYNCHRONOUS entry point (the call waits for its stream), so no two queues acquire
# scratch for it at the same moment -- the failure the primer prevents (HSA_STATUS_ERROR_OUT_OF_
# RESOURCES when twenty slot queues grew their scratch at once, round 2).  Every kernel of the batch
# path (aggregate / verify, _dev and submit entry points) must fit the primer; the build fails
# otherwise (check_private_segments).
SYNC_ONLY_KERNELS = {
    "k_sign": "ssb_sign_batch",
    "k_sk_to_pk": "ssb_sk_to_pk_batch",
    "k_pk_validate": "ssb_pk_validate_batch",
    "k_combine_terms": "ssb_unsafe_aggregate_batch (255-bit products of unchecked shares)",
    "k_dleq_verify": "ssb_dleq_verify_batch",
    "k_feldman_share": "ssb_feldman_verify_batch",
    "k_scratch_prime": "the primer itself",
}


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


def _prime_bytes():
    import re
    with open(os.path.join(CSRC, "ssb_k_combine.hip")) as f:
        return 4 * int(re.search(r"constexpr int PRIME_WORDS = (\d+);", f.read()).group(1))


def kernel_resources(objs):
    """{kernel: {"private": bytes, "vgpr": n, "agpr": n, "tu": file}} from the gfx950 code objects
    embedded in the compiled objects (.hip_fatbin -> clang-offload-bundler -> llvm-readelf --notes)."""
    import re
    import tempfile
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for obj in objs:
            fb, co = os.path.join(td, "fatbin"), os.path.join(td, "co")
            if subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fb, obj],
                              capture_output=True).returncode != 0:
                continue   # a host-only translation unit (no device code)
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--" + ARCH, "--input=" + fb, "--output=" + co], check=True)
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            for blk in re.split(r"\n\s+- \.", notes):
                m = re.search(r"\.name:\s+(\S+)", blk)
                p = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
                if not (m and p):
                    continue
                mangled = m.group(1)
                k = re.search(r"(k_[A-Za-z0-9_]+?)(?:I|E[ijPKNSvhmR])", mangled)
                name = k.group(1) if k else mangled
                v = re.search(r"\.vgpr_count:\s+(\d+)", blk)
                a = re.search(r"\.agpr_count:\s+(\d+)", blk)
                ent = dict(private=int(p.group(1)), vgpr=int(v.group(1)) if v else None,
                           agpr=int(a.group(1)) if a else None, tu=os.path.basename(obj))
                if name not in res or ent["private"] > res[name]["private"]:
                    res[name] = ent
    return res


# Headroom the batch-path kernels should keep under the primer (round-4 verdict: >= 512 B, so a small
# code change cannot bring back round 2's abort); kernels closer than this are listed in
# kernel_resources.json ("within_headroom_of_primer"), not refused.
HEADROOM = 512


def check_private_segments(objs, out_json=None):
    """Fails when a batch-path kernel's private segment exceeds the queue primer's per-lane array."""
    import json
    limit = _prime_bytes()
    res = kernel_resources(objs)
    bad = {k: v["private"] for k, v in res.items() if v["private"] > limit and k not in SYNC_ONLY_KERNELS}
    for k, v in res.items():
        v["margin"] = limit - v["private"]   # bytes under the primer's per-lane array (negative: sync-only)
    tight = {k: v["private"] for k, v in res.items()
             if k not in SYNC_ONLY_KERNELS and limit - HEADROOM < v["private"] <= limit}
    if out_json:
        with open(out_json, "w") as f:
            json.dump(dict(primer_bytes=limit, headroom_target=HEADROOM, sync_only=SYNC_ONLY_KERNELS,
                           within_headroom_of_primer=tight, kernels=res), f, indent=1, sort_keys=True)
    if bad:
        raise RuntimeError("private segment above the queue primer's %d B/lane (k_scratch_prime) in batch-path "
                           "kernels: %s" % (limit, bad))
    return res


def _code_object(obj, td):
    """The gfx950 code object embedded in a compiled object (None for a host-only TU)."""
    fb, co = os.path.join(td, "fatbin"), os.path.join(td, "co")
    if subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fb, obj],
                      capture_output=True).returncode != 0:
        return None
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--" + ARCH, "--input=" + fb, "--output=" + co], check=True)
    return co


def long_branch_clobbers(objs):
    """{function: count} of callable (non-kernel) device functions whose long branches go through
    s[30:31], the return address.  The compiler relaxes a branch past +-128 KB into
    s_getpc / s_add / s_setpc on a scratch SGPR pair; when the pre-RA size estimate said no long
    branch was coming (amdgpu-long-branch-factor) no pair is reserved and relaxation takes
    s[30:31] without saving it -- the function then "returns" to its own branch target and spins
    forever (the round-4 and round-5 stalls: horner_step<fp2> in the first k_fb_excl form,
    jac_mul_naf_aff, rc_k_chain).  -mllvm -amdgpu-long-branch-factor did not prevent it; the chains
    call small out-of-line steps instead, and this guard fails the build if one slips through."""
    import re
    import tempfile
    bad = {}
    with tempfile.TemporaryDirectory() as td:
        for obj in objs:
            co = _code_object(obj, td)
            if co is None:
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            kernels = set(re.findall(r"\.name:\s+(\S+)", notes))
            p = subprocess.Popen([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                                 stdout=subprocess.PIPE, text=True)
            for f, c in scan_disassembly(p.stdout, kernels).items():
                bad[f] = bad.get(f, 0) + c
            p.wait()
    return bad


def scan_disassembly(lines, kernels):
    """{function: count} of `s_getpc_b64 s[30:31]` in the non-kernel functions of an llvm-objdump -d
    listing (an iterable of lines; `kernels`: the entry points' symbols, whose s[30:31] holds no return
    address)."""
    bad, cur = {}, None
    for line in lines:
        if line.rstrip("\n").endswith(">:"):
            cur = line[line.index("<") + 1:line.rstrip("\n").rindex(">")]
        elif "s_getpc_b64 s[30:31]" in line and cur is not None and cur not in kernels:
            bad[cur] = bad.get(cur, 0) + 1
    return bad


def _guards(objs):
    try:
        check_private_segments(objs, os.path.join(OBJDIR, "kernel_resources.json"))
    except RuntimeError as e:
        if not VARIANT:
            raise
        print("[ssbls] variant %s: %s" % (VARIANT, e), flush=True)   # experiment builds: reported only
    clob = long_branch_clobbers(objs)
    if clob:
        raise RuntimeError("callable device functions whose long branches overwrite the return address "
                           "s[30:31] (they would never return; split them into smaller out-of-line steps): %s"
                           % clob)


def build(force: bool = False, verbose: bool = True) -> str:
    want = _source_hash()
    if not force and os.path.exists(LIB) and os.path.exists(STAMP) and open(STAMP).read().strip() == want:
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(HERE, "..", "include", "ssbls.h")]
    procs, objs, fresh = [], [], []
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
        fresh.append(stamp)
    # private-segment and long-branch guards (before the library is replaced): kernel_resources.json
    # beside the objects; a refused object's stamp is removed so that it does not pass as built next time
    if os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        try:
            _guards(objs)
        except RuntimeError:
            for st in fresh:
                if os.path.exists(st):
                    os.remove(st)
            raise
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB + ".tmp"] + objs
    if verbose:
        print("[ssbls] linking:", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(STAMP, "w") as f:
        f.write(want + "\n")
    return LIB


COLLBENCH_SRC = os.path.join(HERE, "..", "bench_tools", "collbench.cpp")
COLLBENCH_LIB = os.path.join(HERE, "..", "bench_tools", "libcollbench.so")


def build_collbench(verbose: bool = True) -> str:
    """bench_tools/libcollbench.so: the native submitter threads of bench.py's value_collector
    (benchmark / test infrastructure, linked against libssbls.so)."""
    build(verbose=verbose)
    want = _hash([COLLBENCH_SRC, os.path.join(HERE, "..", "include", "ssbls.h")], "collbench" + os.path.basename(LIB))
    stamp = COLLBENCH_LIB + ".srchash"
    if os.path.exists(COLLBENCH_LIB) and os.path.exists(stamp) and open(stamp).read().strip() == want:
        return COLLBENCH_LIB
    cmd = ["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-o", COLLBENCH_LIB + ".tmp", COLLBENCH_SRC,
           "-L" + HERE, "-l:" + os.path.basename(LIB), "-Wl,-rpath,$ORIGIN/../safestakeoperator_amd"]
    if verbose:
        print("[ssbls] building:", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(COLLBENCH_LIB + ".tmp", COLLBENCH_LIB)
    with open(stamp, "w") as f:
        f.write(want + "\n")
    return COLLBENCH_LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    if not VARIANT:   # (bench_tools/libcollbench.so links the product library only)
        build_collbench()
