"""Static scratch (spill) census of a translation unit's gfx950 code: per function, the scratch
stores / loads in the body and inside loops, and each kernel's private segment.

    python bench_tools/isa_scratch.py safestakeoperator_amd/csrc/ssb_k_fused.hip [filter]
"""
import os
import re
import subprocess
import sys
import tempfile

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def census(src, filt=""):
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "out.s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "-S",
                        "-Wno-unused-result", "-Wno-unused-value", "-o", asm, src], check=True, capture_output=True)
        lines = open(asm).read().split("\n")
    out = []
    i = 0
    while i < len(lines):
        m = re.match(r"\t\.type\t(\S+),@function", lines[i])
        if not m:
            i += 1
            continue
        name, lab = m.group(1), ""
        st = ld = lst = lld = calls = 0
        scratch = None
        j = i + 1
        while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
            l = lines[j]
            if l.startswith(".LBB"):
                lab = l
            if "scratch_store" in l:
                st += 1
                lst += "in Loop" in lab
            elif "scratch_load" in l:
                ld += 1
                lld += "in Loop" in lab
            elif "s_swappc" in l:
                calls += 1
            j += 1
        for k in range(j, min(j + 40, len(lines))):
            mm = re.search(r"; ScratchSize: (\d+)", lines[k])
            if mm:
                scratch = int(mm.group(1))
                break
        if filt in name:
            out.append((name, st, ld, lst, lld, calls, scratch))
        i = j
    return out


if __name__ == "__main__":
    for row in census(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print("%-70s st %4d ld %4d loop st %3d ld %3d calls %2d scratch %s" % ((row[0][:70],) + row[1:]))
