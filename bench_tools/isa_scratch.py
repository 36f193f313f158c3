"""Static scratch (spill) census of a translation unit's gfx950 code: per function, the scratch
stores / loads in the body and inside loops, and each kernel's private segment.

    python bench_tools/isa_scratch.py safestakeoperator_amd/csrc/ssb_k_fused.hip [filter] [--blocks]
(--blocks: also every basic block with spill code or > 500 instructions; the last column is then the
block's instruction count)
"""
import os
import re
import subprocess
import sys
import tempfile

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def blocks(lines, i):
    """per basic block of the function starting at line i: (label, stores, loads, instructions)"""
    out, lab = [], None
    for l in lines[i + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        if l.startswith(".LBB"):
            lab = [l.split(":")[0], 0, 0, 0]
            out.append(lab)
            continue
        if lab is None or not l.startswith("\t") or l.startswith("\t.") or l.startswith("\t;"):
            continue
        lab[3] += 1
        lab[1] += "scratch_store" in l
        lab[2] += "scratch_load" in l
    return out


def census(src, filt="", per_block=False):
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
            if per_block:
                for b in blocks(lines, i):
                    if b[3] > 500 or b[1] or b[2]:
                        out.append(("    " + b[0], b[1], b[2], 0, 0, 0, b[3]))
        i = j
    return out


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--blocks"]
    for row in census(args[0], args[1] if len(args) > 1 else "", "--blocks" in sys.argv):
        print("%-70s st %4d ld %4d loop st %3d ld %3d calls %2d scratch %s" % ((row[0][:70],) + row[1:]))
