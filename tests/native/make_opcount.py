"""Build the instrumented host copy of the device units (SSB_OPCOUNT) and write
bench_tools/opcount.json: Fp mul/sqr and Fr mul counts per work unit of every kernel
(SURVEY.md §8d).  Run from the repo root: python tests/native/make_opcount.py [--check]"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(ROOT, "bench_tools", "opcount.json")
CXX = os.environ.get("SSB_HOST_CXX", "/opt/rocm/llvm/bin/clang++")


def build_host(opcount: bool) -> str:
    exe = os.path.join(tempfile.gettempdir(), "ssb_host_math%s" % ("_cnt" if opcount else ""))
    src = os.path.join(HERE, "host_math.cpp")
    cmd = [CXX, "-std=c++17", "-O2", "-o", exe, src] + (["-DSSB_OPCOUNT"] if opcount else [])
    subprocess.run(cmd, check=True)
    return exe


def measure():
    exe = build_host(True)
    with open(os.path.join(ROOT, "tests", "golden", "threshold_cases.json")) as f:
        c = json.load(f)["cases"][0]
    line = "opcount %s %s %s\n" % (c["pks"][0], c["sigs"][0], c["root"])
    out = subprocess.run([exe], input=line, capture_output=True, text=True, check=True).stdout.strip()
    d = json.loads(out)
    d["_doc"] = ("per-unit Fp mul / Fp sqr / Fr mul counts of the exact device code (ssb_units.h), from "
                 "tests/native/make_opcount.py; MADs/unit = 300*(fp_mul+fp_sqr) + 136*fr_mul (SURVEY.md 8d)")
    return d


if __name__ == "__main__":
    d = measure()
    if "--check" in sys.argv:
        with open(OUT) as f:
            old = json.load(f)
        sys.exit(0 if old == d else 1)
    with open(OUT, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    print("wrote", OUT)
