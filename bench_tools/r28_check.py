"""Host check of bench_tools/r28_bench's samples: r == a * b^3 * 2^(-392*3) (mod p) for the 3-step
chain a <- a b / 2^392 (r < 2p, compared mod p).  Reads the JSON on stdin, prints the verdict."""
import json
import sys

P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab


def val(h):
    limbs = [int(x, 16) for x in h.strip(",").split(",")]   # most significant first
    v = 0
    for l in limbs:
        v = (v << 28) + l
    return v


d = json.load(sys.stdin)
Ri = pow(2 ** 392, -1, P)
ok = all((val(a) * pow(val(b), 3, P) * pow(Ri, 3, P) - val(r)) % P == 0 and val(r) < 2 * P for a, b, r in d["samples"])
print(json.dumps({"samples_ok": ok, "short": d["short_Gmul_s"], "sustained": d["sustained_2s"]}))
sys.exit(0 if ok else 1)
