"""Host check of bench_tools/fp28_bench samples: r == a * b * 2^-392 mod p (14 x 28-bit limbs)."""
import json
import sys

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
d = json.load(open(sys.argv[1]))
ok = True
for a, b, r in d["samples"]:
    a, b, r = int(a, 16), int(b, 16), int(r, 16)
    ok &= r == a * b * pow(2, -392, P) % P
print("fp28 samples exact:", ok)
sys.exit(0 if ok else 1)
