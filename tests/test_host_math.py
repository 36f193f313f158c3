"""CPU: the device math headers compiled for the host (test-only build, never shipped) against
the oracle's golden fixtures; and the committed op counts match the current device code."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "native"))
import make_opcount  # noqa: E402

GOLD = os.path.join(HERE, "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def host_exe():
    return make_opcount.build_host(False)


def _run(exe, lines):
    r = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    return r.stdout.strip().split("\n")


def test_hash_to_g2(host_exe):
    hc = _load("hash_to_g2.json")["cases"]
    out = _run(host_exe, ["h2g2 " + c["msg"] for c in hc])
    assert out == [c["out192"] for c in hc]
    # RFC 9380 Appendix K.2 (QUUX DST, empty message) through the device code compiled for the host
    v = _load("known_answers.json")["rfc9380_g2"][0]
    o = _run(host_exe, ["h2g2 %s %s" % (v["msg"].encode().hex() or "-", v["dst"].encode().hex())])[0]
    assert [o[0:96], o[96:192], o[192:288], o[288:384]] == [v["P_x"][1], v["P_x"][0], v["P_y"][1], v["P_y"][0]]


def test_point_decoding(host_exe):
    pts = _load("points.json")
    out = _run(host_exe, ["g2dec " + p["compressed"] for p in pts["g2"]] + ["g1dec " + p["compressed"] for p in pts["g1"]])
    for p, line in zip(pts["g2"], out):
        st, sub, unc, cmp_ = line.split()
        assert int(st) & 1 and sub == "1" and unc == p["uncompressed"] and cmp_ == p["compressed"]
    for p, line in zip(pts["g1"], out[len(pts["g2"]):]):
        st, cmp_, x, y = line.split()
        assert int(st) & 1 and cmp_ == p["compressed"]
        if p["x"] is not None:
            assert x == p["x"] and y == p["y"]


def test_share_decoding_and_verify(host_exe):
    cases = _load("threshold_cases.json")["cases"]
    lines = []
    for c in cases[:6]:
        for s, p in zip(c["sigs"], c["pks"]):
            lines.append("verify %s %s %s" % (p, s, c["root"]))
    out = _run(host_exe, lines)
    want = [v for c in cases[:6] for v in c["share_verdicts"]]
    assert [o == "1" for o in out] == want


def test_bad_encodings_rejected(host_exe):
    c = [x for x in _load("threshold_cases.json")["cases"] if x["name"] == "bad_encoding_shares"][0]
    out = _run(host_exe, ["g2dec " + s for s in c["sigs"][:3]])
    assert all(line.split()[0] == "0" for line in out)
    c = [x for x in _load("threshold_cases.json")["cases"] if x["name"] == "non_subgroup_share"][0]
    st, sub = _run(host_exe, ["g2dec " + c["sigs"][0]])[0].split()[:2]
    assert st == "1" and sub == "0"


def test_opcount_is_current():
    with open(make_opcount.OUT) as f:
        committed = json.load(f)
    assert make_opcount.measure() == committed


def test_rlc_scalars_match_restatement(host_exe):
    """The device's RLC scalar derivation (ssb_units.h: ChaCha12 of the batch key and the share
    index, odd) compiled for the host == oracle/rlc.py, for seed-expanded and explicit keys."""
    from oracle import rlc
    lines, want = [], []
    for seed in (0, 1, 0x5AFE57A4E, 2**64 - 1):
        for i in (0, 1, 2, 16383, 2**32 + 5):
            lines.append("rlc %d %d" % (seed, i))
            want.append(rlc.rlc_scalar_odd(rlc.key_from_seed(seed), i))
    key = [0x03020100 + 0x04040404 * k for k in range(8)]
    for i in (0, 7, 2**40):
        lines.append("rlc 0 %d %s" % (i, " ".join("%08x" % w for w in key)))
        want.append(rlc.rlc_scalar_odd(key, i))
    assert [int(x) for x in _run(host_exe, lines)] == want


def test_lane_programs_match_single_lane(host_exe):
    """The generated lane-group programs (G2/G1 dbl, add, mixed add with exception checks, the
    windowed 64-bit multiplication, the subgroup check) reproduce the single-lane code."""
    for seed in ("00" * 31 + "01", "5a" * 32):
        ok, n = _run(host_exe, ["lane " + seed])[0].split()
        assert ok == n, (ok, n)


def test_lane_programs_are_current():
    import subprocess, sys
    gen = os.path.join(HERE, "..", "safestakeoperator_amd", "csrc", "gen_lane_progs.py")
    hdr = os.path.join(HERE, "..", "safestakeoperator_amd", "csrc", "ssb_lane_progs.h")
    before = open(hdr).read()
    subprocess.run([sys.executable, gen], check=True, capture_output=True)
    assert open(hdr).read() == before


def test_small_lagrange_fast_path(host_exe):
    """Integer Lagrange coefficients (ids 1..t and other id sets whose lambda_i are integers) give
    the same combined signature as the 255-bit lambda_i mod r path; other sets are not eligible."""
    cases = {(1, 2, 3): 1, (3, 1, 2): 1, (2, 3, 4): 1, (1, 2, 3, 4, 5): 1, tuple(range(1, 11)): 1,
             (4, 2, 7, 1, 5, 6, 3): 1, (1, 2, 4): 0, (5, 9, 100): 0, (1, 1, 2): 0}
    lines = ["lagsmall %d %s" % (len(k), " ".join(map(str, k))) for k in cases]
    out = _run(host_exe, lines)
    for (ids, elig), line in zip(cases.items(), out):
        e, same = map(int, line.split())
        assert e == elig, (ids, line)
        if elig:
            assert same == 1, ids


def test_registry_ratio_path(host_exe):
    """Registry ids (arbitrary, < 2^16): T = sum c_i sig_i and [M^-1 mod r] T by its four GLS digits
    (unit_lagrange_ratio / unit_combine_ratio_w4: lane-uniform joint windows) == the 255-bit lambda_i path, with
    M = lcm |prod_{j!=i}(x_j - x_i)|; repeated ids and values past 62 bits are not eligible."""
    import random
    rnd = random.Random(7)
    cases = [(5, 9, 100), (1, 2, 4), (65535, 1, 40000), (17, 3, 60001, 2), (1, 2, 3)]
    cases += [tuple(rnd.sample(range(1, 1 << 16), t)) for t in (3, 3, 3, 4, 4, 5)]
    lines = ["lagratio %d %s" % (len(k), " ".join(map(str, k))) for k in cases]
    lines += ["lagratio 3 1 1 2", "lagratio 3 %d 2 3" % (1 << 62)]
    out = _run(host_exe, lines)
    from math import lcm, prod
    n_elig = 0
    for ids, line in zip(cases, out):
        e, same, M = map(int, line.split())
        D = [prod(x - y for x in ids if x != y) for y in ids]
        L = lcm(*[abs(d) for d in D])
        c = [prod(x for x in ids if x != y) * (L // d) for y, d in zip(ids, D)]
        want = L < 2**62 and all(abs(v) < 2**62 for v in c)   # t = 3 always; wider committees rarely
        assert e == int(want), (ids, line)
        if e:
            n_elig += 1
            assert same == 1 and M == L, (ids, line)
    assert n_elig >= 8
    assert [l.split()[0] for l in out[len(cases):]] == ["0", "0"]


def test_ratio_combine_infinity(host_exe):
    """The windowed ratio combine (unit_combine_ratio_w4) when T = sum c_i sig_i is the point at
    infinity: shares [x_i] P make T = M (sum lambda_i x_i) P = O, and the output is INFINITY_SIGNATURE
    (0xc0 || 0^95), as blst's sum of the 255-bit terms."""
    out = _run(host_exe, ["ratiozero 3 5 9 100", "ratiozero 3 1 2 4", "ratiozero 4 1 2 4 5"])
    for line in out:
        e, sig = line.split()
        assert e == "1" and sig == "c0" + "00" * 95


def test_small_inverse_and_gls_digits(host_exe):
    """inv_small_mod_r (extended Euclid on 64-bit integers + one exact division) == pow(M, -1, r), and
    gls_digits4 (three divisions by u) are the base-u digits, for edge and pseudo-random M < 2^62."""
    import random
    r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    u = 0xd201000000010000
    rnd = random.Random(5)
    Ms = [1, 2, 3, 7, 2**32, 2**32 + 1, 2**61 - 1, 2**62 - 1, 65535 * 65534, 6] + [rnd.randrange(1, 2**62) for _ in range(40)]
    out = _run(host_exe, ["invsmall %d" % M for M in Ms])
    for M, line in zip(Ms, out):
        y, *d = line.split()
        y, d = int(y, 16), list(map(int, d))
        assert y == pow(M, -1, r), M
        assert all(0 <= x < u for x in d[:3]) and sum(x * u ** q for q, x in enumerate(d)) == y, M


def test_lagrange_fast_matches_definition(host_exe):
    """unit_lagrange_fast (ratio form: 64-bit Euclid inverse of M + one Montgomery product per share;
    otherwise unit_lagrange) == prod_{j!=i} x_j / (x_j - x_i) mod r, blst's inverse(0) = 0 for repeated
    ids, for sequential, registry-like and wide id sets."""
    import random
    r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    rnd = random.Random(11)
    cases = [(1, 2, 3), (1, 2, 4), (2, 3, 4), (5, 9, 100), (65535, 1, 40000), (1, 1, 2), (7,), (2**40, 3, 5)]
    cases += [tuple(rnd.sample(range(1, 1 << 16), t)) for t in (3, 3, 4, 4, 5, 7, 10)]
    out = _run(host_exe, ["lagfast %d %s" % (len(k), " ".join(map(str, k))) for k in cases])
    for ids, line in zip(cases, out):
        want = []
        for i, xi in enumerate(ids):
            num, den = 1, 1
            for j, xj in enumerate(ids):
                if j != i:
                    num, den = num * xj % r, den * (xj - xi) % r
            want.append(num * (pow(den, -1, r) if den else 0) % r)
        assert [int(h, 16) for h in line.split()] == want, ids


def test_bucket_madd_matches_generic(host_exe):
    """jac_madd_at (the MSM bucket loops' in-place mixed addition) == jac_add_aff_inl coordinate for
    coordinate, on G2 and G1, including infinity on either side, doubling and opposite points."""
    ok, n = _run(host_exe, ["madd 12"])[0].split()
    assert ok == n and int(n) == 12 * 7


def test_accumulator_engine_reduction(host_exe):
    """la_fin (the lane programs' sum of scaled +-terms in the reduced radix, one signed accumulator per
    28-bit limb, folded below 2p) equals the modular sum, including the edge values 0, p-1 and 2p-1
    (the slot bound) and coefficients up to 60 per term; the unfolded form is congruent."""
    assert _run(host_exe, ["lafin 20000"]) == ["0"]


def test_safegcd_inversion(host_exe):
    """fp_inv (Bernstein-Yang divsteps, ssb_field.h) against Fermat a^(p-2) on 20,000 pseudo-random
    elements and the edge cases 1, 2, p-1, p-2, 2^32, 2^380; inv(0) = 0 (blst semantics)."""
    ok, n = _run(host_exe, ["invtest 20000"])[0].split()
    assert ok == n and int(n) == 20007


def test_reduced_radix_subgroup_check(host_exe):
    """The 14 x 28-bit reduced-radix G2 membership test (ssb_f28.h, the per-share subgroup kernels'
    form since round 6) gives the engine's answer (g2_in_subgroup_inl) on infinity, hash_to_G2
    outputs, their negations and multiples (in G2) and raw isogeny images and their sums with G2
    points (on E2, not in G2); and its products, two-product sums, squarings (the square roots'
    powers) and fold / canon equal the engine's arithmetic on 2,000 random triples, including values
    next to the 64p bound and a 2p - 1 operand."""
    agree, tot, nin, nout, aok, an = map(int, _run(host_exe, ["sg28 200"])[0].split())
    assert agree == tot == 1001 and nin > 500 and nout == 400
    assert aok == an == 10000


def test_reduced_radix_msm_additions(host_exe):
    """The G2 MSM's reduced-radix complete additions (ssb_f28.h pt2_madd / pt2_add / pt2_dbl: the
    bucket and window sums of k_msm_bucket2 / k_msm_window2) give the engine's points for random
    inputs, equal points (doubling), opposite points (infinity), infinity on either side, a chained
    bucket sum and a window recurrence; and the G1 form (pt1_madd, the merged G1 MSM's buckets) the
    same way."""
    ok, n = _run(host_exe, ["pt28 40"])[0].split()
    assert ok == n and int(n) == 40 * 18
