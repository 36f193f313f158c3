"""CPU oracle: pure-Python restatement of the BLS12-381 arithmetic on SafeStake's threshold path.

TEST INFRASTRUCTURE ONLY.  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import this module, and only as the checker.  The product path
(`safestakeoperator_amd`, `libssbls.so`) never imports or calls anything under `oracle/`.

What it restates (the reference's own arithmetic lives in blst 0.3.10, a crates.io dependency
that is NOT vendored in /root/reference):

* curve BLS12-381, `min_pk` variant: public keys in G1, signatures in G2
  (reference: src/crypto/impls/blst.rs:7 `pub use blst::min_pk as blst_core`);
* DST ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_`` (src/crypto/impls/blst.rs:11);
* hash_to_G2 = RFC 9380 suite BLS12381G2_XMD:SHA-256_SSWU_RO_ (expand_message_xmd, SSWU on the
  3-isogenous curve, 3-isogeny, clear_cofactor by h_eff);
* ZCash compressed serialisation (96-byte G2 / 48-byte G1, flags 0x80/0x40/0x20), the format
  `Signature::serialize()` / `blst_p2_compress` produce (src/crypto/impls/blst.rs:77,86);
* `Signature::verify(pk, msg)` = blst `verify(sig_groupcheck=true, msg, DST, aug=[], pk,
  pk_validate=false)` (SafeStake's direct use of the same convention:
  src/network/io_committee.rs:536-539), i.e. subgroup check of the signature, then
  e(pk, H(m)) == e(g1, sig);
* optimal-ate pairing with the final exponentiation (p^12-1)/r.

Parity status: pinned by known-answer vectors held in tests/golden/known_answers.json
(RFC 9380 Appendix K.2 hash_to_curve vectors, the Ethereum consensus BLS `sign` vectors and the
Ethereum interop keypair), and by the reference's own relational test
(tests/test_generic_threshold.rs:26-35: threshold combine == master signature, both verify).
"""
from __future__ import annotations

import hashlib

# ----------------------------------------------------------------------------------------------
# Parameters
# ----------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
# r: src/crypto/define.rs:27-28 ("0x73eda753...00000001")
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # |x|, the BLS parameter x = -0xd201000000010000
X = -X_ABS

DST_POP = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"

# ----------------------------------------------------------------------------------------------
# Fp
# ----------------------------------------------------------------------------------------------

def fp_inv(a: int) -> int:
    return pow(a, P - 2, P)


def fp_sqrt(a: int):
    """Square root in Fp (p = 3 mod 4); None if a is a non-residue."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_sgn0(a: int) -> int:
    return a % 2


def fp_is_lex_largest(a: int) -> bool:
    """ZCash 'sign' bit for Fp: a > (p-1)/2."""
    return a > (P - 1) // 2

# ----------------------------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2+1), elements are tuples (c0, c1)
# ----------------------------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_muls(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = fp_inv((a[0] * a[0] + a[1] * a[1]) % P)
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_pow(a, e):
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


def f2_sqrt(a):
    """A square root of a in Fp2, or None.  Any root is returned (callers fix the sign)."""
    if f2_is_zero(a):
        return F2_ZERO
    a0, a1 = a
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0 % P)
        return (0, s)
    n = (a0 * a0 + a1 * a1) % P
    s = fp_sqrt(n)
    if s is None:
        return None
    inv2 = (P + 1) // 2
    c = (a0 + s) * inv2 % P
    x0 = fp_sqrt(c)
    if x0 is None:
        c = (a0 - s) * inv2 % P
        x0 = fp_sqrt(c)
        if x0 is None:
            return None
    x1 = a1 * fp_inv(2 * x0 % P) % P
    r = (x0, x1)
    return r if f2_sqr(r) == (a0 % P, a1 % P) else None


def f2_sgn0(a):
    """RFC 9380 sgn0 for Fp2."""
    sign_0 = a[0] % 2
    zero_0 = a[0] == 0
    sign_1 = a[1] % 2
    return sign_0 | (zero_0 and sign_1)


def f2_is_lex_largest(a):
    """ZCash sign bit for Fp2: compare c1 first, c0 if c1 == 0."""
    if a[1] != 0:
        return a[1] > (P - 1) // 2
    return a[0] > (P - 1) // 2


XI = (1, 1)  # xi = 1 + u, the non-residue defining Fp6 and the sextic twist


def f2_mul_xi(a):
    # (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
    return ((a[0] - a[1]) % P, (a[0] + a[1]) % P)

# ----------------------------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v)
# ----------------------------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_add(f2_mul(a1, b2), f2_mul(a2, b1))))
    c1 = f2_add(f2_add(f2_mul(a0, b1), f2_mul(a1, b0)), f2_mul_xi(t2))
    c2 = f2_add(f2_add(f2_mul(a0, b2), f2_mul(a2, b0)), t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    # (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    c0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    c1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    c2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    t = f2_add(f2_mul(a0, c0), f2_mul_xi(f2_add(f2_mul(a2, c1), f2_mul(a1, c2))))
    ti = f2_inv(t)
    return (f2_mul(c0, ti), f2_mul(c1, ti), f2_mul(c2, ti))


F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c0 = f6_add(t0, f6_mul_v(t1))
    c1 = f6_add(f6_mul(a0, b1), f6_mul(a1, b0))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e):
    r = F12_ONE
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


def f12_from_f2_coeffs(cs):
    """cs[k] = coefficient of w^k, k=0..5 (w^2 = v): returns the Fp12 element."""
    # w^k: k even -> c0 part, v^(k/2); k odd -> c1 part, v^((k-1)/2)
    return ((cs[0], cs[2], cs[4]), (cs[1], cs[3], cs[5]))


def f12_is_one(a):
    return a == F12_ONE

# ----------------------------------------------------------------------------------------------
# Curves.  E1: y^2 = x^3 + 4 over Fp;  E2 (twist): y^2 = x^3 + 4(1+u) over Fp2.
# Points are affine tuples (x, y) or None for the point at infinity.
# ----------------------------------------------------------------------------------------------
B1 = 4
B2 = (4, 4)

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)


class _Fp:  # field-op namespace for the generic curve code
    zero = 0
    one = 1
    add = staticmethod(lambda a, b: (a + b) % P)
    sub = staticmethod(lambda a, b: (a - b) % P)
    mul = staticmethod(lambda a, b: a * b % P)
    neg = staticmethod(lambda a: (-a) % P)
    inv = staticmethod(fp_inv)


class _Fp2:
    zero = F2_ZERO
    one = F2_ONE
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    neg = staticmethod(f2_neg)
    inv = staticmethod(f2_inv)


def _ec_add(F, p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if y1 == y2 and y1 != F.zero:
            lam = F.mul(F.mul(F.mul(x1, x1), F.add(F.one, F.add(F.one, F.one))), F.inv(F.add(y1, y1)))
        else:
            return None
    else:
        lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
    x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
    y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
    return (x3, y3)


def _ec_neg(F, p1):
    return None if p1 is None else (p1[0], F.neg(p1[1]))


def _ec_mul(F, pt, k):
    if k < 0:
        return _ec_mul(F, _ec_neg(F, pt), -k)
    acc = None
    add = pt
    while k:
        if k & 1:
            acc = _ec_add(F, acc, add)
        add = _ec_add(F, add, add)
        k >>= 1
    return acc


def g1_add(a, b):
    return _ec_add(_Fp, a, b)


def g1_neg(a):
    return _ec_neg(_Fp, a)


def g1_mul(a, k):
    return _ec_mul(_Fp, a, k)


def g2_add(a, b):
    return _ec_add(_Fp2, a, b)


def g2_neg(a):
    return _ec_neg(_Fp2, a)


def g2_mul(a, k):
    return _ec_mul(_Fp2, a, k)


def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g2_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO

# psi = untwist-Frobenius-twist endomorphism on E2 (acts as [p] = [x] on G2)
PSI_CX = f2_inv(f2_pow(XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(XI, (P - 1) // 2))


def g2_psi(pt):
    if pt is None:
        return None
    x, y = pt
    return (f2_mul(f2_conj(x), PSI_CX), f2_mul(f2_conj(y), PSI_CY))


def g2_in_subgroup_slow(pt):
    return g2_mul(pt, R) is None


def g2_in_subgroup(pt):
    """G2 membership: psi(P) == [x]P (Scott 2021; equivalent to [r]P == O on BLS12-381)."""
    if pt is None:
        return True
    return g2_psi(pt) == g2_mul(pt, X)


def g1_in_subgroup_slow(pt):
    return g1_mul(pt, R) is None

# ----------------------------------------------------------------------------------------------
# Serialisation (ZCash format, as blst_p1_compress / blst_p2_compress / *_uncompress)
# ----------------------------------------------------------------------------------------------

def g1_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(47)
    x, y = pt
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80
    if fp_is_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


class DecodeError(Exception):
    pass


def g1_decompress(b: bytes):
    """blst_p1_uncompress semantics (no subgroup check); raises DecodeError."""
    if len(b) != 48:
        raise DecodeError("length")
    b0 = b[0]
    if not (b0 & 0x80):
        raise DecodeError("not compressed")
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise DecodeError("bad infinity")
    x = int.from_bytes(bytes([b0 & 0x1F]) + b[1:], "big")
    if x >= P:
        raise DecodeError("x >= p")
    y = fp_sqrt((x * x * x + B1) % P)
    if y is None:
        raise DecodeError("not on curve")
    if fp_is_lex_largest(y) != bool(b0 & 0x20):
        y = (-y) % P
    return (x, y)


def g2_compress(pt) -> bytes:
    if pt is None:
        return bytes([0xC0]) + bytes(95)
    x, y = pt
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80
    if f2_is_lex_largest(y):
        b[0] |= 0x20
    return bytes(b)


def g2_decompress(b: bytes):
    """blst_p2_uncompress semantics (no subgroup check); raises DecodeError."""
    if len(b) != 96:
        raise DecodeError("length")
    b0 = b[0]
    if not (b0 & 0x80):
        raise DecodeError("not compressed")
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return None
        raise DecodeError("bad infinity")
    x1 = int.from_bytes(bytes([b0 & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x0 >= P or x1 >= P:
        raise DecodeError("x >= p")
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B2))
    if y is None:
        raise DecodeError("not on curve")
    if f2_is_lex_largest(y) != bool(b0 & 0x20):
        y = f2_neg(y)
    return (x, y)


def g2_serialize_uncompressed(pt) -> bytes:
    """blst_p2_serialize: 192 bytes x.c1|x.c0|y.c1|y.c0, 0x40 flag for infinity."""
    if pt is None:
        return bytes([0x40]) + bytes(191)
    x, y = pt
    return (x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big")
            + y[1].to_bytes(48, "big") + y[0].to_bytes(48, "big"))

# ----------------------------------------------------------------------------------------------
# Pairing: optimal ate, computed on the untwisted point in E(Fp12) with affine chord/tangent
# lines (deliberately the plain textbook form; the device uses projective formulas).
# ----------------------------------------------------------------------------------------------
# w in Fp12 (coefficient 1 at w^1), and its inverse powers for the untwist (x/w^2, y/w^3).
_W = f12_from_f2_coeffs([F2_ZERO, F2_ONE, F2_ZERO, F2_ZERO, F2_ZERO, F2_ZERO])
_W_INV = f12_inv(_W)
_W_INV2 = f12_mul(_W_INV, _W_INV)
_W_INV3 = f12_mul(_W_INV2, _W_INV)


def _f2_to_f12(a):
    return ((a, F2_ZERO, F2_ZERO), F6_ZERO)


def _fp_to_f12(a):
    return _f2_to_f12((a % P, 0))


def _untwist(q):
    x, y = q
    return (f12_mul(_f2_to_f12(x), _W_INV2), f12_mul(_f2_to_f12(y), _W_INV3))


def _f12_sub(a, b):
    return (f6_sub(a[0], b[0]), f6_sub(a[1], b[1]))


def _f12_add(a, b):
    return (f6_add(a[0], b[0]), f6_add(a[1], b[1]))


def miller_loop(p_g1, q_g2):
    """f_{|x|,Q}(P), conjugated for negative x.  Returns an Fp12 element before final exp."""
    if p_g1 is None or q_g2 is None:
        return F12_ONE
    xp, yp = _fp_to_f12(p_g1[0]), _fp_to_f12(p_g1[1])
    Q = _untwist(q_g2)
    T = Q
    f = F12_ONE
    three = _fp_to_f12(3)
    two = _fp_to_f12(2)
    for bit in bin(X_ABS)[3:]:
        # tangent at T
        xt, yt = T
        lam = f12_mul(f12_mul(three, f12_sqr(xt)), f12_inv(f12_mul(two, yt)))
        line = _f12_sub(_f12_sub(yp, yt), f12_mul(lam, _f12_sub(xp, xt)))
        f = f12_mul(f12_sqr(f), line)
        x3 = _f12_sub(_f12_sub(f12_sqr(lam), xt), xt)
        y3 = _f12_sub(f12_mul(lam, _f12_sub(xt, x3)), yt)
        T = (x3, y3)
        if bit == "1":
            xt, yt = T
            xq, yq = Q
            lam = f12_mul(_f12_sub(yq, yt), f12_inv(_f12_sub(xq, xt)))
            line = _f12_sub(_f12_sub(yp, yt), f12_mul(lam, _f12_sub(xp, xt)))
            f = f12_mul(f, line)
            x3 = _f12_sub(_f12_sub(f12_sqr(lam), xt), xq)
            y3 = _f12_sub(f12_mul(lam, _f12_sub(xt, x3)), yt)
            T = (x3, y3)
    return f12_conj(f)  # x < 0


FINAL_EXP = (P ** 12 - 1) // R


def final_exponentiation(f):
    return f12_pow(f, FINAL_EXP)


def pairing(p_g1, q_g2):
    return final_exponentiation(miller_loop(p_g1, q_g2))


def pairing_product_is_one(pairs):
    f = F12_ONE
    for p1, q2 in pairs:
        f = f12_mul(f, miller_loop(p1, q2))
    return f12_is_one(final_exponentiation(f))

# ----------------------------------------------------------------------------------------------
# hash_to_G2: RFC 9380, suite BLS12381G2_XMD:SHA-256_SSWU_RO_
# ----------------------------------------------------------------------------------------------

def expand_message_xmd(msg: bytes, dst: bytes, len_in_bytes: int) -> bytes:
    b_in_bytes, r_in_bytes = 32, 64
    ell = (len_in_bytes + b_in_bytes - 1) // b_in_bytes
    assert ell <= 255 and len(dst) <= 255
    dst_prime = dst + bytes([len(dst)])
    msg_prime = bytes(r_in_bytes) + msg + len_in_bytes.to_bytes(2, "big") + b"\x00" + dst_prime
    b0 = hashlib.sha256(msg_prime).digest()
    b = [hashlib.sha256(b0 + b"\x01" + dst_prime).digest()]
    for i in range(2, ell + 1):
        b.append(hashlib.sha256(bytes(x ^ y for x, y in zip(b0, b[-1])) + bytes([i]) + dst_prime).digest())
    return b"".join(b)[:len_in_bytes]


def hash_to_field_fp2(msg: bytes, dst: bytes, count: int = 2):
    L = 64
    data = expand_message_xmd(msg, dst, count * 2 * L)
    out = []
    for i in range(count):
        e = [int.from_bytes(data[L * (j + i * 2): L * (j + i * 2 + 1)], "big") % P for j in range(2)]
        out.append((e[0], e[1]))
    return out

SSWU_A = (0, 240)
SSWU_B = (1012, 1012)
SSWU_Z = f2_neg((2, 1))


def map_to_curve_sswu_e2p(u):
    """Simplified SWU onto E2': y^2 = x^3 + A'x + B' (RFC 9380 §6.6.2).  Output is unique:
    x = x1 if g(x1) is square else Z u^2 x1, and sgn0(y) == sgn0(u)."""
    A, B, Z = SSWU_A, SSWU_B, SSWU_Z
    zu2 = f2_mul(Z, f2_sqr(u))
    den = f2_add(f2_sqr(zu2), zu2)
    if f2_is_zero(den):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(den)))

    def g(x):
        return f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(A, x)), B)

    y = f2_sqrt(g(x1))
    if y is not None:
        x = x1
    else:
        x = f2_mul(zu2, x1)
        y = f2_sqrt(g(x))
        assert y is not None
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)

# 3-isogeny E2' -> E2 (RFC 9380 Appendix E.3)
_ISO_XNUM = [
    (0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    (0,
     0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1,
     0),
]
_ISO_XDEN = [
    (0,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
    (0xC,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
    (1, 0),
]
_ISO_YNUM = [
    (0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
     0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    (0,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10,
     0),
]
_ISO_YDEN = [
    (0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB),
    (0,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
    (0x12,
     0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
    (1, 0),
]
ISO3_CONSTANTS = {"xnum": _ISO_XNUM, "xden": _ISO_XDEN, "ynum": _ISO_YNUM, "yden": _ISO_YDEN}


def _poly_eval(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def iso3_map(pt):
    if pt is None:
        return None
    xp, yp = pt
    xden = _poly_eval(_ISO_XDEN, xp)
    yden = _poly_eval(_ISO_YDEN, xp)
    if f2_is_zero(xden) or f2_is_zero(yden):
        return None
    x = f2_mul(_poly_eval(_ISO_XNUM, xp), f2_inv(xden))
    y = f2_mul(yp, f2_mul(_poly_eval(_ISO_YNUM, xp), f2_inv(yden)))
    return (x, y)


H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551


def clear_cofactor_g2(pt):
    """h_eff * P via Budroni-Pintore: [x^2-x-1]P + [x-1]psi(P) + psi^2(2P) (RFC 9380 G.3)."""
    if pt is None:
        return None
    t1 = g2_mul(pt, X)                      # [x]P
    t2 = g2_psi(pt)                          # psi(P)
    t3 = g2_add(pt, pt)                      # 2P
    t3 = g2_psi(g2_psi(t3))                  # psi^2(2P)
    t3 = g2_add(t3, g2_neg(t2))              # psi^2(2P) - psi(P)
    t2 = g2_add(t1, t2)                      # [x]P + psi(P)
    t2 = g2_mul(t2, X)                       # [x^2]P + [x]psi(P)
    t3 = g2_add(t3, t2)
    t3 = g2_add(t3, g2_neg(t1))
    return g2_add(t3, g2_neg(pt))


def hash_to_g2(msg: bytes, dst: bytes = DST_POP):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    q0 = iso3_map(map_to_curve_sswu_e2p(u0))
    q1 = iso3_map(map_to_curve_sswu_e2p(u1))
    return clear_cofactor_g2(g2_add(q0, q1))

# ----------------------------------------------------------------------------------------------
# BLS signatures (min_pk, PoP ciphersuite)
# ----------------------------------------------------------------------------------------------

def sk_to_pk(sk: int):
    return g1_mul(G1_GEN, sk % R)


def sign(sk: int, msg: bytes, dst: bytes = DST_POP):
    """SecretKey::sign = H(m)*sk (src/node/dvfcore.rs:241-243)."""
    return g2_mul(hash_to_g2(msg, dst), sk % R)


def verify_points(pk, sig, msg: bytes, dst: bytes = DST_POP, h=None) -> bool:
    """blst Signature::verify(sig_groupcheck=true, msg, dst, aug=[], pk, pk_validate=false)."""
    if pk is None:
        return False  # BLST_PK_IS_INFINITY
    if not g2_in_subgroup(sig):
        return False
    if h is None:
        h = hash_to_g2(msg, dst)
    return pairing_product_is_one([(pk, h), (g1_neg(G1_GEN), sig)])


def verify(pk48: bytes, sig96: bytes, msg: bytes, dst: bytes = DST_POP) -> bool:
    try:
        pk = g1_decompress(pk48)
        sig = g2_decompress(sig96)
    except DecodeError:
        return False
    return verify_points(pk, sig, msg, dst)

# ----------------------------------------------------------------------------------------------
# Threshold layer (src/crypto/impls/blst.rs, src/crypto/generic_threshold.rs)
# ----------------------------------------------------------------------------------------------

def lagrange_coeffs(ids):
    """src/crypto/impls/blst.rs:19-39: lambda_i = prod_{j!=i} x_j * (x_j - x_i)^{-1} mod r,
    with blst_sk_inverse(0) == 0 (only reachable with duplicate ids)."""
    out = []
    for i, xi in enumerate(ids):
        p = 1
        for j, xj in enumerate(ids):
            if i != j:
                d = (xj - xi) % R
                dinv = pow(d, R - 2, R) if d else 0
                p = p * (xj % R) % R * dinv % R
        out.append(p)
    return out


def unsafe_aggregate_points(sigs, ids, t):
    """src/crypto/impls/blst.rs:67-87: sum_{i<t} lambda_i * sig_i, started from infinity."""
    if len(ids) != t:
        raise ValueError("Different length")  # require() panics (src/utils/error.rs:4-8)
    lam = lagrange_coeffs(ids)
    acc = None
    for i in range(t):
        acc = g2_add(acc, g2_mul(sigs[i], lam[i]))
    return acc


# DvfError tags used across the C ABI (include/ssbls.h)
OK = 0
DIFFERENT_LENGTH = 1
INSUFFICIENT_SIGNATURES = 2
INVALID_OPERATOR_ID = 3
INSUFFICIENT_VALID_SIGNATURES = 4


def threshold_aggregate(t, sigs96, pks48, ids, msg, verify_fn=None):
    """src/crypto/generic_threshold.rs:132-175, exact selection and error order.

    Returns (status, payload) where payload is the 96-byte combined signature on success, or
    the error fields (x, y) / (got, expected) / (id,)."""
    if len(sigs96) != len(pks48):
        return DIFFERENT_LENGTH, (len(sigs96), len(pks48))
    if len(sigs96) != len(ids):
        return DIFFERENT_LENGTH, (len(sigs96), len(ids))
    if len(sigs96) < t:
        return INSUFFICIENT_SIGNATURES, (len(sigs96), t)
    vf = verify_fn or (lambda i: verify(pks48[i], sigs96[i], msg))
    sel_sigs, sel_ids, seen = [], [], set()
    for i in range(len(sigs96)):
        if ids[i] == 0:
            return INVALID_OPERATOR_ID, (ids[i],)
        if ids[i] in seen:
            continue
        if vf(i):
            sel_sigs.append(sigs96[i])
            sel_ids.append(ids[i])
            seen.add(ids[i])
            if len(sel_ids) >= t:
                break
    if len(sel_ids) < t:
        return INSUFFICIENT_VALID_SIGNATURES, (len(sel_ids), t)
    pts = [g2_decompress(s) for s in sel_sigs]
    return OK, g2_compress(unsafe_aggregate_points(pts, sel_ids, t))

# ----------------------------------------------------------------------------------------------
# Key split (fixture side): src/crypto/generic_threshold.rs:59-80, src/math/polynomial.rs:39-51
# ----------------------------------------------------------------------------------------------

def poly_eval(coeffs, x):
    """Horner, as Polynomial::eval; reduced mod r as Ring::reduce (src/math/bigint_ext.rs:9-18)."""
    acc = 0
    for c in reversed(coeffs):
        acc = acc * x + c
    return acc % R


def key_split(sk: int, coeffs_tail, ids):
    coeffs = [sk] + list(coeffs_tail)
    return {i: poly_eval(coeffs, i) for i in ids}


# ---- wire format of a partial signature ----
# bincode::serialize(&sig) (src/node/dvfcore.rs:245-251) of lighthouse's bls::Signature, whose serde
# form is the string "0x" + lowercase hex of the 96-byte compressed point; bincode 1.x (fixint,
# little endian) writes a string as a u64 length and the bytes.  (The lighthouse serde macro is
# upstream, not in the reference tree: this layout follows SURVEY.md §8a-6.)
def bincode_signature(sig96: bytes) -> bytes:
    s = b"0x" + sig96.hex().encode()
    return len(s).to_bytes(8, "little") + s


def bincode_signature_decode(rec: bytes):
    """(status, sig96 or None): 0 ok, 1 length field not 194, 2 no "0x", 3 non-hex digit, 4 the
    point does not decompress (bincode::deserialize::<Signature> runs Signature::deserialize, i.e.
    blst uncompress: flags, x < p, on the curve; src/validation/operator.rs:108-113 drops the
    record on any of these)."""
    if int.from_bytes(rec[:8], "little") != 194:
        return 1, None
    if rec[8:10] != b"0x":
        return 2, None
    try:
        sig = bytes.fromhex(rec[10:204].decode("ascii"))
    except ValueError:
        return 3, None
    try:
        g2_decompress(sig)
    except DecodeError:
        return 4, None
    return 0, sig


# ---- DKG / VSS share verification ----
def committed_poly_from_bytes(comm48):
    """CommittedPoly::from_bytes (src/math/polynomial.rs:101-118): blst_p1_uncompress's return
    code is ignored, so bytes that do not decode leave the zeroed affine point, which
    blst_p1_from_affine maps to the identity (None here)."""
    out = []
    for b in comm48:
        try:
            out.append(g1_decompress(b))
        except DecodeError:
            out.append(None)
    return out


def committed_poly_eval(commitments, x: int):
    """CommittedPoly::eval (src/math/polynomial.rs:68-81): C_0 + sum_{i>=1} [x^i mod r] C_i with
    x^i accumulated by blst_sk_mul_n_check (mod r)."""
    y = commitments[0]
    xp = x % R
    for c in commitments[1:]:
        y = g1_add(y, g1_mul(c, xp))
        xp = xp * x % R
    return y


def feldman_share_verify(h, share: int, commitments, party: int) -> bool:
    """DKG share_verification (src/crypto/dkg.rs:433-450): blst_p1_mult(h, s) (255-bit scalar, s
    from LE bytes; blst reads its low 255 bits) == committed_poly.eval(party).
    PARITY UNPINNED for a commitment outside G1: blst_p1_mult uses GLV for 255-bit scalars, which
    is [k]P only on G1, so the reference's result there is blst-defined; like the engine, this
    restatement rejects such a commitment (an honest dealer never sends one)."""
    if any(c is not None and not g1_in_subgroup_slow(c) for c in commitments):
        return False
    return g1_mul(h, share & ((1 << 255) - 1)) == committed_poly_eval(commitments, party)


def hash_points_to_scalar(points) -> int:
    """hash_points_to_blst_scalar (src/utils/blst_utils.rs:273-278): the compressed points
    concatenated, read as ONE little-endian integer and reduced mod r (blst_scalar_from_le_bytes)."""
    return int.from_bytes(b"".join(g1_compress(p) for p in points), "little") % R


def dleq_prove(x1, x2, alpha: int, w: int):
    """DKG::dleq_prove (src/crypto/dkg.rs:649-672) with a given nonce w: (y1, y2, c, r)."""
    y1, y2 = g1_mul(x1, alpha), g1_mul(x2, alpha)
    t1, t2 = g1_mul(x1, w), g1_mul(x2, w)
    c = hash_points_to_scalar([x1, y1, x2, y2, t1, t2])
    return y1, y2, c, (w - alpha * c) % R


def dleq_verify(x1, y1, x2, y2, c: int, r: int) -> bool:
    """DKG::dleq_verify (src/crypto/dkg.rs:674-692): t_i = [r]x_i + [c]y_i (255-bit scalars),
    accept iff c == hash_points_to_scalar(x1, y1, x2, y2, t1, t2)."""
    m = (1 << 255) - 1
    t1 = g1_add(g1_mul(x1, r & m), g1_mul(y1, c & m))
    t2 = g1_add(g1_mul(x2, r & m), g1_mul(y2, c & m))
    return c == hash_points_to_scalar([x1, y1, x2, y2, t1, t2])
