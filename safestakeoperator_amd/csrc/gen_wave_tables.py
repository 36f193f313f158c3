"""Build-time generator for ssb_wave_tables.h: lane-parallel ("bilinear phase") programs of the
BLS12-381 tower operations used by the latency-bound parts of the engine (final exponentiation,
Miller loops).

Each operation is traced SYMBOLICALLY through the same formulas as the single-lane code in
ssb_field.h / ssb_pairing.h.  Every Fp value becomes a linear form (integer coefficients) over
"slots": the op's inputs, constants, and the products the op computes.  A product's operands are
linear forms over earlier slots, so products are grouped into phases by dependency depth; inside
a phase every product is independent and runs on its own lane of a wavefront.  The outputs are
linear forms over inputs and products.  Coefficient c is emitted as |c| repeated +-terms.

Run: python safestakeoperator_amd/csrc/gen_wave_tables.py
"""
import os

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


class Ctx:
    def __init__(self):
        self.products = []  # (phase, xform, yform)
        self.mats = []      # (phase, form): linear values materialised at the end of `phase`

    def product(self, x, y):
        ph = 1 + max([self.phase_of(s) for s in list(x.c) + list(y.c)] + [0])
        self.products.append((ph, x, y))
        return L({("P", len(self.products) - 1): 1})

    def mat(self, form):
        ph = max([self.phase_of(s) for s in form.c] + [0])
        assert ph >= 1, "materialise only forms that depend on products"
        # level inside the phase's linear stage: after every same-phase materialisation it reads
        lvl = 1 + max([self.mats[s[1]][2] for s in form.c if s[0] == "M" and self.mats[s[1]][0] == ph] + [-1])
        self.mats.append((ph, form, lvl))
        return L({("M", len(self.mats) - 1): 1})

    def phase_of(self, sym):
        if sym[0] == "P":
            return self.products[sym[1]][0]
        if sym[0] == "M":
            return self.mats[sym[1]][0]
        return 0


CTX = None


class L:
    """A linear form over symbols: ("A", i) input a, ("B", i) input b, ("K", i) constant, ("P", i) product."""
    __slots__ = ("c",)

    def __init__(self, c=None):
        self.c = {k: v for k, v in (c or {}).items() if v}

    def __add__(self, o):
        d = dict(self.c)
        for k, v in o.c.items():
            d[k] = d.get(k, 0) + v
        return L(d)

    def __sub__(self, o):
        d = dict(self.c)
        for k, v in o.c.items():
            d[k] = d.get(k, 0) - v
        return L(d)

    def __neg__(self):
        return L({k: -v for k, v in self.c.items()})

    def __mul__(self, o):
        if isinstance(o, int):
            return L({k: v * o for k, v in self.c.items()})
        return CTX.product(self, o)

    __rmul__ = __mul__


ZERO = L()


def mat(form):
    return CTX.mat(form)


def mat2(a):
    return (mat(a[0]), mat(a[1]))

# ---------------- tower, mirroring ssb_field.h ----------------


def f2(a, b):
    return (a, b)


def f2_add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def f2_sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def f2_neg(a):
    return (-a[0], -a[1])


def f2_dbl(a):
    return (a[0] * 2, a[1] * 2)


def f2_conj(a):
    return (a[0], -a[1])


def f2_mul(a, b):  # fp2_mul: Karatsuba
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    t2 = (a[0] + a[1]) * (b[0] + b[1])
    return (t0 - t1, t2 - t0 - t1)


def f2_sqr(a):  # fp2_sqr
    m = a[0] * a[1]
    return ((a[0] + a[1]) * (a[0] - a[1]), m * 2)


def f2_mul_fp(a, s):
    return (a[0] * s, a[1] * s)


def f2_mul_xi(a):
    return (a[0] - a[1], a[0] + a[1])


def f6_add(a, b):
    return tuple(f2_add(x, y) for x, y in zip(a, b))


def f6_sub(a, b):
    return tuple(f2_sub(x, y) for x, y in zip(a, b))


def f6_neg(a):
    return tuple(f2_neg(x) for x in a)


def f6_mul(a, b):  # fp6_mul
    t0 = f2_mul(a[0], b[0])
    t1 = f2_mul(a[1], b[1])
    t2 = f2_mul(a[2], b[2])
    u = f2_mul(f2_add(a[1], a[2]), f2_add(b[1], b[2]))
    u = f2_sub(f2_sub(u, t1), t2)
    c0 = f2_add(f2_mul_xi(u), t0)
    u = f2_mul(f2_add(a[0], a[1]), f2_add(b[0], b[1]))
    u = f2_sub(f2_sub(u, t0), t1)
    c1 = f2_add(u, f2_mul_xi(t2))
    u = f2_mul(f2_add(a[0], a[2]), f2_add(b[0], b[2]))
    u = f2_sub(f2_sub(u, t0), t2)
    c2 = f2_add(u, t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_mul_01(a, b0, b1):
    aa = f2_mul(a[0], b0)
    bb = f2_mul(a[1], b1)
    t1 = f2_add(f2_mul_xi(f2_mul(a[2], b1)), aa)
    t2 = f2_sub(f2_sub(f2_mul(f2_add(b0, b1), f2_add(a[0], a[1])), aa), bb)
    t3 = f2_add(f2_mul(a[2], b0), bb)
    return (t1, t2, t3)


def f6_mul_1(a, b1):
    return (f2_mul_xi(f2_mul(a[2], b1)), f2_mul(a[0], b1), f2_mul(a[1], b1))


def f12_mul(a, b):  # fp12_mul
    t0 = f6_mul(a[0], b[0])
    t1 = f6_mul(a[1], b[1])
    c1 = f6_mul(f6_add(a[0], a[1]), f6_add(b[0], b[1]))
    c1 = f6_sub(f6_sub(c1, t0), t1)
    return (f6_add(t0, f6_mul_v(t1)), c1)


def f12_sqr(a):  # fp12_sqr
    ab = f6_mul(a[0], a[1])
    s0 = f6_add(a[0], a[1])
    s1 = f6_add(a[0], f6_mul_v(a[1]))
    s0 = f6_sub(f6_mul(s0, s1), ab)
    c0 = f6_sub(s0, f6_mul_v(ab))
    return (c0, f6_add(ab, ab))


def f12_mul_014(f, o0, o1, o4):  # fp12_mul_014
    aa = f6_mul_01(f[0], o0, o1)
    bb = f6_mul_1(f[1], o4)
    o = f2_add(o1, o4)
    s = f6_mul_01(f6_add(f[1], f[0]), o0, o)
    c1 = f6_sub(f6_sub(s, aa), bb)
    c0 = f6_add(f6_mul_v(bb), aa)
    return (c0, c1)


def fp4_sqr(a, b):
    t0 = f2_sqr(a)
    t1 = f2_sqr(b)
    c0 = f2_add(f2_mul_xi(t1), t0)
    t2 = f2_sub(f2_sub(f2_sqr(f2_add(a, b)), t0), t1)
    return c0, t2


def f12_cyc_sqr(f):  # fp12_cyc_sqr
    z0, z4, z3 = f[0]
    z2, z1, z5 = f[1]
    t0, t1 = fp4_sqr(z0, z1)
    z0 = f2_add(f2_dbl(f2_sub(t0, z0)), t0)
    z1 = f2_add(f2_dbl(f2_add(t1, z1)), t1)
    t0, t1 = fp4_sqr(z2, z3)
    t2, t3 = fp4_sqr(z4, z5)
    z4 = f2_add(f2_dbl(f2_sub(t0, z4)), t0)
    z5 = f2_add(f2_dbl(f2_add(t1, z5)), t1)
    t0 = f2_mul_xi(t3)
    z2 = f2_add(f2_dbl(f2_add(t0, z2)), t0)
    z3 = f2_add(f2_dbl(f2_sub(t2, z3)), t2)
    return ((z0, z4, z3), (z2, z1, z5))


def f12_frob(a, consts):
    """consts[k] = gamma_k as a pair of constant symbols (Fp2), k = 1..5; conj for odd n."""
    c = [a[0][0], a[1][0], a[0][1], a[1][1], a[0][2], a[1][2]]
    out = []
    for k in range(6):
        x = c[k]
        if consts["odd"]:
            x = f2_conj(x)
        if k:
            x = f2_mul(x, consts[k])
        out.append(x)
    return ((out[0], out[2], out[4]), (out[1], out[3], out[5]))


def f12_conj(a):
    return (a[0], f6_neg(a[1]))

# ---------------- Miller loop steps, mirroring ssb_pairing.h ----------------


def miller_dbl(T, P):
    X, Y, Z = T
    xP, yP = P
    A = f2_sqr(X)
    B = f2_sqr(Y)
    C = f2_sqr(B)
    t = mat2(f2_sub(f2_sub(f2_sqr(f2_add(X, B)), A), C))
    D = mat2(f2_dbl(t))
    E = mat2(f2_add(f2_dbl(A), A))
    F = f2_sqr(E)
    ZZ = f2_sqr(Z)
    l0 = f2_sub(f2_mul(E, X), f2_dbl(B))
    l1 = f2_mul_fp(mat2(f2_neg(f2_mul(E, ZZ))), xP)
    x3 = mat2(f2_sub(F, f2_dbl(D)))
    z3 = mat2(f2_dbl(f2_mul(Y, Z)))
    y3 = f2_mul(E, mat2(f2_sub(D, x3)))
    C2 = mat2(f2_dbl(C))
    C4 = mat2(f2_dbl(C2))
    C8 = mat2(f2_dbl(C4))
    y3 = f2_sub(y3, C8)
    l4 = f2_mul_fp(mat2(f2_mul(z3, ZZ)), yP)
    return (x3, y3, z3), (l0, l1, l4)


def miller_add(T, Q, P):
    X, Y, Z = T
    xQ, yQ = Q
    xP, yP = P
    ZZ = mat2(f2_sqr(Z))
    U2 = f2_mul(xQ, ZZ)
    S2 = f2_mul(mat2(f2_mul(yQ, Z)), ZZ)
    H = mat2(f2_sub(U2, X))
    rr = mat2(f2_dbl(f2_sub(S2, Y)))
    HH = mat2(f2_sqr(H))
    I = mat2(f2_dbl(f2_dbl(HH)))
    J = mat2(f2_mul(H, I))
    V = mat2(f2_mul(X, I))
    x3 = mat2(f2_sub(f2_sub(f2_sqr(rr), J), f2_dbl(V)))
    y3 = f2_sub(f2_mul(rr, f2_sub(V, x3)), f2_dbl(f2_mul(Y, J)))
    z3 = mat2(f2_sub(f2_sub(f2_sqr(f2_add(Z, H)), ZZ), HH))
    l0 = f2_sub(f2_mul(rr, xQ), f2_mul(yQ, z3))
    l1 = f2_mul_fp(f2_neg(rr), xP)
    l4 = f2_mul_fp(z3, yP)
    return (x3, y3, z3), (l0, l1, l4)

# ---------------- tracing ----------------


def sym_fp12(tag):
    s = [L({(tag, i): 1}) for i in range(12)]
    f2s = [(s[2 * k], s[2 * k + 1]) for k in range(6)]
    return ((f2s[0], f2s[1], f2s[2]), (f2s[3], f2s[4], f2s[5]))


def flat_fp12(a):
    return [c for f6 in a for f2_ in f6 for c in f2_]


def sym_vec(tag, n):
    return [L({(tag, i): 1}) for i in range(n)]


OUT_CHUNK = 8


def _nterms(form):
    return sum(abs(c) for c in form.c.values())


def split_outputs(outs):
    """Outputs longer than OUT_CHUNK terms become sums of partial materialisations computed by
    other lanes at the end of the last phase (the output lanes then add <= OUT_CHUNK terms)."""
    if not CTX.products:
        return outs
    last = max(p[0] for p in CTX.products)
    res = []
    for o in outs:
        if _nterms(o) <= OUT_CHUNK:
            res.append(o)
            continue
        chunks, cur, n = [], {}, 0
        for sym, c in sorted(o.c.items()):
            if n + abs(c) > OUT_CHUNK and cur:
                chunks.append(cur)
                cur, n = {}, 0
            cur[sym] = c
            n += abs(c)
        if cur:
            chunks.append(cur)
        acc = L()
        for ch in chunks:
            f_ = L(ch)
            ph = max([CTX.phase_of(s_) for s_ in f_.c] + [0])
            if ph >= 1:
                acc = acc + CTX.mat(f_)
            else:
                acc = acc + f_
        res.append(acc)
    return res


def trace(fn):
    global CTX
    CTX = Ctx()
    outs = split_outputs(fn())
    TRACED_MATS[0] = CTX.mats
    return CTX.products, outs


TRACED_MATS = [()]


# slot index space inside a program: 0 = zero, then A (na), B (nb), K (nk constants), P (products)
def encode(name, products, outs, na, nb, consts, mats=()):
    nk = len(consts)
    base = {"A": 1, "B": 1 + na, "K": 1 + na + nb, "P": 1 + na + nb + nk}
    base["M"] = base["P"] + len(products)

    def idx(sym):
        return base[sym[0]] + sym[1]

    def terms(form):
        pos, neg = [], []
        for sym, c in sorted(form.c.items(), key=lambda kv: (kv[0][0], kv[0][1])):
            (pos if c > 0 else neg).extend([idx(sym)] * abs(c))
        return pos, neg

    nphase = max([p[0] for p in products] + [0])
    # renumber products phase-major so each phase is a contiguous lane range
    order = sorted(range(len(products)), key=lambda i: products[i][0])
    remap = {old: new for new, old in enumerate(order)}
    morder = sorted(range(len(mats)), key=lambda i: (mats[i][0], mats[i][2]))
    mremap = {old: new for new, old in enumerate(morder)}

    def fix(form):
        d = {}
        for s, c in form.c.items():
            s2 = ("P", remap[s[1]]) if s[0] == "P" else (("M", mremap[s[1]]) if s[0] == "M" else s)
            d[s2] = c
        return L(d)

    prods = [(products[i][0], fix(products[i][1]), fix(products[i][2])) for i in order]
    mts = [(mats[i][0], fix(mats[i][1]), mats[i][2]) for i in morder]
    outs = [fix(o) for o in outs]
    phase_end = [sum(1 for p in prods if p[0] <= ph) for ph in range(1, nphase + 1)]
    # linear stages: per phase, per level -> (phase, end index into mats)
    stages = []
    for ph in range(1, nphase + 1):
        lv = sorted(set(m[2] for m in mts if m[0] == ph))
        for l_ in lv:
            stages.append((ph, sum(1 for m in mts if (m[0], m[2]) <= (ph, l_))))
    mat_end = stages
    rows = []
    for ph, x, y in prods:
        xp, xn = terms(x)
        yp, yn = terms(y)
        rows.append((xp, xn, yp, yn))
    mrows = [terms(m) for _, m, _ in mts]
    orows = [terms(o) for o in outs]
    return dict(name=name, na=na, nb=nb, nk=nk, consts=consts, nprod=len(prods), nphase=nphase, nmat=len(mts),
                phase_start=phase_end, mat_end=mat_end, rows=rows, mrows=mrows, orows=orows, nout=len(outs))


def programs():
    progs = []
    # fp12 mul: A = a (12), B = b (12)
    pr, o = trace(lambda: flat_fp12(f12_mul(sym_fp12("A"), sym_fp12("B"))))
    progs.append(encode("FP12_MUL", pr, o, 12, 12, [], TRACED_MATS[0]))
    pr, o = trace(lambda: flat_fp12(f12_sqr(sym_fp12("A"))))
    progs.append(encode("FP12_SQR", pr, o, 12, 0, [], TRACED_MATS[0]))
    pr, o = trace(lambda: flat_fp12(f12_cyc_sqr(sym_fp12("A"))))
    progs.append(encode("FP12_CYC_SQR", pr, o, 12, 0, [], TRACED_MATS[0]))

    # sparse line multiply: B = (l0.c0, l0.c1, l1.c0, l1.c1, l4.c0, l4.c1)
    def mul014():
        b = sym_vec("B", 6)
        return flat_fp12(f12_mul_014(sym_fp12("A"), (b[0], b[1]), (b[2], b[3]), (b[4], b[5])))
    pr, o = trace(mul014)
    progs.append(encode("FP12_MUL_014", pr, o, 12, 6, [], TRACED_MATS[0]))
    # frobenius n = 1, 2, 3: constants gamma_{n,k}, k = 1..5 (10 Fp)
    for n in (1, 2, 3):
        def frob(n=n):
            k = sym_vec("K", 10)
            consts = {"odd": n & 1}
            for i in range(1, 6):
                consts[i] = (k[2 * (i - 1)], k[2 * (i - 1) + 1])
            return flat_fp12(f12_frob(sym_fp12("A"), consts))
        pr, o = trace(frob)
        progs.append(encode("FP12_FROB%d" % n, pr, o, 12, 0, [(n, k, c) for k in range(1, 6) for c in range(2)], TRACED_MATS[0]))
    pr, o = trace(lambda: flat_fp12(f12_conj(sym_fp12("A"))))
    progs.append(encode("FP12_CONJ", pr, o, 12, 0, [], TRACED_MATS[0]))

    # Miller doubling step: A = T (6: X, Y, Z as Fp2), B = P (2: xP, yP); out T'(6) + line(6)
    def mdbl():
        a = sym_vec("A", 6)
        b = sym_vec("B", 2)
        T, l = miller_dbl(((a[0], a[1]), (a[2], a[3]), (a[4], a[5])), (b[0], b[1]))
        return [c for f2_ in T for c in f2_] + [c for f2_ in l for c in f2_]
    pr, o = trace(mdbl)
    progs.append(encode("MILLER_DBL", pr, o, 6, 2, [], TRACED_MATS[0]))

    # Miller addition step: A = T (6), B = (xQ, yQ, xP, yP) as (4 + 2) Fp
    def madd():
        a = sym_vec("A", 6)
        b = sym_vec("B", 6)
        T, l = miller_add(((a[0], a[1]), (a[2], a[3]), (a[4], a[5])), ((b[0], b[1]), (b[2], b[3])), (b[4], b[5]))
        return [c for f2_ in T for c in f2_] + [c for f2_ in l for c in f2_]
    pr, o = trace(madd)
    progs.append(encode("MILLER_ADD", pr, o, 6, 6, [], TRACED_MATS[0]))
    return progs


def emit(progs):
    out = ["// GENERATED by gen_wave_tables.py -- do not edit.",
           "// Lane-parallel programs of the tower ops: see gen_wave_tables.py and ssb_wave.h.",
           "#pragma once", "#include <cstdint>", "namespace ssb {", "namespace wave {"]
    TX = max(max(len(r[0]), len(r[1]), len(r[2]), len(r[3])) for p in progs for r in p["rows"])
    TO = max(max(len(r[0]), len(r[1])) for p in progs for r in p["orows"])
    out.append("constexpr int MAX_PROD = %d;" % max(p["nprod"] for p in progs))
    out.append("constexpr int MAX_OUT = %d;" % max(p["nout"] for p in progs))
    out.append("constexpr int MAX_SLOTS_OP = %d;" % max(1 + p["na"] + p["nb"] + p["nk"] + p["nprod"] + p["nmat"] for p in progs))
    out.append("constexpr int MAX_MAT = %d;" % max(p["nmat"] for p in progs))
    out.append("struct prog { int na, nb, nk, nprod, nmat, nphase, nout, nlin; const uint8_t* phase_end;")
    out.append("  const uint8_t* lin;   // linear stages: (after phase index, end of its materialisation range)")
    out.append("  const uint8_t* cnt;   // per product: |x+|, |x-|, |y+|, |y-|")
    out.append("  const uint16_t* off;  // per product: offset of its term list in terms[]")
    out.append("  const uint8_t* ocnt;  // per materialisation, then per output: |+|, |-|")
    out.append("  const uint16_t* ooff; const uint8_t* terms; const uint8_t* kconst; };")
    for p in progs:
        nm = p["name"]
        terms, cnt, off, ocnt, ooff = [], [], [], [], []
        for xp, xn, yp, yn in p["rows"]:
            off.append(len(terms))
            cnt += [len(xp), len(xn), len(yp), len(yn)]
            terms += xp + xn + yp + yn
        for pos, neg in list(p["mrows"]) + list(p["orows"]):  # materialisations first, then outputs
            ooff.append(len(terms))
            ocnt += [len(pos), len(neg)]
            terms += pos + neg
        assert max(terms + [0]) < 256
        kc = []
        for (n, k, c) in p["consts"]:
            kc += [n, k, c]  # K slot = component c of gamma_{n,k} (FROBn[k])
        out.append("constexpr uint8_t %s_PH[] = {%s};" % (nm, ", ".join(map(str, p["phase_start"])) or "0"))
        me = []
        for (ph, end) in p["mat_end"]:
            me += [ph - 1, end]   # (phase index, end) pairs: linear stages in order
        out.append("constexpr uint8_t %s_ME[] = {%s};" % (nm, ", ".join(map(str, me)) or "0"))
        out.append("constexpr uint8_t %s_CNT[] = {%s};" % (nm, ", ".join(map(str, cnt)) or "0"))
        out.append("constexpr uint16_t %s_OFF[] = {%s};" % (nm, ", ".join(map(str, off)) or "0"))
        out.append("constexpr uint8_t %s_OCNT[] = {%s};" % (nm, ", ".join(map(str, ocnt))))
        out.append("constexpr uint16_t %s_OOFF[] = {%s};" % (nm, ", ".join(map(str, ooff))))
        out.append("constexpr uint8_t %s_TERMS[] = {%s};" % (nm, ", ".join(map(str, terms))))
        out.append("constexpr uint8_t %s_K[] = {%s};" % (nm, ", ".join(map(str, kc)) or "0"))
        out.append("constexpr prog %s = {%d, %d, %d, %d, %d, %d, %d, %d, %s_PH, %s_ME, %s_CNT, %s_OFF, %s_OCNT, %s_OOFF, %s_TERMS, %s_K};"
                   % (nm, p["na"], p["nb"], p["nk"], p["nprod"], p["nmat"], p["nphase"], p["nout"], len(p["mat_end"]),
                      nm, nm, nm, nm, nm, nm, nm, nm))
        out.append("// %s: %d products in %d phases, %d materialised, %d outputs, max terms/form %d" %
                   (nm, p["nprod"], p["nphase"], p["nmat"], p["nout"],
                    max([max(len(r[0]) + len(r[1]), len(r[2]) + len(r[3])) for r in p["rows"]] + [0])))
    out.append("}  // namespace wave")
    out.append("}  // namespace ssb")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ssb_wave_tables.h")
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")
    print("wrote", path, "max form terms", TX, "max output terms", TO)


if __name__ == "__main__":
    ps = programs()
    for p in ps:
        print(p["name"], "products", p["nprod"], "phases", p["nphase"], "phase_ends", p["phase_start"],
              "mats", p["mat_end"], "outs", p["nout"],
              "max_form", max([max(len(r[0]) + len(r[1]), len(r[2]) + len(r[3])) for r in p["rows"]] + [0]),
              "max_lin", max([len(r[0]) + len(r[1]) for r in list(p["mrows"]) + list(p["orows"])] + [0]))
    emit(ps)
