"""Build-time generator for ssb_lane_progs.h: straight-line LANE-GROUP programs of the BLS12-381
point and tower operations.

Why: the per-share work of the engine (subgroup check, RLC multiples, Lagrange terms, cofactor
clearing, the sums, Miller loops, the final exponentiation) is long chains of point / Fp12
operations.  On one lane each Fp2 multiply is 3 dependent-issue Fp multiplies and a G2 point
doubling 16, so the latency of a chain, not the ALU rate, bounds every stage (the C2 batch has only
16k shares: 256 waves on a 1024-SIMD chip).  A program here runs ONE operation on a group of G
lanes (G = 8 for point operations, 64 for Fp12 operations); the 64/G groups of a wave run
independent operations in lockstep.  Every lane computes one Fp product per round, operands being
short +-sums of LDS slots; between product rounds some lanes "materialise" longer linear forms
(reduced mod p) into slots.

How: each operation is traced SYMBOLICALLY through the same formulas as the single-lane code
(ssb_curve.h / ssb_field.h / ssb_pairing.h), giving products (x_form * y_form) and linear forms
over inputs, constants, products and materialisations.  A list scheduler packs ready products into
rounds of <= G, materialises operand forms with more than 3 terms (operands < 3p are legal for the
Montgomery product: 3p * 3p < p * 2^384) and outputs / long forms with up to 8 terms (< 8p < 2^384,
reduced by conditional subtraction), and allocates LDS slots by liveness.  The emitted C++ runs on
the device with one role per lane and on the host (tests) with a loop over roles, so the programs
are checked against the single-lane code on the CPU.

Slot codes (8 bit): 0..47 shared constants (0 = zero), 48..175 group scratch, 176..199 input A,
200..223 input B, 224..255 output D.

Run: python safestakeoperator_amd/csrc/gen_lane_progs.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))

MAXT = 3     # max terms of an inlined product operand (value < 3p)
MAXM = 8     # max terms of a materialised form (value < 8p < 2^384)
C_SCR, C_A, C_B, C_D = 48, 176, 200, 224
N_SCR = C_A - C_SCR

# shared constants (Fp components, Montgomery form, from ssb_consts.h): name -> code
CONSTS = ["ZERO"]
for nm in ["PSI_CX", "PSI_CY", "FP2_B2"]:
    CONSTS += [nm + ".c0", nm + ".c1"]
CONSTS += ["FP_B1", "FP_ONE"]
for n in (1, 2, 3):
    for k in range(1, 6):
        CONSTS += ["FROB%d[%d].c0" % (n, k), "FROB%d[%d].c1" % (n, k)]
assert len(CONSTS) <= C_SCR
CCODE = {nm: i for i, nm in enumerate(CONSTS)}


# ------------------------------------------------------------------------------------------
# symbolic linear forms over symbols ('A', i) ('B', i) ('K', name) ('P', i) ('M', i)
# ------------------------------------------------------------------------------------------
class L:
    __slots__ = ("c",)

    def __init__(self, c=None):
        self.c = {k: v for k, v in (c or {}).items() if v}

    def __add__(self, o):
        d = dict(self.c)
        for k, v in o.c.items():
            d[k] = d.get(k, 0) + v
        return L(d)

    def __sub__(self, o):
        return self + (-o)

    def __neg__(self):
        return L({k: -v for k, v in self.c.items()})

    def __mul__(self, o):
        if isinstance(o, int):
            return L({k: v * o for k, v in self.c.items()})
        return PROG.product(self, o)

    __rmul__ = __mul__

    def weight(self):
        return sum(abs(v) for v in self.c.values())


def K(name):
    return L({("K", name): 1})


class Prog:
    def __init__(self, name, na, nb, G):
        self.name, self.na, self.nb, self.G = name, na, nb, G
        self.prods = []    # (x, y)
        self.mats = []     # L
        self.checks = []   # list of lists of L (a check fires when ALL its components are zero)

    def product(self, x, y):
        self.prods.append((x, y))
        return L({("P", len(self.prods) - 1): 1})

    def mat(self, f):
        if f.weight() == 0:
            return f
        if len(f.c) == 1 and list(f.c.values())[0] == 1 and list(f.c)[0][0] in "PM":
            return f
        self.mats.append(f)
        return L({("M", len(self.mats) - 1): 1})


PROG = None


def A(i):
    return L({("A", i): 1})


def B(i):
    return L({("B", i): 1})


def mat(f):
    return PROG.mat(f)


def mat2(a):
    return (mat(a[0]), mat(a[1]))


def check_zero(*comps):
    PROG.checks.append(list(comps))


# ---------------- Fp2 tower, mirroring ssb_field.h ----------------
def f2_add(a, b): return (a[0] + b[0], a[1] + b[1])
def f2_sub(a, b): return (a[0] - b[0], a[1] - b[1])
def f2_neg(a): return (-a[0], -a[1])
def f2_dbl(a): return (a[0] * 2, a[1] * 2)
def f2_conj(a): return (a[0], -a[1])
def f2_mul_xi(a): return (a[0] - a[1], a[0] + a[1])


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    t2 = (a[0] + a[1]) * (b[0] + b[1])
    return (t0 - t1, t2 - t0 - t1)


def f2_sqr(a):
    m = a[0] * a[1]
    return ((a[0] + a[1]) * (a[0] - a[1]), m * 2)


def f2_mul_fp(a, s): return (a[0] * s, a[1] * s)


def K2(nm): return (K(nm + ".c0"), K(nm + ".c1"))


# field-generic helpers: an Fp element is an L, an Fp2 element a 2-tuple of L
def is2(a): return isinstance(a, tuple)
def g_add(a, b): return f2_add(a, b) if is2(a) else a + b
def g_sub(a, b): return f2_sub(a, b) if is2(a) else a - b
def g_dbl(a): return f2_dbl(a) if is2(a) else a * 2
def g_mul(a, b): return f2_mul(a, b) if is2(a) else a * b
def g_sqr(a): return f2_sqr(a) if is2(a) else a * a
def g_mat(a): return mat2(a) if is2(a) else mat(a)
def g_comps(a): return list(a) if is2(a) else [a]


# ---------------- curve formulas, mirroring ssb_curve.h ----------------
def jac_dbl(X, Y, Z):  # dbl-2009-l, a = 0
    A_ = g_sqr(X)
    B_ = g_mat(g_sqr(Y))
    C = g_sqr(B_)
    D = g_mat(g_dbl(g_sub(g_sub(g_sqr(g_add(X, B_)), A_), C)))
    E = g_mat(g_add(g_dbl(A_), A_))
    F = g_sqr(E)
    x3 = g_mat(g_sub(F, g_dbl(D)))
    z3 = g_dbl(g_mul(Y, Z))
    C2 = g_mat(g_dbl(C))
    C8 = g_mat(g_dbl(g_dbl(C2)))
    y3 = g_sub(g_mul(E, g_sub(D, x3)), C8)
    return x3, y3, z3


def jac_add(X1, Y1, Z1, X2, Y2, Z2):  # add-2007-bl
    check_zero(*g_comps(Z1))
    check_zero(*g_comps(Z2))
    Z1Z1 = g_mat(g_sqr(Z1))
    Z2Z2 = g_mat(g_sqr(Z2))
    U1 = g_mat(g_mul(X1, Z2Z2))
    U2 = g_mul(X2, Z1Z1)
    S1 = g_mat(g_mul(g_mat(g_mul(Y1, Z2)), Z2Z2))
    S2 = g_mul(g_mat(g_mul(Y2, Z1)), Z1Z1)
    H = g_mat(g_sub(U2, U1))
    check_zero(*g_comps(H))
    rr = g_mat(g_dbl(g_sub(S2, S1)))
    I = g_mat(g_sqr(g_dbl(H)))
    J = g_mat(g_mul(H, I))
    V = g_mat(g_mul(U1, I))
    x3 = g_mat(g_sub(g_sub(g_sqr(rr), J), g_dbl(V)))
    y3 = g_sub(g_mul(rr, g_sub(V, x3)), g_dbl(g_mul(S1, J)))
    z3 = g_mul(g_mat(g_sub(g_sub(g_sqr(g_add(Z1, Z2)), Z1Z1), Z2Z2)), H)
    return x3, y3, z3


def jac_add_aff(X1, Y1, Z1, x2, y2):  # madd-2007-bl (q affine, not infinity)
    check_zero(*g_comps(Z1))
    Z1Z1 = g_mat(g_sqr(Z1))
    U2 = g_mul(x2, Z1Z1)
    S2 = g_mul(g_mat(g_mul(y2, Z1)), Z1Z1)
    H = g_mat(g_sub(U2, X1))
    check_zero(*g_comps(H))
    rr = g_mat(g_dbl(g_sub(S2, Y1)))
    HH = g_mat(g_sqr(H))
    I = g_mat(g_dbl(g_dbl(HH)))
    J = g_mat(g_mul(H, I))
    V = g_mat(g_mul(X1, I))
    x3 = g_mat(g_sub(g_sub(g_sqr(rr), J), g_dbl(V)))
    y3 = g_sub(g_mul(rr, g_sub(V, x3)), g_dbl(g_mul(Y1, J)))
    z3 = g_sub(g_sub(g_sqr(g_add(Z1, H)), Z1Z1), HH)
    return x3, y3, z3


def sym_pt2(T, off=0):
    return ((T(off), T(off + 1)), (T(off + 2), T(off + 3)), (T(off + 4), T(off + 5)))


def flat(*vals):
    out = []
    for v in vals:
        out += g_comps(v)
    return out


# ---------------- program list ----------------
def programs():
    ps = []

    def define(name, na, nb, G, fn):
        global PROG
        PROG = Prog(name, na, nb, G)
        outs = fn()
        ps.append((PROG, outs))

    # G2 (Fp2) Jacobian: A = (X0, X1, Y0, Y1, Z0, Z1)
    define("G2_DBL", 6, 0, 8, lambda: flat(*jac_dbl(*sym_pt2(A))))
    define("G2_ADD", 6, 6, 8, lambda: flat(*jac_add(*sym_pt2(A), *sym_pt2(B))))
    define("G2_MADD", 6, 4, 8, lambda: flat(*jac_add_aff(*sym_pt2(A), (B(0), B(1)), (B(2), B(3)))))

    def g2_psi():  # psi(X, Y, Z) = (conj(X) cx, conj(Y) cy, conj(Z))
        X, Y, Z = sym_pt2(A)
        return flat(f2_mul(f2_conj(X), K2("PSI_CX")), f2_mul(f2_conj(Y), K2("PSI_CY")), f2_conj(Z))
    define("G2_PSI", 6, 0, 8, g2_psi)

    def g2_npsi_aff():  # -psi(x, y) = (conj(x) cx, -conj(y) cy) for an affine A = (x0, x1, y0, y1)
        x, y = (A(0), A(1)), (A(2), A(3))
        return flat(f2_mul(f2_conj(x), K2("PSI_CX")), f2_neg(f2_mul(f2_conj(y), K2("PSI_CY"))))
    define("G2_NPSI_AFF", 4, 0, 8, g2_npsi_aff)

    def g2_eq_aff():  # (x Z^2 - X, y Z^3 - Y) for Jacobian A vs affine B = (x0, x1, y0, y1)
        X, Y, Z = sym_pt2(A)
        zz = g_mat(f2_sqr(Z))
        zzz = g_mat(f2_mul(zz, Z))
        return flat(f2_sub(f2_mul((B(0), B(1)), zz), X), f2_sub(f2_mul((B(2), B(3)), zzz), Y))
    define("G2_EQ_AFF", 6, 4, 8, g2_eq_aff)

    # G1 (Fp) Jacobian: A = (X, Y, Z)
    define("G1_DBL", 3, 0, 4, lambda: flat(*jac_dbl(A(0), A(1), A(2))))
    define("G1_ADD", 3, 3, 4, lambda: flat(*jac_add(A(0), A(1), A(2), B(0), B(1), B(2))))
    define("G1_MADD", 3, 2, 4, lambda: flat(*jac_add_aff(A(0), A(1), A(2), B(0), B(1))))
    return ps


# ------------------------------------------------------------------------------------------
# scheduling
# ------------------------------------------------------------------------------------------
def syms_of(f):
    return list(f.c.keys())


class Sched:
    """Turns a traced program into stages.  A stage is ("lin", items) -- materialisations whose
    inputs are ready, reduced mod p and stored --, ("prod", items) -- at most G products -- ,
    ("chk", items) -- zero tests -- or ("out", items).  Items: ("P", i), ("M", j), ("O", k),
    ("C", c, k)."""

    def __init__(self, prog, outs):
        self.p, self.G = prog, prog.G
        # operand forms with > MAXT terms become materialisations
        self.prods = [(self._limit(x), self._limit(y)) for x, y in prog.prods]
        # every materialisation (including the ones created here) has <= MAXM terms
        j = 0
        while j < len(prog.mats):
            prog.mats[j] = self._chunk(prog.mats[j])
            j += 1
        self.outs = [self._chunk(o) for o in outs]
        self.checks = [[self._chunk(c) for c in chk] for chk in prog.checks]
        j = 0
        while j < len(prog.mats):
            prog.mats[j] = self._chunk(prog.mats[j])
            j += 1
        self.mats = prog.mats

    def _chunk(self, f):
        """f with <= MAXM terms, splitting it into materialised parts when longer."""
        if f.weight() <= MAXM:
            return f
        parts, cur, w = [], {}, 0
        for s, c in sorted(f.c.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
            sg = 1 if c > 0 else -1
            n = abs(c)
            while n:
                take = min(n, MAXM - w)
                cur[s] = cur.get(s, 0) + sg * take
                w += take
                n -= take
                if w == MAXM:
                    parts.append(L(cur))
                    cur, w = {}, 0
        if cur:
            parts.append(L(cur))
        acc = L()
        for q in parts:
            acc = acc + self.p.mat(q)
        return self._chunk(acc)

    def _limit(self, f):
        if f.weight() <= MAXT:
            return f
        return self.p.mat(self._chunk(f))

    def schedule(self):
        P, G = self.p, self.G
        mats = self.mats
        # dependency heights for priorities
        users = {}
        for i, (x, y) in enumerate(self.prods):
            for s in syms_of(x) + syms_of(y):
                users.setdefault(s, []).append(("P", i))
        for j, f in enumerate(mats):
            for s in syms_of(f):
                users.setdefault(s, []).append(("M", j))
        memo = {}

        def height(s):
            if s in memo:
                return memo[s]
            h = 0
            for u in users.get(s, []):
                h = max(h, height(u) + (1 if u[0] == "P" else 0))
            memo[s] = h
            return h

        avail = set()
        stages = []
        done_p, done_m = set(), set()

        def ready(f):
            return all(s[0] in "ABK" or s in avail for s in syms_of(f))

        n_rounds = 0
        while len(done_p) < len(self.prods) or len(done_m) < len(mats):
            # linear stage: every ready materialisation, in dependency levels
            while True:
                lvl = [("M", j) for j in range(len(mats)) if ("M", j) not in done_m and ready(mats[j])]
                if not lvl:
                    break
                stages.append(("lin", lvl))
                for it in lvl:
                    done_m.add(it)
                    avail.add(it)
            rp = [("P", i) for i in range(len(self.prods))
                  if ("P", i) not in done_p and ready(self.prods[i][0]) and ready(self.prods[i][1])]
            if not rp:
                if len(done_p) < len(self.prods) or len(done_m) < len(mats):
                    raise RuntimeError("%s: deadlock" % P.name)
                break
            rp.sort(key=lambda it: -height(it))
            pick = rp[:G]
            stages.append(("prod", pick))
            n_rounds += 1
            for it in pick:
                done_p.add(it)
                avail.add(it)
        # checks: as soon as ready -> put them in a final check stage (cheap, no store)
        chk_items = [("C", c, k) for c, chk in enumerate(self.checks) for k in range(len(chk))]
        if chk_items:
            stages.append(("chk", chk_items))
        outs = [("O", k) for k in range(len(self.outs))]
        stages.append(("out", outs))
        self.stages = stages
        self.n_rounds = n_rounds
        return stages

    def form_of(self, it):
        if it[0] == "M":
            return self.mats[it[1]]
        if it[0] == "O":
            return self.outs[it[1]]
        if it[0] == "C":
            return self.checks[it[1]][it[2]]
        raise KeyError(it)

    def allocate(self):
        """Scratch slots by liveness at stage granularity."""
        last_use = {}
        for si, (kind, items) in enumerate(self.stages):
            for it in items:
                forms = self.prods[it[1]] if it[0] == "P" else (self.form_of(it),)
                for f in forms:
                    for s in syms_of(f):
                        if s[0] in "PM":
                            last_use[s] = si
        slot = {}
        free = list(range(N_SCR))
        busy = {}  # slot -> symbol
        for si, (kind, items) in enumerate(self.stages):
            # release values whose last use is before this stage
            for sl, s in list(busy.items()):
                if last_use.get(s, -1) < si:
                    del busy[sl]
                    free.append(sl)
            free.sort()
            for it in items:
                if it[0] in "PM":
                    if it not in last_use:
                        slot[it] = None  # dead value (never read): junk slot
                        continue
                    if not free:
                        raise RuntimeError("%s: out of scratch slots" % self.p.name)
                    sl = free.pop(0)
                    busy[sl] = it
                    slot[it] = sl
        self.slot = slot
        self.n_scratch = max([s for s in slot.values() if s is not None] + [-1]) + 2  # + junk slot
        self.junk = self.n_scratch - 1
        return slot

    def code(self, s):
        k = s[0]
        if k == "A":
            assert s[1] < C_B - C_A
            return C_A + s[1]
        if k == "B":
            assert s[1] < C_D - C_B
            return C_B + s[1]
        if k == "K":
            return CCODE[s[1]]
        sl = self.slot[s]
        assert sl is not None
        return C_SCR + sl


# ------------------------------------------------------------------------------------------
# emission
# ------------------------------------------------------------------------------------------
def terms_of(f):
    """-> list of (sign, sym) with |coef| repetition, positives first."""
    pos, neg = [], []
    for s, c in sorted(f.c.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
        (pos if c > 0 else neg).extend([s] * abs(c))
    return [(0, s) for s in pos] + [(1, s) for s in neg]


class Emitter:
    def __init__(self, sch):
        self.s, self.G = sch, sch.G
        self.lines = []
        self.tables = []  # for G > 8: (name, bytes)

    def sel(self, codes, tag):
        """per-role 8-bit codes -> a C expression of `role`."""
        G = self.G
        codes = list(codes) + [0] * (G - len(codes))
        if G <= 8:
            v = 0
            for r, c in enumerate(codes):
                v |= (c & 0xFF) << (8 * r)
            return "LP_SEL8(0x%016xull)" % v
        name = "%s_t%d" % (self.s.p.name, len(self.tables))
        self.tables.append((name, codes))
        return "LP_SELT(%s)" % name

    def bits(self, bits):
        v = 0
        for r, b in enumerate(bits):
            v |= (b & 1) << r
        return "0x%xull" % v

    def emit_form(self, var, forms):
        """forms: per role (L or None). Accumulates var = sum of +-terms (value < weight * p)."""
        G = self.G
        tl = [terms_of(f) if f is not None else [] for f in forms]
        T = max([len(t) for t in tl] + [1])
        for k in range(T):
            codes, sg = [], []
            for r in range(G):
                if r < len(tl) and k < len(tl[r]):
                    sgn, sym = tl[r][k]
                    codes.append(self.s.code(sym)); sg.append(sgn)
                else:
                    codes.append(0); sg.append(0)
            src = self.sel(codes, var)
            uni = "pos" if all(b == 0 for b in sg) else ("neg" if all(b == 1 for b in sg) else "mix")
            if k == 0:
                if uni == "pos":
                    self.lines.append("      lp_ld(%s, g, %s);" % (var, src))
                elif uni == "neg":
                    self.lines.append("      lp_ld_neg(%s, g, %s);" % (var, src))
                else:
                    self.lines.append("      lp_ld_sgn(%s, g, %s, LP_BIT(%s));" % (var, src, self.bits(sg)))
            else:
                if uni == "pos":
                    self.lines.append("      lp_acc(%s, g, %s);" % (var, src))
                elif uni == "neg":
                    self.lines.append("      lp_acc_neg(%s, g, %s);" % (var, src))
                else:
                    self.lines.append("      lp_acc_sgn(%s, g, %s, LP_BIT(%s));" % (var, src, self.bits(sg)))
        return T

    def reduce_line(self, forms):
        """Forms evaluate to values <= w*p (negative terms enter as p - v); reduce to [0, p)."""
        w = max(f.weight() for f in forms)
        neg = any(c < 0 for f in forms for c in f.c.values())
        if w <= 1 and not neg:
            return None
        steps = 1 if w <= 1 else (2 if w <= 2 else (3 if w <= 4 else 4))
        return "      lp_reduce%d(LP_T);" % steps

    def emit(self):
        s, G = self.s, self.G
        P = s.p
        out = self.lines
        nout = len(s.outs)
        staged = nout > G
        stage_base = s.n_scratch  # output staging after the scratch area
        n_scr_total = s.n_scratch + (nout if staged else 0)
        assert n_scr_total <= N_SCR, (P.name, n_scr_total)
        junk = C_SCR + s.junk
        # check bits: component k of check c -> bit (offset(c) + k); fires when all set
        cbit, masks, b = {}, [], 0
        for c, chk in enumerate(s.checks):
            for k in range(len(chk)):
                cbit[(c, k)] = 1 << (b + k)
            masks.append(((1 << len(chk)) - 1) << b)
            b += len(chk)
        assert b <= 32
        self.masks = masks
        for (kind, items) in s.stages:
            for p0 in range(0, len(items), G):
                chunk = items[p0:p0 + G]
                out.append("  {  // %s %s" % (kind, " ".join("".join(str(x) for x in it) for it in chunk)))
                out.append("    LP_DECL_T;")
                if kind == "prod":
                    out.append("    LP_FOR(%d) {" % G)
                    out.append("      fp x, y;")
                    self.emit_form("x", [s.prods[it[1]][0] for it in chunk])
                    self.emit_form("y", [s.prods[it[1]][1] for it in chunk])
                    out.append("      fp_mul(LP_T, x, y);")
                    out.append("    }")
                    dst = [C_SCR + s.slot[it] if s.slot[it] is not None else junk for it in chunk]
                    dst += [junk] * (G - len(dst))
                    out.append("    LP_FOR(%d) lp_st(g, %s, LP_T);" % (G, self.sel(dst, "d")))
                else:
                    forms = [s.form_of(it) for it in chunk]
                    out.append("    LP_FOR(%d) {" % G)
                    self.emit_form("LP_T", forms)
                    red = self.reduce_line(forms)
                    if red:
                        out.append(red)
                    out.append("    }")
                    if kind == "chk":
                        bits = [cbit[(it[1], it[2])] for it in chunk] + [0] * (G - len(chunk))
                        v = 0
                        for r, bb in enumerate(bits):  # per-role bit index (5 bits) packed, 0x1f = none
                            idx = bb.bit_length() - 1 if bb else 31
                            v |= idx << (5 * r) if G <= 12 else 0
                        if G <= 12:
                            out.append("    LP_FOR(%d) lp_chk(g, LP_T, (uint32_t)((0x%xull >> (5 * role)) & 31u));" % (G, v))
                        else:
                            self.tables.append(("%s_c%d" % (P.name, len(self.tables)),
                                                [(bb.bit_length() - 1) if bb else 31 for bb in bits]))
                            out.append("    LP_FOR(%d) lp_chk(g, LP_T, LP_SELT(%s));" % (G, self.tables[-1][0]))
                    else:
                        if kind == "lin":
                            dst = [C_SCR + s.slot[it] if s.slot[it] is not None else junk for it in chunk]
                        elif staged:
                            dst = [C_SCR + stage_base + it[1] for it in chunk]
                        else:
                            dst = [C_D + it[1] for it in chunk]
                        dst += [junk] * (G - len(dst))
                        out.append("    LP_FOR(%d) lp_st(g, %s, LP_T);" % (G, self.sel(dst, "d")))
                out.append("    LP_SYNC();")
                out.append("  }")
        if staged:
            for p0 in range(0, nout, G):
                n = min(G, nout - p0)
                src = [C_SCR + stage_base + p0 + r for r in range(n)] + [0] * (G - n)
                dst = [C_D + p0 + r for r in range(n)] + [junk] * (G - n)
                out.append("  {  // copy outputs %d..%d" % (p0, p0 + n - 1))
                out.append("    LP_DECL_T;")
                out.append("    LP_FOR(%d) lp_ld(LP_T, g, %s);" % (G, self.sel(src, "s")))
                out.append("    LP_FOR(%d) lp_st(g, %s, LP_T);" % (G, self.sel(dst, "d")))
                out.append("    LP_SYNC();")
                out.append("  }")
        self.n_scr_total = n_scr_total
        return out


def emit_header(progs):
    hdr = ["// GENERATED by gen_lane_progs.py -- do not edit.",
           "// Lane-group programs: see gen_lane_progs.py (scheduling) and ssb_lane.h (runtime).",
           "#pragma once", "#include \"ssb_lane.h\"", "namespace ssb {", "namespace lane {"]
    hdr.append("// shared constant slots (code -> value), filled by lp_init_consts")
    hdr.append("constexpr int N_CONSTS = %d;" % len(CONSTS))
    summary = []
    for P, outs in progs:
        sch = Sched(P, outs)
        sch.schedule()
        sch.allocate()
        em = Emitter(sch)
        body = em.emit()
        nprod = len(sch.prods)
        for name, codes in em.tables:
            hdr.append("SSB_LP_TABLE uint8_t %s[%d] = {%s};" % (name, len(codes), ", ".join(map(str, codes))))
        hdr.append("// %s: G=%d, %d products in %d rounds (%.0f%% lane use), %d materialisations, %d outputs, "
                   "%d scratch slots, %d stages"
                   % (P.name, P.G, nprod, sch.n_rounds, 100.0 * nprod / max(1, sch.n_rounds * P.G), len(sch.mats),
                      len(sch.outs), em.n_scr_total, len(sch.stages)))
        summary.append((P.name, P.G, nprod, sch.n_rounds, len(sch.stages), em.n_scr_total))
        hdr.append("constexpr int %s_G = %d, %s_SCRATCH = %d, %s_NOUT = %d, %s_ROUNDS = %d;"
                   % (P.name, P.G, P.name, em.n_scr_total, P.name, len(sch.outs), P.name, sch.n_rounds))
        hdr.append("constexpr uint32_t %s_CHECK_MASKS[%d] = {%s};"
                   % (P.name, max(1, len(em.masks)), ", ".join("0x%xu" % m for m in em.masks) or "0u"))
        hdr.append("constexpr int %s_NCHECK = %d;" % (P.name, len(em.masks)))
        hdr.append("template <class GR> SSB_LP_FN void lp_%s(GR& g) {" % P.name.lower())
        hdr += body
        hdr.append("}")
    hdr.append("}  // namespace lane")
    hdr.append("}  // namespace ssb")
    return "\n".join(hdr) + "\n", summary


def const_init_table():
    """C initialiser of the shared constants, in code order."""
    out = []
    for nm in CONSTS:
        if nm == "ZERO":
            out.append("fp_zero()")
        elif nm == "FP_ONE":
            out.append("fp_one()")
        elif nm == "FP_B1":
            out.append("fp_from_c(FP_B1)")
        else:
            base, comp = nm.rsplit(".", 1)
            out.append("fp_from_c(%s.%s)" % (base, comp))
    return out


def main():
    ps = programs()
    txt, summary = emit_header(ps)
    consts = const_init_table()
    init = ["template <class GR> SSB_LP_FN void lp_init_consts(GR& g) {",
            "  LP_FOR_ALL_CONSTS(i) {"]
    init.append("    fp v;")
    init.append("    switch (i) {")
    for i, c in enumerate(consts):
        init.append("      case %d: v = %s; break;" % (i, c))
    init.append("      default: v = fp_zero();")
    init.append("    }")
    init.append("    g.k[i] = v;")
    init.append("  }")
    init.append("  LP_SYNC();")
    init.append("}")
    txt = txt.replace("}  // namespace lane\n}  // namespace ssb\n", "\n".join(init) + "\n}  // namespace lane\n}  // namespace ssb\n")
    path = os.path.join(HERE, "ssb_lane_progs.h")
    with open(path, "w") as f:
        f.write(txt)
    for row in summary:
        print("%-10s G=%-2d products=%-3d rounds=%-3d stages=%-3d scratch=%d" % row)
    print("wrote", path)


if __name__ == "__main__":
    main()
