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

Slot codes (16 bit): 0..47 shared constants (0 = zero), 48..447 group scratch, 448..479 input A,
480..511 input B, 512..543 output D.

Run: python safestakeoperator_amd/csrc/gen_lane_progs.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))

MAXT = 3     # max unit terms of a plain-summed product operand (value <= 3p)
MAXM = 8     # max unit terms of a plain-summed materialised form (value <= 8p < 2^384)
TMAX = 16    # max terms of any form (longer ones, and scaled ones, use the accumulator engine)
C_SCR, C_A, C_B, C_D = 48, 448, 480, 512
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


# ---------------- Fp6 / Fp12 tower, mirroring ssb_field.h ----------------
def f6_add(a, b): return tuple(f2_add(x, y) for x, y in zip(a, b))
def f6_sub(a, b): return tuple(f2_sub(x, y) for x, y in zip(a, b))
def f6_neg(a): return tuple(f2_neg(x) for x in a)
def f6_mul_v(a): return (f2_mul_xi(a[2]), a[0], a[1])


def f6_mul(a, b):
    t0 = f2_mul(a[0], b[0])
    t1 = f2_mul(a[1], b[1])
    t2 = f2_mul(a[2], b[2])
    u = f2_sub(f2_sub(f2_mul(f2_add(a[1], a[2]), f2_add(b[1], b[2])), t1), t2)
    c0 = f2_add(f2_mul_xi(u), t0)
    u = f2_sub(f2_sub(f2_mul(f2_add(a[0], a[1]), f2_add(b[0], b[1])), t0), t1)
    c1 = f2_add(u, f2_mul_xi(t2))
    u = f2_sub(f2_sub(f2_mul(f2_add(a[0], a[2]), f2_add(b[0], b[2])), t0), t2)
    c2 = f2_add(u, t1)
    return (c0, c1, c2)


def f6_mul_01(a, b0, b1):
    aa = f2_mul(a[0], b0)
    bb = f2_mul(a[1], b1)
    t1 = f2_add(f2_mul_xi(f2_mul(a[2], b1)), aa)
    t2 = f2_sub(f2_sub(f2_mul(f2_add(b0, b1), f2_add(a[0], a[1])), aa), bb)
    t3 = f2_add(f2_mul(a[2], b0), bb)
    return (t1, t2, t3)


def f6_mul_1(a, b1):
    return (f2_mul_xi(f2_mul(a[2], b1)), f2_mul(a[0], b1), f2_mul(a[1], b1))


def f12_mul(a, b):
    t0 = f6_mul(a[0], b[0])
    t1 = f6_mul(a[1], b[1])
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a[0], a[1]), f6_add(b[0], b[1])), t0), t1)
    return (f6_add(t0, f6_mul_v(t1)), c1)


def f12_sqr(a):
    ab = f6_mul(a[0], a[1])
    s0 = f6_add(a[0], a[1])
    s1 = f6_add(a[0], f6_mul_v(a[1]))
    s0 = f6_sub(f6_mul(s0, s1), ab)
    c0 = f6_sub(s0, f6_mul_v(ab))
    return (c0, f6_add(ab, ab))


def f12_mul_014(f, o0, o1, o4):
    aa = f6_mul_01(f[0], o0, o1)
    bb = f6_mul_1(f[1], o4)
    o = f2_add(o1, o4)
    s_ = f6_mul_01(f6_add(f[1], f[0]), o0, o)
    c1 = f6_sub(f6_sub(s_, aa), bb)
    c0 = f6_add(f6_mul_v(bb), aa)
    return (c0, c1)


def fp4_sqr(a, b):
    t0 = f2_sqr(a)
    t1 = f2_sqr(b)
    c0 = f2_add(f2_mul_xi(t1), t0)
    t2 = f2_sub(f2_sub(f2_sqr(f2_add(a, b)), t0), t1)
    return c0, t2


def f12_cyc_sqr(f):
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


def f12_frob(a, n):
    c = [a[0][0], a[1][0], a[0][1], a[1][1], a[0][2], a[1][2]]
    out = []
    for k in range(6):
        x = c[k]
        if n & 1:
            x = f2_conj(x)
        if k:
            x = f2_mul(x, K2("FROB%d[%d]" % (n, k)))
        out.append(x)
    return ((out[0], out[2], out[4]), (out[1], out[3], out[5]))


def f12_conj(a): return (a[0], f6_neg(a[1]))


def sym_fp12(T, off=0):
    s_ = [T(off + i) for i in range(12)]
    f2s = [(s_[2 * k], s_[2 * k + 1]) for k in range(6)]
    return ((f2s[0], f2s[1], f2s[2]), (f2s[3], f2s[4], f2s[5]))


def flat12(a):
    return [c for f6 in a for f2_ in f6 for c in f2_]


# ---------------- Miller loop steps, mirroring ssb_pairing.h ----------------
def miller_dbl(T, P):
    X, Y, Z = T
    xP, yP = P
    A_ = f2_sqr(X)
    B_ = f2_sqr(Y)
    C = f2_sqr(B_)
    D = f2_dbl(f2_sub(f2_sub(f2_sqr(f2_add(X, B_)), A_), C))
    E = mat2(f2_add(f2_dbl(A_), A_))
    F = f2_sqr(E)
    ZZ = mat2(f2_sqr(Z))
    l0 = f2_sub(f2_mul(E, X), f2_dbl(B_))
    l1 = f2_mul_fp(mat2(f2_neg(f2_mul(E, ZZ))), xP)
    x3 = mat2(f2_sub(F, f2_dbl(D)))
    z3 = mat2(f2_dbl(f2_mul(Y, Z)))
    y3 = f2_sub(f2_mul(E, mat2(f2_sub(D, x3))), f2_dbl(f2_dbl(f2_dbl(C))))
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


def f2_scale(a, k): return (a[0] * k, a[1] * k)


# Homogeneous-projective Miller steps (x = X/Z, y = Y/Z; Costello-Lange-Naehrig 2010, Aranha et al.
# 2011, every doubling output scaled by 4 so nothing is halved).  A line differs from the Jacobian
# step's line above by a factor in Fp2 (doubling: Z^2 vs Z_J^6 times the affine tangent line
# (y^2 - 3b', -3x^2 xP, 2y yP); addition: Z vs 2 Z_J^3 times (yQ x - y xQ, -(yQ - y) xP, (xQ - x) yP)),
# and the final exponentiation -- a multiple of p^2 - 1 -- removes every Fp2 factor.  The doubling's
# lines are ready after two product rounds instead of three, so a Miller iteration is one product
# round shorter.  b' = 4(1 + i): 3b' Z^2 = 12 (1 + i) Z^2.
def miller_dbl_h(T, P):
    X, Y, Z = T
    xP, yP = P
    Bq = f2_sqr(Y)                                          # Y^2
    xiC = f2_mul_xi(f2_sqr(Z))                              # (1 + i) Z^2
    XY = f2_mul(X, Y)
    XX = f2_sqr(X)
    YZ = f2_mul(Y, Z)
    E = f2_scale(xiC, 12)                                   # 3b' Z^2
    F = f2_scale(xiC, 36)                                   # 9b' Z^2
    x3 = mat2(f2_dbl(f2_mul(XY, f2_sub(Bq, F))))            # 2 XY (B - F)
    y3 = mat2(f2_sub(f2_sqr(f2_add(Bq, F)), f2_scale(f2_sqr(xiC), 1728)))   # (B + F)^2 - 12 E^2
    z3 = mat2(f2_scale(f2_mul(Bq, YZ), 8))                  # 4 B H, H = 2 YZ
    l0 = f2_sub(Bq, E)                                      # Y^2 - 3b' Z^2
    l1 = f2_mul_fp(f2_scale(XX, -3), xP)                    # -3 X^2 xP
    l4 = f2_mul_fp(f2_dbl(YZ), yP)                          # 2 YZ yP
    return (x3, y3, z3), (l0, l1, l4)


def miller_add_h(T, Q, P):
    X, Y, Z = T
    xQ, yQ = Q
    xP, yP = P
    th = mat2(f2_sub(Y, f2_mul(yQ, Z)))                     # theta = Y - yQ Z
    la = mat2(f2_sub(X, f2_mul(xQ, Z)))                     # lambda = X - xQ Z
    C = f2_sqr(th)
    D = mat2(f2_sqr(la))
    E = mat2(f2_mul(la, D))
    F = f2_mul(Z, C)
    G = mat2(f2_mul(X, D))
    H = mat2(f2_sub(f2_add(E, F), f2_dbl(G)))
    x3 = mat2(f2_mul(la, H))
    y3 = f2_sub(f2_mul(th, f2_sub(G, H)), f2_mul(Y, E))
    z3 = mat2(f2_mul(Z, E))
    l0 = f2_sub(f2_mul(la, yQ), f2_mul(th, xQ))             # lambda yQ - theta xQ
    l1 = f2_mul_fp(th, xP)                                  # theta xP
    l4 = f2_mul_fp(f2_neg(la), yP)                          # -lambda yP
    return (x3, y3, z3), (l0, l1, l4)


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
    # ---- Fp12 (G = 64, one program per wave): A = a (12), B = b (12) ----
    define("FP12_MUL", 12, 12, 64, lambda: flat12(f12_mul(sym_fp12(A), sym_fp12(B))))
    define("FP12_SQR", 12, 0, 64, lambda: flat12(f12_sqr(sym_fp12(A))))
    define("FP12_CYC_SQR", 12, 0, 64, lambda: flat12(f12_cyc_sqr(sym_fp12(A))))
    # two cyclotomic squarings in one program: the second squaring's operands are formed from the
    # first one's products directly (accumulator forms), so the first output stage disappears
    define("FP12_CYC_SQR2", 12, 0, 64, lambda: flat12(f12_cyc_sqr(f12_cyc_sqr(sym_fp12(A)))))
    define("FP12_CONJ", 12, 0, 64, lambda: flat12(f12_conj(sym_fp12(A))))
    for n in (1, 2, 3):
        define("FP12_FROB%d" % n, 12, 0, 64, lambda n=n: flat12(f12_frob(sym_fp12(A), n)))

    # Miller iteration, fused: f <- f^2 * l_{T,T}(P), T <- 2T.  A = f (12) | T (6), B = (xP, yP)
    def miller_iter(first=False):
        f = sym_fp12(A)
        T = ((A(12), A(13)), (A(14), A(15)), (A(16), A(17)))
        T2, (l0, l1, l4) = miller_dbl_h(T, (B(0), B(1)))
        f2 = f if first else f12_sqr(f)
        return flat12(f12_mul_014(f2, l0, l1, l4)) + flat(*T2)
    define("MILLER_ITER", 18, 2, 64, miller_iter)

    # Miller addition step: f <- f * l_{T,Q}(P), T <- T + Q.  A = f | T, B = (xQ, yQ, xP, yP)
    def miller_addstep():
        f = sym_fp12(A)
        T = ((A(12), A(13)), (A(14), A(15)), (A(16), A(17)))
        T2, (l0, l1, l4) = miller_add_h(T, ((B(0), B(1)), (B(2), B(3))), (B(4), B(5)))
        return flat12(f12_mul_014(f, l0, l1, l4)) + flat(*T2)
    define("MILLER_ADDSTEP", 18, 6, 64, miller_addstep)

    # Two Miller loops in one (a pairing check's e(P1, Q1) e(P2, Q2) before the final
    # exponentiation): f <- f^2 l_{T1,T1}(P1) l_{T2,T2}(P2), both T doubled -- the squaring of f is
    # shared, and the two lines' products ride in the same rounds.  A = f (12) | T1 (6) | T2 (6),
    # B = (xP1, yP1, xP2, yP2)
    def miller_iter2():
        f = sym_fp12(A)
        T1 = ((A(12), A(13)), (A(14), A(15)), (A(16), A(17)))
        T2 = ((A(18), A(19)), (A(20), A(21)), (A(22), A(23)))
        T1n, la = miller_dbl_h(T1, (B(0), B(1)))
        T2n, lb = miller_dbl_h(T2, (B(2), B(3)))
        g = f12_mul_014(f12_mul_014(f12_sqr(f), *la), *lb)
        return flat12(g) + flat(*T1n) + flat(*T2n)
    define("MILLER_ITER2", 24, 4, 64, miller_iter2)

    # f <- f l_{T1,Q1}(P1) l_{T2,Q2}(P2), T1 += Q1, T2 += Q2.  B = (xQ1, yQ1, xP1, yP1, xQ2, yQ2, xP2, yP2)
    def miller_addstep2():
        f = sym_fp12(A)
        T1 = ((A(12), A(13)), (A(14), A(15)), (A(16), A(17)))
        T2 = ((A(18), A(19)), (A(20), A(21)), (A(22), A(23)))
        T1n, la = miller_add_h(T1, ((B(0), B(1)), (B(2), B(3))), (B(4), B(5)))
        T2n, lb = miller_add_h(T2, ((B(6), B(7)), (B(8), B(9))), (B(10), B(11)))
        g = f12_mul_014(f12_mul_014(f, *la), *lb)
        return flat12(g) + flat(*T1n) + flat(*T2n)
    define("MILLER_ADDSTEP2", 24, 12, 64, miller_addstep2)
    return ps



# ------------------------------------------------------------------------------------------
# scheduling
# ------------------------------------------------------------------------------------------
def syms_of(f):
    return list(f.c.keys())


def wt(f):
    """Bound of a form's value in units of p: every term (|c| v mod p, or p minus it) is <= p."""
    return len(f.c)


def subst(f, sym, g):
    c = f.c.get(sym, 0)
    if not c:
        return f
    d = dict(f.c)
    del d[sym]
    return L(d) + g * c


class Sched:
    """Turns a traced program into stages.  A stage is ("lin", items) -- materialisations,
    reduced mod p and stored, and zero checks --, ("prod", items) -- at most G products -- or
    ("out", items) -- outputs (and leftover checks).  Items: ("P", i), ("M", j), ("O", k),
    ("C", c, k).  Materialisations written in the formulas are SOFT: one is inlined into its
    consumers whenever the consumers stay within the bounds (product operands wx * wy <= 9,
    other forms <= 8 terms), which removes linear stages from the dependency chain."""

    def __init__(self, prog, outs):
        self.p, self.G = prog, prog.G
        self.prods = [list(xy) for xy in prog.prods]
        self.mats = list(prog.mats)
        self.alive = [True] * len(self.mats)
        self.outs = list(outs)
        self.checks = [list(c) for c in prog.checks]
        self._eliminate()
        self._enforce()

    # -- every form that may reference a symbol --
    def _consumers(self):
        for i, xy in enumerate(self.prods):
            yield ("P", i)
        for j in range(len(self.mats)):
            if self.alive[j]:
                yield ("M", j)
        for k in range(len(self.outs)):
            yield ("O", k)
        for c, chk in enumerate(self.checks):
            for k in range(len(chk)):
                yield ("C", c, k)

    def _ok(self, it, forms):
        # the accumulator engine (ssb_lane.h la_*) reduces any form to < 2p: only the cost,
        # i.e. the number of distinct terms, is bounded
        return all(len(f.c) <= TMAX for f in forms)

    def _get(self, it):
        if it[0] == "P":
            return self.prods[it[1]]
        if it[0] == "M":
            return [self.mats[it[1]]]
        if it[0] == "O":
            return [self.outs[it[1]]]
        return [self.checks[it[1]][it[2]]]

    def _set(self, it, forms):
        if it[0] == "P":
            self.prods[it[1]] = forms
        elif it[0] == "M":
            self.mats[it[1]] = forms[0]
        elif it[0] == "O":
            self.outs[it[1]] = forms[0]
        else:
            self.checks[it[1]][it[2]] = forms[0]

    def _eliminate(self):
        changed = True
        while changed:
            changed = False
            for j in range(len(self.mats)):
                if not self.alive[j]:
                    continue
                sym = ("M", j)
                g = self.mats[j]
                trial = []
                ok = True
                for it in self._consumers():
                    if it == ("M", j):
                        continue
                    fs = self._get(it)
                    if not any(sym in f.c for f in fs):
                        continue
                    nf = [subst(f, sym, g) for f in fs]
                    if not self._ok(it, nf):
                        ok = False
                        break
                    trial.append((it, nf))
                if ok:
                    for it, nf in trial:
                        self._set(it, nf)
                    self.alive[j] = False
                    changed = True

    def _new_mat(self, f):
        self.mats.append(f)
        self.alive.append(True)
        return L({("M", len(self.mats) - 1): 1})

    def _chunk(self, f):
        """f with <= TMAX terms: longer forms become sums of materialised parts."""
        if len(f.c) <= TMAX:
            return f
        items = sorted(f.c.items(), key=lambda kv: (kv[0][0], str(kv[0][1])))
        acc = L()
        for i in range(0, len(items), TMAX):
            acc = acc + self._new_mat(L(dict(items[i:i + TMAX])))
        return self._chunk(acc)

    def _enforce(self):
        self.prods = [[self._chunk(x), self._chunk(y)] for x, y in self.prods]
        j = 0
        while j < len(self.mats):
            if self.alive[j]:
                self.mats[j] = self._chunk(self.mats[j])
            j += 1
        self.outs = [self._chunk(o) for o in self.outs]
        self.checks = [[self._chunk(c) for c in chk] for chk in self.checks]

    def schedule(self):
        G = self.G
        mats = [j for j in range(len(self.mats)) if self.alive[j]]
        users = {}
        for i, (x, y) in enumerate(self.prods):
            for s in syms_of(x) + syms_of(y):
                users.setdefault(s, []).append(("P", i))
        for j in mats:
            for s in syms_of(self.mats[j]):
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
        pend_chk = [("C", c, k) for c, chk in enumerate(self.checks) for k in range(len(chk))]

        def ready(f):
            return all(s[0] in "ABK" or s in avail for s in syms_of(f))

        def take_checks(n):
            got = [it for it in pend_chk if ready(self.checks[it[1]][it[2]])][:n]
            for it in got:
                pend_chk.remove(it)
            return got

        n_rounds = 0
        while len(done_p) < len(self.prods) or len(done_m) < len(mats):
            while True:
                lvl = [("M", j) for j in mats if ("M", j) not in done_m and ready(self.mats[j])]
                if not lvl:
                    break
                pad = (-len(lvl)) % G
                stages.append(("lin", lvl + take_checks(pad)))
                for it in lvl:
                    done_m.add(it)
                    avail.add(it)
            rp = [("P", i) for i in range(len(self.prods))
                  if ("P", i) not in done_p and ready(self.prods[i][0]) and ready(self.prods[i][1])]
            if not rp:
                if len(done_p) < len(self.prods) or len(done_m) < len(mats):
                    raise RuntimeError("%s: deadlock" % self.p.name)
                break
            rp.sort(key=lambda it: -height(it))
            pick = rp[:G]
            stages.append(("prod", pick))
            n_rounds += 1
            for it in pick:
                done_p.add(it)
                avail.add(it)
        outs = [("O", k) for k in range(len(self.outs))]
        stages.append(("out", outs + take_checks(len(pend_chk))))
        assert not pend_chk
        self.stages = stages
        self.n_rounds = n_rounds
        self.n_mats = len(mats)
        return stages

    def form_of(self, it):
        if it[0] == "M":
            return self.mats[it[1]]
        if it[0] == "O":
            return self.outs[it[1]]
        if it[0] == "C":
            return self.checks[it[1]][it[2]]
        raise KeyError(it)

    def forms_of(self, it):
        return self.prods[it[1]] if it[0] == "P" else [self.form_of(it)]

    def allocate(self):
        """Scratch slots by liveness at stage granularity (a value's slot is reusable from the
        stage after its last read; never within a stage, whose passes may run in sequence)."""
        last_use = {}
        for si, (kind, items) in enumerate(self.stages):
            for it in items:
                for f in self.forms_of(it):
                    for s in syms_of(f):
                        if s[0] in "PM":
                            last_use[s] = si
        slot = {}
        free = list(range(N_SCR))
        busy = {}
        for si, (kind, items) in enumerate(self.stages):
            for sl, s in list(busy.items()):
                if last_use.get(s, -1) < si:
                    del busy[sl]
                    free.append(sl)
            free.sort()
            for it in items:
                if it[0] in "PM":
                    if it not in last_use:
                        slot[it] = None
                        continue
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
    """-> list of (sign, magnitude, sym): unit terms first (cheap), then scaled ones."""
    items = sorted(f.c.items(), key=lambda kv: (abs(kv[1]) != 1, kv[1] < 0, kv[0][0], str(kv[0][1])))
    return [(1 if c < 0 else 0, abs(c), s) for s, c in items]


class Emitter:
    def __init__(self, sch):
        self.s, self.G = sch, sch.G
        self.lines = []
        self.tables = []      # (name, words): per-stage packed code rows, [role][NW] uint32
        self.cur = None       # codes of the stage being emitted (lists of G values)

    def sel(self, codes):
        """per-role values (< 2^16) -> a C expression of `role`: packed immediates for small
        groups, a table otherwise."""
        G = self.G
        codes = list(codes) + [0] * (G - len(codes))
        assert all(0 <= c < 65536 for c in codes)
        if G <= 8 and max(codes) < 256:
            v = 0
            for r, c in enumerate(codes):
                v |= c << (8 * r)
            return "LP_SEL8(0x%016xull)" % v
        if G <= 4:
            v = 0
            for r, c in enumerate(codes):
                v |= c << (16 * r)
            return "LP_SEL16(0x%016xull)" % v
        if G <= 8:
            lo = hi = 0
            for r, c in enumerate(codes):
                if r < 4:
                    lo |= c << (16 * r)
                else:
                    hi |= c << (16 * (r - 4))
            return "LP_SEL16X2(0x%016xull, 0x%016xull)" % (lo, hi)
        if len(set(codes)) == 1:
            return "%du" % codes[0]
        # one packed row per lane and stage (LP_CODES at the stage's top loads the lane's row with
        # 16-byte loads, one memory round trip per stage instead of one per table)
        idx = len(self.cur)
        self.cur.append(codes)
        return "LP_CW(@TAB@, @NW@, %d)" % idx

    def begin_stage(self):
        self.cur = []
        self.stage_start = len(self.lines)

    def end_stage(self):
        """Pack the stage's code lists into a table and patch the stage's lines."""
        codes, self.cur = self.cur, None
        if not codes:
            return
        G = self.G
        nw = (len(codes) + 1) // 2
        nw = (nw + 3) // 4 * 4
        name = "%s_s%d" % (self.s.p.name, len(self.tables))
        words = []
        for r in range(G):
            row = [0] * nw
            for i, c in enumerate(codes):
                row[i // 2] |= c[r] << (16 * (i & 1))
            words += row
        self.tables.append((name, words))
        for k in range(self.stage_start, len(self.lines)):
            self.lines[k] = self.lines[k].replace("@TAB@", name).replace("@NW@", str(nw))
        self.lines.insert(self.stage_start + 2, "    LP_CODES(%s, %d);" % (name, nw))

    def bits(self, bits):
        v = 0
        for r, b in enumerate(bits):
            v |= (b & 1) << r
        return "0x%xull" % v

    def emit_form(self, var, forms):
        """var = sum over terms of (+-)(|c| v mod p): each term <= p, so var <= wt * p."""
        G, out = self.G, self.lines
        tl = [terms_of(f) if f is not None else [] for f in forms]
        T = max([len(t) for t in tl] + [1])
        for k in range(T):
            codes, sg, mg = [], [], []
            for r in range(G):
                if r < len(tl) and k < len(tl[r]):
                    sgn, m, sym = tl[r][k]
                    codes.append(self.s.code(sym)); sg.append(sgn); mg.append(m)
                else:
                    codes.append(0); sg.append(0); mg.append(1)
            src = self.sel(codes)
            first = k == 0
            if all(m == 1 for m in mg):
                val = None
            else:
                # u = m * v mod p, left to right over the bits of m (per-role m)
                nb = max(m.bit_length() for m in mg)
                out.append("      { lv v_, u_; lp_ld(v_, g, %s);" % src)
                top = [(m >> (nb - 1)) & 1 for m in mg]
                if all(top):
                    out.append("        u_ = v_;")
                else:
                    out.append("        u_ = lv_zero(); lp_sel(u_, v_, u_, LP_BIT(%s));" % self.bits(top))
                for bit in range(nb - 2, -1, -1):
                    out.append("        lp_dbl_mod(u_);")
                    bs = [(m >> bit) & 1 for m in mg]
                    if all(bs):
                        out.append("        lp_add_mod(u_, v_);")
                    elif any(bs):
                        out.append("        lp_add_mod_sel(u_, v_, LP_BIT(%s));" % self.bits(bs))
                val = "u_"
            uni = "pos" if all(b == 0 for b in sg) else ("neg" if all(b == 1 for b in sg) else "mix")
            if val is None:
                if first:
                    fn = {"pos": "lp_ld(%s, g, %s);", "neg": "lp_ld_neg(%s, g, %s);",
                          "mix": "lp_ld_sgn(%s, g, %s, LP_BIT(" + self.bits(sg) + "));"}[uni]
                else:
                    fn = {"pos": "lp_acc(%s, g, %s);", "neg": "lp_acc_neg(%s, g, %s);",
                          "mix": "lp_acc_sgn(%s, g, %s, LP_BIT(" + self.bits(sg) + "));"}[uni]
                out.append("      " + fn % (var, src))
            else:
                if first:
                    fn = {"pos": "%s = u_;", "neg": "lp_pminus(%s, u_);",
                          "mix": "{ lv n_; lp_pminus(n_, u_); lp_sel(%s, n_, u_, LP_BIT(" + self.bits(sg) + ")); }"}[uni]
                else:
                    fn = {"pos": "lp_add_raw(%s, u_);", "neg": "{ lv n_; lp_pminus(n_, u_); lp_add_raw(%s, n_); }",
                          "mix": "{ lv n_; lp_pminus(n_, u_); lp_sel(n_, n_, u_, LP_BIT(" + self.bits(sg) + ")); lp_add_raw(%s, n_); }"}[uni]
                out.append("        " + fn % var + " }")
        return T

    @staticmethod
    def simple(f, maxw):
        return f is None or (len(f.c) <= maxw and all(abs(c) == 1 for c in f.c.values()))

    def emit_acc(self, var, forms, fold):
        """var = the forms' values via the accumulator engine: folded below 2p (a stored value, or an
        operand whose bound needs it), else < 2p sum|c| (acc_bound)."""
        G, out = self.G, self.lines
        tl = [terms_of(f) if f is not None else [] for f in forms]
        T = max([len(t) for t in tl] + [1])
        out.append("      { lacc A_; la_zero(A_);")
        Ks = []
        for r in range(G):
            Ks.append(sum(m for (sg, m, sym) in (tl[r] if r < len(tl) else []) if sg))
        for k in range(T):
            codes, cp, cn = [], [], []
            for r in range(G):
                if r < len(tl) and k < len(tl[r]):
                    sg, m, sym = tl[r][k]
                    codes.append(self.s.code(sym)); cp.append(0 if sg else m); cn.append(m if sg else 0)
                else:
                    codes.append(0); cp.append(0); cn.append(0)
            src = self.sel(codes)
            if all(c == 0 for c in cn):
                out.append("        la_ld_pos(A_, g, %s, %s);" % (src, self.sel(cp)))
            elif all(c == 0 for c in cp):
                out.append("        la_ld_neg(A_, g, %s, %s);" % (src, self.sel(cn)))
            else:
                out.append("        la_ld_mix(A_, g, %s, %s, %s);" % (src, self.sel(cp), self.sel(cn)))
        out.append("        la_fin(%s, A_, %s, %s); }" % (var, self.sel(Ks), "true" if fold else "false"))

    def reduce_line(self, forms):
        """Plain sums (terms < 4p, every limb < 2^29, <= MAXM terms: limbs < 2^32) -> a slot value
        (< 2p): normalized and folded, except single positive unit terms (copies)."""
        exact = all(wt(f) <= 1 and all(c == 1 for c in f.c.values()) for f in forms)
        if exact:
            return None
        return "      lp_reduce(LP_T);"

    # bounds of the reduced-radix runtime (ssb_lane.h): slot values < 2p with limbs < 2^28; a plain
    # sum's negative term K4P - v is < 4p with limbs < 2^29; an accumulator form without its fold is
    # < 2p sum|c| with normalized limbs.  A product needs x y < 2^392 p (~2521 p^2; kept <= 2400 p^2)
    # and limb products <= 2^60 (its 64-bit columns).
    @staticmethod
    def simple_bound(forms):
        return max(sum(4 if sg else 2 for (sg, m, sym) in terms_of(f)) for f in forms if f is not None)

    @staticmethod
    def simple_limb_bits(forms):
        import math
        return max(math.log2(sum((1 << 29) if sg else (1 << 28) for (sg, m, sym) in terms_of(f)))
                   for f in forms if f is not None)

    @staticmethod
    def acc_bound(forms):
        return max(2 * sum(m for (sg, m, sym) in terms_of(f)) for f in forms if f is not None)

    def emit(self):
        s, G = self.s, self.G
        P = s.p
        out = self.lines
        nout = len(s.outs)
        staged = nout > G
        stage_base = s.n_scratch
        n_scr_total = s.n_scratch + (nout if staged else 0)
        assert n_scr_total <= N_SCR, (P.name, n_scr_total)
        junk = C_SCR + s.junk
        cbit, masks, b = {}, [], 0
        for c, chk in enumerate(s.checks):
            for k in range(len(chk)):
                cbit[(c, k)] = b + k
            masks.append(((1 << len(chk)) - 1) << b)
            b += len(chk)
        assert b <= 30
        self.masks = masks
        for (kind, items) in s.stages:
            for p0 in range(0, len(items), G):
                chunk = items[p0:p0 + G]
                self.begin_stage()
                out.append("  {  // %s %s" % (kind, " ".join("".join(str(x) for x in it) for it in chunk)))
                out.append("    LP_DECL_T;")
                if kind == "prod":
                    out.append("    LP_FOR(%d) {" % G)
                    out.append("      lv x, y;")
                    xs = [s.prods[it[1]][0] for it in chunk]
                    ys = [s.prods[it[1]][1] for it in chunk]
                    xp = all(self.simple(f, MAXT) for f in xs)
                    yp = all(self.simple(f, MAXT) for f in ys)
                    bx = max(len(f.c) for f in xs) if xp else 2
                    by = max(len(f.c) for f in ys) if yp else 2
                    if bx * by > 9:  # plain sums too wide for the Montgomery bound: reduce one side
                        if xp and (bx >= by or not yp):
                            xp, bx = False, 2
                        else:
                            yp, by = False, 2
                    if bx * by > 9:
                        xp = yp = False
                    Bx = self.simple_bound(xs) if xp else self.acc_bound(xs)
                    By = self.simple_bound(ys) if yp else self.acc_bound(ys)
                    fx = fy = False
                    while Bx * By > 2400:
                        if not xp and not fx and (Bx >= By or yp or fy):
                            fx, Bx = True, 2
                        elif not yp and not fy:
                            fy, By = True, 2
                        else:
                            raise AssertionError((P.name, Bx, By))
                    nx = ny = False
                    if xp and yp:
                        lx, ly = self.simple_limb_bits(xs), self.simple_limb_bits(ys)
                        if lx + ly > 60:
                            if lx >= ly:
                                nx, lx = True, 28
                            else:
                                ny, ly = True, 28
                        assert lx + ly <= 60, (P.name, lx, ly)
                    if xp:
                        self.emit_form("x", xs)
                        if nx:
                            out.append("      lp_norm(x);")
                    else:
                        self.emit_acc("x", xs, fx)
                    if yp:
                        self.emit_form("y", ys)
                        if ny:
                            out.append("      lp_norm(y);")
                    else:
                        self.emit_acc("y", ys, fy)
                    out.append("      lp_mul(LP_T, x, y);")
                    out.append("    }")
                    dst = [C_SCR + s.slot[it] if s.slot[it] is not None else junk for it in chunk]
                    dst += [junk] * (G - len(dst))
                    out.append("    LP_FOR(%d) lp_st(g, %s, LP_T);" % (G, self.sel(dst)))
                else:
                    forms = [s.form_of(it) for it in chunk]
                    out.append("    LP_FOR(%d) {" % G)
                    if all(self.simple(f, MAXM) for f in forms):
                        self.emit_form("LP_T", forms)
                        red = self.reduce_line(forms)
                        if red:
                            out.append(red)
                    else:
                        self.emit_acc("LP_T", forms, True)
                    out.append("    }")
                    dst, cb = [], []
                    for it in chunk:
                        if it[0] == "C":
                            dst.append(junk); cb.append(cbit[(it[1], it[2])])
                        elif it[0] == "M":
                            dst.append(C_SCR + s.slot[it] if s.slot[it] is not None else junk); cb.append(31)
                        elif staged:
                            dst.append(C_SCR + stage_base + it[1]); cb.append(31)
                        else:
                            dst.append(C_D + it[1]); cb.append(31)
                    dst += [junk] * (G - len(dst))
                    cb += [31] * (G - len(cb))
                    out.append("    LP_FOR(%d) lp_st(g, %s, LP_T);" % (G, self.sel(dst)))
                    if any(c != 31 for c in cb):
                        out.append("    LP_FOR(%d) lp_chk(g, LP_T, %s);" % (G, self.sel(cb)))
                out.append("    LP_SYNC();")
                out.append("  }")
                self.end_stage()
        if staged:
            for p0 in range(0, nout, G):
                n = min(G, nout - p0)
                src = [C_SCR + stage_base + p0 + r for r in range(n)] + [0] * (G - n)
                dst = [C_D + p0 + r for r in range(n)] + [junk] * (G - n)
                self.begin_stage()
                out.append("  {  // copy outputs %d..%d" % (p0, p0 + n - 1))
                out.append("    LP_DECL_T;")
                out.append("    LP_FOR(%d) lp_ld(LP_T, g, %s);" % (G, self.sel(src)))
                out.append("    LP_FOR(%d) lp_st(g, %s, LP_T);" % (G, self.sel(dst)))
                out.append("    LP_SYNC();")
                out.append("  }")
                self.end_stage()
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
        nmat = sch.n_mats
        for name, words in em.tables:
            hdr.append("SSB_LP_TABLE uint32_t %s[%d] = {%s};" % (name, len(words), ", ".join("0x%x" % w for w in words)))
        hdr.append("// %s: G=%d, %d products in %d rounds (%.0f%% lane use), %d materialisations, %d outputs, "
                   "%d scratch slots, %d stages"
                   % (P.name, P.G, nprod, sch.n_rounds, 100.0 * nprod / max(1, sch.n_rounds * P.G), nmat,
                      len(sch.outs), em.n_scr_total, len(sch.stages)))
        summary.append((P.name, P.G, nprod, sch.n_rounds, len(sch.stages), em.n_scr_total))
        hdr.append("constexpr int %s_G = %d, %s_SCRATCH = %d, %s_NOUT = %d, %s_ROUNDS = %d;"
                   % (P.name, P.G, P.name, em.n_scr_total, P.name, len(sch.outs), P.name, sch.n_rounds))
        hdr.append("constexpr uint32_t %s_CHECK_MASKS[%d] = {%s};"
                   % (P.name, max(1, len(em.masks)), ", ".join("0x%xu" % m for m in em.masks) or "0u"))
        hdr.append("constexpr int %s_NCHECK = %d;" % (P.name, len(em.masks)))
        hdr.append("template <class GR> SSB_LP_FN void lp_%s(GR g) {" % P.name.lower())
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
            out.append("lv_zero()")
        elif nm == "FP_ONE":
            out.append("lv_one()")
        elif nm == "FP_B1":
            out.append("lv_in(fp_from_c(FP_B1))")
        else:
            base, comp = nm.rsplit(".", 1)
            out.append("lv_in(fp_from_c(%s.%s))" % (base, comp))
    return out


def main():
    ps = programs()
    txt, summary = emit_header(ps)
    consts = const_init_table()
    init = ["template <class GR> SSB_LP_FN void lp_init_consts(GR g) {",
            "  LP_FOR_ALL_CONSTS(i) {"]
    init.append("    lv v;")
    init.append("    switch (i) {")
    for i, c in enumerate(consts):
        init.append("      case %d: v = %s; break;" % (i, c))
    init.append("      default: v = lv_zero();")
    init.append("    }")
    init.append("    lp_put(g.k + i, v);")
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
