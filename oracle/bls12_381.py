"""BLS12-381 CPU restatement — TEST INFRASTRUCTURE ONLY (the checker, never the product).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import
anything under `oracle/`.  The shipped path is the HIP library in `coconut-rust_amd/csrc/`
and it fails loudly when that library is missing; nothing here is a fallback.

What this restates
------------------
The reference (`/root/reference`, coconut 0.1.0) delegates all arithmetic to third-party crates
that are NOT present in this container (marked [EXT]):

* `amcl_wrapper 0.1.7` (feature `bls381`; reference `Cargo.toml:16-19`) wrapping
  `miracl_amcl` (AMCL v3.2 Rust): FP/FP2/FP4/FP12 tower, ECP (G1), ECP2 (G2), `pair::ate2`,
  `pair::fexp`, `to_bytes`/`from_bytes`.
* `ps_sig 0.1.2` (reference `Cargo.toml:21-22`): group aliases and `ate_2_pairing`.

This module restates the published algorithms of those crates for BLS12-381:

* Fp = GF(p); Fp2 = Fp[i]/(i^2+1); the sextic extension is represented FLAT here as
  Fp12 = Fp2[W]/(W^6 - xi), xi = 1+i.  AMCL's tower Fp4 = Fp2[s]/(s^2 - xi),
  Fp12 = Fp4[w]/(w^3 - s) is the same field with w = W, s = W^3; `gt_to_bytes` applies the
  coefficient permutation.  The flat form is deliberately a different
  representation from the device code (which uses the AMCL tower) and from the C oracle (which
  uses the Fp2->Fp6->Fp12 tower): three representations must agree byte-for-byte.
* G1: y^2 = x^3 + 4 over Fp.  G2: the M-type sextic twist y^2 = x^3 + 4*xi over Fp2, untwisted by
  psi(x, y) = (x / W^2, y / W^3).
* Pairing = AMCL `ate2` + `fexp`: optimal-ate Miller loop over |x| = 0xd201000000010000, a
  conjugation because x < 0, then the final exponentiation (p^6-1)(p^2+1) * 3*Phi_12(p)/r.  The
  factor 3 comes from AMCL's BLS12 hard-part chain, whose exponent is
  (x-1)^2 (x+p)(x^2+p^2-1) + 3 = 3*Phi_12(p)/r (checked by `tests/test_oracle.py`).  Line
  normalisations (Fp2 multiples times powers of W) are killed by the easy part, so the GT value is
  fixed by the Miller function alone.
* Serialisation (amcl_wrapper `to_bytes`): Fr 48 B big-endian; G1 97 B = 0x04 || x || y;
  G2 192 B = x.a || x.b || y.a || y.b; GT 576 B in AMCL FP12 order a.a.a, a.a.b, a.b.a, a.b.b,
  b.a.a, ..., c.b.b (each 48 B BE).  Identity encodes as AMCL's projective infinity (x = 0, y = 1);
  any encoding that is not on the curve decodes to the identity (AMCL `ECP::new_bigs`).

Parity status: verdicts and group elements are pinned algebraically by the
reference's own tests (see tests/test_oracle.py); GT bytes and the infinity encoding are
"parity unpinned" — the AMCL sources are not available offline.
"""

from __future__ import annotations

# ----------------------------------------------------------------------------------------------
# Curve constants (BLS12-381; AMCL rom for BLS381)
# ----------------------------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
X_ABS = 0xD201000000010000  # |x|, x = -X_ABS (AMCL SIGN_OF_X = NEGATIVEX)
B1 = 4                       # G1: y^2 = x^3 + 4
XI = (1, 1)                  # xi = 1 + i
B2 = (4, 4)                  # G2 twist: y^2 = x^3 + 4*xi

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

FP_BYTES = 48


# ----------------------------------------------------------------------------------------------
# Fp2 = Fp[i]/(i^2 + 1), elements are tuples (a, b) = a + b*i
# ----------------------------------------------------------------------------------------------
def f2_add(x, y):
    return ((x[0] + y[0]) % P, (x[1] + y[1]) % P)


def f2_sub(x, y):
    return ((x[0] - y[0]) % P, (x[1] - y[1]) % P)


def f2_neg(x):
    return ((-x[0]) % P, (-x[1]) % P)


def f2_mul(x, y):
    a, b = x
    c, d = y
    return ((a * c - b * d) % P, (a * d + b * c) % P)


def f2_sqr(x):
    return f2_mul(x, x)


def f2_muls(x, k):
    return ((x[0] * k) % P, (x[1] * k) % P)


def f2_conj(x):
    return (x[0], (-x[1]) % P)


def f2_inv(x):
    a, b = x
    t = pow((a * a + b * b) % P, -1, P)
    return ((a * t) % P, (-b * t) % P)


def f2_mul_xi(x):
    a, b = x
    return ((a - b) % P, (a + b) % P)


def f2_pow(x, e):
    r = (1, 0)
    base = x
    while e:
        if e & 1:
            r = f2_mul(r, base)
        base = f2_sqr(base)
        e >>= 1
    return r


def f2_is_zero(x):
    return x[0] == 0 and x[1] == 0


F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def fp_sqrt(a):
    """p = 3 mod 4 square root; returns None if a is a non-residue."""
    s = pow(a, (P + 1) // 4, P)
    return s if (s * s) % P == a % P else None


# ----------------------------------------------------------------------------------------------
# Fp12 flat: list of 6 Fp2 coefficients of W^0..W^5, W^6 = xi
# ----------------------------------------------------------------------------------------------
def f12_one():
    return [F2_ONE] + [F2_ZERO] * 5


def f12_mul(x, y):
    acc = [[0, 0] for _ in range(11)]
    for i in range(6):
        xa, xb = x[i]
        if xa == 0 and xb == 0:
            continue
        for j in range(6):
            ya, yb = y[j]
            if ya == 0 and yb == 0:
                continue
            t = acc[i + j]
            t[0] += xa * ya - xb * yb
            t[1] += xa * yb + xb * ya
    out = []
    for k in range(6):
        a, b = acc[k]
        if k + 6 < 11:
            ha, hb = acc[k + 6]
            # h * xi = (ha - hb) + (ha + hb) i
            a += ha - hb
            b += ha + hb
        out.append((a % P, b % P))
    return out


def f12_sqr(x):
    return f12_mul(x, x)


def f12_conj(x):
    """x^(p^6): W^(p^6) = -W, so odd coefficients flip sign (checked in tests)."""
    return [c if k % 2 == 0 else f2_neg(c) for k, c in enumerate(x)]


def f12_eq(x, y):
    return all(a == b for a, b in zip(x, y))


def f12_is_one(x):
    return f12_eq(x, f12_one())


def _f6_inv(g0, g1, g2):
    """Inverse in Fp2[V]/(V^3 - xi) of g0 + g1 V + g2 V^2."""
    A = f2_sub(f2_sqr(g0), f2_mul_xi(f2_mul(g1, g2)))
    B = f2_sub(f2_mul_xi(f2_sqr(g2)), f2_mul(g0, g1))
    C = f2_sub(f2_sqr(g1), f2_mul(g0, g2))
    F = f2_add(f2_mul(g0, A), f2_mul_xi(f2_add(f2_mul(g2, B), f2_mul(g1, C))))
    Fi = f2_inv(F)
    return f2_mul(A, Fi), f2_mul(B, Fi), f2_mul(C, Fi)


def f12_inv(x):
    c = f12_conj(x)
    g = f12_mul(x, c)  # lies in Fp6 = Fp2[W^2]
    assert all(f2_is_zero(g[k]) for k in (1, 3, 5))
    i0, i1, i2 = _f6_inv(g[0], g[2], g[4])
    gi = [i0, F2_ZERO, i1, F2_ZERO, i2, F2_ZERO]
    return f12_mul(c, gi)


def f12_pow(x, e):
    r = f12_one()
    base = x
    while e:
        if e & 1:
            r = f12_mul(r, base)
        base = f12_sqr(base)
        e >>= 1
    return r


# Frobenius: (c W^k)^p = conj(c) * gamma_k * W^k, gamma_k = xi^(k(p-1)/6)
FROB_GAMMA = [f2_pow(XI, k * (P - 1) // 6) for k in range(6)]


def f12_frob(x):
    return [f2_mul(f2_conj(c), FROB_GAMMA[k]) for k, c in enumerate(x)]


# ----------------------------------------------------------------------------------------------
# Elliptic curves, affine; None is the point at infinity.  Generic over Fp / Fp2 via small ops.
# ----------------------------------------------------------------------------------------------
class _FpOps:
    zero = 0
    one = 1
    b = B1

    @staticmethod
    def add(a, b): return (a + b) % P
    @staticmethod
    def sub(a, b): return (a - b) % P
    @staticmethod
    def mul(a, b): return (a * b) % P
    @staticmethod
    def neg(a): return (-a) % P
    @staticmethod
    def inv(a): return pow(a, -1, P)
    @staticmethod
    def muls(a, k): return (a * k) % P
    @staticmethod
    def is_zero(a): return a % P == 0


class _Fp2Ops:
    zero = F2_ZERO
    one = F2_ONE
    b = B2
    add = staticmethod(f2_add)
    sub = staticmethod(f2_sub)
    mul = staticmethod(f2_mul)
    neg = staticmethod(f2_neg)
    inv = staticmethod(f2_inv)
    muls = staticmethod(f2_muls)
    is_zero = staticmethod(f2_is_zero)


class Curve:
    def __init__(self, F, gen, name):
        self.F = F
        self.gen = gen
        self.name = name

    def on_curve(self, Pt):
        if Pt is None:
            return True
        F = self.F
        x, y = Pt
        return F.sub(F.mul(y, y), F.add(F.mul(F.mul(x, x), x), F.b)) == F.zero

    def neg(self, Pt):
        if Pt is None:
            return None
        return (Pt[0], self.F.neg(Pt[1]))

    def add(self, A, B):
        F = self.F
        if A is None:
            return B
        if B is None:
            return A
        x1, y1 = A
        x2, y2 = B
        if x1 == x2:
            if y1 == y2 and not F.is_zero(y1):
                lam = F.mul(F.muls(F.mul(x1, x1), 3), F.inv(F.muls(y1, 2)))
            else:
                return None
        else:
            lam = F.mul(F.sub(y2, y1), F.inv(F.sub(x2, x1)))
        x3 = F.sub(F.sub(F.mul(lam, lam), x1), x2)
        y3 = F.sub(F.mul(lam, F.sub(x1, x3)), y1)
        return (x3, y3)

    def dbl(self, A):
        return self.add(A, A)

    def mul(self, A, k):
        """Scalar multiplication (double-and-add); k reduced mod r like an Fr exponent."""
        k %= R
        Rp = None
        Q = A
        while k:
            if k & 1:
                Rp = self.add(Rp, Q)
            Q = self.dbl(Q)
            k >>= 1
        return Rp

    def mul_any(self, A, k):
        """Scalar multiplication without reducing k mod r (for subgroup / cofactor checks)."""
        Rp = None
        Q = A
        while k > 0:
            if k & 1:
                Rp = self.add(Rp, Q)
            Q = self.dbl(Q)
            k >>= 1
        return Rp

    def msm(self, points, scalars):
        """sum k_i P_i — amcl_wrapper `multi_scalar_mul_{var,const}_time` output (same element)."""
        if len(points) != len(scalars):
            raise ValueError("UnequalNoOfBasesExponents")
        acc = None
        for Pt, k in zip(points, scalars):
            acc = self.add(acc, self.mul(Pt, k))
        return acc


G1 = Curve(_FpOps, G1_GEN, "G1")
G2 = Curve(_Fp2Ops, G2_GEN, "G2")


# ----------------------------------------------------------------------------------------------
# Pairing (AMCL ate2 + fexp semantics)
# ----------------------------------------------------------------------------------------------
def _line(lam, xt, yt, Pg1):
    """Line through psi(T) with twist-slope lam, evaluated at P, scaled by W^3 (a monomial, killed
    by the easy part):  y_P W^3 - lam x_P W^2 + (lam x_T - y_T)."""
    xp, yp = Pg1
    c0 = f2_sub(f2_mul(lam, xt), yt)
    c2 = f2_neg(f2_muls(lam, xp))
    c3 = (yp % P, 0)
    return [c0, F2_ZERO, c2, c3, F2_ZERO, F2_ZERO]


def miller_loop(Qg2, Pg1):
    """f_{x,Q}(P) up to subfield factors; Q on the twist (affine Fp2), P in G1 (affine Fp).
    Returns the Fp12 identity when either point is infinity (AMCL ate: e(O, .) = 1)."""
    if Qg2 is None or Pg1 is None:
        return f12_one()
    f = f12_one()
    T = Qg2
    xq, yq = Qg2
    nbits = X_ABS.bit_length()
    for i in range(nbits - 2, -1, -1):
        xt, yt = T
        lam = f2_mul(f2_muls(f2_sqr(xt), 3), f2_inv(f2_muls(yt, 2)))
        f = f12_mul(f12_sqr(f), _line(lam, xt, yt, Pg1))
        T = G2.dbl(T)
        if (X_ABS >> i) & 1:
            xt, yt = T
            lam = f2_mul(f2_sub(yq, yt), f2_inv(f2_sub(xq, xt)))
            f = f12_mul(f, _line(lam, xt, yt, Pg1))
            T = G2.add(T, Qg2)
    return f12_conj(f)  # x < 0


PHI12 = P ** 4 - P ** 2 + 1
assert PHI12 % R == 0
HARD_EXP = 3 * PHI12 // R  # AMCL hard part exponent (3 * Phi_12(p) / r)


def final_exp(f):
    """AMCL `fexp`: easy part f^((p^6-1)(p^2+1)), hard part ^(3*Phi_12(p)/r)."""
    t = f12_mul(f12_conj(f), f12_inv(f))           # f^(p^6 - 1)
    t = f12_mul(f12_frob(f12_frob(t)), t)          # ^(p^2 + 1)
    return f12_pow(t, HARD_EXP)


def pairing(Pg1, Qg2):
    """amcl_wrapper GT::ate_pairing(g1, g2) = fexp(ate(g2, g1))."""
    return final_exp(miller_loop(Qg2, Pg1))


def ate_2_pairing(P1, Q1, P2, Q2):
    """amcl_wrapper GT::ate_2_pairing(g1, g2, h1, h2) = e(g1, g2) * e(h1, h2), one shared fexp."""
    return final_exp(f12_mul(miller_loop(Q1, P1), miller_loop(Q2, P2)))


# ----------------------------------------------------------------------------------------------
# amcl_wrapper / AMCL byte codec
# ----------------------------------------------------------------------------------------------
def int_to_be(v, n=FP_BYTES):
    return int(v).to_bytes(n, "big")


def be_to_int(b):
    return int.from_bytes(bytes(b), "big")


def fr_to_bytes(k):
    return int_to_be(k % R)


def fr_from_bytes(b):
    return be_to_int(b) % R


G1_BYTES = 97
G2_BYTES = 192
GT_BYTES = 576


def g1_to_bytes(Pt):
    if Pt is None:
        return b"\x04" + int_to_be(0) + int_to_be(1)
    return b"\x04" + int_to_be(Pt[0]) + int_to_be(Pt[1])


def g1_from_bytes(b):
    """AMCL ECP::frombytes (uncompressed): off-curve -> infinity."""
    b = bytes(b)
    assert len(b) == G1_BYTES
    if b[0] != 0x04:
        return None  # only the uncompressed form amcl_wrapper writes is accepted
    x = be_to_int(b[1:49]) % P
    y = be_to_int(b[49:97]) % P
    Pt = (x, y)
    return Pt if G1.on_curve(Pt) else None


def g2_to_bytes(Pt):
    if Pt is None:
        return int_to_be(0) + int_to_be(0) + int_to_be(1) + int_to_be(0)
    (xa, xb), (ya, yb) = Pt
    return int_to_be(xa) + int_to_be(xb) + int_to_be(ya) + int_to_be(yb)


def g2_from_bytes(b):
    b = bytes(b)
    assert len(b) == G2_BYTES
    v = [be_to_int(b[k * 48:(k + 1) * 48]) % P for k in range(4)]
    Pt = ((v[0], v[1]), (v[2], v[3]))
    return Pt if G2.on_curve(Pt) else None


# AMCL FP12 = a + b w + c w^2 over FP4 (a = a.a + a.b s), s = W^3, w = W.
# Flat index of each AMCL FP2 slot, in serialisation order a.a, a.b, b.a, b.b, c.a, c.b:
AMCL_SLOT_TO_W = [0, 3, 1, 4, 2, 5]


def gt_to_bytes(f):
    out = b""
    for k in AMCL_SLOT_TO_W:
        a, b = f[k]
        out += int_to_be(a) + int_to_be(b)
    return out


def gt_from_bytes(b):
    b = bytes(b)
    f = [F2_ZERO] * 6
    for slot, k in enumerate(AMCL_SLOT_TO_W):
        a = be_to_int(b[slot * 96: slot * 96 + 48])
        c = be_to_int(b[slot * 96 + 48: slot * 96 + 96])
        f[k] = (a, c)
    return f
