"""Subgroup membership for G1 / G2 points — CPU restatement (TEST INFRASTRUCTURE ONLY: imported by
tests/ and the fixture generator, never by the product path).

SURVEY.md §8(f) row 1 ("on-GPU decode and subgroup/on-curve checks, which the reference does not do
on verify").  The reference (amcl_wrapper 0.1.7 `from_bytes` [EXT]) only maps off-curve encodings to
the identity; membership in the order-r subgroup is never tested, so verdict parity keeps that
behaviour and the check is an extra, separate entry point (and the RLC batch mode's soundness guard).

Two definitions, one used to pin the other:
  * in_subgroup_def(P)  : [r] P == O  (the definition; slow)
  * in_g1_endo(P)       : phi(P) == -[x^2] P,  phi(x, y) = (beta x, y)           (eprint 2021/1130 §6,
                          proof corrected in eprint 2022/352)
  * in_g2_endo(Q)       : psi(Q) == [x] Q,     psi = untwist-Frobenius-twist     (eprint 2021/1130 §4)
with x = -0xd201000000010000 the BLS parameter.  The cube root beta and the psi coefficients are
selected below by checking them against the generators.
"""
from . import bls12_381 as B

P, R = B.P, B.R
X = -0xD201000000010000

# the two primitive cube roots of unity in Fp; phi with the right one acts as [-x^2] on G1
_w = pow(2, (P - 1) // 3, P)
if _w == 1:
    _w = pow(3, (P - 1) // 3, P)
_BETAS = (_w, _w * _w % P)


def _phi(Pt, beta):
    return None if Pt is None else (Pt[0] * beta % P, Pt[1])


def _mul_signed(curve, Pt, k):
    Q = curve.mul_any(Pt, abs(k))
    return curve.neg(Q) if k < 0 else Q


BETA = next(b for b in _BETAS if _phi(B.G1.gen, b) == _mul_signed(B.G1, B.G1.gen, -(X * X)))

# psi(x, y) = (conj(x) * PSI_X, conj(y) * PSI_Y), PSI_X = 1/xi^((p-1)/3), PSI_Y = 1/xi^((p-1)/2)
XI = (1, 1)
PSI_X = B.f2_inv(B.f2_pow(XI, (P - 1) // 3))
PSI_Y = B.f2_inv(B.f2_pow(XI, (P - 1) // 2))


def psi(Q):
    if Q is None:
        return None
    return (B.f2_mul(B.f2_conj(Q[0]), PSI_X), B.f2_mul(B.f2_conj(Q[1]), PSI_Y))


assert psi(B.G2.gen) == _mul_signed(B.G2, B.G2.gen, X), "psi coefficients"


def in_subgroup_def(curve, Pt):
    return curve.mul_any(Pt, R) is None


def in_g1_endo(Pt):
    return _phi(Pt, BETA) == _mul_signed(B.G1, Pt, -(X * X))


def in_g2_endo(Q):
    return psi(Q) == _mul_signed(B.G2, Q, X)


# ---------------------------------------------------------------- points outside the subgroups
def f2_sqrt(a):
    """Square root in Fp2 = Fp[i]/(i^2+1), p = 3 mod 4 (Adj & Rodriguez-Henriquez, Alg. 9); None if
    a is not a square."""
    a1 = B.f2_pow(a, (P - 3) // 4)
    alpha = B.f2_mul(B.f2_mul(a1, a1), a)
    a0 = B.f2_mul(B.f2_pow(alpha, P), alpha)
    if a0 == (P - 1, 0):
        return None
    x0 = B.f2_mul(a1, a)
    if alpha == (P - 1, 0):
        return B.f2_mul((0, 1), x0)
    b = B.f2_pow(B.f2_add((1, 0), alpha), (P - 1) // 2)
    return B.f2_mul(b, x0)


def random_curve_point(curve, seed_x):
    """First point with x = seed_x, seed_x + 1, ... on the curve (almost surely NOT in the subgroup:
    the cofactors are ~2^126 and ~2^380)."""
    if curve is B.G1:
        x = seed_x % P
        while True:
            rhs = (x * x * x + 4) % P
            y = B.fp_sqrt(rhs)
            if y is not None and y * y % P == rhs:
                return (x, y)
            x += 1
    x = (seed_x % P, (seed_x * 7 + 3) % P)
    while True:
        rhs = B.f2_add(B.f2_mul(B.f2_mul(x, x), x), B.B2)
        y = f2_sqrt(rhs)
        if y is not None and B.f2_mul(y, y) == rhs:
            return (x, y)
        x = ((x[0] + 1) % P, x[1])
