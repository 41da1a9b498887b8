"""amcl_wrapper `from_msg_hash` — CPU restatement (TEST INFRASTRUCTURE ONLY: imported by tests/ and
the fixture generator, never by the product path).  PARITY UNPINNED: the algorithm below is restated
from recalled upstream sources that are not in this container (amcl_wrapper 0.1.7, miracl_amcl /
AMCL v3.2 Rust), and the reference ships no output to compare with.

Reference call sites: Params::new (src/signature.rs:22-32) hashes label || " : g", " : g_tilde",
" : y" || i; SignatureRequest::compute_h (src/signature.rs:197-206) hashes commitment.to_bytes() ||
known messages' to_bytes().

  hash_msg(msg)      = SHAKE256(msg) read to 48 bytes (MODBYTES)              [amcl_wrapper utils]
  G1 from_msg_hash   = ECP::mapit(hash): x = BIG::frombytes(h) mod p; loop { P = ECP::new_bigint(x, 0)
                       (y = rhs^((p+1)/4), negated if its integer value is odd; infinity when rhs is
                       not a square); x += 1; if P finite: P = [h1] P (cfp: the G1 cofactor), stop if
                       finite }
  G2 from_msg_hash   = ECP2::mapit(hash): x as above; loop { X = 1 + x i; Q = ECP2::new_fp2(X) (y =
                       FP2::sqrt(X^3 + 4(1+i)), AMCL's root); stop if finite; x += 1 }; then the
                       Budroni-Pintore cofactor clearing  [x^2 - x - 1] Q + psi([x - 1] Q) + psi^2(2 Q)
with x the (negative) BLS parameter and psi the untwist-Frobenius-twist map (AMCL ECP2::frob).
"""
import hashlib

from . import bls12_381 as B
from . import subgroup as S

P = B.P
H1 = 0x396C8C005555E1568C00AAAB0000AAAB  # G1 cofactor (x - 1)^2 / 3 (AMCL rom CURVE_Cof)
X = S.X


def hash_msg(msg: bytes) -> bytes:
    return hashlib.shake_256(msg).digest(48)


def fp_sqrt_amcl(a):
    """FP::sqrt for p = 3 mod 4: a^((p+1)/4) (a root only when a is a square)."""
    return pow(a % P, (P + 1) // 4, P)


def fp_is_qr(a):
    a %= P
    return a != 0 and pow(a, (P - 1) // 2, P) == 1


def f2_sqrt_amcl(x):
    """FP2::sqrt of AMCL v3.2: sqrt(a + ib) = s + i b / (2 s), s = sqrt((a +- sqrt(a^2 + b^2)) / 2);
    returns None when x is not a square."""
    a, b = x
    if a % P == 0 and b % P == 0:
        return (0, 0)
    w1 = (b * b + a * a) % P
    if not fp_is_qr(w1):
        return None
    w1 = fp_sqrt_amcl(w1)
    inv2 = (P + 1) // 2
    w2 = (a + w1) * inv2 % P
    if not fp_is_qr(w2):
        w2 = (a - w1) * inv2 % P
        if not fp_is_qr(w2):
            return None
    s = fp_sqrt_amcl(w2)
    return (s, b * pow(2 * s, P - 2, P) % P)


def _mul_signed(curve, Pt, k):
    Q = curve.mul_any(Pt, abs(k))
    return curve.neg(Q) if k < 0 else Q


def g1_from_msg_hash(msg: bytes):
    x = int.from_bytes(hash_msg(msg), "big") % P
    while True:
        rhs = (x * x * x + 4) % P
        x_cur = x
        x = (x + 1) % P
        if not fp_is_qr(rhs):
            continue
        y = fp_sqrt_amcl(rhs)
        if y & 1:
            y = (P - y) % P
        Pt = B.G1.mul_any((x_cur, y), H1)
        if Pt is not None:
            return Pt


def g2_from_msg_hash(msg: bytes):
    x = int.from_bytes(hash_msg(msg), "big") % P
    while True:
        X2 = (1, x)
        rhs = B.f2_add(B.f2_mul(B.f2_mul(X2, X2), X2), B.B2)
        y = f2_sqrt_amcl(rhs)
        x = (x + 1) % P
        if y is not None:
            Q = (X2, y)
            break
    G = B.G2
    xQ = _mul_signed(G, Q, X)
    x2Q = _mul_signed(G, xQ, X)
    t1 = G.add(G.add(x2Q, G.neg(xQ)), G.neg(Q))        # [x^2 - x - 1] Q
    t2 = S.psi(G.add(xQ, G.neg(Q)))                     # psi([x - 1] Q)
    t3 = S.psi(S.psi(G.dbl(Q)))                         # psi^2(2 Q)
    return G.add(G.add(t3, t1), t2)


def params_new(grp_mode: str, msg_count: int, label: bytes):
    """Params::new (src/signature.rs:22-32): (g, g_tilde, h[]) with SignatureGroup = G2 under SigG2."""
    sig = g2_from_msg_hash if grp_mode == "G2" else g1_from_msg_hash
    oth = g1_from_msg_hash if grp_mode == "G2" else g2_from_msg_hash
    g = sig(label + b" : g")
    g_tilde = oth(label + b" : g_tilde")
    h = [sig(label + b" : y" + str(i).encode()) for i in range(msg_count)]
    return g, g_tilde, h
