"""Keygen-side pieces — CPU restatement (TEST INFRASTRUCTURE ONLY: tests/ and the fixture generator
import it, never the product path).  SURVEY.md §8(f) row 4.

  keygen_from_shares   reference src/keygen.rs:17-45: alpha_i = g~ * x_i, beta_ij = g~ * y_ij
  PedersenVSS (secret_sharing@6bca50d [EXT, recalled]; used by trusted_party_PVSS_keygen
  src/keygen.rs:74-122 and the test at keygen.rs:309-349):
    gens(label)        = (G1::from_msg_hash(label || " : g"), G1::from_msg_hash(label || " : h"))
    deal(t, n, g, h)   : f, f' of degree t-1; C_i = g * f_i + h * f'_i (i < t); shares (f(j), f'(j)), j = 1..n
    verify_share(t, id, (s, s'), C, g, h) : g * s + h * s' == sum_{i<t} C_i * id^i
PARITY UNPINNED for gens() (AMCL mapit restated, oracle/hash_to_curve.py); verify_share is the
standard Pedersen VSS identity, pinned by the reference's own assertion (keygen.rs:334-349: every
dealt share verifies).
"""
from . import bls12_381 as B
from . import hash_to_curve as H

R = B.R


def pedersen_gens(label: bytes):
    return H.g1_from_msg_hash(label + b" : g"), H.g1_from_msg_hash(label + b" : h")


def _poly(c, x):
    acc = 0
    for a in reversed(c):
        acc = (acc * x + a) % R
    return acc


def pedersen_deal(t, n, g, h, rng):
    f = [rng.fr() for _ in range(t)]
    ft = [rng.fr() for _ in range(t)]
    comm = [B.G1.add(B.G1.mul(g, a), B.G1.mul(h, b)) for a, b in zip(f, ft)]
    shares = {j: (_poly(f, j), _poly(ft, j)) for j in range(1, n + 1)}
    return f[0], ft[0], comm, shares


def verify_share(t, i, share, comm, g, h):
    s, st = share
    lhs = B.G1.add(B.G1.mul(g, s), B.G1.mul(h, st))
    rhs = None
    for k in range(t):
        rhs = B.G1.add(rhs, B.G1.mul(comm[k], pow(i, k, R)))
    return lhs == rhs
