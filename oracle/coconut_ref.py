"""Coconut / PS verifier-side semantics — TEST INFRASTRUCTURE ONLY (the checker).

Restates, over `oracle/bls12_381.py`:

* `Signature::verify`        reference `src/signature.rs:473-478`  -> ps_sig `Signature::verify` [EXT]
* `Signature::aggregate`     reference `src/signature.rs:448-470`
* `Verkey::aggregate`        reference `src/signature.rs:483-526`
* `Polynomial::lagrange_basis_at_0`  secret_sharing@6bca50d [EXT], called at `signature.rs:460,502`
* `PoKOfSignature::{init, gen_proof}` and `PoKOfSignatureProof::verify`  ps_sig 0.1.2 [EXT],
  exercised by reference `src/pok_sig.rs:17-106`
* `trusted_party_SSS_keygen` reference `src/keygen.rs:53-71` (+ `keygen_from_shares` `17-45`)

Group assignment (reference `src/lib.rs:3-4,12-13`; ps_sig feature default): mode "G2" puts
sigma, g, h in G2 and X~, Y~, g~ in G1 (the reference default build); mode "G1" is the other
assignment (north_star layout).  Only the first `threshold` entries are aggregated, sigma_1 comes
from entry 0, and the Lagrange set is the de-duplicated id set (HashSet) — exactly as the
reference does.
"""

from __future__ import annotations

import hashlib

from . import bls12_381 as B

R = B.R


# ----------------------------------------------------------------------------------------------
# deterministic randomness: SHAKE256(seed || counter), rejection-sampled < r
# ----------------------------------------------------------------------------------------------
class Drbg:
    def __init__(self, seed: bytes | int | str):
        if isinstance(seed, int):
            seed = seed.to_bytes(8, "big")
        elif isinstance(seed, str):
            seed = seed.encode()
        self.seed = bytes(seed)
        self.ctr = 0

    def block(self, n=32) -> bytes:
        out = hashlib.shake_256(self.seed + self.ctr.to_bytes(8, "big")).digest(n)
        self.ctr += 1
        return out

    def fr(self) -> int:
        while True:
            v = int.from_bytes(self.block(32), "big") & ((1 << 255) - 1)
            if v < R:
                return v

    def bits(self, nbits: int) -> int:
        return int.from_bytes(self.block((nbits + 7) // 8), "big") & ((1 << nbits) - 1)

    def below(self, n: int) -> int:
        return int.from_bytes(self.block(8), "big") % n


# ----------------------------------------------------------------------------------------------
# group assignment
# ----------------------------------------------------------------------------------------------
class Groups:
    def __init__(self, mode: str):
        assert mode in ("G1", "G2")
        self.mode = mode
        if mode == "G2":   # reference default: SignatureGroup = G2, OtherGroup = G1
            self.sig, self.other = B.G2, B.G1
            self.sig_to_bytes, self.sig_from_bytes = B.g2_to_bytes, B.g2_from_bytes
            self.oth_to_bytes, self.oth_from_bytes = B.g1_to_bytes, B.g1_from_bytes
        else:
            self.sig, self.other = B.G1, B.G2
            self.sig_to_bytes, self.sig_from_bytes = B.g1_to_bytes, B.g1_from_bytes
            self.oth_to_bytes, self.oth_from_bytes = B.g2_to_bytes, B.g2_from_bytes

    def ate_2_pairing(self, s1, o1, s2, o2):
        """ps_sig `ate_2_pairing(sig1, other1, sig2, other2)`: e(.,.)*e(.,.) with the G1 argument
        first for amcl_wrapper (arguments swapped under SignatureG2)."""
        if self.mode == "G1":
            return B.ate_2_pairing(s1, o1, s2, o2)
        return B.ate_2_pairing(o1, s1, o2, s2)


# ----------------------------------------------------------------------------------------------
# secret sharing (secret_sharing@6bca50d [EXT])
# ----------------------------------------------------------------------------------------------
def lagrange_basis_at_0(ids, i: int) -> int:
    """l_i(0) = prod_{j in set, j != i} x_j / (x_j - x_i) mod r; ids is a set (duplicates collapse)."""
    num, den = 1, 1
    for x in set(ids):
        if x == i:
            continue
        num = num * x % R
        den = den * ((x - i) % R) % R
    return num * pow(den, -1, R) % R if den else 0


def get_shared_secret(threshold: int, total: int, rng: Drbg):
    """Shamir: random degree-(t-1) polynomial, secret = f(0), share_i = f(i) for i in 1..total."""
    coeffs = [rng.fr() for _ in range(threshold)]
    shares = {}
    for i in range(1, total + 1):
        acc = 0
        for c in reversed(coeffs):
            acc = (acc * i + c) % R
        shares[i] = acc
    return coeffs[0], shares


def reconstruct_secret(threshold, shares: dict) -> int:
    ids = set(list(shares.keys())[:threshold])
    return sum(lagrange_basis_at_0(ids, i) * shares[i] for i in ids) % R


# ----------------------------------------------------------------------------------------------
# Params / keys / signatures
# ----------------------------------------------------------------------------------------------
def params_from_rng(grp: Groups, msg_count: int, rng: Drbg):
    """Params{g, g_tilde, h[q]} as known multiples of the standard generators.
    (Params::new hashes a label to the curve — signature.rs:22-32 — a §8f 'next' row.)"""
    g = grp.sig.mul(grp.sig.gen, rng.fr())
    g_tilde = grp.other.mul(grp.other.gen, rng.fr())
    h = [grp.sig.mul(grp.sig.gen, rng.fr()) for _ in range(msg_count)]
    return {"g": g, "g_tilde": g_tilde, "h": h}


def trusted_party_sss_keygen(grp: Groups, threshold, total, params, rng: Drbg):
    """keygen.rs:53-71 + keygen_from_shares 17-45: Verkey_i = (g~ * x_i, [g~ * y_ij])."""
    q = len(params["h"])
    secret_x, x_shares = get_shared_secret(threshold, total, rng)
    secret_y, y_shares = [], []
    for _ in range(q):
        s, sh = get_shared_secret(threshold, total, rng)
        secret_y.append(s)
        y_shares.append(sh)
    signers = []
    for i in range(total):
        sid = i + 1
        x_i = x_shares[sid]
        y_i = [y_shares[j][sid] for j in range(q)]
        X = grp.other.mul(params["g_tilde"], x_i)
        Y = [grp.other.mul(params["g_tilde"], y) for y in y_i]
        signers.append({"id": sid, "sk": (x_i, y_i), "vk": (X, Y)})
    return secret_x, secret_y, signers


def sign(grp: Groups, sk, msgs, h_point):
    """PS signature (h, h^(x + sum y_j m_j)) — what BlindSignature::new + unblind produce
    (signature.rs:382-443) for an issuer holding sk."""
    x, y = sk
    e = (x + sum(yj * mj for yj, mj in zip(y, msgs))) % R
    return (h_point, grp.sig.mul(h_point, e))


def signature_aggregate(grp: Groups, threshold, sigs):
    """signature.rs:448-470."""
    if len(sigs) < threshold:
        raise ValueError("threshold")  # reference: assert! panic (line 449)
    sigma_1 = sigs[0][1][0]
    ids = {sid for sid, _ in sigs[:threshold]}
    pts, exps = [], []
    for sid, sig in sigs[:threshold]:
        pts.append(sig[1])
        exps.append(lagrange_basis_at_0(ids, sid))
    return (sigma_1, grp.sig.msm(pts, exps))


def verkey_aggregate(grp: Groups, threshold, keys):
    """signature.rs:483-526."""
    if len(keys) < threshold:
        raise ValueError("threshold")
    q = len(keys[0][1][1])
    for _, vk in keys[1:]:
        if len(vk[1]) != q:
            raise ValueError("ragged")
    ids = {sid for sid, _ in keys[:threshold]}
    ls = [lagrange_basis_at_0(ids, sid) for sid, _ in keys[:threshold]]
    X = grp.other.msm([vk[0] for _, vk in keys[:threshold]], ls)
    Y = [grp.other.msm([vk[1][j] for _, vk in keys[:threshold]], ls) for j in range(q)]
    return (X, Y)


def verify_gt(grp: Groups, sig, msgs, vk, g_tilde):
    """ps_sig Signature::verify [EXT] body; returns (verdict, GT or None).

    len check -> identity check -> pr = MSM([X~, Y~_1..q], [1, m_1..q]) ->
    ate_2_pairing(sigma_1, pr, -sigma_2, g~).is_one()."""
    X, Y = vk
    if len(Y) != len(msgs):
        raise ValueError("UnsupportedNoOfMessages")
    s1, s2 = sig
    pr = grp.other.msm([X] + list(Y), [1] + list(msgs))
    gt = grp.ate_2_pairing(s1, pr, grp.sig.neg(s2), g_tilde)
    if s1 is None or s2 is None:
        return False, gt
    return B.f12_is_one(gt), gt


def verify(grp: Groups, sig, msgs, vk, g_tilde) -> bool:
    return verify_gt(grp, sig, msgs, vk, g_tilde)[0]


# ----------------------------------------------------------------------------------------------
# PoK of signature (ps_sig 0.1.2 pok_sig.rs [EXT]; flow in reference pok_sig.rs:80-105)
# ----------------------------------------------------------------------------------------------
def pok_init(grp: Groups, sig, vk, g_tilde, msgs, revealed: set, rng: Drbg):
    """PoKOfSignature::init: blind sigma with r1, r2; J = g~^r2 * prod_{hidden} Y~_i^m_i;
    Schnorr commitment T = sum b_i * base_i with random blindings."""
    X, Y = vk
    r1, r2 = rng.fr(), rng.fr()
    s1p = grp.sig.mul(sig[0], r1)
    s2p = grp.sig.mul(grp.sig.add(sig[1], grp.sig.mul(sig[0], r2)), r1)
    bases = [g_tilde] + [Y[i] for i in range(len(msgs)) if i not in revealed]
    secrets = [r2] + [msgs[i] for i in range(len(msgs)) if i not in revealed]
    J = grp.other.msm(bases, secrets)
    blindings = [rng.fr() for _ in bases]
    T = grp.other.msm(bases, blindings)
    return {"sig": (s1p, s2p), "J": J, "T": T, "bases": bases, "secrets": secrets,
            "blindings": blindings}


def pok_to_bytes(grp: Groups, pok) -> bytes:
    """PoKOfSignature::to_bytes ordering (sig, J, committed bases?, commitment) — used only to
    derive a challenge for fixtures; the verifier takes `chal` as input (pok_sig.rs:94,103)."""
    out = grp.sig_to_bytes(pok["sig"][0]) + grp.sig_to_bytes(pok["sig"][1])
    out += grp.oth_to_bytes(pok["J"])
    for b in pok["bases"]:
        out += grp.oth_to_bytes(b)
    out += grp.oth_to_bytes(pok["T"])
    return out


def pok_gen_proof(pok, chal: int):
    """ProverCommitted::gen_proof: response_i = blinding_i - chal * secret_i."""
    resp = [(b - chal * s) % R for b, s in zip(pok["blindings"], pok["secrets"])]
    return {"sig": pok["sig"], "J": pok["J"], "T": pok["T"], "responses": resp}


def pok_verify_gt(grp: Groups, proof, vk, g_tilde, revealed_msgs: dict, chal: int):
    """PoKOfSignatureProof::verify [EXT]:
      identity check on sigma'; Schnorr: MSM(bases || J, responses || chal) - T == O;
      J' = X~ + J + sum_{revealed} Y~_i m_i; ate_2_pairing(sigma'_1, J', -sigma'_2, g~).is_one().
    Returns (verdict, GT or None)."""
    X, Y = vk
    s1, s2 = proof["sig"]
    if s1 is None or s2 is None:
        return False, None
    bases = [g_tilde] + [Y[i] for i in range(len(Y)) if i not in revealed_msgs]
    if len(bases) != len(proof["responses"]):
        raise ValueError("UnequalNoOfBasesExponents")
    chk = grp.other.msm(bases + [proof["J"]], list(proof["responses"]) + [chal])
    chk = grp.other.add(chk, grp.other.neg(proof["T"]))
    if chk is not None:
        return False, None
    j = grp.other.add(X, proof["J"])
    for i, m in revealed_msgs.items():
        j = grp.other.add(j, grp.other.mul(Y[i], m))
    gt = grp.ate_2_pairing(s1, j, grp.sig.neg(s2), g_tilde)
    return B.f12_is_one(gt), gt
