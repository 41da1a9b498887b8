"""Issuer-side Coconut flow — CPU restatement (TEST INFRASTRUCTURE ONLY: tests/ and the fixture
generator import it; the product path never does).  SURVEY.md §8(f) row 3.

Follows reference src/signature.rs step for step:
  SignatureRequest::new           124-189   commitment = MSM(h_1..h_k, g; m_1..m_k, r); h = compute_h;
                                            ciphertext_i = elgamal_encrypt(g, pk, h * m_i)  (elgamal.rs:11-19)
  SignatureRequest::compute_h     197-206   from_msg_hash(commitment.to_bytes() || m_j.to_bytes() ...)
  SignatureRequestPoK::init       215-270   Schnorr commitments (impl_PoK_VC!, ps_sig [EXT])
  SignatureRequestPoK::gen_proof  283-320   response = blinding - challenge * secret
  SignatureRequestProof::verify   324-377   four kinds of Schnorr checks + response equality
  BlindSignature::new             382-433   (h, (sum y_i a_i, sum y_i b_i + h (x + sum y_{k+j} m_j)))
  BlindSignature::unblind         436-443   sigma = (h, c2 - sk c1)
impl_PoK_VC! ProofX::verify [EXT, recalled]: MSM(bases || commitment, responses || challenge) - T == O,
UnequalNoOfBasesExponents when the counts differ.
"""
from . import bls12_381 as B
from . import hash_to_curve as H

R = B.R


def compute_h(grp, commitment, known_msgs):
    data = grp.sig_to_bytes(commitment) + b"".join(B.fr_to_bytes(m) for m in known_msgs)
    return H.g2_from_msg_hash(data) if grp.mode == "G2" else H.g1_from_msg_hash(data)


def elgamal_keygen(grp, params, rng):
    sk = rng.fr()
    return sk, grp.sig.mul(params["g"], sk)


def signature_request_new(grp, msgs, k, pk, params, rng):
    assert len(msgs) >= k and len(msgs) == len(params["h"])
    r = rng.fr()
    commitment = grp.sig.msm(list(params["h"][:k]) + [params["g"]], list(msgs[:k]) + [r])
    randomness = [r]
    known = list(msgs[k:])
    cts = []
    if k > 0:
        h = compute_h(grp, commitment, known)
        for m in msgs[:k]:
            kk = rng.fr()
            c1 = grp.sig.mul(params["g"], kk)
            c2 = grp.sig.add(grp.sig.mul(pk, kk), grp.sig.mul(h, m))
            randomness.append(kk)
            cts.append((c1, c2))
    return {"known": known, "commitment": commitment, "ciphertexts": cts}, randomness


def _committed(grp, bases, blindings):
    return {"bases": bases, "blindings": blindings, "T": grp.sig.msm(bases, blindings)}


def sigreq_pok_init(grp, req, pk, params, rng):
    k = len(req["ciphertexts"])
    sk_c = _committed(grp, [params["g"]], [rng.fr()])
    hb = [rng.fr() for _ in range(k)]
    comm_c = _committed(grp, list(params["h"][:k]) + [params["g"]], hb + [rng.fr()])
    cts = []
    if k:
        h = compute_h(grp, req["commitment"], req["known"])
        for i in range(k):
            c1 = _committed(grp, [params["g"]], [rng.fr()])
            c2 = _committed(grp, [pk, h], [rng.fr(), hb[i]])
            cts.append((c1, c2))
    return {"sk": sk_c, "comm": comm_c, "cts": cts}


def _proof(c, secrets, chal):
    return {"T": c["T"], "responses": [(b - chal * s) % R for b, s in zip(c["blindings"], secrets)]}


def sigreq_gen_proof(pok, hidden, randomness, sk, chal):
    return {"sk": _proof(pok["sk"], [sk], chal),
            "comm": _proof(pok["comm"], list(hidden) + [randomness[0]], chal),
            "cts": [(_proof(c1, [randomness[i + 1]], chal), _proof(c2, [randomness[i + 1], hidden[i]], chal))
                    for i, (c1, c2) in enumerate(pok["cts"])]}


def schnorr_verify(grp, bases, commitment, proof, chal):
    if len(bases) != len(proof["responses"]):
        raise ValueError("UnequalNoOfBasesExponents")
    pr = grp.sig.msm(list(bases) + [commitment], list(proof["responses"]) + [chal])
    return grp.sig.add(pr, grp.sig.neg(proof["T"])) is None


def sigreq_proof_verify(grp, proof, req, pk, chal, params):
    k = len(req["ciphertexts"])
    assert len(proof["cts"]) == k and len(proof["comm"]["responses"]) == k + 1
    if not schnorr_verify(grp, [params["g"]], pk, proof["sk"], chal):
        return False
    if not schnorr_verify(grp, list(params["h"][:k]) + [params["g"]], req["commitment"], proof["comm"], chal):
        return False
    h = compute_h(grp, req["commitment"], req["known"])
    for i, (p1, p2) in enumerate(proof["cts"]):
        if p2["responses"][1] % R != proof["comm"]["responses"][i] % R:
            return False
        if not schnorr_verify(grp, [params["g"]], req["ciphertexts"][i][0], p1, chal):
            return False
        if not schnorr_verify(grp, [pk, h], req["ciphertexts"][i][1], p2, chal):
            return False
    return True


def blind_sign(grp, req, sigkey):
    x, y = sigkey
    k = len(req["ciphertexts"])
    assert k + len(req["known"]) == len(y)
    h = compute_h(grp, req["commitment"], req["known"])
    c1 = grp.sig.msm([a for a, _ in req["ciphertexts"]], list(y[:k]))
    e = (x + sum(y[k + i] * m for i, m in enumerate(req["known"]))) % R
    c2 = grp.sig.msm([b for _, b in req["ciphertexts"]] + [h], list(y[:k]) + [e])
    return h, c1, c2


def unblind(grp, blinded, sk):
    h, c1, c2 = blinded
    return (h, grp.sig.add(c2, grp.sig.neg(grp.sig.mul(c1, sk))))
