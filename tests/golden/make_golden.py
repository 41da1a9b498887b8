"""Generate the committed golden fixtures under tests/golden/ from the Python oracle.

    python tests/golden/make_golden.py          (~2-4 minutes, single core)

The reference holds no golden vectors or known-answer tests (all its tests use an unseeded RNG;
SURVEY.md §4, §8c), so every fixture here is produced by the CPU restatement in `oracle/` from a
seeded SHAKE256 DRBG and is pinned by the algebraic identities the reference's tests assert
(see tests/test_oracle.py).  Files are data (inputs + expected outputs), hex-encoded JSON.
"""

from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as B          # noqa: E402
from oracle import coconut_ref as C        # noqa: E402


def hx(b: bytes) -> str:
    return b.hex()


def fr_hex(k: int) -> str:
    return B.fr_to_bytes(k).hex()


def setup(mode, q, t, n, seed):
    grp = C.Groups(mode)
    rng = C.Drbg(seed)
    params = C.params_from_rng(grp, q, rng)
    sx, sy, signers = C.trusted_party_sss_keygen(grp, t, n, params, rng)
    vk = C.verkey_aggregate(grp, t, [(s["id"], s["vk"]) for s in signers])
    return grp, rng, params, sx, sy, signers, vk


def vk_json(grp, vk):
    return {"X": hx(grp.oth_to_bytes(vk[0])), "Y": [hx(grp.oth_to_bytes(y)) for y in vk[1]]}


KINDS = ["valid", "sigma2_plus_g", "msg_plus_1", "swapped", "sigma1_inf", "sigma2_inf",
         "wrong_key", "both_inf", "offcurve_sigma1", "neg_sigma2"]


def make_verify(mode, q, ncred, seed, per_cred_vk=False):
    t, n = 3, 5
    grp, rng, params, sx, sy, signers, vk = setup(mode, q, t, n, seed)
    secret = (sx, sy)
    # a second key pair for "wrong_key"
    wrong = (rng.fr(), [rng.fr() for _ in range(q)])
    creds = []
    for c in range(ncred):
        kind = "valid" if (c % 3 != 1) else KINDS[1 + (c // 3) % (len(KINDS) - 1)]
        if per_cred_vk:
            sk = (rng.fr(), [rng.fr() for _ in range(q)])
            cvk = (grp.other.mul(params["g_tilde"], sk[0]),
                   [grp.other.mul(params["g_tilde"], y) for y in sk[1]])
        else:
            sk, cvk = secret, vk
        msgs = [rng.fr() for _ in range(q)]
        h = grp.sig.mul(grp.sig.gen, rng.fr())
        sig = C.sign(grp, sk, msgs, h)
        s1b = grp.sig_to_bytes(sig[0])
        s2b = grp.sig_to_bytes(sig[1])
        if kind == "sigma2_plus_g":
            sig = (sig[0], grp.sig.add(sig[1], grp.sig.gen))
        elif kind == "msg_plus_1":
            j = c % q
            msgs = list(msgs)
            msgs[j] = (msgs[j] + 1) % B.R
        elif kind == "swapped":
            sig = (sig[1], sig[0])
        elif kind == "sigma1_inf":
            sig = (None, sig[1])
        elif kind == "sigma2_inf":
            sig = (sig[0], None)
        elif kind == "wrong_key":
            sig = C.sign(grp, wrong, msgs, h)
        elif kind == "both_inf":
            sig = (None, None)
        elif kind == "neg_sigma2":
            sig = (sig[0], grp.sig.neg(sig[1]))
        s1b = grp.sig_to_bytes(sig[0])
        s2b = grp.sig_to_bytes(sig[1])
        if kind == "offcurve_sigma1":
            # flip a bit of y: not on the curve -> AMCL decodes to infinity -> reject
            bb = bytearray(s1b)
            bb[-1] ^= 1
            s1b = bytes(bb)
        s1 = grp.sig_from_bytes(s1b)
        s2 = grp.sig_from_bytes(s2b)
        verdict, gt = C.verify_gt(grp, (s1, s2), msgs, cvk, params["g_tilde"])
        if kind == "valid":
            assert verdict, "valid credential rejected by the oracle"
        else:
            assert not verdict, kind
        rec = {"kind": kind, "sigma1": hx(s1b), "sigma2": hx(s2b),
               "msgs": [fr_hex(m) for m in msgs], "verdict": int(verdict),
               "gt": hx(B.gt_to_bytes(gt))}
        if per_cred_vk:
            rec["vk"] = vk_json(grp, cvk)
        creds.append(rec)
        print(f"  verify {mode} q={q} cred {c} {kind} -> {int(verdict)}", flush=True)
    out = {"mode": mode, "q": q, "seed": seed, "threshold": t, "total": n,
           "g_tilde": hx(grp.oth_to_bytes(params["g_tilde"])),
           "creds": creds}
    if not per_cred_vk:
        out["vk"] = vk_json(grp, vk)
    return out


PERVK_EDGES = ["vk_x_identity", "vk_y_identity", "vk_dup_bases", "vk_y_offcurve", "msg_zero", "msg_r_minus_1",
               "msg_nibbles_8", "msg_noncanonical", "msg_top_nibble"]


def make_verify_pervk_edges(mode, q, seed):
    """Per-credential verkeys (Signature::verify takes the verkey per call, signature.rs:473-478) at
    msg_count q: the corruption kinds of make_verify, each under its own key, then the edge cases of
    a variable-base MSM over [X~, Y~_1..q]: identity X~ or Y~_j (x = 0 / y_j = 0), repeated bases, an
    off-curve Y~_j (AMCL decodes it to the identity, so the credential fails), scalars 0, r - 1, all
    radix-16 digits 8 (the signed recoding's carry chain), a message given as m + r (48 bytes: decoded
    mod r) and one whose top nibble is set."""
    grp, rng, params, sx, sy, signers, vk = setup(mode, q, 3, 5, seed)
    base = make_verify(mode, q, 28, seed, per_cred_vk=True)
    creds = base["creds"]
    for kind in PERVK_EDGES:
        sk = (rng.fr(), [rng.fr() for _ in range(q)])
        msgs = [rng.fr() for _ in range(q)]
        enc_msgs = None
        if kind == "vk_x_identity":
            sk = (0, sk[1])
        elif kind == "vk_y_identity":
            sk = (sk[0], [0 if j % 2 == 1 else y for j, y in enumerate(sk[1])])
        elif kind == "vk_dup_bases":
            sk = (sk[0], [sk[1][0]] * q)
        elif kind == "msg_zero":
            msgs = [0] + msgs[1:]
        elif kind == "msg_r_minus_1":
            msgs = [B.R - 1] * q
        elif kind == "msg_nibbles_8":
            msgs = [int("8" * 63, 16) % B.R] + [int("8" * 62, 16)] * (q - 1)
        elif kind == "msg_noncanonical":
            enc_msgs = [(m + B.R).to_bytes(48, "big").hex() for m in msgs]
        elif kind == "msg_top_nibble":
            msgs = [B.R - (1 << 200) - j for j in range(q)]
        cvk = (grp.other.mul(params["g_tilde"], sk[0]) if sk[0] else None,
               [grp.other.mul(params["g_tilde"], y) if y else None for y in sk[1]])
        h = grp.sig.mul(grp.sig.gen, rng.fr())
        sig = C.sign(grp, sk, msgs, h)
        vkj = vk_json(grp, cvk)
        vk_used = cvk
        if kind == "vk_y_offcurve":
            bb = bytearray.fromhex(vkj["Y"][1])
            bb[-1] ^= 1  # y flipped: off the curve -> decoded as the identity
            vkj["Y"][1] = bb.hex()
            vk_used = (cvk[0], [None if j == 1 else y for j, y in enumerate(cvk[1])])
        s1b, s2b = grp.sig_to_bytes(sig[0]), grp.sig_to_bytes(sig[1])
        verdict, gt = C.verify_gt(grp, (grp.sig_from_bytes(s1b), grp.sig_from_bytes(s2b)), msgs, vk_used,
                                  params["g_tilde"])
        assert verdict == (kind != "vk_y_offcurve"), kind
        creds.append({"kind": kind, "sigma1": hx(s1b), "sigma2": hx(s2b),
                      "msgs": enc_msgs or [fr_hex(m) for m in msgs], "verdict": int(verdict),
                      "gt": hx(B.gt_to_bytes(gt)), "vk": vkj})
        print(f"  verify-pervk {mode} q={q} {kind} -> {int(verdict)}", flush=True)
    return base


def make_aggregate(mode, seed, q=6, t=3, n=6, big=False):
    """Config 1-style keygen + the reference's aggregation test shapes
    (signature.rs:537-580 ids 1..t and gaps {1,3,5}; 761-822 sig set {1,3,5} vs vk set {2,4,6};
    duplicate ids; more than t entries)."""
    grp, rng, params, sx, sy, signers, _ = setup(mode, q, t, n, seed)
    msgs = [rng.fr() for _ in range(q)]
    h = grp.sig.mul(grp.sig.gen, rng.fr())
    partial = {s["id"]: C.sign(grp, s["sk"], msgs, h) for s in signers}
    cases = []
    id_lists = [[1, 2, 3], [1, 3, 5], [2, 4, 6], [5, 1, 3, 2, 6], [1, 1, 3], [6, 5, 4, 3]]
    if big:
        id_lists = [list(range(1, n + 1))[:t]]
    for ids in id_lists:
        sigs = [(i, partial[i]) for i in ids]
        keys = [(i, signers[i - 1]["vk"]) for i in ids]
        asig = C.signature_aggregate(grp, t, sigs)
        avk = C.verkey_aggregate(grp, t, keys)
        distinct = len(set(ids[:t])) == t
        if distinct:
            # signature.rs:554-559 — aggregated vk == g~ * secret
            assert avk[0] == grp.other.mul(params["g_tilde"], sx)
            assert all(avk[1][j] == grp.other.mul(params["g_tilde"], sy[j]) for j in range(q))
            assert C.verify(grp, asig, msgs, avk, params["g_tilde"])
        cases.append({
            "ids": ids,
            "sigma1": [hx(grp.sig_to_bytes(partial[i][0])) for i in ids],
            "sigma2": [hx(grp.sig_to_bytes(partial[i][1])) for i in ids],
            "X": [hx(grp.oth_to_bytes(signers[i - 1]["vk"][0])) for i in ids],
            "Y": [[hx(grp.oth_to_bytes(y)) for y in signers[i - 1]["vk"][1]] for i in ids],
            "out_sigma1": hx(grp.sig_to_bytes(asig[0])),
            "out_sigma2": hx(grp.sig_to_bytes(asig[1])),
            "out_X": hx(grp.oth_to_bytes(avk[0])),
            "out_Y": [hx(grp.oth_to_bytes(y)) for y in avk[1]],
            "lagrange": [fr_hex(C.lagrange_basis_at_0(set(ids[:t]), i)) for i in ids[:t]],
            "verifies": int(C.verify(grp, asig, msgs, avk, params["g_tilde"])),
        })
        print(f"  aggregate {mode} ids={ids[:8]}", flush=True)
    return {"mode": mode, "q": q, "threshold": t, "total": n, "seed": seed,
            "g_tilde": hx(grp.oth_to_bytes(params["g_tilde"])),
            "msgs": [fr_hex(m) for m in msgs],
            "secret_X": hx(grp.oth_to_bytes(grp.other.mul(params["g_tilde"], sx))),
            "secret_Y": [hx(grp.oth_to_bytes(grp.other.mul(params["g_tilde"], y))) for y in sy],
            "cases": cases}


def make_aggregate_subsets(mode, seed, q=6, t=67, n=100, ncase=3):
    """BASELINE config 4 shape: t = 67 of n = 100 issuers, each case a seeded random 67-subset of ids
    1..100 (gaps, shuffled order); case 1 also carries entries beyond t (ignored by the reference) and
    case 2 a duplicated id inside the first t (HashSet de-duplication, signature.rs:454-458)."""
    import random
    grp, rng, params, sx, sy, signers, _ = setup(mode, q, t, n, seed)
    msgs = [rng.fr() for _ in range(q)]
    h = grp.sig.mul(grp.sig.gen, rng.fr())
    partial = {s["id"]: C.sign(grp, s["sk"], msgs, h) for s in signers}
    pick = random.Random(seed)
    cases = []
    for c in range(ncase):
        ids = pick.sample(range(1, n + 1), t + (3 if c == 1 else 0))
        if c == 2:
            ids[5] = ids[40]
        sigs = [(i, partial[i]) for i in ids]
        keys = [(i, signers[i - 1]["vk"]) for i in ids]
        asig = C.signature_aggregate(grp, t, sigs)
        avk = C.verkey_aggregate(grp, t, keys)
        if len(set(ids[:t])) == t:
            assert avk[0] == grp.other.mul(params["g_tilde"], sx)
            assert C.verify(grp, asig, msgs, avk, params["g_tilde"])
        cases.append({
            "ids": ids,
            "sigma1": [hx(grp.sig_to_bytes(partial[i][0])) for i in ids],
            "sigma2": [hx(grp.sig_to_bytes(partial[i][1])) for i in ids],
            "X": [hx(grp.oth_to_bytes(signers[i - 1]["vk"][0])) for i in ids],
            "Y": [[hx(grp.oth_to_bytes(y)) for y in signers[i - 1]["vk"][1]] for i in ids],
            "out_sigma1": hx(grp.sig_to_bytes(asig[0])),
            "out_sigma2": hx(grp.sig_to_bytes(asig[1])),
            "out_X": hx(grp.oth_to_bytes(avk[0])),
            "out_Y": [hx(grp.oth_to_bytes(y)) for y in avk[1]],
            "verifies": int(C.verify(grp, asig, msgs, avk, params["g_tilde"])),
        })
        print(f"  aggregate-subsets {mode} case {c} ids={ids[:6]}...", flush=True)
    return {"mode": mode, "q": q, "threshold": t, "total": n, "seed": seed,
            "g_tilde": hx(grp.oth_to_bytes(params["g_tilde"])),
            "msgs": [fr_hex(m) for m in msgs],
            "secret_X": hx(grp.oth_to_bytes(grp.other.mul(params["g_tilde"], sx))),
            "secret_Y": [hx(grp.oth_to_bytes(grp.other.mul(params["g_tilde"], y))) for y in sy],
            "cases": cases}


POK_KINDS = ["valid", "valid", "bad_chal", "bad_revealed", "bad_response", "sigma1_inf",
             "bad_J", "valid"]


def make_pok(mode, q, revealed, nproof, seed):
    t, n = 3, 5
    grp, rng, params, sx, sy, signers, vk = setup(mode, q, t, n, seed)
    proofs = []
    for c in range(nproof):
        kind = POK_KINDS[c % len(POK_KINDS)]
        msgs = [rng.fr() for _ in range(q)]
        h = grp.sig.mul(grp.sig.gen, rng.fr())
        sig = C.sign(grp, (sx, sy), msgs, h)
        pok = C.pok_init(grp, sig, vk, params["g_tilde"], msgs, set(revealed), rng)
        chal = int.from_bytes(__import__("hashlib").shake_256(C.pok_to_bytes(grp, pok)).digest(48),
                              "big") % B.R
        proof = C.pok_gen_proof(pok, chal)
        rev = {i: msgs[i] for i in revealed}
        if kind == "bad_chal":
            chal = (chal + 1) % B.R
        elif kind == "bad_revealed":
            i0 = revealed[0]
            rev[i0] = (rev[i0] + 1) % B.R
        elif kind == "bad_response":
            proof["responses"] = list(proof["responses"])
            proof["responses"][-1] = (proof["responses"][-1] + 5) % B.R
        elif kind == "sigma1_inf":
            proof["sig"] = (None, proof["sig"][1])
        elif kind == "bad_J":
            proof["J"] = grp.other.add(proof["J"], grp.other.gen)
        verdict, gt = C.pok_verify_gt(grp, proof, vk, params["g_tilde"], rev, chal)
        assert verdict == kind.startswith("valid"), kind
        proofs.append({
            "kind": kind,
            "sigma1": hx(grp.sig_to_bytes(proof["sig"][0])),
            "sigma2": hx(grp.sig_to_bytes(proof["sig"][1])),
            "J": hx(grp.oth_to_bytes(proof["J"])),
            "T": hx(grp.oth_to_bytes(proof["T"])),
            "responses": [fr_hex(x) for x in proof["responses"]],
            "chal": fr_hex(chal),
            "revealed_msgs": [fr_hex(rev[i]) for i in revealed],
            "verdict": int(verdict),
            "gt": hx(B.gt_to_bytes(gt)) if gt is not None else None,
        })
        print(f"  pok {mode} q={q} proof {c} {kind} -> {int(verdict)}", flush=True)
    return {"mode": mode, "q": q, "revealed": list(revealed), "seed": seed,
            "g_tilde": hx(grp.oth_to_bytes(params["g_tilde"])), "vk": vk_json(grp, vk),
            "proofs": proofs}


def make_subgroup(seed):
    """Encodings with their codec status (0 identity / invalid, 1 on-curve outside the order-r
    subgroup, 2 in G1 / G2), status by the DEFINITION [r] P == O and cross-checked by the
    endomorphism tests the device runs (oracle/subgroup.py)."""
    from oracle import subgroup as S
    rng = C.Drbg(seed)
    h1 = 0x396C8C005555E1568C00AAAB0000AAAB
    out = {}
    for name, curve, enc, endo in (("G1", B.G1, B.g1_to_bytes, S.in_g1_endo), ("G2", B.G2, B.g2_to_bytes, S.in_g2_endo)):
        pts = [curve.mul(curve.gen, rng.fr()) for _ in range(3)]
        pts += [S.random_curve_point(curve, rng.fr()) for _ in range(4)]
        if name == "G1":
            pts.append(curve.mul_any(S.random_curve_point(curve, rng.fr()), h1))  # cofactor-cleared
        recs = []
        for Pt in pts:
            st = 2 if S.in_subgroup_def(curve, Pt) else 1
            assert (st == 2) == endo(Pt)
            recs.append({"point": hx(enc(Pt)), "status": st})
        recs.append({"point": hx(enc(None)), "status": 0})
        bad = bytearray(enc(pts[0]))
        bad[-1] ^= 1  # off the curve
        recs.append({"point": hx(bytes(bad)), "status": 0})
        out[name] = recs
        print(f"  subgroup {name}: {[r['status'] for r in recs]}", flush=True)
    return out


def make_hash_to_curve():
    """amcl_wrapper from_msg_hash vectors (PARITY UNPINNED: AMCL mapit restated, oracle/hash_to_curve.py):
    messages across the SHAKE256 block boundary (rate 136) and Params::new(6, "test") in both group
    assignments (the reference's test label, signature.rs:668-679)."""
    from oracle import hash_to_curve as H
    import hashlib
    msgs = [b"", b"a", bytes(range(47)), bytes(135), bytes(range(136)), bytes(137), b"x" * 271, b"y" * 272,
            bytes((7 * i) & 0xFF for i in range(300))]
    out = {"messages": []}
    for m in msgs:
        out["messages"].append({"msg": hx(m), "shake256_48": hashlib.shake_256(m).hexdigest(48),
                                "g1": hx(B.g1_to_bytes(H.g1_from_msg_hash(m))),
                                "g2": hx(B.g2_to_bytes(H.g2_from_msg_hash(m)))})
        print(f"  h2c msg len {len(m)}", flush=True)
    for mode in ("G2", "G1"):
        g, gt, h = H.params_new(mode, 6, b"test")
        sig_enc = B.g2_to_bytes if mode == "G2" else B.g1_to_bytes
        oth_enc = B.g1_to_bytes if mode == "G2" else B.g2_to_bytes
        out[f"params_{mode}"] = {"label": "test", "msg_count": 6, "g": hx(sig_enc(g)), "g_tilde": hx(oth_enc(gt)),
                                 "h": [hx(sig_enc(x)) for x in h]}
    return out


ISSUE_KINDS = ["valid", "bad_sk_response", "bad_comm_response", "resp_mismatch", "bad_ct_proof", "wrong_chal", "valid"]


def make_issuance(mode, q, k, nreq, seed):
    """SignatureRequest -> SignatureRequestPoK proof -> verify, and BlindSignature::new -> unblind ->
    Signature::verify (reference check_signing_on_random_msgs, signature.rs:582-638)."""
    from oracle import issuance as I
    grp = C.Groups(mode)
    rng = C.Drbg(seed)
    params = C.params_from_rng(grp, q, rng)
    x, y = rng.fr(), [rng.fr() for _ in range(q)]
    vk = (grp.other.mul(params["g_tilde"], x), [grp.other.mul(params["g_tilde"], v) for v in y])
    fr = lambda v: hx(B.fr_to_bytes(v % B.R))  # noqa: E731
    se = lambda pt: hx(grp.sig_to_bytes(pt))  # noqa: E731
    reqs = []
    for c in range(nreq):
        kind = ISSUE_KINDS[c % len(ISSUE_KINDS)]
        sk, pk = I.elgamal_keygen(grp, params, rng)
        msgs = [rng.fr() for _ in range(q)]
        req, rnd = I.signature_request_new(grp, msgs, k, pk, params, rng)
        pok = I.sigreq_pok_init(grp, req, pk, params, rng)
        chal = rng.fr()
        proof = I.sigreq_gen_proof(pok, msgs[:k], rnd, sk, chal)
        if kind == "bad_sk_response":
            proof["sk"]["responses"][0] += 1
        elif kind == "bad_comm_response":
            proof["comm"]["responses"][-1] += 1
        elif kind == "resp_mismatch" and k:
            proof["cts"][0][1]["responses"][1] += 1
        elif kind == "bad_ct_proof" and k:
            proof["cts"][0][0]["T"] = grp.sig.add(proof["cts"][0][0]["T"], grp.sig.gen)
        elif kind == "wrong_chal":
            chal += 1
        verdict = I.sigreq_proof_verify(grp, proof, req, pk, chal, params)
        assert verdict == (kind == "valid" or (k == 0 and kind in ("resp_mismatch", "bad_ct_proof"))), kind
        rec_p = se(proof["sk"]["T"]) + fr(proof["sk"]["responses"][0]) + se(proof["comm"]["T"])
        rec_p += "".join(fr(v) for v in proof["comm"]["responses"])
        for p1, p2 in proof["cts"]:
            rec_p += se(p1["T"]) + fr(p1["responses"][0]) + se(p2["T"]) + fr(p2["responses"][0]) + fr(p2["responses"][1])
        h, c1, c2 = I.blind_sign(grp, req, (x, y))
        sig = I.unblind(grp, (h, c1, c2), sk)
        assert C.verify(grp, sig, msgs, vk, params["g_tilde"]), "unblinded signature must verify"
        reqs.append({"kind": kind, "commitment": se(req["commitment"]), "known": [fr(m) for m in req["known"]],
                     "ciphertexts": [[se(a), se(b)] for a, b in req["ciphertexts"]], "pk": se(pk), "proof": rec_p,
                     "chal": fr(chal), "verdict": int(verdict), "h": se(h), "c1": se(c1), "c2": se(c2),
                     "sigma2": se(sig[1]), "msgs": [fr(m) for m in msgs], "elgamal_sk": fr(sk)})
        print(f"  issuance {mode} k={k} req {c} {kind} -> {int(verdict)}", flush=True)
    return {"mode": mode, "q": q, "k": k, "g": se(params["g"]), "h": [se(v) for v in params["h"]],
            "g_tilde": hx(grp.oth_to_bytes(params["g_tilde"])), "x": fr(x), "y": [fr(v) for v in y],
            "vk": {"X": hx(grp.oth_to_bytes(vk[0])), "Y": [hx(grp.oth_to_bytes(v)) for v in vk[1]]},
            "requests": reqs}


def make_keygen(seed, t=3, n=5, q=7):
    """keygen_from_shares (keygen.rs:17-45) derivations and Pedersen VSS dealings / share checks
    (trusted_party_PVSS_keygen keygen.rs:74-122, verify_share test keygen.rs:334-349), gens from the
    reference test label "testPVSS" (parity unpinned: AMCL mapit restated)."""
    from oracle import keygen as K
    rng = C.Drbg(seed)
    g, h = K.pedersen_gens(b"testPVSS")
    sets, checks = [], []
    shares_x = None
    for d in range(1 + q):
        sec, sec_t, comm, shares = K.pedersen_deal(t, n, g, h, rng)
        sets.append([hx(B.g1_to_bytes(c)) for c in comm])
        for i in range(1, n + 1):
            s_, st = shares[i]
            bad = (d + i) % 4 == 0
            if bad:
                s_ = (s_ + 1) % B.R
            ok = K.verify_share(t, i, (s_, st), comm, g, h)
            assert ok == (not bad)
            checks.append({"set": d, "id": i, "s": fr_hex(s_), "s_t": fr_hex(st), "ok": int(ok)})
        if d == 0:
            shares_x = {i: shares[i][0] for i in shares}
    grp = C.Groups("G2")
    g_tilde = B.G1.mul(B.G1.gen, rng.fr())
    derive = [{"x": fr_hex(v), "alpha": hx(B.g1_to_bytes(B.G1.mul(g_tilde, v)))} for v in shares_x.values()]
    g2t = B.G2.mul(B.G2.gen, rng.fr())
    derive_g2 = [{"x": fr_hex(v), "alpha": hx(B.g2_to_bytes(B.G2.mul(g2t, v)))} for v in shares_x.values()]
    return {"t": t, "n": n, "q": q, "g": hx(B.g1_to_bytes(g)), "h": hx(B.g1_to_bytes(h)), "commitments": sets,
            "checks": checks, "g_tilde_g1": hx(B.g1_to_bytes(g_tilde)), "derive_g1": derive,
            "g_tilde_g2": hx(B.g2_to_bytes(g2t)), "derive_g2": derive_g2}


def make_pairing_kat(seed):
    """Single-pairing KATs: e(a*G1, b*G2) bytes + the generator pairing."""
    rng = C.Drbg(seed)
    out = []
    for k in range(4):
        a, b = (1, 1) if k == 0 else (rng.fr(), rng.fr())
        Pp = B.G1.mul(B.G1.gen, a)
        Qq = B.G2.mul(B.G2.gen, b)
        gt = B.pairing(Pp, Qq)
        ml = B.miller_loop(Qq, Pp)
        out.append({"a": fr_hex(a), "b": fr_hex(b), "P": hx(B.g1_to_bytes(Pp)),
                    "Q": hx(B.g2_to_bytes(Qq)), "gt": hx(B.gt_to_bytes(gt)),
                    "miller_fexp_check": hx(B.gt_to_bytes(B.final_exp(ml)))})
    return {"pairings": out}


def write(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=0, sort_keys=True)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    which = set(sys.argv[1:])

    def want(tag):
        return not which or tag in which

    if want("kat"):
        write("pairing_kat.json", make_pairing_kat(11))
    if want("keygen"):
        write("keygen_vss.json", make_keygen(31))
    if want("issue"):
        for mode in ("G2", "G1"):
            write(f"issuance_{mode.lower()}.json", {"cases": [make_issuance(mode, 6, 2, 7, 21), make_issuance(mode, 4, 0, 3, 22),
                                                              make_issuance(mode, 3, 3, 3, 23)]})
    if want("h2c"):
        write("hash_to_curve.json", make_hash_to_curve())
    if want("subgroup"):
        write("subgroup.json", make_subgroup(13))
    for mode in ("G2", "G1"):
        if want("verify"):
            write(f"verify_{mode.lower()}_q6.json", make_verify(mode, 6, 30, 2))
            write(f"verify_{mode.lower()}_q16_pervk.json", make_verify(mode, 16, 6, 3, per_cred_vk=True))
        if want("pervk6"):
            write(f"verify_{mode.lower()}_q6_pervk.json", make_verify_pervk_edges(mode, 6, 12))
        if want("aggregate"):
            write(f"aggregate_{mode.lower()}.json", make_aggregate(mode, 4))
        if want("pok"):
            write(f"pok_{mode.lower()}_q6.json", make_pok(mode, 6, [3, 5], 8, 5))
            write(f"pok_{mode.lower()}_q32.json", make_pok(mode, 32, [3, 5, 7, 11, 13, 17, 19, 23], 8, 6))
        if want("rlc16"):
            write(f"verify_{mode.lower()}_q16.json", make_verify(mode, 16, 12, 8))
        if want("agg67"):
            write(f"aggregate_{mode.lower()}_t67_subsets.json", make_aggregate_subsets(mode, 9))
    if want("aggbig"):
        write("aggregate_g2_t67.json", make_aggregate("G2", 7, q=6, t=67, n=100, big=True))


if __name__ == "__main__":
    main()
