"""The reference's own test flows, run through the HIP entry points.

The reference ships no golden vectors (its tests draw from an unseeded RNG); what it does pin is the
assertions of its own tests.  Each test here replays one of them with every issuer- and verifier-side
step on the GPU, in both group modes, with full-size Fr scalars:

  Params::new(q, "test")          cc_hash_to_curve (params_new)                 signature.rs:22-32
  keygen_from_shares              cc_fixed_base_mul (g~ x_i, g~ y_ij)           keygen.rs:17-45
  PedersenVSS::gens / verify_share cc_hash_to_curve, cc_vss_verify_batch        keygen.rs:74-122, 332-351
  SignatureRequestProof::verify   cc_sigreq_verify_batch                        signature.rs:324-377
  BlindSignature::new             cc_blind_sign_batch                           signature.rs:382-433
  Signature::verify               cc_verify_batch (per-credential verkeys)      signature.rs:473-478
  Signature::aggregate            cc_signature_aggregate_batch                  signature.rs:448-470
  Verkey::aggregate               cc_verkey_aggregate_batch, cc_verkey_aggregate_ids   signature.rs:483-526
  PoKOfSignatureProof::verify     cc_pok_verify_batch                           pok_sig.rs:103-105

The requester's side is not on the verifier path: the Shamir/Pedersen polynomials (host
Fr arithmetic, as trusted_party_*_keygen runs them), ElGamal keygen, SignatureRequest::new,
SignatureRequestPoK, BlindSignature::unblind and PoKOfSignature::init / gen_proof come from the CPU
restatement (oracle/issuance.py, oracle/coconut_ref.py: test infrastructure), fed the GPU's own
Params and signatures.  Challenges are FieldElement::from_msg_hash on the GPU (cc_hash_msg).
"""
import numpy as np
import pytest

from test_gpu_parity import MODES

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


@pytest.fixture(scope="module")
def ctxs():
    import coconut
    c = {m: coconut.Context(0, coconut.GroupMode(v)) for m, v in MODES.items()}
    yield c
    for x in c.values():
        x.close()


def _fr(v):
    return (v % R).to_bytes(48, "big")


def _poly(coeffs, x):
    acc = 0
    for a in reversed(coeffs):
        acc = (acc * x + a) % R
    return acc


class Flow:
    """One reference test's world: a context, GPU Params, the requester's RNG and group helpers."""

    def __init__(self, ctx, mode, seed, q, label=b"test"):
        import coconut
        from oracle import coconut_ref as C
        self.co, self.ctx, self.mode = coconut, ctx, mode
        self.grp = C.Groups(mode)
        self.rng = C.Drbg(seed)
        self.params = coconut.params_new(ctx, q, label)
        self.q = q
        self.og = 1 if mode == "G2" else 2        # OtherGroup (verkeys) as cc group id
        self.ob = 97 if mode == "G2" else 192
        self.sb = 192 if mode == "G2" else 97
        self.pts = {"g": self.grp.sig_from_bytes(self.params.g),
                    "g_tilde": self.grp.oth_from_bytes(self.params.g_tilde),
                    "h": [self.grp.sig_from_bytes(h) for h in self.params.h]}

    # ---------------------------------------------------------------- keygen
    def signers_from_shares(self, n, x_shares, y_shares):
        """keygen_from_shares (keygen.rs:17-45): every alpha_i = g~ x_i, beta_ij = g~ y_ij on the GPU."""
        q = self.q
        scal = b"".join(_fr(x_shares[i]) + b"".join(_fr(y_shares[j][i]) for j in range(q)) for i in range(1, n + 1))
        pts = self.co.fixed_base_mul(self.ctx, self.og, self.params.g_tilde, scal)
        ob, signers = self.ob, []
        for i in range(1, n + 1):
            row = pts[(i - 1) * (q + 1) * ob:i * (q + 1) * ob]
            vk = self.co.Verkey(row[:ob], [row[(j + 1) * ob:(j + 2) * ob] for j in range(q)])
            signers.append({"id": i, "x": x_shares[i], "y": [y_shares[j][i] for j in range(q)], "vk": vk})
        return signers

    def sss_keygen(self, t, n):
        """trusted_party_SSS_keygen (keygen.rs:53-71): Shamir over Fr on the host, keys on the GPU."""
        def shared():
            c = [self.rng.fr() for _ in range(t)]
            return c[0], {i: _poly(c, i) for i in range(1, n + 1)}
        sx, xs = shared()
        sy, ys = zip(*[shared() for _ in range(self.q)])
        return sx, list(sy), self.signers_from_shares(n, xs, ys)

    def pvss_keygen(self, t, n):
        """trusted_party_PVSS_keygen (keygen.rs:74-122) with PedersenVSS::gens("testPVSS") hashed on the
        GPU; the dealer's commitments C_k = g f_k + h f'_k on the host (the dealer's side); every share of
        every dealing checked by verify_share on the GPU (the reference's keygen.rs:334-349 assertion)."""
        from oracle import bls12_381 as B
        from oracle import keygen as K
        gb, hb = self.co.hash_to_curve(self.ctx, 1, [b"testPVSS : g", b"testPVSS : h"])
        g, h = B.g1_from_bytes(gb), B.g1_from_bytes(hb)
        secrets, share_maps, comms = [], [], []
        for _ in range(1 + self.q):
            sec, _sec_t, comm, shares = K.pedersen_deal(t, n, g, h, self.rng)
            secrets.append(sec)
            share_maps.append(shares)
            comms.append([B.g1_to_bytes(c) for c in comm])
        set_of = [d for d in range(1 + self.q) for _ in range(n)]
        ids = [i for _ in range(1 + self.q) for i in range(1, n + 1)]
        shares = [(_fr(share_maps[d][i][0]), _fr(share_maps[d][i][1])) for d, i in zip(set_of, ids)]
        assert self.co.vss_verify_batch(self.ctx, t, gb, hb, comms, set_of, ids, shares).all()
        bad = list(shares)
        bad[3] = (_fr(share_maps[set_of[3]][ids[3]][0] + 1), bad[3][1])
        v = self.co.vss_verify_batch(self.ctx, t, gb, hb, comms, set_of, ids, bad)
        assert v[3] == 0 and v.sum() == len(ids) - 1
        xs = {i: share_maps[0][i][0] for i in range(1, n + 1)}
        ys = [{i: share_maps[1 + j][i][0] for i in range(1, n + 1)} for j in range(self.q)]
        return secrets[0], secrets[1:], self.signers_from_shares(n, xs, ys)

    # ---------------------------------------------------------------- issuance
    def blind_signatures(self, msgs, k, signers):
        """SignatureRequest::new + SignatureRequestPoK (requester, host) -> per signer:
        SignatureRequestProof::verify and BlindSignature::new on the GPU -> unblind (requester, host).
        Returns the unblinded signatures."""
        from oracle import issuance as I
        grp, P = self.grp, self.pts
        sk, pk = I.elgamal_keygen(grp, P, self.rng)
        req, rnd = I.signature_request_new(grp, msgs, k, pk, P, self.rng)
        pok = I.sigreq_pok_init(grp, req, pk, P, self.rng)
        se = grp.sig_to_bytes
        pok_bytes = se(pok["sk"]["T"]) + se(pok["comm"]["T"]) + b"".join(se(a["T"]) + se(b["T"]) for a, b in pok["cts"])
        chal = int.from_bytes(self.co.hash_msg(self.ctx, [pok_bytes])[0], "big")  # from_msg_hash(pok.to_bytes())
        proof = I.sigreq_gen_proof(pok, msgs[:k], rnd, sk, chal)
        pb = se(proof["sk"]["T"]) + _fr(proof["sk"]["responses"][0]) + se(proof["comm"]["T"])
        pb += b"".join(_fr(v) for v in proof["comm"]["responses"])
        for p1, p2 in proof["cts"]:
            pb += se(p1["T"]) + _fr(p1["responses"][0]) + se(p2["T"]) + _fr(p2["responses"][0]) + _fr(p2["responses"][1])
        cm = se(req["commitment"])
        known = [_fr(m) for m in req["known"]]
        cts = [(se(a), se(b)) for a, b in req["ciphertexts"]]
        # every signer checks the request proof before signing (signature.rs:614-618): one batch of t
        t = len(signers)
        v = self.co.sigreq_verify_batch(self.ctx, self.q, k, self.params.g, self.params.h, [cm] * t, [known] * t,
                                        [cts] * t, [se(pk)] * t, [pb] * t, [_fr(chal)] * t)
        assert v.all()
        wrong = self.co.sigreq_verify_batch(self.ctx, self.q, k, self.params.g, self.params.h, [cm], [known], [cts],
                                            [se(pk)], [pb], [_fr(chal + 1)])
        assert not wrong.any()
        sigs = []
        for s in signers:
            hs, c1s, c2s = self.co.blind_sign_batch(self.ctx, self.q, k, [cm], [known], [cts], _fr(s["x"]),
                                                    [_fr(y) for y in s["y"]])
            h_pt, c1, c2 = (grp.sig_from_bytes(v[0]) for v in (hs, c1s, c2s))
            _, s2 = I.unblind(grp, (h_pt, c1, c2), sk)
            sigs.append(self.co.Signature(hs[0], se(s2)))
        return sigs

    def verify_each(self, sigs, msgs, signers):
        """Per-signer Signature::verify (signature.rs:623): one call per signer through the single-
        credential API, and the same t credentials as ONE batch with per-credential verkeys."""
        mb = [_fr(m) for m in msgs]
        for sig, s in zip(sigs, signers):
            assert sig.verify(mb, s["vk"], self.params, ctx=self.ctx)
        n = len(sigs)
        X = b"".join(s["vk"].X_tilde for s in signers)
        Y = b"".join(y for s in signers for y in s["vk"].Y_tilde)
        self.ctx.set_params(self.params.g_tilde)
        v = self.co.verify_batch(self.ctx, n, self.q, b"".join(s.sigma_1 for s in sigs),
                                 b"".join(s.sigma_2 for s in sigs), b"".join(mb) * n, vk=(X, Y))
        assert v.all()

    def verify_aggregate(self, sig, msgs, vk, expect=True):
        """Aggregate Signature::verify (signature.rs:637) through the single-credential API and through
        the shared-verkey batch path; a changed message is rejected."""
        mb = [_fr(m) for m in msgs]
        assert sig.verify(mb, vk, self.params, ctx=self.ctx) == expect
        self.ctx.set_params(self.params.g_tilde)
        self.ctx.set_verkey(vk.X_tilde, vk.Y_tilde)
        v = self.co.verify_batch(self.ctx, 2, self.q, sig.sigma_1 * 2, sig.sigma_2 * 2,
                                 b"".join(mb) + b"".join(mb[:-1]) + _fr(msgs[-1] + 1))
        assert list(v) == [int(expect), 0]


def check_signing_on_random_msgs(f, t, q, hidden, signers):
    """signature.rs:582-638."""
    msgs = [f.rng.fr() for _ in range(q)]
    sigs = f.blind_signatures(msgs, hidden, signers[:t])
    f.verify_each(sigs, msgs, signers[:t])
    aggr_sig = f.co.Signature.aggregate(t, [(s["id"], sig) for s, sig in zip(signers, sigs)], ctx=f.ctx)
    aggr_vk = f.co.Verkey.aggregate(t, [(s["id"], s["vk"]) for s in signers], ctx=f.ctx)
    f.verify_aggregate(aggr_sig, msgs, aggr_vk)
    return msgs, aggr_sig, aggr_vk


def check_key_aggregation(f, t, secret_x, secret_y, keys):
    """signature.rs:537-580: Verkey::aggregate of t signers' keys equals g~ * secret, element for element
    (byte-equal encodings), through the caller-supplied-verkey MSM and through resident issuer tables."""
    co = f.co
    aggr = co.Verkey.aggregate(t, keys, ctx=f.ctx)
    want = co.fixed_base_mul(f.ctx, f.og, f.params.g_tilde, b"".join(_fr(v) for v in [secret_x] + list(secret_y)))
    ob = f.ob
    assert aggr.X_tilde == want[:ob]
    for j in range(f.q):
        assert aggr.Y_tilde[j] == want[(j + 1) * ob:(j + 2) * ob], j
    ids = [i for i, _ in keys]
    f.ctx.set_issuers(ids, b"".join(vk.X_tilde for _, vk in keys),
                      b"".join(y for _, vk in keys for y in vk.Y_tilde), f.q)
    oX, oY = co.verkey_aggregate_ids(f.ctx, 1, len(ids), t, np.array([ids], np.uint64))
    assert oX == want[:ob] and oY == want[ob:]


@pytest.mark.parametrize("mode", ["G2", "G1"])
@pytest.mark.parametrize("keygen", ["sss", "pvss"])
def test_verkey_aggregation(ctxs, mode, keygen):
    """test_verkey_aggregation_{shamir,verifiable}_secret_sharing_keygen (signature.rs:640-666) and the
    gaps-in-ids variants (:710-759): t = 3 of 5, msg_count = 7; ids {1, 2, 3} and {1, 3, 5}."""
    f = Flow(ctxs[mode], mode, seed=501 + (keygen == "pvss"), q=7)
    sx, sy, signers = (f.sss_keygen if keygen == "sss" else f.pvss_keygen)(3, 5)
    check_key_aggregation(f, 3, sx, sy, [(s["id"], s["vk"]) for s in signers[:3]])
    check_key_aggregation(f, 3, sx, sy, [(signers[k]["id"], signers[k]["vk"]) for k in (0, 2, 4)])


@pytest.mark.parametrize("mode", ["G2", "G1"])
@pytest.mark.parametrize("keygen", ["sss", "pvss"])
def test_sign_verify(ctxs, mode, keygen):
    """test_sign_verify_{shamir,verifiable}_secret_sharing_keygen (signature.rs:668-708): t = 3 of 5,
    msg_count = 6, 2 hidden messages -> check_signing_on_random_msgs."""
    f = Flow(ctxs[mode], mode, seed=601 + (keygen == "pvss"), q=6)
    _, _, signers = (f.sss_keygen if keygen == "sss" else f.pvss_keygen)(3, 5)
    check_signing_on_random_msgs(f, 3, 6, 2, signers)


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_sign_verify_1(ctxs, mode):
    """signature.rs:761-822: t = 3 of 6; the signature is requested from signers {1, 3, 5} and verified
    under the verkey aggregated from the different threshold group {2, 4, 6}."""
    f = Flow(ctxs[mode], mode, seed=701, q=6)
    _, _, signers = f.sss_keygen(3, 6)
    msgs = [f.rng.fr() for _ in range(6)]
    group = [signers[i - 1] for i in (1, 3, 5)]
    sigs = f.blind_signatures(msgs, 2, group)
    f.verify_each(sigs, msgs, group)
    aggr_sig = f.co.Signature.aggregate(3, [(s["id"], sig) for s, sig in zip(group, sigs)], ctx=f.ctx)
    aggr_vk = f.co.Verkey.aggregate(3, [(signers[k]["id"], signers[k]["vk"]) for k in (1, 3, 5)], ctx=f.ctx)
    f.verify_aggregate(aggr_sig, msgs, aggr_vk)
    # a threshold group that overlaps with neither and holds only 2 keys cannot stand in for 3
    short = f.co.Verkey.aggregate(2, [(signers[k]["id"], signers[k]["vk"]) for k in (1, 3)], ctx=f.ctx)
    f.verify_aggregate(aggr_sig, msgs, short, expect=False)


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_PoK_sig(ctxs, mode):
    """pok_sig.rs:17-106: issuance and aggregation as check_signing_on_random_msgs (t = 3 of 5, q = 6,
    2 hidden), then PoKOfSignature over the aggregate with messages {3, 5} revealed; the proof verifies
    under the aggregated verkey with the GPU's challenge, and not with a changed revealed message."""
    from oracle import coconut_ref as C
    f = Flow(ctxs[mode], mode, seed=801, q=6)
    _, _, signers = f.sss_keygen(3, 5)
    msgs, aggr_sig, aggr_vk = check_signing_on_random_msgs(f, 3, 6, 2, signers)
    grp = f.grp
    sig = (grp.sig_from_bytes(aggr_sig.sigma_1), grp.sig_from_bytes(aggr_sig.sigma_2))
    vk = (grp.oth_from_bytes(aggr_vk.X_tilde), [grp.oth_from_bytes(y) for y in aggr_vk.Y_tilde])
    revealed = {3, 5}
    pok = C.pok_init(grp, sig, vk, f.pts["g_tilde"], msgs, revealed, f.rng)
    chal = int.from_bytes(f.co.hash_msg(f.ctx, [C.pok_to_bytes(grp, pok)])[0], "big")
    proof = C.pok_gen_proof(pok, chal)
    P = f.co.PoKOfSignatureProof(grp.sig_to_bytes(proof["sig"][0]), grp.sig_to_bytes(proof["sig"][1]),
                                 grp.oth_to_bytes(proof["J"]), grp.oth_to_bytes(proof["T"]),
                                 [_fr(r) for r in proof["responses"]])
    rev = {i: msgs[i] for i in revealed}
    assert P.verify(aggr_vk, f.params, rev, chal, ctx=f.ctx)
    rev[5] += 1
    assert not P.verify(aggr_vk, f.params, rev, chal, ctx=f.ctx)
