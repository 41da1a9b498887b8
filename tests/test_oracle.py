"""CPU tests of the oracle (test infrastructure): the Python restatement against the algebraic
identities the reference's own tests assert, and the C restatement against the golden fixtures
(an independent representation: 64-bit limbs, Fp6 tower).  See DESIGN.md §Oracle for what is
pinned by the reference and what is "parity unpinned"."""
import ctypes

import pytest

from conftest import golden
from oracle import bls12_381 as B
from oracle import coconut_ref as C


def test_hard_part_chain_is_3_phi_over_r():
    x = -B.X_ABS
    assert (x - 1) ** 2 * (x + B.P) * (x * x + B.P * B.P - 1) + 3 == 3 * B.PHI12 // B.R


def test_conj_is_p6_frobenius():
    assert B.f2_pow(B.XI, (B.P ** 6 - 1) // 6) == (B.P - 1, 0)
    f = [(k + 3, 2 * k + 1) for k in range(6)]
    g = f
    for _ in range(6):
        g = B.f12_frob(g)
    assert B.f12_eq(g, B.f12_conj(f))


def test_generators_and_orders():
    assert B.G1.on_curve(B.G1.gen) and B.G2.on_curve(B.G2.gen)
    assert B.G1.mul_any(B.G1.gen, B.R) is None
    assert B.G2.mul_any(B.G2.gen, B.R) is None


def test_pairing_bilinear_and_order_r():
    e = B.pairing(B.G1.gen, B.G2.gen)
    assert not B.f12_is_one(e)
    assert B.f12_is_one(B.f12_pow(e, B.R))
    e2 = B.pairing(B.G1.mul(B.G1.gen, 6), B.G2.mul(B.G2.gen, 5))
    assert B.f12_eq(e2, B.f12_pow(e, 30))


def test_pairing_kat_fixture_consistent():
    kat = golden("pairing_kat.json")["pairings"]
    for k in kat[:2]:
        P = B.g1_from_bytes(bytes.fromhex(k["P"]))
        Q = B.g2_from_bytes(bytes.fromhex(k["Q"]))
        assert B.gt_to_bytes(B.pairing(P, Q)).hex() == k["gt"]
        assert k["gt"] == k["miller_fexp_check"]


def test_gt_codec_roundtrip():
    e = B.pairing(B.G1.gen, B.G2.gen)
    assert B.f12_eq(B.gt_from_bytes(B.gt_to_bytes(e)), e)


def test_codec_identity_and_offcurve():
    assert B.g1_from_bytes(B.g1_to_bytes(None)) is None
    assert B.g2_from_bytes(B.g2_to_bytes(None)) is None
    b = bytearray(B.g1_to_bytes(B.G1.gen))
    b[-1] ^= 1
    assert B.g1_from_bytes(bytes(b)) is None
    b = bytearray(B.g1_to_bytes(B.G1.gen))
    b[0] = 0x02
    assert B.g1_from_bytes(bytes(b)) is None


def test_lagrange_reconstructs_secret():
    rng = C.Drbg(99)
    s, shares = C.get_shared_secret(3, 6, rng)
    for ids in ([1, 2, 3], [1, 3, 5], [2, 4, 6], [6, 5, 4]):
        assert sum(C.lagrange_basis_at_0(set(ids), i) * shares[i] for i in ids) % B.R == s


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_reference_flow_sign_verify_1(mode):
    """Restates reference signature.rs:761-822 (test_sign_verify_1) and the key-aggregation
    checks of 537-580 with seeded randomness: sigma aggregated from signers {1,3,5} verifies under
    the verkey aggregated from {2,4,6}; aggregated verkey == g~ * secret."""
    grp = C.Groups(mode)
    rng = C.Drbg(b"flow" + mode.encode())
    q, t, n = 6, 3, 6
    params = C.params_from_rng(grp, q, rng)
    sx, sy, signers = C.trusted_party_sss_keygen(grp, t, n, params, rng)
    msgs = [rng.fr() for _ in range(q)]
    h = grp.sig.mul(grp.sig.gen, rng.fr())
    sigs = []
    for i in (1, 3, 5):
        s = C.sign(grp, signers[i - 1]["sk"], msgs, h)
        assert C.verify(grp, s, msgs, signers[i - 1]["vk"], params["g_tilde"])  # signature.rs:808
        sigs.append((i, s))
    asig = C.signature_aggregate(grp, t, sigs)
    avk = C.verkey_aggregate(grp, t, [(i, signers[i - 1]["vk"]) for i in (2, 4, 6)])
    assert avk[0] == grp.other.mul(params["g_tilde"], sx)
    assert C.verify(grp, asig, msgs, avk, params["g_tilde"])  # signature.rs:821


def _verify_fixture_c(oc, name):
    d = golden(name)
    mode = 0 if d["mode"] == "G2" else 1
    q = d["q"]
    cr = d["creds"]
    n = len(cr)
    s1 = b"".join(bytes.fromhex(c["sigma1"]) for c in cr)
    s2 = b"".join(bytes.fromhex(c["sigma2"]) for c in cr)
    msgs = b"".join(bytes.fromhex(m) for c in cr for m in c["msgs"])
    if "vk" in d:
        X = bytes.fromhex(d["vk"]["X"])
        Y = b"".join(bytes.fromhex(y) for y in d["vk"]["Y"])
        per = 0
    else:
        X = b"".join(bytes.fromhex(c["vk"]["X"]) for c in cr)
        Y = b"".join(bytes.fromhex(y) for c in cr for y in c["vk"]["Y"])
        per = 1
    ver = ctypes.create_string_buffer(n)
    gts = ctypes.create_string_buffer(576 * n)
    oc.oc_verify_batch(mode, ctypes.c_size_t(n), ctypes.c_size_t(q), s1, s2, msgs, X, Y, per,
                       bytes.fromhex(d["g_tilde"]), ver, gts, 4)
    return d, ver.raw, gts.raw


@pytest.mark.parametrize("name", ["verify_g2_q6.json", "verify_g1_q6.json", "verify_g2_q16_pervk.json",
                                  "verify_g2_q6_pervk.json", "verify_g1_q6_pervk.json",
                                  "verify_g1_q16_pervk.json", "verify_g2_q16.json", "verify_g1_q16.json"])
def test_c_oracle_matches_golden_verify(oc, name):
    d, ver, gts = _verify_fixture_c(oc, name)
    for i, c in enumerate(d["creds"]):
        assert ver[i] == c["verdict"], (i, c["kind"])
        assert gts[576 * i:576 * (i + 1)].hex() == c["gt"], (i, c["kind"])
    kinds = {c["kind"] for c in d["creds"]}
    assert "valid" in kinds and len(kinds) >= 3


def test_c_oracle_pairing_kat(oc):
    for k in golden("pairing_kat.json")["pairings"]:
        out = ctypes.create_string_buffer(576)
        oc.oc_pairing(bytes.fromhex(k["P"]), bytes.fromhex(k["Q"]), out)
        assert out.raw.hex() == k["gt"]


@pytest.mark.parametrize("name", ["aggregate_g2.json", "aggregate_g1.json", "aggregate_g2_t67.json",
                                  "aggregate_g2_t67_subsets.json", "aggregate_g1_t67_subsets.json"])
def test_c_oracle_matches_golden_aggregate(oc, name):
    d = golden(name)
    mode = 0 if d["mode"] == "G2" else 1
    t, q = d["threshold"], d["q"]
    sb, ob = (192, 97) if mode == 0 else (97, 192)
    for case in d["cases"]:
        ids = case["ids"]
        L = len(ids)
        idarr = (ctypes.c_uint64 * L)(*ids)
        s1 = b"".join(bytes.fromhex(x) for x in case["sigma1"])
        s2 = b"".join(bytes.fromhex(x) for x in case["sigma2"])
        o1 = ctypes.create_string_buffer(sb)
        o2 = ctypes.create_string_buffer(sb)
        assert oc.oc_signature_aggregate(mode, ctypes.c_size_t(L), ctypes.c_size_t(t), idarr, s1, s2, o1, o2) == 0
        assert o1.raw.hex() == case["out_sigma1"] and o2.raw.hex() == case["out_sigma2"]
        X = b"".join(bytes.fromhex(x) for x in case["X"])
        Y = b"".join(bytes.fromhex(y) for row in case["Y"] for y in row)
        oX = ctypes.create_string_buffer(ob)
        oY = ctypes.create_string_buffer(ob * q)
        assert oc.oc_verkey_aggregate(mode, ctypes.c_size_t(L), ctypes.c_size_t(t), ctypes.c_size_t(q), idarr,
                                      X, Y, oX, oY) == 0
        assert oX.raw.hex() == case["out_X"]
        assert [oY.raw[j * ob:(j + 1) * ob].hex() for j in range(q)] == case["out_Y"]
        if len(set(ids[:t])) == t:
            # reference signature.rs:554-559: aggregated verkey == g~ * secret
            assert case["out_X"] == d["secret_X"] and case["out_Y"] == d["secret_Y"]
            assert case["verifies"] == 1


@pytest.mark.parametrize("name", ["pok_g2_q6.json", "pok_g1_q6.json", "pok_g2_q32.json", "pok_g1_q32.json"])
def test_c_oracle_matches_golden_pok(oc, name):
    d = golden(name)
    mode = 0 if d["mode"] == "G2" else 1
    q = d["q"]
    rev = d["revealed"]
    X = bytes.fromhex(d["vk"]["X"])
    Y = b"".join(bytes.fromhex(y) for y in d["vk"]["Y"])
    g = bytes.fromhex(d["g_tilde"])
    idx = (ctypes.c_uint64 * len(rev))(*rev)
    for p in d["proofs"]:
        resp = b"".join(bytes.fromhex(x) for x in p["responses"])
        gt = ctypes.create_string_buffer(576)
        v = oc.oc_pok_verify(mode, ctypes.c_size_t(q), ctypes.c_size_t(len(rev)), bytes.fromhex(p["sigma1"]),
                             bytes.fromhex(p["sigma2"]), bytes.fromhex(p["J"]), bytes.fromhex(p["T"]), resp,
                             ctypes.c_size_t(len(p["responses"])), bytes.fromhex(p["chal"]), idx,
                             b"".join(bytes.fromhex(m) for m in p["revealed_msgs"]), X, Y, g, gt)
        assert v == p["verdict"], p["kind"]
        if p["gt"] is not None:
            assert gt.raw.hex() == p["gt"], p["kind"]


def test_c_oracle_lagrange(oc):
    ids = [1, 3, 5]
    out = ctypes.create_string_buffer(48 * 3)
    oc.oc_lagrange(ctypes.c_size_t(3), (ctypes.c_uint64 * 3)(*ids), out)
    for k, i in enumerate(ids):
        assert int.from_bytes(out.raw[48 * k:48 * (k + 1)], "big") == C.lagrange_basis_at_0(set(ids), i)


def test_subgroup_fixture_definition_and_endomorphism_tests_agree():
    """tests/golden/subgroup.json: status by the definition [r] P == O equals the endomorphism tests
    (G1 phi(P) == -[x^2] P, G2 psi(Q) == [x] Q) the device runs; off-curve / bad encodings decode to
    the identity (status 0) as AMCL does."""
    from oracle import bls12_381 as B
    from oracle import subgroup as S
    d = golden("subgroup.json")
    for name, curve, dec, endo in (("G1", B.G1, B.g1_from_bytes, S.in_g1_endo),
                                   ("G2", B.G2, B.g2_from_bytes, S.in_g2_endo)):
        for rec in d[name]:
            Pt = dec(bytes.fromhex(rec["point"]))
            if Pt is None:
                assert rec["status"] == 0
                continue
            assert curve.on_curve(Pt)
            assert rec["status"] == (2 if S.in_subgroup_def(curve, Pt) else 1)
            assert endo(Pt) == (rec["status"] == 2)


def test_hash_to_curve_fixture_is_consistent():
    """hash_to_curve.json (parity unpinned: AMCL mapit restated): digests are SHAKE256 (hashlib), every
    point is on its curve and in the order-r subgroup (cofactor cleared), and the oracle reproduces
    every vector."""
    import hashlib
    from oracle import bls12_381 as B
    from oracle import hash_to_curve as H
    from oracle import subgroup as S
    d = golden("hash_to_curve.json")
    for rec in d["messages"][:4]:
        m = bytes.fromhex(rec["msg"])
        assert hashlib.shake_256(m).hexdigest(48) == rec["shake256_48"] == H.hash_msg(m).hex()
        p1 = B.g1_from_bytes(bytes.fromhex(rec["g1"]))
        q2 = B.g2_from_bytes(bytes.fromhex(rec["g2"]))
        assert S.in_g1_endo(p1) and S.in_g2_endo(q2)
        assert B.g1_to_bytes(H.g1_from_msg_hash(m)).hex() == rec["g1"]
        assert B.g2_to_bytes(H.g2_from_msg_hash(m)).hex() == rec["g2"]


def test_issuance_and_keygen_fixtures_are_consistent():
    """Oracle self-consistency on the §8(f) rows 3-4 fixtures: every generated request's proof verdict
    and every VSS share verdict re-derive from the restatements."""
    from oracle import bls12_381 as B
    from oracle import keygen as K
    d = golden("keygen_vss.json")
    g, h = B.g1_from_bytes(bytes.fromhex(d["g"])), B.g1_from_bytes(bytes.fromhex(d["h"]))
    for c in d["checks"][:8]:
        comm = [B.g1_from_bytes(bytes.fromhex(x)) for x in d["commitments"][c["set"]]]
        ok = K.verify_share(d["t"], c["id"], (int(c["s"], 16), int(c["s_t"], 16)), comm, g, h)
        assert ok == bool(c["ok"])
