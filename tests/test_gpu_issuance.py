"""GPU tests of the issuer-side batch against the oracle's fixtures:
BlindSignature::new (src/signature.rs:382-433) byte-for-byte, SignatureRequestProof::verify
(src/signature.rs:324-377) verdicts on valid and corrupted proofs, k = 0 / k = q edge cases, and the
reference's end-to-end property (check_signing_on_random_msgs, signature.rs:582-638): the GPU's
blinded signature, unblinded, verifies under the issuer's verkey."""
import pytest

from conftest import golden
from test_gpu_parity import MODES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    import coconut
    c = {m: coconut.Context(0, coconut.GroupMode(v)) for m, v in MODES.items()}
    yield c
    for x in c.values():
        x.close()


def _b(h):
    return bytes.fromhex(h)


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_blind_sign_and_request_proofs(ctxs, mode):
    from coconut import blind_sign_batch, sigreq_verify_batch
    ctx = ctxs[mode]
    for case in golden(f"issuance_{mode.lower()}.json")["cases"]:
        q, k, rq = case["q"], case["k"], case["requests"]
        cms = [_b(r["commitment"]) for r in rq]
        kn = [[_b(m) for m in r["known"]] for r in rq]
        cts = [[(_b(a), _b(b)) for a, b in r["ciphertexts"]] for r in rq]
        hs, c1s, c2s = blind_sign_batch(ctx, q, k, cms, kn, cts, _b(case["x"]), [_b(v) for v in case["y"]])
        for r, h, c1, c2 in zip(rq, hs, c1s, c2s):
            assert (h.hex(), c1.hex(), c2.hex()) == (r["h"], r["c1"], r["c2"]), (k, r["kind"])
        v = sigreq_verify_batch(ctx, q, k, _b(case["g"]), [_b(x) for x in case["h"]], cms, kn, cts,
                                [_b(r["pk"]) for r in rq], [_b(r["proof"]) for r in rq], [_b(r["chal"]) for r in rq])
        assert list(v) == [r["verdict"] for r in rq], k


def test_unblinded_gpu_signature_verifies(ctxs):
    """unblind(c~) = (h, c~2 - sk c~1) from the GPU's blind signature verifies on the GPU under vk."""
    from oracle import bls12_381 as B
    from coconut import Params, Signature, Verkey, blind_sign_batch
    case = golden("issuance_g2.json")["cases"][0]
    ctx = ctxs["G2"]
    r = case["requests"][0]
    h, c1, c2 = blind_sign_batch(ctx, case["q"], case["k"], [_b(r["commitment"])], [[_b(m) for m in r["known"]]],
                                 [[(_b(a), _b(b)) for a, b in r["ciphertexts"]]], _b(case["x"]), [_b(v) for v in case["y"]])
    sk = int(r["elgamal_sk"], 16)
    P1, P2 = B.g2_from_bytes(c1[0]), B.g2_from_bytes(c2[0])
    s2 = B.g2_to_bytes(B.G2.add(P2, B.G2.neg(B.G2.mul(P1, sk))))
    assert s2.hex() == r["sigma2"]
    vk = Verkey(_b(case["vk"]["X"]), [_b(v) for v in case["vk"]["Y"]])
    sig = Signature(h[0], s2)
    assert sig.verify([_b(m) for m in r["msgs"]], vk, Params(g=b"", g_tilde=_b(case["g_tilde"])), ctx=ctx)


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_compute_h_hashes_canonical_encodings(ctxs, mode):
    """compute_h (signature.rs:197-206) hashes commitment.to_bytes() || known_m.to_bytes(): a known
    message sent as m + r (a 48-byte value >= r) must give the same h, and so the same blind
    signature, as the canonical m."""
    from coconut import blind_sign_batch
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    ctx = ctxs[mode]
    case = next(c for c in golden(f"issuance_{mode.lower()}.json")["cases"] if c["q"] > c["k"])
    q, k, rq = case["q"], case["k"], case["requests"]
    cms = [_b(r["commitment"]) for r in rq]
    kn = [[_b(m) for m in r["known"]] for r in rq]
    kn_big = [[(int.from_bytes(m, "big") + R).to_bytes(48, "big") for m in row] for row in kn]
    cts = [[(_b(a), _b(b)) for a, b in r["ciphertexts"]] for r in rq]
    x, y = _b(case["x"]), [_b(v) for v in case["y"]]
    h0, c10, c20 = blind_sign_batch(ctx, q, k, cms, kn, cts, x, y)
    h1, c11, c21 = blind_sign_batch(ctx, q, k, cms, kn_big, cts, x, y)
    assert [h.hex() for h in h1] == [h.hex() for h in h0] == [r["h"] for r in rq]
    assert [c.hex() for c in c21] == [c.hex() for c in c20]
