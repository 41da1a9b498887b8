"""GPU tests of the codec-side rows of SURVEY.md §8(f): batched amcl_wrapper `from_msg_hash`
(Params::new, src/signature.rs:22-32; SignatureRequest::compute_h, src/signature.rs:197-206) against
the oracle's vectors (parity unpinned: AMCL `mapit` restated), and SHAKE256 against hashlib."""
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


def test_shake256_digests(ctxs):
    from coconut import hash_msg
    d = golden("hash_to_curve.json")["messages"]
    got = hash_msg(ctxs["G2"], [bytes.fromhex(r["msg"]) for r in d])
    assert [g.hex() for g in got] == [r["shake256_48"] for r in d]


@pytest.mark.parametrize("group", [1, 2])
def test_from_msg_hash_vectors(ctxs, group):
    from coconut import hash_to_curve
    d = golden("hash_to_curve.json")["messages"]
    got = hash_to_curve(ctxs["G2"], group, [bytes.fromhex(r["msg"]) for r in d])
    key = "g1" if group == 1 else "g2"
    for g, r in zip(got, d):
        assert g.hex() == r[key], len(r["msg"]) // 2


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_params_new_label_test(ctxs, mode):
    """Params::new(6, "test"): the reference's own test parameters (signature.rs:668-679)."""
    from coconut import params_new
    want = golden("hash_to_curve.json")[f"params_{mode}"]
    p = params_new(ctxs[mode], 6, b"test")
    assert p.g.hex() == want["g"]
    assert p.g_tilde.hex() == want["g_tilde"]
    assert [h.hex() for h in p.h] == want["h"]


def test_hash_to_curve_batch_is_in_subgroup(ctxs):
    """A 4,096-message batch (compute_h-shaped inputs: 192-byte commitment || 48-byte messages): every
    output is in G2 (cofactor cleared) and equal inputs hash equally."""
    from coconut import hash_to_curve, subgroup_check
    msgs = [bytes([i & 0xFF, i >> 8]) * 96 + bytes(48 * (i % 4)) for i in range(4096)]
    out = hash_to_curve(ctxs["G2"], 2, msgs)
    st = subgroup_check(ctxs["G2"], 2, b"".join(out))
    assert (st == 2).all()
    again = hash_to_curve(ctxs["G2"], 2, msgs[:64])
    assert again == out[:64]
