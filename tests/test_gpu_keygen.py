"""GPU tests of the keygen row of SURVEY.md §8(f) (row 4): the verkey derivation of
keygen_from_shares (reference src/keygen.rs:17-45, alpha_i = g~ x_i) through cc_fixed_base_mul, and
Pedersen VSS share verification (keygen.rs:334-349) through cc_vss_verify_batch, against the oracle."""
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import coconut
    c = coconut.Context(0, coconut.GroupMode.SIG_G2)
    yield c
    c.close()


@pytest.mark.parametrize("group", [1, 2])
def test_keygen_derivation_fixed_base(ctx, group):
    from coconut import fixed_base_mul
    d = golden("keygen_vss.json")
    key = "g1" if group == 1 else "g2"
    rows = d[f"derive_{key}"]
    out = fixed_base_mul(ctx, group, bytes.fromhex(d[f"g_tilde_{key}"]), b"".join(bytes.fromhex(r["x"]) for r in rows))
    eb = 97 if group == 1 else 192
    assert [out[i * eb:(i + 1) * eb].hex() for i in range(len(rows))] == [r["alpha"] for r in rows]


def test_pedersen_vss_verify_share(ctx):
    from coconut import vss_verify_batch
    d = golden("keygen_vss.json")
    ch = d["checks"]
    v = vss_verify_batch(ctx, d["t"], bytes.fromhex(d["g"]), bytes.fromhex(d["h"]),
                         [[bytes.fromhex(c) for c in s] for s in d["commitments"]], [c["set"] for c in ch],
                         [c["id"] for c in ch], [(bytes.fromhex(c["s"]), bytes.fromhex(c["s_t"])) for c in ch])
    assert list(v) == [c["ok"] for c in ch]
    assert 0 < sum(v) < len(ch)
