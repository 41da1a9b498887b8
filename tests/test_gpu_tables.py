"""GPU tests of every table width and size-dependent launch path the library can select, and of the
context state after a failed table build (C ABI cc_set_table_bits / cc_table_bits /
cc_device_error):

* shared-verkey tables at 8 to 22 bits: the golden verify and PoK fixtures (both group modes) give
  the oracle's verdicts and GT bytes with every width;
* the default table budget (4 GiB: config 2's q = 6 gets 18 bits) and the boundary's idempotence: a
  repeated identical cc_set_params / cc_set_verkey returns without rebuilding (< 1 ms), a changed
  width or key rebuilds;
* issuer tables at every width the budget can pick (8, 10, 12, 13, 16): the golden Verkey::aggregate
  cases;
* a verkey too large for wide tables (q = 2,048 in SigG1: 410 GB at 16 bits) falls back to 8 bits and verifies;
  forcing 16 bits there fails and leaves the context WITHOUT a verkey (CC_ERR_STATE afterwards);
* Lagrange with t > 3,968 (ids past the 64 KiB LDS staging, read from global memory): Shamir-shared
  signatures and verkeys aggregate to the master values (signature.rs:554-559 identity);
* an unknown issuer id in the device entry point: identity output and CC_DEVERR_UNKNOWN_ID.
"""
import ctypes
import sys

import numpy as np
import pytest

from conftest import ROOT, golden
from test_gpu_parity import _cat

sys.path.insert(0, ROOT)
pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _ctx(mode):
    import coconut
    return coconut.Context(0, coconut.GroupMode(0 if mode == "G2" else 1))


@pytest.mark.parametrize("bits", [8, 12, 16, 18, 20, 22])
@pytest.mark.parametrize("name", ["verify_g2_q6.json", "verify_g1_q6.json"])
def test_verkey_table_widths_verify_golden(name, bits):
    from coconut import verify_batch
    d = golden(name)
    ctx = _ctx(d["mode"])
    try:
        ctx.set_table_bits(bits, 0)
        ctx.set_params(bytes.fromhex(d["g_tilde"]))
        ctx.set_verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
        assert ctx.table_bits()[0] == bits
        cr = d["creds"]
        v, gts = verify_batch(ctx, len(cr), d["q"], _cat(c["sigma1"] for c in cr), _cat(c["sigma2"] for c in cr),
                              _cat(m for c in cr for m in c["msgs"]), want_gt=True)
        for i, c in enumerate(cr):
            assert v[i] == c["verdict"], (i, c["kind"])
            assert gts[576 * i:576 * (i + 1)].hex() == c["gt"], (i, c["kind"])
        # the RLC form reads the same tables (delta-MSM and fold points)
        vr = verify_batch(ctx, len(cr), d["q"], _cat(c["sigma1"] for c in cr), _cat(c["sigma2"] for c in cr),
                          _cat(m for c in cr for m in c["msgs"]), rlc=True)
        assert [int(x) for x in vr] == [c["verdict"] for c in cr]
    finally:
        ctx.close()


@pytest.mark.parametrize("bits", [8, 16])
@pytest.mark.parametrize("name", ["pok_g2_q6.json", "pok_g1_q6.json"])
def test_verkey_table_widths_pok_golden(name, bits):
    from coconut import pok_verify_batch
    d = golden(name)
    ctx = _ctx(d["mode"])
    try:
        ctx.set_table_bits(bits, 0)
        ctx.set_params(bytes.fromhex(d["g_tilde"]))
        ctx.set_verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
        pr = d["proofs"]
        nresp = len(pr[0]["responses"])
        v, gts = pok_verify_batch(ctx, len(pr), d["q"], d["revealed"], nresp, _cat(p["sigma1"] for p in pr),
                                  _cat(p["sigma2"] for p in pr), _cat(p["J"] for p in pr), _cat(p["T"] for p in pr),
                                  _cat(x for p in pr for x in p["responses"]), _cat(p["chal"] for p in pr),
                                  _cat(m for p in pr for m in p["revealed_msgs"]), want_gt=True)
        for i, p in enumerate(pr):
            assert v[i] == p["verdict"], (i, p["kind"])
            if p["gt"] is not None:
                assert gts[576 * i:576 * (i + 1)].hex() == p["gt"], (i, p["kind"])
    finally:
        ctx.close()


@pytest.mark.parametrize("bits", [8, 10, 12, 13, 16])
@pytest.mark.parametrize("name", ["aggregate_g2_t67_subsets.json", "aggregate_g1_t67_subsets.json"])
def test_issuer_table_widths_golden(name, bits):
    from coconut import verkey_aggregate_ids
    d = golden(name)
    ctx = _ctx(d["mode"])
    try:
        ctx.set_table_bits(0, bits)
        q, t = d["q"], d["threshold"]
        table = {}
        for case in d["cases"]:
            for i, x, ys in zip(case["ids"], case["X"], case["Y"]):
                table[i] = (x, ys)
        ids = sorted(table)
        ctx.set_issuers(ids, _cat(table[i][0] for i in ids), _cat(y for i in ids for y in table[i][1]), q)
        assert ctx.table_bits()[1] == bits
        ob = ctx.mode.other_bytes
        L = max(len(c["ids"]) for c in d["cases"])
        rows = [c["ids"] + [c["ids"][0]] * (L - len(c["ids"])) for c in d["cases"]]
        oX, oY = verkey_aggregate_ids(ctx, len(rows), L, t, rows)
        for r, c in enumerate(d["cases"]):
            assert oX[r * ob:(r + 1) * ob].hex() == c["out_X"]
            assert [oY[(r * q + j) * ob:(r * q + j + 1) * ob].hex() for j in range(q)] == c["out_Y"]
    finally:
        ctx.close()


def _be(v):
    return int(v % R).to_bytes(48, "big")


def _table_gib(mode_other_group, q, bits):
    nwin = (256 + bits - 1) // bits
    entry = 96 if mode_other_group == 1 else 192
    return (q + 2) * nwin * ((1 << bits) - 1) * entry / 2**30


def test_default_table_budget_and_idempotent_boundary():
    """Library default: the widest window whose q + 2 bases fit 4 GiB (q = 6 SigG2: 18 bits, 3.0 GB);
    a repeated identical cc_set_params / cc_set_verkey through the C ABI (no Python cache in the way)
    returns in < 1 ms without rebuilding; a new key or a new forced width rebuilds; verdicts stay the
    oracle's throughout."""
    import time
    from coconut import _lib, verify_batch
    d = golden("verify_g2_q6.json")
    ctx = _ctx("G2")
    try:
        g = bytes.fromhex(d["g_tilde"])
        X = bytes.fromhex(d["vk"]["X"])
        Y = b"".join(bytes.fromhex(y) for y in d["vk"]["Y"])
        q = d["q"]
        L = _lib.lib
        assert L.cc_set_params(ctx.h, g) == 0
        t0 = time.perf_counter()
        assert L.cc_set_verkey(ctx.h, X, Y, q) == 0
        build_ms = (time.perf_counter() - t0) * 1e3
        bits = ctx.table_bits()[0]
        assert bits == 18, bits
        assert _table_gib(1, q, bits) <= 4.0
        times = []
        for _ in range(5):
            t0 = time.perf_counter()
            assert L.cc_set_params(ctx.h, g) == 0
            assert L.cc_set_verkey(ctx.h, X, Y, q) == 0
            times.append((time.perf_counter() - t0) * 1e3)
        assert min(times) < 1.0, (times, build_ms)
        ctx._gtilde, ctx._vk = g, (X, Y)
        cr = d["creds"]
        args = (ctx, len(cr), q, _cat(c["sigma1"] for c in cr), _cat(c["sigma2"] for c in cr),
                _cat(m for c in cr for m in c["msgs"]))
        assert [int(v) for v in verify_batch(*args)] == [c["verdict"] for c in cr]
        # another key (X~ and Y~_0 swapped) rebuilds: the honest credentials now fail
        Ysw = X + Y[97:]
        assert L.cc_set_verkey(ctx.h, Y[:97], Ysw, q) == 0
        assert not any(int(v) for v in verify_batch(*args))
        assert L.cc_set_verkey(ctx.h, X, Y, q) == 0
        # a new forced width rebuilds the same key at that width
        assert L.cc_set_table_bits(ctx.h, 12, 0) == 0
        assert L.cc_set_verkey(ctx.h, X, Y, q) == 0
        assert ctx.table_bits()[0] == 12
        assert [int(v) for v in verify_batch(*args)] == [c["verdict"] for c in cr]
    finally:
        ctx.close()


def test_large_verkey_falls_back_to_8_bits_and_failed_build_leaves_no_verkey():
    """SigG1 (verkey in G2), q = 2,048: 16-bit tables would need 2,050 x 200 MB.  Chosen by memory the
    tables are 8-bit and verify works; forced to 16 bits the build fails, and the context then refuses
    verification (CC_ERR_STATE) instead of reading a half-built table."""
    import coconut
    from coconut import CoconutError, verify_batch
    ctx = _ctx("G1")
    try:
        q = 2048
        rng = np.random.default_rng(46)
        x = int(rng.integers(1, 2**62))
        y = [int(v) for v in rng.integers(1, 2**62, size=q)]
        gk = 987654321
        vk = coconut.fixed_base_mul(ctx, 2, coconut.G2_GENERATOR, b"".join(_be(s * gk) for s in [x] + y + [1]))
        X, Y, g_tilde = vk[:192], vk[192:192 * (q + 1)], vk[192 * (q + 1):]
        ctx.set_params(g_tilde)
        ctx.set_verkey(X, [Y[j * 192:(j + 1) * 192] for j in range(q)])
        assert ctx.table_bits()[0] == 8
        n = 3
        msgs = [[int(v) for v in rng.integers(0, 2**62, size=q)] for _ in range(n)]
        ks = [int(v) for v in rng.integers(1, 2**62, size=n)]
        e2 = [k * (x + sum(a * b for a, b in zip(y, m))) for k, m in zip(ks, msgs)]
        e2[2] += 1  # a bad one
        s1 = coconut.fixed_base_mul(ctx, 1, coconut.G1_GENERATOR, b"".join(_be(k) for k in ks))
        s2 = coconut.fixed_base_mul(ctx, 1, coconut.G1_GENERATOR, b"".join(_be(e) for e in e2))
        mb = b"".join(_be(v) for m in msgs for v in m)
        v = verify_batch(ctx, n, q, s1, s2, mb)
        assert [int(a) for a in v] == [1, 1, 0]
        ctx.set_table_bits(16, 0)
        with pytest.raises(CoconutError):
            ctx.set_verkey(X, [Y[j * 192:(j + 1) * 192] for j in range(q)])
        assert ctx.table_bits()[0] == 0
        with pytest.raises(CoconutError) as e:
            verify_batch(ctx, n, q, s1, s2, mb)
        assert e.value.code == -7  # CC_ERR_STATE
    finally:
        ctx.close()


def test_lagrange_large_threshold_global_ids():
    """t = 4,000 (> 3,968: k_lagrange reads the ids from global memory).  Shares of a degree-2
    polynomial f (exact for any t >= 3 points): sigma_2,i = k f(i) G, X~_i = f(i) g~; both aggregates
    must equal the master values k f(0) G and f(0) g~."""
    import coconut
    from coconut import signature_aggregate_batch, verkey_aggregate_ids
    ctx = _ctx("G2")
    try:
        t = 4000
        a, b, c, k = 1234567, 7654321, 1111111, 424242
        ids = list(range(1, t + 1))
        f = [(a + b * i + c * i * i) % R for i in ids]
        s1one = coconut.fixed_base_mul(ctx, 2, coconut.G2_GENERATOR, _be(k))
        s2 = coconut.fixed_base_mul(ctx, 2, coconut.G2_GENERATOR, b"".join(_be(k * v) for v in f))
        want_s2 = coconut.fixed_base_mul(ctx, 2, coconut.G2_GENERATOR, _be(k * a))
        g1, g2 = signature_aggregate_batch(ctx, 1, t, t, [ids], s1one * t, s2)
        assert g1 == s1one and g2 == want_s2
        Xs = coconut.fixed_base_mul(ctx, 1, coconut.G1_GENERATOR, b"".join(_be(v) for v in f))
        want_X = coconut.fixed_base_mul(ctx, 1, coconut.G1_GENERATOR, _be(a))
        ctx.set_issuers(ids, Xs, b"", 0)
        oX, _ = verkey_aggregate_ids(ctx, 1, t, t, [ids])
        assert oX == want_X
    finally:
        ctx.close()


def test_unknown_issuer_id_device_entry_raises_device_error():
    import torch
    from coconut import _lib
    d = golden("aggregate_g2.json")
    ctx = _ctx("G2")
    try:
        case = d["cases"][0]
        q = d["q"]
        ctx.set_issuers(case["ids"], _cat(case["X"]), _cat(y for row in case["Y"] for y in row), q)
        assert ctx.device_error() == 0
        dev = torch.device("cuda", 0)
        rows = np.array([case["ids"][:3], [case["ids"][0], case["ids"][1], 999999]], dtype=np.uint64)
        d_ids = torch.from_numpy(rows.view(np.int64).copy()).to(dev)
        oX = torch.zeros(2 * 97, dtype=torch.uint8, device=dev)
        oY = torch.zeros(2 * q * 97, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
        assert _lib.lib.cc_verkey_aggregate_ids_device(ctx.h, 2, 3, 3, P(d_ids), P(oX), P(oY), None) == 0
        assert ctx.device_error() == 1  # CC_DEVERR_UNKNOWN_ID
        assert ctx.device_error() == 0  # cleared by the read
        ox = bytes(oX.cpu().numpy())
        assert ox[:97].hex() == case["out_X"]  # the valid row is unaffected
        ident = bytes(ox[97:])
        from coconut import verkey_aggregate_ids
        zX, _ = verkey_aggregate_ids(ctx, 1, 3, 0, [case["ids"][:3]])  # t = 0: the identity encoding
        assert ident == zX
    finally:
        ctx.close()
