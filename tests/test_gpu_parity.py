"""GPU parity tests (run on the MI355X box: pytest -m gpu).  The HIP path, called through the C ABI,
must reproduce the oracle bit-for-bit: verdicts, GT bytes (AMCL order) and aggregated group
elements, on the committed golden fixtures and on generated batches (checked against the C oracle
and against verdicts known by construction)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import golden, host_threads, oracle_lib

pytestmark = pytest.mark.gpu

MODES = {"G2": 0, "G1": 1}


@pytest.fixture(scope="module")
def ctxs():
    import coconut
    c = {m: coconut.Context(0, coconut.GroupMode(v)) for m, v in MODES.items()}
    yield c
    for x in c.values():
        x.close()


def _cat(hexes):
    return b"".join(bytes.fromhex(h) for h in hexes)


@pytest.mark.parametrize("name", ["verify_g2_q6.json", "verify_g1_q6.json"])
def test_verify_shared_vk_golden(ctxs, name):
    from coconut import verify_batch
    d = golden(name)
    ctx = ctxs[d["mode"]]
    cr = d["creds"]
    ctx.set_params(bytes.fromhex(d["g_tilde"]))
    ctx.set_verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
    v, gts = verify_batch(ctx, len(cr), d["q"], _cat(c["sigma1"] for c in cr), _cat(c["sigma2"] for c in cr),
                          _cat(m for c in cr for m in c["msgs"]), want_gt=True)
    for i, c in enumerate(cr):
        assert v[i] == c["verdict"], (i, c["kind"])
        assert gts[576 * i:576 * (i + 1)].hex() == c["gt"], (i, c["kind"])


@pytest.mark.parametrize("name", ["verify_g2_q16_pervk.json", "verify_g1_q16_pervk.json", "verify_g2_q6_pervk.json",
                                  "verify_g1_q6_pervk.json"])
def test_verify_per_credential_vk_golden(ctxs, name):
    from coconut import verify_batch
    d = golden(name)
    ctx = ctxs[d["mode"]]
    cr = d["creds"]
    ctx.set_params(bytes.fromhex(d["g_tilde"]))
    X = _cat(c["vk"]["X"] for c in cr)
    Y = _cat(y for c in cr for y in c["vk"]["Y"])
    v, gts = verify_batch(ctx, len(cr), d["q"], _cat(c["sigma1"] for c in cr), _cat(c["sigma2"] for c in cr),
                          _cat(m for c in cr for m in c["msgs"]), vk=(X, Y), want_gt=True)
    for i, c in enumerate(cr):
        assert v[i] == c["verdict"], (i, c["kind"])
        assert gts[576 * i:576 * (i + 1)].hex() == c["gt"], (i, c["kind"])


@pytest.mark.parametrize("name", ["verify_g2_q6_pervk.json", "verify_g1_q6_pervk.json"])
def test_verify_pervk_device_entry_golden(ctxs, name):
    """cc_verify_batch_pervk_device (HBM-resident batch, one verkey per credential): the q = 6 per-verkey
    fixture — every corruption kind plus the variable-base MSM's edge cases (identity / repeated /
    off-curve bases, scalars 0, r - 1, all digits 8, m + r, a high top nibble) — gives the oracle's
    verdicts and GT bytes; ragged batch sizes 1 and 3 reuse the same scratch."""
    import torch
    from coconut import _lib
    d = golden(name)
    ctx = ctxs[d["mode"]]
    ctx.set_params(bytes.fromhex(d["g_tilde"]))
    dev = torch.device("cuda", 0)
    to = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    for sel in (slice(None), slice(0, 1), slice(5, 8)):
        cr = d["creds"][sel]
        n = len(cr)
        D = [to(_cat(c[k] for c in cr)) for k in ("sigma1", "sigma2")]
        D.append(to(_cat(m for c in cr for m in c["msgs"])))
        D.append(to(_cat(c["vk"]["X"] for c in cr)))
        D.append(to(_cat(y for c in cr for y in c["vk"]["Y"])))
        v = torch.zeros(n, dtype=torch.uint8, device=dev)
        gt = torch.zeros(n * 576, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        assert _lib.lib.cc_verify_batch_pervk_device(ctx.h, n, d["q"], *[P(x) for x in D], P(v), P(gt), None) == 0
        torch.cuda.synchronize()
        v, gt = v.cpu().numpy(), bytes(gt.cpu().numpy())
        for i, c in enumerate(cr):
            assert v[i] == c["verdict"], (i, c["kind"])
            assert gt[576 * i:576 * (i + 1)].hex() == c["gt"], (i, c["kind"])


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_pervk_full_size_65536_distinct_verkeys(ctxs, mode):
    """Config 2's size with a DISTINCT verkey per credential (65,536 credentials, q = 6): verdicts equal
    construction through cc_verify_batch_pervk_device; a 128-credential sample's GT bytes equal the C
    oracle's (per-credential verkeys)."""
    import torch
    from coconut import _lib
    m = MODES[mode]
    n, q = 65536, 6
    ctx = ctxs[mode]
    from bench_modes import make_pervk_batch
    b = make_pervk_batch(ctx, m, n, q, seed=777 + m)
    ctx.set_params(b["g_tilde"])
    dev = torch.device("cuda", 0)
    to = lambda x: torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev)  # noqa: E731
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    D = [to(b[k]) for k in ("s1", "s2", "msgs", "X", "Y")]
    v = torch.zeros(n, dtype=torch.uint8, device=dev)
    k0, k = 40000, 128
    gt = torch.zeros(n * 576, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    assert _lib.lib.cc_verify_batch_pervk_device(ctx.h, n, q, *[P(x) for x in D], P(v), P(gt), None) == 0
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), b["expect"])
    sb, ob = (192, 97) if m == 0 else (97, 192)
    oc = oracle_lib()
    ver = ctypes.create_string_buffer(k)
    gts = ctypes.create_string_buffer(576 * k)
    oc.oc_verify_batch(m, ctypes.c_size_t(k), ctypes.c_size_t(q), b["s1"][k0 * sb:(k0 + k) * sb],
                       b["s2"][k0 * sb:(k0 + k) * sb], b["msgs"][k0 * q * 48:(k0 + k) * q * 48],
                       b["X"][k0 * ob:(k0 + k) * ob], b["Y"][k0 * q * ob:(k0 + k) * q * ob], 1, b["g_tilde"], ver, gts,
                       host_threads())
    assert np.array_equal(np.frombuffer(ver.raw, np.uint8), b["expect"][k0:k0 + k])
    assert bytes(gt[k0 * 576:(k0 + k) * 576].cpu().numpy()) == gts.raw


def test_single_signature_verify_api(ctxs):
    """The reference's per-call API (signature.rs:473) through a batch of one."""
    from coconut import Params, Signature, Verkey
    d = golden("verify_g2_q6.json")
    ctx = ctxs["G2"]
    vk = Verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
    params = Params(g=b"", g_tilde=bytes.fromhex(d["g_tilde"]))
    for c in d["creds"][:4]:
        sig = Signature(bytes.fromhex(c["sigma1"]), bytes.fromhex(c["sigma2"]))
        assert sig.verify([bytes.fromhex(m) for m in c["msgs"]], vk, params, ctx=ctx) == bool(c["verdict"])


def test_verify_length_mismatch_is_an_error(ctxs):
    from coconut import CoconutError, verify_batch
    d = golden("verify_g2_q6.json")
    ctx = ctxs["G2"]
    ctx.set_params(bytes.fromhex(d["g_tilde"]))
    ctx.set_verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
    c = d["creds"][0]
    with pytest.raises(CoconutError) as e:
        verify_batch(ctx, 1, 5, bytes.fromhex(c["sigma1"]), bytes.fromhex(c["sigma2"]), _cat(c["msgs"][:5]))
    assert e.value.code == -1


@pytest.mark.parametrize("name", ["aggregate_g2.json", "aggregate_g1.json", "aggregate_g2_t67.json",
                                  "aggregate_g2_t67_subsets.json", "aggregate_g1_t67_subsets.json"])
def test_aggregate_golden(ctxs, name):
    from coconut import signature_aggregate_batch, verkey_aggregate_batch
    d = golden(name)
    ctx = ctxs[d["mode"]]
    t, q = d["threshold"], d["q"]
    ob = ctx.mode.other_bytes
    for case in d["cases"]:
        ids = case["ids"]
        L = len(ids)
        o1, o2 = signature_aggregate_batch(ctx, 1, L, t, [ids], _cat(case["sigma1"]), _cat(case["sigma2"]))
        assert o1.hex() == case["out_sigma1"] and o2.hex() == case["out_sigma2"], ids
        oX, oY = verkey_aggregate_batch(ctx, 1, L, t, q, [ids], _cat(case["X"]),
                                        _cat(y for row in case["Y"] for y in row))
        assert oX.hex() == case["out_X"], ids
        assert [oY[j * ob:(j + 1) * ob].hex() for j in range(q)] == case["out_Y"], ids


def test_aggregate_api_and_threshold_error(ctxs):
    from coconut import CoconutError, Signature, Verkey
    d = golden("aggregate_g2.json")
    ctx = ctxs["G2"]
    case = d["cases"][1]
    sigs = [(i, Signature(bytes.fromhex(a), bytes.fromhex(b)))
            for i, a, b in zip(case["ids"], case["sigma1"], case["sigma2"])]
    s = Signature.aggregate(d["threshold"], sigs, ctx=ctx)
    assert s.sigma_2.hex() == case["out_sigma2"]
    keys = [(i, Verkey(bytes.fromhex(x), [bytes.fromhex(y) for y in ys]))
            for i, x, ys in zip(case["ids"], case["X"], case["Y"])]
    vk = Verkey.aggregate(d["threshold"], keys, ctx=ctx)
    assert vk.X_tilde.hex() == d["secret_X"]
    with pytest.raises(CoconutError):
        Signature.aggregate(5, sigs, ctx=ctx)


@pytest.mark.parametrize("name", ["pok_g2_q6.json", "pok_g1_q6.json", "pok_g2_q32.json", "pok_g1_q32.json"])
def test_pok_verify_golden(ctxs, name):
    from coconut import pok_verify_batch
    d = golden(name)
    ctx = ctxs[d["mode"]]
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


def _full_fr(rng, n):
    """n full-size Fr scalars (uniform below 2^254 < r: every 4-bit window, the top ones included,
    carries non-zero digits) from a numpy Generator, as Python ints and as 48-byte big-endian rows."""
    raw = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    raw[:, 0] &= 0x3F
    rows = np.zeros((n, 48), np.uint8)
    rows[:, 16:] = raw
    b = rows.tobytes()
    return [int.from_bytes(b[48 * i:48 * (i + 1)], "big") for i in range(n)], b


def _gen_batch(mode, n, q, seed, bad_every=16):
    """Valid-by-construction credentials (sigma1 = k G, sigma2 = k (x + sum y m) G) generated by the
    C oracle with full-size Fr scalars (x, y_j, every message and k); every `bad_every`-th has sigma2
    off by G.  Returns inputs and expected verdicts."""
    from oracle import coconut_ref as C
    oc = oracle_lib()
    rng = np.random.default_rng(seed)
    R = C.R
    (x, *y), _ = _full_fr(rng, q + 1)
    g_other = 1 if mode == 0 else 2  # OtherGroup generator (G1 for SigG2)
    sig_group = 2 if mode == 0 else 1
    ob, sb = (97, 192) if mode == 0 else (192, 97)
    gk = 123456789
    scal = [x * gk % R] + [yj * gk % R for yj in y] + [gk]  # X = x g~, Y_j = y_j g~ with g~ = gk G
    pts = ctypes.create_string_buffer(ob * (q + 2))
    oc.oc_gen_mul(g_other, ctypes.c_size_t(q + 2), b"".join(s.to_bytes(48, "big") for s in scal), pts)
    X, Y, gtil = pts.raw[:ob], pts.raw[ob:ob * (q + 1)], pts.raw[ob * (q + 1):]
    msgs, mb = _full_fr(rng, n * q)
    ks, _ = _full_fr(rng, n)
    e1, e2, expect = [], [], np.ones(n, dtype=np.uint8)
    for i in range(n):
        k = ks[i] or 1
        s = x
        for j in range(q):
            s += y[j] * msgs[i * q + j]
        e = k * s % R
        if i % bad_every == bad_every - 1:
            e = (e + 1) % R
            expect[i] = 0
        e1.append(k.to_bytes(48, "big"))
        e2.append(e.to_bytes(48, "big"))
    nth = host_threads()
    s1 = ctypes.create_string_buffer(sb * n)
    s2 = ctypes.create_string_buffer(sb * n)
    oc.oc_gen_mul_mt(sig_group, ctypes.c_size_t(n), b"".join(e1), s1, nth)
    oc.oc_gen_mul_mt(sig_group, ctypes.c_size_t(n), b"".join(e2), s2, nth)
    return dict(X=X, Y=Y, g_tilde=gtil, s1=s1.raw, s2=s2.raw, msgs=mb, expect=expect)


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_generated_batch_against_c_oracle(ctxs, mode):
    """4,096 generated credentials: verdicts by construction; GT bytes of a 256-credential sample
    against the C oracle (independent representation)."""
    from coconut import verify_batch
    m = MODES[mode]
    q, n = 6, 4096
    b = _gen_batch(m, n, q, seed=7 + m)
    ctx = ctxs[mode]
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    v, gts = verify_batch(ctx, n, q, b["s1"], b["s2"], b["msgs"], want_gt=True)
    assert np.array_equal(v, b["expect"])
    oc = oracle_lib()
    sb = 192 if m == 0 else 97
    k = 256
    ver = ctypes.create_string_buffer(k)
    ref = ctypes.create_string_buffer(576 * k)
    oc.oc_verify_batch(m, ctypes.c_size_t(k), ctypes.c_size_t(q), b["s1"][:k * sb], b["s2"][:k * sb],
                       b["msgs"][:k * q * 48], b["X"], b["Y"], 0, b["g_tilde"], ver, ref, host_threads())
    assert ref.raw == gts[:576 * k]
    assert np.array_equal(np.frombuffer(ver.raw, np.uint8), v[:k])


@pytest.mark.parametrize("n", [1, 3, 129, 257])
def test_ragged_batch_sizes_pair_lanes(ctxs, n):
    """Batch sizes that leave lane pairs / blocks partly filled (one credential per lane pair, 128
    per block): every verdict and GT byte against the C oracle."""
    from coconut import verify_batch
    q = 6
    b = _gen_batch(0, n, q, seed=100 + n)
    ctx = ctxs["G2"]
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    v, gts = verify_batch(ctx, n, q, b["s1"], b["s2"], b["msgs"], want_gt=True)
    assert np.array_equal(v, b["expect"])
    oc = oracle_lib()
    ver = ctypes.create_string_buffer(n)
    ref = ctypes.create_string_buffer(576 * n)
    oc.oc_verify_batch(0, ctypes.c_size_t(n), ctypes.c_size_t(q), b["s1"], b["s2"], b["msgs"], b["X"], b["Y"], 0,
                       b["g_tilde"], ver, ref, host_threads())
    assert ref.raw == gts
    assert np.array_equal(np.frombuffer(ver.raw, np.uint8), v)


WIDE_MAX, FEXP_WIDE_MAX, PREP_WIDE_MAX = 4096, 2048, 1024  # slots.h kWideMax, kFexpWideMax, kPrepWideMax
WIDE2_MAX_CREDS = 128  # fexp_pl.hip kWide2Max = 256 pairs: k_miller_wide2 (two waves a pair) up to 128 credentials


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_small_batch_wide_miller_path_matches_pair_lane_path(ctxs, mode):
    """Batches of <= 4,096 credentials take the one-wave-per-pair Miller path (capi.cpp kWideMax:
    k_wide_pairs -> k_miller_wide -> k_f12_reduce_wide), those of <= 2,048 also the one-wave-per-
    credential final exponentiation (kFexpWideMax: k_fexp1) and the one-wave prep; larger ones the
    pair-lane loop, the quad-lane fexp and the lane-pair prep; up to 128 credentials (256 pairs,
    fexp_pl.hip kWide2Max) the wide loop runs two waves a pair (k_miller_wide2).  The same credentials (a
    4,104 batch; its first 4,096, 2,049, 2,048, 1,025, 129, 128 and a ragged 37; then single credentials)
    give the same verdicts and GT bytes, with every corruption kind (identity sigmas included) in the
    batch."""
    import bench
    from coconut import verify_batch
    m = MODES[mode]
    q, n = 6, WIDE_MAX + 8
    ctx = ctxs[mode]
    b = bench.make_verify_batch(ctx, m, n, q, seed=4242 + m, bad_every=4)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    sb = 192 if m == 0 else 97
    v_big, gt_big = verify_batch(ctx, n, q, b["s1"], b["s2"], b["msgs"], want_gt=True)
    assert np.array_equal(v_big, b["expect"])
    for k in (WIDE_MAX, FEXP_WIDE_MAX + 1, FEXP_WIDE_MAX, PREP_WIDE_MAX + 1, WIDE2_MAX_CREDS + 1, WIDE2_MAX_CREDS, 37):
        v_w, gt_w = verify_batch(ctx, k, q, b["s1"][:k * sb], b["s2"][:k * sb], b["msgs"][:k * q * 48], want_gt=True)
        assert np.array_equal(v_w, b["expect"][:k]), k
        assert gt_w == gt_big[:576 * k], k
    for i in (0, 3, 7, 11, 15, 19, 23, FEXP_WIDE_MAX - 1, WIDE_MAX - 1, n - 1):  # every corruption kind
        v1, g1 = verify_batch(ctx, 1, q, b["s1"][i * sb:(i + 1) * sb], b["s2"][i * sb:(i + 1) * sb],
                              b["msgs"][i * q * 48:(i + 1) * q * 48], want_gt=True)
        assert v1[0] == b["expect"][i], (i, b["kind"][i])
        assert g1 == gt_big[576 * i:576 * (i + 1)], (i, b["kind"][i])


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_small_batch_pok_paths_agree(ctxs, mode):
    """PoK batches of <= 1,024 proofs take the one-block-per-proof prep (aggregate.hip
    k_prep_pok_wide_*: chal J on one wave, the Schnorr and J' table terms spread over the other), up to
    2,048 the one-wave fexp, up to 4,096 the one-wave Miller loop, larger ones the lane-pair prep and
    Miller loop and the quad fexp: the same proofs (1/4 with a bad response) give the same verdicts and
    GT bytes through every mix (4,102 / 2,049 / 2,048 / one at a time)."""
    import bench_modes
    from coconut import pok_verify_batch
    m = MODES[mode]
    ctx = ctxs[mode]
    n, q = WIDE_MAX + 6, 32
    b = bench_modes.make_pok_batch(ctx, m, n, q=q, seed=777 + m, bad_every=4)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    sb, ob = (192, 97) if m == 0 else (97, 192)
    nr, r = b["nresp"], len(b["revealed"])

    def run(lo, hi):
        return pok_verify_batch(ctx, hi - lo, q, b["revealed"], nr, b["s1"][lo * sb:hi * sb], b["s2"][lo * sb:hi * sb],
                                b["J"][lo * ob:hi * ob], b["T"][lo * ob:hi * ob],
                                b["resp"][lo * nr * 48:hi * nr * 48], b["chal"][lo * 48:hi * 48],
                                b["rev"][lo * r * 48:hi * r * 48], want_gt=True)
    v_big, gt_big = run(0, n)
    assert np.array_equal(v_big, b["expect"])
    for k in (FEXP_WIDE_MAX + 1, FEXP_WIDE_MAX):
        v_w, gt_w = run(0, k)
        assert np.array_equal(v_w, b["expect"][:k]), k
        assert gt_w == gt_big[:576 * k], k
    for i in (0, 3, 4, 7, n - 1):
        v1, g1 = run(i, i + 1)
        assert v1[0] == b["expect"][i], i
        assert g1 == gt_big[576 * i:576 * (i + 1)], i


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_small_batch_pok_degenerate_challenges(ctxs, mode):
    """chal J runs on the one-wave prep as a chain of spread doublings and additions (curve_wide_lz.h):
    challenges 0, 1, r - 1 and one with only top digits, and (SigG2) J = (0, +-2), a point of order 3
    outside G1 that the reference does not reject, whose windowed multiples hit the addition's
    doubling and identity branches.  Verdicts against the C oracle's PoKOfSignatureProof::verify,
    verdicts and GT bytes between the small-batch and the lane-pair paths."""
    import bench_modes
    from coconut import pok_verify_batch
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
    m = MODES[mode]
    ctx = ctxs[mode]
    n, q, k = WIDE_MAX + 6, 32, 7
    b = bench_modes.make_pok_batch(ctx, m, n, q=q, seed=991 + m, bad_every=0)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    sb, ob = (192, 97) if m == 0 else (97, 192)
    nr, r = b["nresp"], len(b["revealed"])
    chal, J = bytearray(b["chal"]), bytearray(b["J"])
    for i, c in enumerate([0, 1, R - 1, (1 << 254) | (0xF << 248)]):
        chal[48 * i:48 * (i + 1)] = c.to_bytes(48, "big")
    if m == 0:
        for i, y in ((4, 2), (5, P - 2)):
            J[ob * i:ob * (i + 1)] = b"\x04" + bytes(48) + y.to_bytes(48, "big")
            chal[48 * i:48 * (i + 1)] = (7 + i).to_bytes(48, "big")
    chal, J = bytes(chal), bytes(J)

    def run(lo, hi):
        return pok_verify_batch(ctx, hi - lo, q, b["revealed"], nr, b["s1"][lo * sb:hi * sb], b["s2"][lo * sb:hi * sb],
                                J[lo * ob:hi * ob], b["T"][lo * ob:hi * ob], b["resp"][lo * nr * 48:hi * nr * 48],
                                chal[lo * 48:hi * 48], b["rev"][lo * r * 48:hi * r * 48], want_gt=True)
    v_w, gt_w = run(0, k)
    v_big, gt_big = run(0, n)
    assert np.array_equal(v_big[:k], v_w)
    assert gt_big[:576 * k] == gt_w
    assert np.array_equal(v_big[k:], b["expect"][k:])
    oc = oracle_lib()
    idx = (ctypes.c_uint64 * r)(*b["revealed"])
    Yb = b["Y"] if isinstance(b["Y"], (bytes, bytearray)) else b"".join(b["Y"])
    for i in range(k):
        gt = ctypes.create_string_buffer(576)
        v = oc.oc_pok_verify(m, ctypes.c_size_t(q), ctypes.c_size_t(r), b["s1"][i * sb:(i + 1) * sb],
                             b["s2"][i * sb:(i + 1) * sb], J[i * ob:(i + 1) * ob], b["T"][i * ob:(i + 1) * ob],
                             b["resp"][i * nr * 48:(i + 1) * nr * 48], ctypes.c_size_t(nr), chal[48 * i:48 * (i + 1)],
                             idx, b["rev"][i * r * 48:(i + 1) * r * 48], b["X"], Yb, b["g_tilde"], gt)
        assert v_w[i] == v, i


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_small_batch_pervk_paths_agree(ctxs, mode):
    """Per-credential-verkey batches of <= 1,024 take the one-wave-per-credential prep (pervk.hip
    k_prep_*_var_wide: one lane group per base, spread point arithmetic), larger ones the lane-pair
    Straus (beyond 2,048 the quad fexp, beyond 4,096 the batch Miller loop): the same credentials (every
    corruption kind of make_pervk_batch) agree in verdicts and GT bytes through every mix."""
    import bench_modes
    from coconut import verify_batch
    m = MODES[mode]
    ctx = ctxs[mode]
    n, q = WIDE_MAX + 6, 6
    b = bench_modes.make_pervk_batch(ctx, m, n, q, seed=888 + m, bad_every=4)
    ctx.set_params(b["g_tilde"])
    sb, ob = (192, 97) if m == 0 else (97, 192)

    def run(lo, hi):
        return verify_batch(ctx, hi - lo, q, b["s1"][lo * sb:hi * sb], b["s2"][lo * sb:hi * sb],
                            b["msgs"][lo * q * 48:hi * q * 48],
                            vk=(b["X"][lo * ob:hi * ob], b["Y"][lo * q * ob:hi * q * ob]), want_gt=True)
    v_big, gt_big = run(0, n)
    assert np.array_equal(v_big, b["expect"])
    for k in (FEXP_WIDE_MAX + 1, FEXP_WIDE_MAX):
        v_w, gt_w = run(0, k)
        assert np.array_equal(v_w, b["expect"][:k]), k
        assert gt_w == gt_big[:576 * k], k
    for i in (0, 3, 7, 11, n - 1):
        v1, g1 = run(i, i + 1)
        assert v1[0] == b["expect"][i], i
        assert g1 == gt_big[576 * i:576 * (i + 1)], i


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_small_batch_pervk_degenerate_bases(ctxs, mode):
    """The one-wave per-credential-verkey prep runs each base's Straus on its own lane group and adds the
    groups' sums in a butterfly of spread additions (curve_wide_lz.h): equal group sums (the doubling
    branch), opposite ones (the identity), an identity base, a zero scalar and all bases equal reach
    the exceptional cases.  Verdicts and GT bytes against the C oracle, on the small-batch path and on
    the lane-pair path (the same credentials inside a batch of > 4,096)."""
    import bench_modes
    from coconut import verify_batch
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    m = MODES[mode]
    ctx = ctxs[mode]
    n, q, k = WIDE_MAX + 6, 6, 6
    b = bench_modes.make_pervk_batch(ctx, m, n, q, seed=4242 + m, bad_every=0)
    ctx.set_params(b["g_tilde"])
    sb, ob = (192, 97) if m == 0 else (97, 192)
    ident = (b"\x04" + bytes(ob - 1)) if m == 0 else bytes(ob)
    Y = bytearray(b["Y"])
    msgs = bytearray(b["msgs"])

    def ybase(i, j):
        return bytes(Y[(i * q + j) * ob:(i * q + j + 1) * ob])

    def set_y(i, j, v):
        Y[(i * q + j) * ob:(i * q + j + 1) * ob] = v

    def msg(i, j):
        return int.from_bytes(msgs[(i * q + j) * 48:(i * q + j + 1) * 48], "big")

    def set_m(i, j, v):
        msgs[(i * q + j) * 48:(i * q + j + 1) * 48] = (v % R).to_bytes(48, "big")
    set_y(0, 1, ybase(0, 0))                  # equal group sums: Y1 = Y0, m1 = m0
    set_m(0, 1, msg(0, 0))
    set_y(1, 1, ybase(1, 0))                  # opposite group sums: m1 = -m0
    set_m(1, 1, R - msg(1, 0))
    set_y(2, 2, ident)                        # an identity base
    set_m(3, 4, 0)                            # a zero scalar
    for j in range(1, q):                     # all bases and scalars equal
        set_y(4, j, ybase(4, 0))
        set_m(4, j, msg(4, 0))
    for j in range(q):                        # every term cancels but X~
        set_y(5, j, ybase(5, 0))
        set_m(5, j, msg(5, 0) if j % 2 == 0 else R - msg(5, 0))
    Y, msgs = bytes(Y), bytes(msgs)

    def run(lo, hi):
        return verify_batch(ctx, hi - lo, q, b["s1"][lo * sb:hi * sb], b["s2"][lo * sb:hi * sb],
                            msgs[lo * q * 48:hi * q * 48], vk=(b["X"][lo * ob:hi * ob], Y[lo * q * ob:hi * q * ob]),
                            want_gt=True)
    v_w, gt_w = run(0, k)
    oc = oracle_lib()
    ver = ctypes.create_string_buffer(k)
    ref = ctypes.create_string_buffer(576 * k)
    oc.oc_verify_batch(m, ctypes.c_size_t(k), ctypes.c_size_t(q), b["s1"][:k * sb], b["s2"][:k * sb],
                       msgs[:k * q * 48], b["X"][:k * ob], Y[:k * q * ob], 1, b["g_tilde"], ver, ref, host_threads())
    assert np.array_equal(v_w, np.frombuffer(ver.raw, np.uint8))
    assert gt_w == ref.raw
    v_big, gt_big = run(0, n)
    assert np.array_equal(v_big[:k], v_w)
    assert gt_big[:576 * k] == gt_w
    assert np.array_equal(v_big[k:], b["expect"][k:])


@pytest.mark.parametrize("mode", ["G2", "G1"])
@pytest.mark.parametrize("which", ["X", "Y2"])
def test_identity_verkey_component_both_paths(ctxs, mode, which):
    """A verkey component that decodes to the identity (an off-curve encoding, as AMCL reads it) is
    skipped by the MSM the same way on the one-wave-per-credential prep (small batches) and the
    lane-pair prep: verdicts and GT bytes of both against the C oracle."""
    from coconut import verify_batch
    m = MODES[mode]
    q, n, k = 6, WIDE_MAX + 6, 40
    b = _gen_batch(m, n, q, seed=55 + m, bad_every=5)
    ob, sb = (97, 192) if m == 0 else (192, 97)
    ident = (b"\x04" + bytes(ob - 1)) if m == 0 else bytes(ob)
    X, Y = b["X"], b["Y"]
    if which == "X":
        X = ident
    else:
        Y = Y[:2 * ob] + ident + Y[3 * ob:]
    ctx = ctxs[mode]
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(X, [Y[j * ob:(j + 1) * ob] for j in range(q)])
    v_big, gt_big = verify_batch(ctx, n, q, b["s1"], b["s2"], b["msgs"], want_gt=True)
    v_w, gt_w = verify_batch(ctx, k, q, b["s1"][:k * sb], b["s2"][:k * sb], b["msgs"][:k * q * 48], want_gt=True)
    oc = oracle_lib()
    ver = ctypes.create_string_buffer(k)
    ref = ctypes.create_string_buffer(576 * k)
    oc.oc_verify_batch(m, ctypes.c_size_t(k), ctypes.c_size_t(q), b["s1"][:k * sb], b["s2"][:k * sb],
                       b["msgs"][:k * q * 48], X, Y, 0, b["g_tilde"], ver, ref, host_threads())
    assert np.array_equal(v_w, np.frombuffer(ver.raw, np.uint8))
    assert gt_w == ref.raw
    assert np.array_equal(v_big[:k], v_w)
    assert gt_big[:576 * k] == gt_w


def test_full_size_batch_config2(ctxs):
    """BASELINE config 2 size (65,536 credentials, q = 6, shared vk): every verdict equals the one
    known by construction (size-independent property; 1/16 corrupted)."""
    from coconut import verify_batch
    q, n = 6, 65536
    b = _gen_batch(0, n, q, seed=2)
    ctx = ctxs["G2"]
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    v = verify_batch(ctx, n, q, b["s1"], b["s2"], b["msgs"])
    assert np.array_equal(v, b["expect"])


@pytest.mark.parametrize("mode,n", [("G2", 65536), ("G1", 4096)])
def test_config2_survey_batch_every_corruption_kind(ctxs, mode, n):
    """bench.py's timed config-2 batch: verkey aggregated 3-of-5 on the GPU, 1/16
    corrupted split evenly over sigma_2 + G, m_j + 1, swapped, sigma_1 = O, sigma_2 = O, wrong vk —
    every verdict equals construction; a slice's GT bytes equal the C oracle's."""
    import bench
    from coconut import verify_batch
    m = MODES[mode]
    ctx = ctxs[mode]
    q = 6
    b = bench.make_verify_batch(ctx, m, n, q, seed=2)
    kinds = {k for k in b["kind"] if k}
    assert kinds == set(bench.CORRUPT_KINDS)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    v = verify_batch(ctx, n, q, b["s1"], b["s2"], b["msgs"])
    assert np.array_equal(v, b["expect"])
    k = 192  # covers every kind twice
    sb = 192 if m == 0 else 97
    vk_, gts = verify_batch(ctx, k, q, b["s1"][:k * sb], b["s2"][:k * sb], b["msgs"][:k * q * 48], want_gt=True)
    oc = oracle_lib()
    ver = ctypes.create_string_buffer(k)
    ref = ctypes.create_string_buffer(576 * k)
    oc.oc_verify_batch(m, ctypes.c_size_t(k), ctypes.c_size_t(q), b["s1"][:k * sb], b["s2"][:k * sb],
                       b["msgs"][:k * q * 48], b["X"], b["Y"], 0, b["g_tilde"], ver, ref, host_threads())
    assert ref.raw == gts
    assert np.array_equal(np.frombuffer(ver.raw, np.uint8), vk_)


# ---------------------------------------------------------------- RLC batch mode
@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_rlc_batch_accepts_valid_and_falls_back_exactly(ctxs, mode):
    """cc_verify_batch(rlc=1): an all-valid batch is accepted by one final exponentiation; a batch
    with corrupted credentials falls back to per-credential verdicts, identical to the reference
    semantics (verdicts known by construction)."""
    from coconut import verify_batch
    m = MODES[mode]
    q, n = 6, 1024
    b = _gen_batch(m, n, q, seed=31 + m, bad_every=n + 1)  # no corrupted credential
    ctx = ctxs[mode]
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    v = verify_batch(ctx, n, q, b["s1"], b["s2"], b["msgs"], rlc=True)
    assert b["expect"].all() and np.array_equal(v, b["expect"])
    b2 = _gen_batch(m, n, q, seed=41 + m, bad_every=97)
    ctx.set_params(b2["g_tilde"])
    ctx.set_verkey(b2["X"], b2["Y"])
    v2 = verify_batch(ctx, n, q, b2["s1"], b2["s2"], b2["msgs"], rlc=True)
    assert not b2["expect"].all() and np.array_equal(v2, b2["expect"])


def test_rlc_golden_fixture_with_identity_and_offcurve(ctxs):
    """The golden fixture mixes valid, corrupted, identity and off-curve credentials: RLC must reject
    the batch as a whole and reproduce every per-credential verdict."""
    from coconut import verify_batch
    for name in ("verify_g2_q6.json", "verify_g1_q6.json"):
        d = golden(name)
        ctx = ctxs[d["mode"]]
        cr = d["creds"]
        ctx.set_params(bytes.fromhex(d["g_tilde"]))
        ctx.set_verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
        v = verify_batch(ctx, len(cr), d["q"], _cat(c["sigma1"] for c in cr), _cat(c["sigma2"] for c in cr),
                         _cat(m for c in cr for m in c["msgs"]), rlc=True)
        assert list(v) == [c["verdict"] for c in cr], name
        valid = [c for c in cr if c["verdict"] == 1]
        v = verify_batch(ctx, len(valid), d["q"], _cat(c["sigma1"] for c in valid),
                         _cat(c["sigma2"] for c in valid), _cat(m for c in valid for m in c["msgs"]), rlc=True)
        assert v.all(), name


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_rlc_partials_gathered_across_shards(ctxs, mode):
    """The multi-GPU form on one device: 4 shards -> 4 partials (independent seeds and base indices)
    -> one finish.  Accepts the valid batch; one corrupted credential in one shard rejects it."""
    import torch
    from coconut.dist import DeviceEngine, shard_bounds
    m = MODES[mode]
    q, n, world = 6, 2048, 4
    b = _gen_batch(m, n, q, seed=51 + m, bad_every=n + 1)
    ctx = ctxs[mode]
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    sb = 192 if m == 0 else 97
    dev = torch.device("cuda", 0)
    s1 = torch.frombuffer(bytearray(b["s1"]), dtype=torch.uint8).to(dev)
    s2 = torch.frombuffer(bytearray(b["s2"]), dtype=torch.uint8).to(dev)
    ms = torch.frombuffer(bytearray(b["msgs"]), dtype=torch.uint8).to(dev)

    def run(s2_dev):
        parts = []
        for r in range(world):
            lo, hi = shard_bounds(n, world, r)
            e = DeviceEngine(ctx, hi - lo, q, s1[lo * sb:hi * sb], s2_dev[lo * sb:hi * sb],
                             ms[lo * q * 48:hi * q * 48], base_index=lo)
            parts.append(e.partial().clone())
        torch.cuda.synchronize()
        return e.finish(torch.stack(parts), world)

    assert run(s2)
    bad = s2.clone()
    i = 3 * n // 4 + 5  # inside shard 3: swap in another credential's sigma_2
    bad[i * sb:(i + 1) * sb] = s2[(i + 1) * sb:(i + 2) * sb]
    assert not run(bad)


@pytest.mark.parametrize("mode", ["G2", "G1"])
def test_concurrent_verify_slots(ctxs, mode):
    """cc_set_concurrency(3): eight cc_verify_batch_device calls on three caller streams with no host
    synchronisation in between (each slot reused, batches of sizes on both sides of every small-batch
    threshold so a slot's buffers grow while the other slots' batches run), an n = 1 call in the middle, then a
    host-buffer call and a set_verkey rebind that must wait for the slots; every verdict equals
    construction.  Then the per-credential-verkey fixture through cc_verify_batch_pervk_device on two
    streams.  The context is returned to one slot."""
    import torch
    from coconut import _lib, verify_batch
    m = MODES[mode]
    q = 6
    ctx = ctxs[mode]
    N = WIDE_MAX + 8
    b = _gen_batch(m, N, q, seed=2024 + m, bad_every=7)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    sb = 192 if m == 0 else 97
    dev = torch.device("cuda", 0)
    to = lambda x: torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev)  # noqa: E731
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    d1, d2, dm = to(b["s1"]), to(b["s2"]), to(b["msgs"])
    ctx.set_concurrency(3)
    try:
        assert ctx.concurrency() == 3
        streams = [torch.cuda.Stream(dev) for _ in range(3)]
        torch.cuda.synchronize()
        # every kernel mix (one-wave Miller / fexp / prep up to their thresholds, the batch kernels past
        # them) on the same slots, their buffers growing across the thresholds
        sizes = [256, N, 1024, FEXP_WIDE_MAX + 1, 1, 768, N, WIDE_MAX]
        outs = []
        for k, n in enumerate(sizes):
            v = torch.zeros(n, dtype=torch.uint8, device=dev)
            st = streams[k % 3]
            st.wait_stream(torch.cuda.current_stream(dev))  # v's zero fill
            assert _lib.lib.cc_verify_batch_device(ctx.h, n, q, P(d1), P(d2), P(dm), P(v), None,
                                                   ctypes.c_void_p(st.cuda_stream)) == 0
            v.record_stream(st)
            outs.append((n, v))
        vh = verify_batch(ctx, N, q, b["s1"], b["s2"], b["msgs"])  # host path: waits for the slots
        assert np.array_equal(vh, b["expect"])
        torch.cuda.synchronize()
        for n, v in outs:
            assert np.array_equal(v.cpu().numpy(), b["expect"][:n]), n
        # a verkey rebind while batches are in flight: the rebuild waits for them, later batches see it
        v0 = torch.zeros(N, dtype=torch.uint8, device=dev)
        assert _lib.lib.cc_verify_batch_device(ctx.h, N, q, P(d1), P(d2), P(dm), P(v0), None,
                                               ctypes.c_void_p(streams[0].cuda_stream)) == 0
        b2 = _gen_batch(m, 512, q, seed=4048 + m, bad_every=5)
        ctx.set_verkey(b2["X"], b2["Y"])
        ctx.set_params(b2["g_tilde"])
        e1, e2, em = to(b2["s1"]), to(b2["s2"]), to(b2["msgs"])
        v1 = torch.zeros(512, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        assert _lib.lib.cc_verify_batch_device(ctx.h, 512, q, P(e1), P(e2), P(em), P(v1), None,
                                               ctypes.c_void_p(streams[1].cuda_stream)) == 0
        torch.cuda.synchronize()
        assert np.array_equal(v0.cpu().numpy(), b["expect"])
        assert np.array_equal(v1.cpu().numpy(), b2["expect"])
        # per-credential verkeys on two streams
        d = golden(f"verify_{mode.lower()}_q6_pervk.json")
        ctx.set_params(bytes.fromhex(d["g_tilde"]))
        cr = d["creds"]
        n = len(cr)
        D = [to(_cat(c[k] for c in cr)) for k in ("sigma1", "sigma2")]
        D.append(to(_cat(mm for c in cr for mm in c["msgs"])))
        D.append(to(_cat(c["vk"]["X"] for c in cr)))
        D.append(to(_cat(y for c in cr for y in c["vk"]["Y"])))
        vs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        torch.cuda.synchronize()
        for k in range(2):
            assert _lib.lib.cc_verify_batch_pervk_device(ctx.h, n, q, *[P(x) for x in D], P(vs[k]), None,
                                                         ctypes.c_void_p(streams[k].cuda_stream)) == 0
        torch.cuda.synchronize()
        for v in vs:
            assert list(v.cpu().numpy()) == [c["verdict"] for c in cr]
    finally:
        ctx.set_concurrency(1)
    assert ctx.concurrency() == 1


@pytest.mark.parametrize("name", ["pok_g2_q32.json", "pok_g1_q6.json"])
def test_concurrent_pok_slots(ctxs, name):
    """cc_pok_verify_batch_device under cc_set_concurrency(2): four calls on two streams (each slot its
    own d J tables and revealed-index buffer), alternating the fixture with a copy whose responses are
    all corrupted, no synchronisation in between; every verdict and GT equals the fixture's."""
    import torch
    from coconut import _lib
    d = golden(name)
    ctx = ctxs[d["mode"]]
    ctx.set_params(bytes.fromhex(d["g_tilde"]))
    ctx.set_verkey(bytes.fromhex(d["vk"]["X"]), [bytes.fromhex(y) for y in d["vk"]["Y"]])
    pr = d["proofs"]
    n, q, r = len(pr), d["q"], len(d["revealed"])
    nresp = len(pr[0]["responses"])
    dev = torch.device("cuda", 0)
    to = lambda x: torch.frombuffer(bytearray(x), dtype=torch.uint8).to(dev)  # noqa: E731
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    resp = _cat(x for p in pr for x in p["responses"])
    bad_resp = bytearray(resp)
    for i in range(n):  # the last response's low byte of every proof
        bad_resp[(i * nresp + nresp) * 48 - 1] ^= 1
    D = {k: to(_cat(p[k] for p in pr)) for k in ("sigma1", "sigma2", "J", "T", "chal")}
    D["rev"] = to(_cat(m for p in pr for m in p["revealed_msgs"]))
    R = [to(resp), to(bytes(bad_resp))]
    ridx = (ctypes.c_uint64 * max(r, 1))(*d["revealed"])
    ctx.set_concurrency(2)
    try:
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        outs = []
        torch.cuda.synchronize()
        for k in range(4):
            v = torch.zeros(n, dtype=torch.uint8, device=dev)
            gt = torch.zeros(n * 576, dtype=torch.uint8, device=dev)
            st = streams[k % 2]
            st.wait_stream(torch.cuda.current_stream(dev))
            assert _lib.lib.cc_pok_verify_batch_device(ctx.h, n, q, r, nresp, P(D["sigma1"]), P(D["sigma2"]), P(D["J"]),
                                                       P(D["T"]), P(R[k % 2]), P(D["chal"]), ridx, P(D["rev"]), P(v),
                                                       P(gt), ctypes.c_void_p(st.cuda_stream)) == 0
            outs.append((k % 2, v, gt))
        torch.cuda.synchronize()
        for bad, v, gt in outs:
            v, gt = v.cpu().numpy(), bytes(gt.cpu().numpy())
            for i, p in enumerate(pr):
                if bad:
                    assert v[i] == 0, (i, p["kind"])
                    continue
                assert v[i] == p["verdict"], (i, p["kind"])
                if p["gt"] is not None:
                    assert gt[576 * i:576 * (i + 1)].hex() == p["gt"], (i, p["kind"])
    finally:
        ctx.set_concurrency(1)
