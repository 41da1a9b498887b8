"""GPU tests of BASELINE configs 4 and 5 at their full sizes and of the new entry points:
the issuer-table Verkey::aggregate (cc_set_issuers + cc_verkey_aggregate_ids), the device-buffer
Signature::aggregate and PoK verify, and the windowed Straus MSM (also covered by every
tests/golden/aggregate_*.json case in test_gpu_parity.py)."""
import ctypes
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, golden
from test_gpu_parity import MODES, _cat

sys.path.insert(0, ROOT)
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    import coconut
    c = {m: coconut.Context(0, coconut.GroupMode(v)) for m, v in MODES.items()}
    yield c
    for x in c.values():
        x.close()


@pytest.mark.parametrize("name", ["aggregate_g2_t67_subsets.json", "aggregate_g1_t67_subsets.json",
                                  "aggregate_g2.json", "aggregate_g1.json"])
def test_issuer_table_verkey_aggregate_golden(ctxs, name):
    """Verkey::aggregate from the resident issuer table equals the oracle on every golden case
    (random 67-subsets with gaps, extra entries beyond t, duplicated ids)."""
    from coconut import verkey_aggregate_ids
    d = golden(name)
    ctx = ctxs[d["mode"]]
    q, t = d["q"], d["threshold"]
    table = {}
    for case in d["cases"]:
        for i, x, ys in zip(case["ids"], case["X"], case["Y"]):
            table[i] = (x, ys)
    ids = sorted(table)
    ctx.set_issuers(ids, _cat(table[i][0] for i in ids), _cat(y for i in ids for y in table[i][1]), q)
    ob = ctx.mode.other_bytes
    for case in d["cases"]:
        oX, oY = verkey_aggregate_ids(ctx, 1, len(case["ids"]), t, [case["ids"]])
        assert oX.hex() == case["out_X"], case["ids"][:5]
        assert [oY[j * ob:(j + 1) * ob].hex() for j in range(q)] == case["out_Y"]
    # all cases in ONE batch (ragged lengths padded with valid ids beyond t, which are ignored)
    L = max(len(c["ids"]) for c in d["cases"])
    rows = [c["ids"] + [c["ids"][0]] * (L - len(c["ids"])) for c in d["cases"]]
    oX, oY = verkey_aggregate_ids(ctx, len(rows), L, t, rows)
    assert [oX[i * ob:(i + 1) * ob].hex() for i in range(len(rows))] == [c["out_X"] for c in d["cases"]]


def test_issuer_table_unknown_id_is_an_error(ctxs):
    from coconut import CoconutError, verkey_aggregate_ids
    d = golden("aggregate_g2.json")
    ctx = ctxs["G2"]
    case = d["cases"][0]
    ctx.set_issuers(case["ids"], _cat(case["X"]), _cat(y for row in case["Y"] for y in row), d["q"])
    with pytest.raises(CoconutError):
        verkey_aggregate_ids(ctx, 1, 3, 3, [[1, 2, 99]])


def test_config4_full_size_property(ctxs):
    """10,000 credentials, t = 67 of n = 100 Shamir-shared issuers, random subsets: every aggregated
    verkey equals g~ * master secret and every aggregated sigma_2 equals (x + sum y m) h — the
    reference's check_key_aggregation identity (signature.rs:554-559) at config-4 scale."""
    import torch
    import bench_modes
    from coconut import _lib
    ctx = ctxs["G2"]
    n = 10000
    b = bench_modes.make_aggregate_batch(ctx, 0, n, seed=44)
    ctx.set_issuers(b["iss"], b["X"], b["Y"], b["q"])
    t, q, sb, ob = b["t"], b["q"], b["sb"], b["ob"]
    dev = torch.device("cuda", 0)
    d_ids = torch.from_numpy(b["ids"].view(np.int64).copy()).to(dev)
    d_s1 = torch.frombuffer(bytearray(b["s1"]), dtype=torch.uint8).to(dev)
    d_s2 = torch.frombuffer(bytearray(b["s2"]), dtype=torch.uint8).to(dev)
    o1, o2 = (torch.zeros(n * sb, dtype=torch.uint8, device=dev) for _ in range(2))
    oX = torch.zeros(n * ob, dtype=torch.uint8, device=dev)
    oY = torch.zeros(n * q * ob, dtype=torch.uint8, device=dev)
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    lib = _lib.lib
    assert lib.cc_signature_aggregate_batch_device(ctx.h, n, t, t, P(d_ids), P(d_s1), P(d_s2), P(o1), P(o2), None) == 0
    assert lib.cc_verkey_aggregate_ids_device(ctx.h, n, t, t, P(d_ids), P(oX), P(oY), None) == 0
    torch.cuda.synchronize()  # the calls ran on the context's own stream
    assert bytes(oX.cpu().numpy()) == b["want_X"] * n
    assert bytes(oY.cpu().numpy()) == b["want_Y"] * n
    assert bytes(o2.cpu().numpy()) == b["want_s2"]
    assert bytes(o1.cpu().numpy()) == b["want_s1"]


def test_config4_fused_entry_one_lagrange(ctxs):
    """cc_aggregate_credential_batch_device (one Lagrange launch for both MSMs) equals the two separate
    entry points on 2,000 config-4 credentials, and the golden t = 67 subsets equal the oracle."""
    import torch
    import bench_modes
    from coconut import _lib
    ctx = ctxs["G2"]
    n = 2000
    b = bench_modes.make_aggregate_batch(ctx, 0, n, seed=45)
    ctx.set_issuers(b["iss"], b["X"], b["Y"], b["q"])
    t, q, sb, ob = b["t"], b["q"], b["sb"], b["ob"]
    dev = torch.device("cuda", 0)
    d_ids = torch.from_numpy(b["ids"].view(np.int64).copy()).to(dev)
    d_s1 = torch.frombuffer(bytearray(b["s1"]), dtype=torch.uint8).to(dev)
    d_s2 = torch.frombuffer(bytearray(b["s2"]), dtype=torch.uint8).to(dev)
    o1, o2 = (torch.zeros(n * sb, dtype=torch.uint8, device=dev) for _ in range(2))
    oX = torch.zeros(n * ob, dtype=torch.uint8, device=dev)
    oY = torch.zeros(n * q * ob, dtype=torch.uint8, device=dev)
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    lib = _lib.lib
    assert lib.cc_aggregate_credential_batch_device(ctx.h, n, t, t, P(d_ids), P(d_s1), P(d_s2), P(o1), P(o2),
                                                    P(oX), P(oY), None) == 0
    assert ctx.device_error() == 0
    assert bytes(oX.cpu().numpy()) == b["want_X"] * n
    assert bytes(oY.cpu().numpy()) == b["want_Y"] * n
    assert bytes(o2.cpu().numpy()) == b["want_s2"][:n * sb]
    assert bytes(o1.cpu().numpy()) == b["want_s1"][:n * sb]
    # golden t = 67 random subsets (oracle outputs), both aggregates through the fused entry
    d = golden("aggregate_g2_t67_subsets.json")
    t = d["threshold"]
    table = {}
    for case in d["cases"]:
        for i, x, ys in zip(case["ids"], case["X"], case["Y"]):
            table[i] = (x, ys)
    ids = sorted(table)
    ctx.set_issuers(ids, _cat(table[i][0] for i in ids), _cat(y for i in ids for y in table[i][1]), d["q"])
    for case in d["cases"]:
        L = len(case["ids"])
        g_ids = torch.from_numpy(np.array(case["ids"], dtype=np.uint64).view(np.int64)).to(dev)
        g1 = torch.frombuffer(bytearray(_cat(case["sigma1"])), dtype=torch.uint8).to(dev)
        g2 = torch.frombuffer(bytearray(_cat(case["sigma2"])), dtype=torch.uint8).to(dev)
        r1, r2 = (torch.zeros(sb, dtype=torch.uint8, device=dev) for _ in range(2))
        rX = torch.zeros(ob, dtype=torch.uint8, device=dev)
        rY = torch.zeros(d["q"] * ob, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        assert lib.cc_aggregate_credential_batch_device(ctx.h, 1, L, t, P(g_ids), P(g1), P(g2), P(r1), P(r2),
                                                        P(rX), P(rY), None) == 0
        assert ctx.device_error() == 0
        assert bytes(r2.cpu().numpy()).hex() == case["out_sigma2"]
        assert bytes(r1.cpu().numpy()).hex() == case["out_sigma1"]
        assert bytes(rX.cpu().numpy()).hex() == case["out_X"]
        oy = bytes(rY.cpu().numpy())
        assert [oy[j * ob:(j + 1) * ob].hex() for j in range(d["q"])] == case["out_Y"]


def test_config4_fused_entry_sigg1_and_unknown_id(ctxs):
    """SigG1 (sigma in G1, issuer keys in G2: the pair-lane issuer-table kernel on the side stream, running
    alongside the G1 Straus): the fused entry's four outputs equal construction on 1,000 credentials, and an
    id without an issuer key raises the device error word through the same entry."""
    import torch
    import bench_modes
    from coconut import _lib
    ctx = ctxs["G1"]
    n = 1000
    b = bench_modes.make_aggregate_batch(ctx, 1, n, seed=46)
    ctx.set_issuers(b["iss"], b["X"], b["Y"], b["q"])
    t, q, sb, ob = b["t"], b["q"], b["sb"], b["ob"]
    dev = torch.device("cuda", 0)
    ids = b["ids"].copy()
    d_ids = torch.from_numpy(ids.view(np.int64).copy()).to(dev)
    d_s1 = torch.frombuffer(bytearray(b["s1"]), dtype=torch.uint8).to(dev)
    d_s2 = torch.frombuffer(bytearray(b["s2"]), dtype=torch.uint8).to(dev)
    o1, o2 = (torch.zeros(n * sb, dtype=torch.uint8, device=dev) for _ in range(2))
    oX = torch.zeros(n * ob, dtype=torch.uint8, device=dev)
    oY = torch.zeros(n * q * ob, dtype=torch.uint8, device=dev)
    P = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    lib = _lib.lib
    assert lib.cc_aggregate_credential_batch_device(ctx.h, n, t, t, P(d_ids), P(d_s1), P(d_s2), P(o1), P(o2),
                                                    P(oX), P(oY), None) == 0
    assert ctx.device_error() == 0
    assert bytes(oX.cpu().numpy()) == b["want_X"] * n
    assert bytes(oY.cpu().numpy()) == b["want_Y"] * n
    assert bytes(o2.cpu().numpy()) == b["want_s2"][:n * sb]
    assert bytes(o1.cpu().numpy()) == b["want_s1"][:n * sb]
    bad = ids.copy().reshape(n, -1)
    bad[7, 3] = 10 ** 9  # no issuer holds this id
    d_bad = torch.from_numpy(bad.reshape(-1).view(np.int64).copy()).to(dev)
    torch.cuda.synchronize()
    assert lib.cc_aggregate_credential_batch_device(ctx.h, n, t, t, P(d_bad), P(d_s1), P(d_s2), P(o1), P(o2),
                                                    P(oX), P(oY), None) == 0
    assert ctx.device_error() == 1  # CC_DEVERR_UNKNOWN_ID


def test_config5_full_size_pok_device(ctxs):
    """65,536 PoK proofs (q = 32, 8 revealed) through cc_pok_verify_batch_device: verdicts equal
    construction (1/16 corrupted responses); the host entry point agrees on a slice."""
    import torch
    import bench_modes
    from coconut import _lib, pok_verify_batch
    ctx = ctxs["G2"]
    n = 65536
    b = bench_modes.make_pok_batch(ctx, 0, n, seed=55)
    ctx.set_params(b["g_tilde"])
    ctx.set_verkey(b["X"], b["Y"])
    q, r, nresp = b["q"], len(b["revealed"]), b["nresp"]
    dev = torch.device("cuda", 0)
    D = {k: torch.frombuffer(bytearray(b[k]), dtype=torch.uint8).to(dev) for k in ("s1", "s2", "J", "T", "resp", "chal", "rev")}
    v = torch.zeros(n, dtype=torch.uint8, device=dev)
    P = lambda k: ctypes.c_void_p(D[k].data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    st = _lib.lib.cc_pok_verify_batch_device(ctx.h, n, q, r, nresp, P("s1"), P("s2"), P("J"), P("T"), P("resp"),
                                             P("chal"), (ctypes.c_uint64 * r)(*b["revealed"]), P("rev"),
                                             ctypes.c_void_p(v.data_ptr()), None, None)
    assert st == 0
    torch.cuda.synchronize()
    assert np.array_equal(v.cpu().numpy(), b["expect"])
    k = 64
    vh = pok_verify_batch(ctx, k, q, b["revealed"], nresp, b["s1"][:k * 192], b["s2"][:k * 192], b["J"][:k * 97],
                          b["T"][:k * 97], b["resp"][:k * nresp * 48], b["chal"][:k * 48], b["rev"][:k * r * 48])
    assert np.array_equal(vh, b["expect"][:k])


def test_signature_aggregate_threshold_zero_and_small_order_safe(ctxs):
    """t = 0 aggregates to the identity with sigma_1 from entry 0 (reference: empty MSM)."""
    from coconut import signature_aggregate_batch
    d = golden("aggregate_g2.json")
    ctx = ctxs["G2"]
    case = d["cases"][0]
    o1, o2 = signature_aggregate_batch(ctx, 1, 3, 0, [case["ids"]], _cat(case["sigma1"]), _cat(case["sigma2"]))
    assert o1.hex() == case["sigma1"][0]
    assert o2 == bytes(96) + (1).to_bytes(48, "big") + bytes(48)


@pytest.mark.parametrize("mode_name", ["aggregate_g2_t67_subsets.json", "aggregate_g1_t67_subsets.json"])
@pytest.mark.parametrize("t", [1, 2, 3, 5, 9])
def test_lagrange_batching_ragged_against_oracle(ctxs, oc, mode_name, t):
    """k_lagrange runs 4 (credential, i) tasks per lane with one shared inversion and scans each
    credential for repeated ids once: batches where n * t is not a multiple of 4, lanes straddling
    credentials, and rows with repeated ids (HashSet semantics, reference secret_sharing
    lagrange_basis_at_0) must give the oracle's Signature::aggregate and Verkey::aggregate per row."""
    import random
    from coconut import signature_aggregate_batch, verkey_aggregate_ids
    d = golden(mode_name)
    ctx = ctxs[d["mode"]]
    mode = 0 if d["mode"] == "G2" else 1
    q = d["q"]
    sb, ob = (192, 97) if mode == 0 else (97, 192)
    keys, sigs = {}, {}
    for case in d["cases"]:
        for k, i in enumerate(case["ids"]):
            keys[i] = (case["X"][k], case["Y"][k])
            sigs[i] = (case["sigma1"][k], case["sigma2"][k])
    pool = sorted(set(keys) & set(sigs))
    ctx.set_issuers(pool, _cat(keys[i][0] for i in pool), _cat(y for i in pool for y in keys[i][1]), q)
    rng = random.Random(1000 + t)
    L, n = 9, 13
    rows = []
    for r in range(n):
        row = rng.sample(pool, L)
        if r % 3 == 1 and t > 1:
            row[rng.randrange(1, t)] = row[0]  # a repeated id inside the first t entries
        rows.append(row)
    s1 = _cat(sigs[i][0] for row in rows for i in row)
    s2 = _cat(sigs[i][1] for row in rows for i in row)
    g1, g2 = signature_aggregate_batch(ctx, n, L, t, rows, s1, s2)
    gX, gY = verkey_aggregate_ids(ctx, n, L, t, rows)
    o1, o2 = ctypes.create_string_buffer(sb), ctypes.create_string_buffer(sb)
    oX, oY = ctypes.create_string_buffer(ob), ctypes.create_string_buffer(ob * q)
    for r, row in enumerate(rows):
        idarr = (ctypes.c_uint64 * L)(*row)
        rs1 = _cat(sigs[i][0] for i in row)
        rs2 = _cat(sigs[i][1] for i in row)
        assert oc.oc_signature_aggregate(mode, ctypes.c_size_t(L), ctypes.c_size_t(t), idarr, rs1, rs2, o1, o2) == 0
        assert g1[r * sb:(r + 1) * sb] == o1.raw and g2[r * sb:(r + 1) * sb] == o2.raw, (r, row[:t])
        X = _cat(keys[i][0] for i in row)
        Y = _cat(y for i in row for y in keys[i][1])
        assert oc.oc_verkey_aggregate(mode, ctypes.c_size_t(L), ctypes.c_size_t(t), ctypes.c_size_t(q), idarr,
                                      X, Y, oX, oY) == 0
        assert gX[r * ob:(r + 1) * ob] == oX.raw and gY[r * q * ob:(r + 1) * q * ob] == oY.raw, (r, row[:t])


@pytest.mark.parametrize("t", [1, 2, 5])
def test_lagrange_with_id_zero_against_oracle(ctxs, oc, t):
    """An id equal to 0 zeroes the shared numerator product P, so such a credential takes the
    per-task numerators in k_lagrange; Signature::aggregate must still equal the oracle's."""
    import random
    from coconut import signature_aggregate_batch
    d = golden("aggregate_g2_t67_subsets.json")
    ctx = ctxs[d["mode"]]
    sigs = {}
    for case in d["cases"]:
        for k, i in enumerate(case["ids"]):
            sigs[i] = (case["sigma1"][k], case["sigma2"][k])
    pool = sorted(sigs)
    rng = random.Random(77 + t)
    L, n = 6, 7
    rows, s1, s2 = [], [], []
    for r in range(n):
        src = rng.sample(pool, L)
        row = list(src)
        if r % 2 == 0:
            row[rng.randrange(t)] = 0  # id 0 among the first t
        if r == 3 and t > 2:
            row[1] = row[0]            # and a repeated id
        rows.append(row)
        s1 += [sigs[i][0] for i in src]
        s2 += [sigs[i][1] for i in src]
    g1, g2 = signature_aggregate_batch(ctx, n, L, t, rows, _cat(s1), _cat(s2))
    sb = 192
    o1, o2 = ctypes.create_string_buffer(sb), ctypes.create_string_buffer(sb)
    for r, row in enumerate(rows):
        idarr = (ctypes.c_uint64 * L)(*row)
        assert oc.oc_signature_aggregate(0, ctypes.c_size_t(L), ctypes.c_size_t(t), idarr, _cat(s1[r * L:(r + 1) * L]),
                                         _cat(s2[r * L:(r + 1) * L]), o1, o2) == 0
        assert g1[r * sb:(r + 1) * sb] == o1.raw and g2[r * sb:(r + 1) * sb] == o2.raw, (r, row[:t])
