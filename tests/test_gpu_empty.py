"""Empty batches and argument ceilings through the batch entry points of include/coconut_hip.h.

The contract the header's entry points share: a call validates its context state and its lengths first
(the reference's own errors: UnsupportedNoOfMessages, UnequalNoOfBasesExponents, the threshold assert
of signature.rs:449,484), and only then treats n = 0 as a no-op returning CC_OK, with every buffer
pointer allowed to be NULL (nothing is read, written or launched).  So an empty batch with a wrong q
still reports CC_ERR_LEN, and one on a context without a verkey still reports CC_ERR_STATE."""
import ctypes
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
pytestmark = pytest.mark.gpu

OK, ERR_LEN, ERR_BASES, ERR_THRESHOLD, ERR_STATE = 0, -1, -2, -3, -7
N = None  # a NULL buffer


@pytest.fixture(scope="module")
def ctx():
    import bench
    import bench_modes
    import coconut
    c = coconut.Context(0, coconut.GroupMode.SIG_G2)
    b = bench.make_verify_batch(c, 0, 4, 6, seed=91)
    c.set_params(b["g_tilde"])
    c.set_verkey(b["X"], b["Y"])
    a = bench_modes.make_aggregate_batch(c, 0, 2, t=3, n_iss=5, seed=92)
    c.set_issuers(a["iss"], a["X"], a["Y"], a["q"])
    yield c
    c.close()


def _lib():
    from coconut._lib import lib
    return lib


def test_empty_verify_batches(ctx):
    lib, h, q = _lib(), ctx.h, 6
    assert lib.cc_verify_batch(h, 0, q, N, N, N, N, N, N, N, 0) == OK
    assert lib.cc_verify_batch(h, 0, q, N, N, N, N, N, N, N, 1) == OK  # RLC requested
    assert lib.cc_verify_batch_device(h, 0, q, N, N, N, N, N, N) == OK
    assert lib.cc_verify_batch_pervk_device(h, 0, q, N, N, N, N, N, N, N, N) == OK
    # the length check comes first: q != the verkey's q is UnsupportedNoOfMessages even when empty
    assert lib.cc_verify_batch(h, 0, q + 1, N, N, N, N, N, N, N, 0) == ERR_LEN
    assert lib.cc_verify_batch_device(h, 0, q + 1, N, N, N, N, N, N) == ERR_LEN


def test_empty_pok_batches(ctx):
    lib, h, q = _lib(), ctx.h, 6
    assert lib.cc_pok_verify_batch(h, 0, q, 0, q + 1, N, N, N, N, N, N, N, N, N, N) == OK
    assert lib.cc_pok_verify_batch_device(h, 0, q, 0, q + 1, N, N, N, N, N, N, N, N, N, N, N) == OK
    # UnequalNoOfBasesExponents before the empty check
    assert lib.cc_pok_verify_batch(h, 0, q, 0, q, N, N, N, N, N, N, N, N, N, N) == ERR_BASES
    assert lib.cc_pok_verify_batch_device(h, 0, q, 0, q, N, N, N, N, N, N, N, N, N, N, N) == ERR_BASES


def test_empty_aggregate_batches(ctx):
    lib, h, q = _lib(), ctx.h, 6
    assert lib.cc_signature_aggregate_batch(h, 0, 3, 3, N, N, N, N, N) == OK
    assert lib.cc_signature_aggregate_batch_device(h, 0, 3, 3, N, N, N, N, N, N) == OK
    assert lib.cc_verkey_aggregate_batch(h, 0, 3, 3, q, N, N, N, N, N) == OK
    assert lib.cc_verkey_aggregate_ids(h, 0, 3, 3, N, N, N) == OK
    assert lib.cc_verkey_aggregate_ids_device(h, 0, 3, 3, N, N, N, N) == OK
    assert lib.cc_aggregate_credential_batch_device(h, 0, 3, 3, N, N, N, N, N, N, N, N) == OK
    # the threshold assert (len < t) before the empty check
    assert lib.cc_signature_aggregate_batch(h, 0, 2, 3, N, N, N, N, N) == ERR_THRESHOLD
    assert lib.cc_verkey_aggregate_ids_device(h, 0, 2, 3, N, N, N, N) == ERR_THRESHOLD


def test_empty_helper_batches(ctx):
    import coconut
    lib, h = _lib(), ctx.h
    g1 = ctypes.create_string_buffer(bytes(coconut.G1_GENERATOR), 97)
    assert lib.cc_fixed_base_mul(h, 1, g1, 0, N, N) == OK
    assert lib.cc_subgroup_check(h, 1, 0, N, N) == OK
    assert lib.cc_subgroup_check(h, 2, 0, N, N) == OK
    off = np.zeros(1, dtype=np.uint64)
    assert lib.cc_hash_msg(h, 0, N, off.ctypes.data_as(ctypes.c_void_p), N) == OK
    assert lib.cc_hash_to_curve(h, 1, 0, N, off.ctypes.data_as(ctypes.c_void_p), N) == OK


def test_empty_batch_still_needs_state():
    """A context with params but no verkey: an empty shared-verkey batch is CC_ERR_STATE (call order
    first), the per-credential-verkey form (which needs no verkey) is CC_OK."""
    import bench
    import coconut
    c = coconut.Context(0, coconut.GroupMode.SIG_G2)
    try:
        b = bench.make_verify_batch(c, 0, 2, 2, seed=93)
        c.set_params(b["g_tilde"])
        lib = _lib()
        assert lib.cc_verify_batch_device(c.h, 0, 2, N, N, N, N, N, N) == ERR_STATE
        assert lib.cc_verify_batch(c.h, 0, 2, N, N, N, N, N, N, N, 0) == ERR_STATE
        assert lib.cc_verify_batch_pervk_device(c.h, 0, 2, N, N, N, N, N, N, N, N) == OK
        assert lib.cc_pok_verify_batch(c.h, 0, 2, 0, 3, N, N, N, N, N, N, N, N, N, N) == ERR_STATE
    finally:
        c.close()


def test_counts_past_the_ceilings_are_decode_errors(ctx):
    """coconut_hip.h CC_MAX_*: a count past its ceiling is CC_ERR_DECODE before anything is read,
    allocated or launched — here with real (tiny) host buffers that a missing check would overrun."""
    lib, h, q = _lib(), ctx.h, 6
    DECODE = -4
    big = (1 << 26) + 1
    tiny = ctypes.create_string_buffer(64)
    t = ctypes.cast(tiny, ctypes.c_void_p)
    assert lib.cc_verify_batch(h, big, q, t, t, t, N, N, t, N, 0) == DECODE
    assert lib.cc_pok_verify_batch(h, big, q, 0, q + 1, t, t, t, t, t, t, N, N, t, N) == DECODE
    assert lib.cc_signature_aggregate_batch(h, big, 3, 3, t, t, t, t, t) == DECODE
    assert lib.cc_verkey_aggregate_ids(h, big, 3, 3, t, t, t) == DECODE
    assert lib.cc_verkey_aggregate_ids(h, 1, (1 << 16) + 1, 3, t, t, t) == DECODE  # len past CC_MAX_IDS
    assert lib.cc_fixed_base_mul(h, 1, t, big, t, t) == DECODE
    assert lib.cc_subgroup_check(h, 1, big, t, t) == DECODE
    assert lib.cc_rlc_finish_device(h, (1 << 16) + 1, t, t, N, N) == DECODE
    assert lib.cc_blind_sign_batch(h, 1, 4097, 1, t, t, t, t, t, t, t, t) == DECODE  # q past CC_MAX_Q


def test_python_mirror_checks_buffer_lengths(ctx):
    """The Python mirror checks every byte count the C ABI will read (the C side trusts the caller's
    counts): a short buffer is CoconutError(Decode) before the call, not a read past its end."""
    import coconut
    from coconut import CoconutError, CoconutErrorKind
    q, sb = 6, 192
    s = bytes(4 * sb)
    with pytest.raises(CoconutError) as e:
        coconut.verify_batch(ctx, 5, q, s, s, bytes(5 * q * 48))  # 4 sigmas for a batch of 5
    assert e.value.kind == CoconutErrorKind.Decode
    with pytest.raises(CoconutError):
        coconut.verify_batch(ctx, 4, q, s, s, bytes(4 * q * 48 - 1))  # one message byte short
    with pytest.raises(CoconutError):
        coconut.fixed_base_mul(ctx, 1, bytes(96), bytes(48))  # a 96-byte G1 base (97 expected)
    from coconut.pok_sig import pok_verify_batch
    with pytest.raises(CoconutError):
        pok_verify_batch(ctx, 2, q, [], q + 1, s, s, bytes(2 * 97), bytes(2 * 97), bytes(2 * (q + 1) * 48 - 48),
                         bytes(2 * 48), b"")
