"""The lazy radix-2^28 field core (coconut-rust_amd/csrc/lazy.h) on the device, at its bounds.

cc_selftest_lazy runs the exact product-scanning Montgomery multiplication, value reduction and limb
squeeze the Miller-loop and final-exponentiation kernels use, on inputs drawn by
tests/test_lazy_algebra.py's generators at the limits the compile-time types allow (limbs up to
A = 1040 x 2^20 against 256 x 2^20, |value| up to 2048 p for the reduction), and checks every
result against Python big integers: congruence mod p, normalised output limbs, and the value bound
the types claim.  Any miscompiled signed mad, carry or shift shows up here.
"""
import ctypes
import random

import numpy as np
import pytest

from test_lazy_algebra import LN, M28, P, RP, rand_lz, value

pytestmark = pytest.mark.gpu


def _lib():
    from coconut._lib import lib
    return lib


def _run(op, a, b=None, c=None, d=None):
    lib = _lib()
    n = len(a)
    arrs = [np.ascontiguousarray(np.array(x, dtype=np.int32)) if x is not None else None for x in (a, b, c, d)]
    out = np.zeros((n, LN), dtype=np.int32)
    ptr = lambda x: x.ctypes.data_as(ctypes.c_void_p) if x is not None else None  # noqa: E731
    rc = lib.cc_selftest_lazy(op, n, *[ptr(x) for x in arrs], out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return [[int(t) for t in row] for row in out]


@pytest.mark.parametrize("a1,a2,b1,b2", [(514, 514, 16, 16), (256, 1040, 100, 30), (1040, 256, 18, 18),
                                         (257, 1036, 2048, 16)])
def test_mont2_on_device_at_the_limb_bound(a1, a2, b1, b2):
    assert 2 * a1 * a2 <= 533000
    rng = random.Random(17 + a1 + a2)
    n = 512
    xs = [rand_lz(a1, b1, rng, extreme=k % 2 == 0) for k in range(n)]
    ys = [rand_lz(a2, b2, rng, extreme=k % 3 == 0) for k in range(n)]
    us = [rand_lz(a1, b1, rng) for _ in range(n)]
    vs = [rand_lz(a2, b2, rng) for _ in range(n)]
    out = _run(0, xs, ys, us, vs)
    rinv = pow(RP, -1, P)
    bout = 16 + (2 * b1 * b2 + 40303) // 40304
    for x, y, u, v, r in zip(xs, ys, us, vs, out):
        assert value(r) % P == (value(x) * value(y) + value(u) * value(v)) * rinv % P
        assert all(0 <= t <= M28 for t in r[:-1])
        assert abs(value(r)) < bout * P // 16


def test_mont1_on_device():
    rng = random.Random(5)
    n = 512
    xs = [rand_lz(2047, 200, rng, extreme=False) for _ in range(n)]
    ys = [rand_lz(260, 200, rng) for _ in range(n)]
    out = _run(1, xs, ys)
    rinv = pow(RP, -1, P)
    for x, y, r in zip(xs, ys, out):
        assert value(r) % P == value(x) * value(y) * rinv % P


def test_reduce_and_squeeze_on_device():
    rng = random.Random(23)
    n = 1024
    xs = [rand_lz(2047, 32768, rng, extreme=k % 2 == 0) for k in range(n)]
    red = _run(2, xs)
    sq = _run(3, xs)
    for x, r, s in zip(xs, red, sq):
        assert value(r) % P == value(x) % P and abs(value(r)) < 9 * P // 16
        assert all(0 <= t <= M28 for t in r[:-1])
        assert value(s) == value(x) and all(abs(t) < (257 << 20) for t in s)


def test_divstep_inversions_on_device():
    """field.h fp_inv_int (one lane) and tower_q.h fp_inv_int_quad (the four lanes of a quad share one
    inversion, each lane carrying one of the divstep vectors) against pow(a, p - 2, p), across a whole
    wave (the upper half-wave's lane ids included) and for a = 0, 1, p - 1."""
    rnd = random.Random(7)
    vals = [0, 1, P - 1, 2, P - 2] + [rnd.randrange(1, P) for _ in range(123)]
    a = [[(v >> (32 * k)) & 0xFFFFFFFF for k in range(12)] + [0, 0] for v in vals]
    a = [[x - (1 << 32) if x >> 31 else x for x in row] for row in a]
    quad = [row for row in a for _ in range(4)]  # each quad holds one value
    words = lambda row: sum((x & 0xFFFFFFFF) << (32 * k) for k, x in enumerate(row[:12]))  # noqa: E731
    one = _run(4, a)
    four = _run(5, quad)
    for k, v in enumerate(vals):
        want = pow(v, P - 2, P)
        assert words(one[k]) == want, k
        assert all(words(four[4 * k + j]) == want for j in range(4)), k
