"""CPU check of the lane-pair Fermat inversion schedule used by the pair-lane tower
(coconut-rust_amd/csrc/tower_pl.h: fp_inv_pair; the inversion sits in the final exponentiation's
easy part, AMCL `pair::fexp` via amcl_wrapper `GT::ate_2_pairing`, reference src/lib.rs:13).

The kernel runs one Montgomery multiplication per step on both lanes of a pair: the real lane
squares s <- s^2 (s = a^(2^i)), the imaginary lane multiplies acc by the partner's s when bit i of
p - 2 is set and by Montgomery one otherwise.  This test simulates that lockstep schedule with the
same 381 steps and the same R = 2^406 Montgomery form and compares it with pow(a, p - 2, p).  The
GPU parity tests cover the kernel itself through the GT bytes of the final exponentiation.
"""
import random

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 1 << 406
RINV = pow(R, -1, P)


def mont_mul(x, y):
    return x * y * RINV % P


def inv_pair_schedule(a):
    """a in Montgomery form; returns a^-1 in Montgomery form via the two-lane schedule."""
    e = P - 2
    assert e.bit_length() == 32 * 11 + 29  # the kernel's loop bound: bits 0 .. 32*11 + 28
    one = R % P
    s, acc = a, one  # real lane, imaginary lane
    for bit in range(e.bit_length()):
        sp = s  # imaginary lane reads the partner's value before this step's update (DPP)
        y_im = sp if (e >> bit) & 1 else one
        s, acc = mont_mul(s, s), mont_mul(acc, y_im)
    return acc


def test_inv_pair_schedule_matches_fermat():
    rng = random.Random(7)
    cases = [1, 2, P - 1, P - 2] + [rng.randrange(1, P) for _ in range(16)]
    for x in cases:
        xm = x * R % P
        got = inv_pair_schedule(xm)
        assert got == pow(x, P - 2, P) * R % P
        assert mont_mul(got, xm) == R % P


def test_inv_pair_schedule_step_count_beats_square_and_multiply():
    e = P - 2
    steps_pair = e.bit_length()
    sqr_mul = (e.bit_length() - 1) + (bin(e).count("1") - 1)
    assert steps_pair == 381 and sqr_mul == 380 + 228
