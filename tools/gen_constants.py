#!/usr/bin/env python3
"""Emit the BLS12-381 constants the device field layer needs (coconut-rust_amd/csrc/*.h).

The device multiplies in radix 2^29 (14 limbs) with Montgomery radix R = 2^406; operands are stored
as 12 x 32-bit little-endian limbs.  Every constant kept in Montgomery form therefore depends on R:
ONE = R mod p, R2 = R^2 mod p, the curve constant b = 4 (G1) / 4(1+i) (G2 twist), and the Frobenius
coefficients gamma_k = xi^(k(p-1)/6), gamma2_k = xi^(k(p^2-1)/6), xi = 1 + i.
Run:  python tools/gen_constants.py      (prints C initialisers)
"""
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R_BITS = 406
R = 1 << R_BITS


def limbs32(x, n=12):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def limbs29(x, n=14):
    return [(x >> (29 * i)) & 0x1FFFFFFF for i in range(n)]


def c_list(v):
    return ", ".join(f"0x{w:08x}u" for w in v)


def mont(x):
    return x * R % P


def f2_mul(x, y):
    """Fp2 product on pairs (a, b) = a + b i, i^2 = -1."""
    return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)


def f2_pow(x, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2_mul(r, x)
        x = f2_mul(x, x)
        e >>= 1
    return r


def main():
    n0 = (-pow(P, -1, 1 << 29)) % (1 << 29)
    print(f"// R = 2^{R_BITS}")
    print(f"#define CC_P29_LIMBS {', '.join(f'0x{w:08x}u' for w in limbs29(P))}")
    print(f"constexpr uint32_t N0_29 = 0x{n0:08x}u;")
    print(f"#define CC_ONE_LIMBS {c_list(limbs32(mont(1)))}")
    print(f"#define CC_R2_LIMBS {c_list(limbs32(R * R % P))}")
    print(f"// curve b = 4 (Montgomery)\n{{{c_list(limbs32(mont(4)))}}}")
    xi = (1, 1)
    print("// kGamma1[k] = xi^(k(p-1)/6), Montgomery (a, b)")
    for k in range(6):
        g = f2_pow(xi, k * (P - 1) // 6)
        print(f"    {{{{{c_list(limbs32(mont(g[0])))}}},\n     {{{c_list(limbs32(mont(g[1])))}}}}},")
    print("// kGamma2[k] = xi^(k(p^2-1)/6) in Fp, Montgomery")
    for k in range(6):
        g = f2_pow(xi, k * (P * P - 1) // 6)
        assert g[1] == 0
        print(f"    {{{c_list(limbs32(mont(g[0])))}}},")


if __name__ == "__main__":
    main()
