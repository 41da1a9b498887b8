#!/usr/bin/env python3
"""Emit the constants of the lazy radix-2^28 field layer (coconut-rust_amd/csrc/lazy.h).

lazy.h multiplies 14 signed 28-bit limbs with Montgomery radix R' = 2^392 (the storage layer,
field.h, uses R = 2^406 on 12 x 32-bit limbs).  Values cross between the two with one Montgomery
multiplication: R -> R' by 2^378 mod p, R' -> R by R mod p.  The Frobenius coefficients are the
same field elements as tools/gen_constants.py's, in R' form.
Run:  python tools/gen_lz_constants.py      (prints C initialisers)
"""
from gen_constants import P, f2_pow

RB = 392
RP = 1 << RB


def limbs28(x, n=14):
    return [(x >> (28 * i)) & 0xFFFFFFF for i in range(n)]


def c_list(v):
    return ", ".join(f"0x{w:07x}" for w in v)


def mont(x):
    return x * RP % P


def main():
    n0 = (-pow(P, -1, 1 << 28)) % (1 << 28)
    print(f"#define LZ_P_LIMBS {c_list(limbs28(P))}")
    print(f"constexpr uint32_t LZ_N0 = 0x{n0:07x}u;")
    print(f"#define LZ_ONE_LIMBS {c_list(limbs28(mont(1)))}")
    print(f"#define LZ_C_IN_LIMBS {c_list(limbs28(pow(2, 378, P)))}   // 2^378: R form -> R' form")
    print(f"#define LZ_C_OUT_LIMBS {c_list(limbs28(pow(2, 406, P)))}  // 2^406: R' form -> R form")
    print(f"#define LZ_R3_LIMBS {c_list(limbs28(pow(RP, 3, P)))}     // R'^3: inversion")
    xi = (1, 1)
    print("// gamma_k = xi^(k(p-1)/6), R' form (a, b)")
    for k in range(6):
        g = f2_pow(xi, k * (P - 1) // 6)
        print(f"    {{{{{c_list(limbs28(mont(g[0])))}}},\n     {{{c_list(limbs28(mont(g[1])))}}}}},")
    print("// gamma2_k = xi^(k(p^2-1)/6) in Fp, R' form")
    for k in range(6):
        g = f2_pow(xi, k * (P * P - 1) // 6)
        assert g[1] == 0
        print(f"    {{{c_list(limbs28(mont(g[0])))}}},")


if __name__ == "__main__":
    main()
