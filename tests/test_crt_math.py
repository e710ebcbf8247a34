"""Host model of the f64 GRM's residue arithmetic (pysnptools_amd/csrc/syrk_crt.hip).

The f64 GRM of packed SNPs runs on the int8 MFMA: LUT values are quantised to integers at the
block's exponent, K_int = sum_s q_is q_js is computed modulo each of R pairwise-coprime moduli
(exact int32 sums of int8 products), and k_crt rebuilds K_int with Garner's algorithm in f32
arithmetic.  These tests restate that arithmetic in NumPy -- same moduli, same f32 operations,
same bounds -- and check that it is exact: no GPU involved.  The GPU path itself is checked
against the f64 oracle by the GRM parity tests (test_gpu_parity.py, tolerance 1e-10 of max
diag and tighter) and against the f64 MFMA kernel by tools/ubench.py syrk --dtype f64.
"""
import math
import os
import re

import numpy as np
import pytest

SRC = os.path.join(os.path.dirname(__file__), "..", "pysnptools_amd", "csrc", "syrk_crt.hip")


def kernel_moduli():
    text = open(SRC).read()
    m = re.search(r"__constant__ int kMod\[kR\] = \{([^}]*)\}", text)
    return [int(x) for x in m.group(1).split(",")]


MODS = kernel_moduli()
R = len(MODS)
LOG2P = sum(math.log2(p) for p in MODS)


def fraction_bits(m):  # crt_fraction_bits
    return min(52, math.floor((LOG2P - 1.0 - math.log2(max(m, 1)) - 1e-9) / 2.0))


def garner_constants():
    inv = [1.0]
    for i in range(1, R):
        p, w = MODS[i], 1
        for j in range(i):
            w = w * (MODS[j] % p) % p
        inv.append(float(pow(w, -1, p)))
    return inv


INV = garner_constants()
f32 = np.float32


def _rint(x):
    return np.rint(x).astype(f32)


def garner(res):
    """k_crt: residues [R, k] in [0, p) -> K_int as f64 (f32 digit arithmetic, f64 Horner)."""
    r0 = res[0].astype(np.int64)
    half0 = MODS[0] // 2
    v = [np.where(r0 >= half0, r0 - MODS[0], r0).astype(f32)]
    for i in range(1, R):
        p, ip = f32(MODS[i]), f32(1.0) / f32(MODS[i])
        y = v[i - 1].copy()
        for j in range(i - 2, -1, -1):
            y = (y * f32(MODS[j]) + v[j]).astype(f32)
            y = (y - p * _rint((y * ip).astype(f32))).astype(f32)
        y = ((res[i].astype(f32) - y) * f32(INV[i])).astype(f32)
        v.append((y - p * _rint((y * ip).astype(f32))).astype(f32))
    X = v[R - 1].astype(np.float64)
    for i in range(R - 2, -1, -1):
        X = X * MODS[i] + v[i]
    return X


def sym_residue(q, p):  # k_crt_lut
    x = q % p
    return x - p if x >= (p + 1) // 2 else x


def test_moduli_pairwise_coprime_and_int8():
    assert R == 15
    for i in range(R):
        assert 2 <= MODS[i] <= 256
        for j in range(i):
            assert math.gcd(MODS[i], MODS[j]) == 1
    # symmetric residues fit int8 and the int32 sums stay exact up to crt_max_snps() = 2^16 SNPs
    for p in MODS:
        lo, hi = -(p // 2), (p - 1) // 2
        assert -128 <= lo and hi <= 127
    assert 128 * 128 * (1 << 16) < 2 ** 31


@pytest.mark.parametrize("m", [1, 64, 1000, 10_000, 65_536])
def test_fraction_bits_keep_k_int_in_range(m):
    F = fraction_bits(m)
    assert F >= 50
    # |K_int| <= m 2^2F must lie in the balanced range [-P/2, P/2)
    P = math.prod(MODS)
    assert m * (1 << (2 * F)) < P // 2


def test_garner_f32_arithmetic_is_exact():
    rng = np.random.default_rng(7)
    P = math.prod(MODS)
    xs = [int(rng.integers(-(2 ** 62), 2 ** 62)) * int(rng.integers(0, 2 ** 53)) for _ in range(3000)]
    xs += [P // 2 - 1, -(P // 2), 0, 1, -1, 2 ** 116, -(2 ** 116), 12345678901234567890]
    res = np.array([[x % p for x in xs] for p in MODS], dtype=np.int64)
    X = garner(res)
    for x, got in zip(xs, X):
        assert got == float(x) or abs(got - x) <= 2 ** -52 * abs(x) * R


def test_residue_grm_matches_f64():
    """The whole per-launch pipeline at a small size: quantise, residue products, CRT, scale."""
    rng = np.random.default_rng(3)
    n, m = 48, 700
    codes = rng.integers(0, 4, size=(m, n))
    lut = rng.standard_normal((m, 4)) * rng.choice([1.0, 7.0, 0.01], size=(m, 1))
    lut[:, 1] = 0.0  # the missing code
    a = lut[np.arange(m)[:, None], codes]  # [m, n] standardized values
    e = math.frexp(np.abs(lut).max())[1]
    F = fraction_bits(m)
    q = np.rint(np.ldexp(lut, F - e)).astype(np.int64)
    qa = q[np.arange(m)[:, None], codes]
    res = []
    for p in MODS:
        rho = np.vectorize(lambda v: sym_residue(int(v), p))(qa).astype(np.int64)
        assert np.abs(rho).max() <= 128
        acc = rho.T @ rho  # the int8 MFMA's exact int32 sums
        res.append(np.mod(acc, p))
    K = np.ldexp(garner(np.array(res).reshape(R, -1)), 2 * (e - F)).reshape(n, n)
    Kref = a.T @ a
    # quantisation error <= 2^(e-F-1) per value
    bound = 2.0 ** (e - F) * np.abs(a).sum(axis=0).max() * 2
    assert np.abs(K - Kref).max() <= bound
    assert np.abs(K - Kref).max() <= 1e-13 * np.abs(np.diag(Kref)).max()


def garner_first(res, Rb):
    """k_crt with the first Rb residues only (digits >= Rb left zero: the per-block moduli)."""
    r0 = res[0].astype(np.int64)
    v = [np.where(r0 >= MODS[0] // 2, r0 - MODS[0], r0).astype(f32)]
    for i in range(1, R):
        if i >= Rb:
            v.append(np.zeros_like(v[0]))
            continue
        p, ip = f32(MODS[i]), f32(1.0) / f32(MODS[i])
        y = v[i - 1].copy()
        for j in range(i - 2, -1, -1):
            y = (y * f32(MODS[j]) + v[j]).astype(f32)
            y = (y - p * _rint((y * ip).astype(f32))).astype(f32)
        y = ((res[i].astype(f32) - y) * f32(INV[i])).astype(f32)
        v.append((y - p * _rint((y * ip).astype(f32))).astype(f32))
    X = v[R - 1].astype(np.float64)
    for i in range(R - 2, -1, -1):
        X = X * MODS[i] + v[i]
    return X


def block_moduli(lgp_i, lgp_j):
    """syrk_crt.hip block_moduli: the fewest R with log2 P_R > 0.5 (lgp_i + lgp_j) + 1."""
    need = 0.5 * (lgp_i + lgp_j) + 1.0
    plog = np.cumsum([math.log2(p) for p in MODS])
    Rb = 1
    while Rb < R and plog[Rb - 1] <= need:
        Rb += 1
    return Rb


def test_per_block_moduli_give_the_same_bits():
    """A block whose iids' bound sums M_i = sum_s q_is^2 are small runs fewer moduli: K_int with
    |K_ij| <= sqrt(M_i M_j) is rebuilt from the first R_b residues to the same f64 bits as from all
    15 (the balanced mixed-radix digits above R_b are zero), and R_b never exceeds the launch-wide R."""
    rng = np.random.default_rng(11)
    for bits in (20, 40, 56, 70, 90, 110):
        M_i, M_j = 2.0 ** bits, 2.0 ** (bits - 7)
        Rb = block_moduli(math.log2(M_i * (1 + 2 ** -20)), math.log2(M_j * (1 + 2 ** -20)))
        Rl = block_moduli(math.log2(M_i * (1 + 2 ** -20)), math.log2(M_i * (1 + 2 ** -20)))
        assert 1 <= Rb <= Rl <= R
        assert math.prod(MODS[:Rb]) > 2 * math.sqrt(M_i * M_j)
        lim = int(math.sqrt(M_i * M_j))
        xs = [int(rng.integers(-(2 ** 62), 2 ** 62)) * (lim >> 62) + int(rng.integers(-min(lim, 2 ** 62), min(lim, 2 ** 62) + 1))
              for _ in range(500)] + [lim, -lim, 0, 1, -1]
        xs = [max(-lim, min(lim, x)) for x in xs]
        res = np.array([[x % p for x in xs] for p in MODS], dtype=np.int64)
        full, first = garner(res), garner_first(res, Rb)
        assert np.array_equal(full, first), bits
        for x, got in zip(xs, first):
            assert got == float(x) or abs(got - x) <= 2 ** -52 * abs(x) * R
