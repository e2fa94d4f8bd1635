"""The backward torus conversion used by every PBS kernel (fft_device.h frac_to_torus):
X = rint_half_even(fr * 2^64) mod 2^64 for fr = m - rint(m) in [-1/2, 1/2] (x86.rs:823-874,
961-1044), computed on the GPU as two magic-number fmas (1.5 * 2^52) whose bit patterns are added
into the u64 accumulator.

Expected values come from exact rational arithmetic (fractions.Fraction; Python's round() on a
Fraction rounds half to even, as the reference's NINT).  The CPU test restates the device
algorithm with exactly rounded fmas (Fraction -> float rounds to nearest even) to pin the math;
the GPU test runs the device code itself through the C ABI diagnostic entry point.
"""
from fractions import Fraction

import numpy as np
import pytest

MB = 1.5 * 2.0 ** 52
MA = MB - 0x43380000


def exact_x(fr: float) -> int:
    return round(Fraction(fr) * 2 ** 64) % 2 ** 64


def fma(a: float, b: float, c: float) -> float:
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def bits(d: float) -> int:
    return int(np.array([d]).view(np.uint64)[0])


def device_algorithm(fr: float) -> int:
    a = fma(fr, 2.0 ** 32, MA)
    h = a - MA
    f = fma(fr, 2.0 ** 32, -h)
    b = fma(f, 2.0 ** 32, MB)
    return (bits(b) + ((bits(a) & 0xFFFFFFFF) << 32)) % 2 ** 64


def sample_fractions(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    edges = [0.5, -0.5, 0.0, -0.0, 2.0 ** -64, -(2.0 ** -64), 2.0 ** -65, 3 * 2.0 ** -65, -3 * 2.0 ** -65,
             2.0 ** -33, -(2.0 ** -33), 2.0 ** -32 + 2.0 ** -65, 0.25, np.nextafter(0.5, 0), -np.nextafter(0.5, 0),
             2.0 ** -1074, 1.5 * 2.0 ** -33, (2 ** 31 + 0.5) * 2.0 ** -64]
    # m - rint(m) for accumulator-like magnitudes (the values the kernels see) ...
    m = rng.standard_normal(n) * np.exp2(rng.integers(-20, 34, n))
    fr = m - np.rint(m)
    # ... ties of fr * 2^64 and of the low word, and uniformly random fractions
    ties = (rng.integers(-(2 ** 40), 2 ** 40, n // 4) * 2 + 1).astype(np.float64) * 2.0 ** -65
    uni = rng.uniform(-0.5, 0.5, n // 4)
    return np.concatenate([np.array(edges), fr, ties, uni])


def test_device_algorithm_exact_on_cpu():
    for fr in sample_fractions(3000, 7):
        assert device_algorithm(float(fr)) == exact_x(float(fr)), fr.hex()


@pytest.mark.gpu
def test_device_conversion_exact_on_gpu():
    import ctypes

    from tfhe_mi355 import _lib

    lib = _lib.load()
    fr = sample_fractions(200000, 11)
    exp = np.array([exact_x(float(x)) for x in fr], dtype=np.uint64)
    rng = np.random.default_rng(5)
    acc0 = rng.integers(0, 2 ** 64, fr.size, dtype=np.uint64)
    acc = acc0.copy()
    got = np.zeros_like(acc)
    rc = lib.tfhe_mi355_debug_torus_from_fraction(
        0, fr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), acc.ctypes.data_as(_lib.u64p),
        got.ctypes.data_as(_lib.u64p), fr.size)
    assert rc == 0, lib.tfhe_mi355_last_error()
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(float(fr[i]).hex(), hex(int(got[i])), hex(int(exp[i]))) for i in bad[:5]]
    assert np.array_equal(acc, acc0 + exp)  # wrapping u64 add


def _scalar_backward(z: complex, n: int):
    """convert_add_backward_torus_scalar (fft/mod.rs:284-302) into zeroed outputs: tmp = inp *
    (conj(w) * (1/n)) as plain c64 arithmetic, then from_torus (commons/math/torus/mod.rs:72-78):
    fract = x - round(x) (half away from zero), * 2^64, round, as i64 as u64."""
    j = np.arange(n)
    wr, wi = np.cos(j * (np.pi / (2.0 * n))), np.sin(j * (np.pi / (2.0 * n)))
    norm = 1.0 / n
    c, d = wr * norm, -wi * norm
    re = z.real * c - z.imag * d
    im = z.real * d + z.imag * c

    def from_torus(x):
        fract = x - np.where(x >= 0, np.floor(x + 0.5), np.ceil(x - 0.5))
        fract = fract * 2.0 ** 64
        r = np.where(fract >= 0, np.floor(fract + 0.5), np.ceil(fract - 0.5))
        return [int(v) % 2 ** 64 for v in r]

    return from_torus(re), from_torus(im), wr, wi


def test_fma_backward_within_reference_simd_bound_of_scalar():
    """x86.rs:1200-1235 (add_backward_torus_v3): the AVX2/FMA backward conversion -- the form the
    oracle and every PBS kernel compute (ws = w/M, fma products, fract = m - rint(m),
    rint_half_even(fract 2^64)) -- stays within 2^38 of the reference's scalar path on the
    reference's own input (z = -34384521907.303154 + 19013399110.689323 i, n = 1024)."""
    n = 1024
    z = complex(-34384521907.303154, 19013399110.689323)
    s_re, s_im, wr, wi = _scalar_backward(z, n)
    zr, zi = Fraction(z.real), Fraction(z.imag)
    for j in range(n):
        wsr, wsi = float(Fraction(wr[j]) / n), float(Fraction(wi[j]) / n)   # w / M: exact (power of two)
        mr = float(zr * Fraction(wsr) + Fraction(float(zi * Fraction(wsi))))  # fma(zr, wsr, zi*wsi)
        mi = float(-zr * Fraction(wsi) + Fraction(float(zi * Fraction(wsr))))  # fma(-zr, wsi, zi*wsr)
        for m, s in ((mr, s_re[j]), (mi, s_im[j])):
            fr = m - float(round(Fraction(m)))          # rint: half to even
            v = exact_x(fr)
            diff = (v - s) % 2 ** 64
            assert min(diff, 2 ** 64 - diff) < 2 ** 38, (j, v, s)
