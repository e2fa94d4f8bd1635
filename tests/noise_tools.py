"""Noise-measurement helpers restating the reference's test tools:
torus_modular_diff (core_crypto/algorithms/misc.rs:67-94) and variance
(core_crypto/commons/mod.rs:77-83), plus the reference FFT tolerance
(core_crypto/fft_impl/fft64/math/fft/tests.rs:166-172)."""
import numpy as np

RELATIVE_TOLERANCE = 0.0625   # lwe_encryption_noise.rs:9-10
NB_TESTS = 1000               # lwe_encryption_noise.rs:12


def torus_modular_diff(first, other) -> np.ndarray:
    """Smallest signed difference first - other on the native torus, in [-1/2, 1/2)."""
    a = np.asarray(first, dtype=np.uint64)
    b = np.asarray(other, dtype=np.uint64)
    d0 = a - b
    d1 = b - a
    return np.where(d0 < d1, d0.astype(np.float64), -d1.astype(np.float64)) / 2.0 ** 64


def variance(samples) -> float:
    s = np.asarray(samples, dtype=np.float64)
    return float(np.sum((s - s.mean()) ** 2) / (len(s) - 1))


def fft_product_tolerance(N: int, int_magnitude: int) -> int:
    """fft/tests.rs:166-172: |FFT product - exact| <= 2^(64 - (52 - integer_magnitude - log2 N))."""
    return 1 << (64 - (52 - int_magnitude - (N.bit_length() - 1)))


def external_product_tolerance(params) -> int:
    """The reference tolerance summed over the (k+1) L products of one output column of an
    external product; signed PBS digits have |d| <= 2^(base_log - 1)."""
    p = params
    return (p.glwe_dimension + 1) * p.pbs_level * fft_product_tolerance(p.polynomial_size, p.pbs_base_log - 1)


def modular_distance(a, b) -> np.ndarray:
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    return np.minimum(a - b, b - a)
