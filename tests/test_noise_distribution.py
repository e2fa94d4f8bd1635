"""Noise-distribution tests on the CPU.

* Port of core_crypto/algorithms/test/noise_distribution/lwe_encryption_noise.rs:14-80
  (lwe_encrypt_decrypt_noise_distribution_custom_mod at TEST_PARAMS_4_BITS_NATIVE_U64):
  NB_TESTS = 1000 encryptions per message, every message of the 4-bit space, decryption exact,
  measured noise variance within RELATIVE_TOLERANCE = 1/16 of lwe_modular_std_dev^2.  Run on the
  engine's client-side encryption (C ABI, used by bench.py and the shortint/integer client keys)
  and on the oracle's (used to build every test key).  The reference draws a fresh secret key per
  sample; the noise does not depend on the key, so one key per message is used here.
* The FFT-free exact PBS oracle: Karatsuba == schoolbook, exact PBS decrypts, and one CMUX of the
  FFT oracle (== the GPU, bit for bit) is within the reference FFT tolerance of exact arithmetic.
"""
import numpy as np
import pytest

from noise_tools import (NB_TESTS, RELATIVE_TOLERANCE, external_product_tolerance, modular_distance,
                         torus_modular_diff, variance)


def _encryption_noise(encrypt, decrypt, keygen, params):
    msg_modulus = 16
    delta = (1 << 63) // msg_modulus          # encoding with padding / msg_modulus
    n = params.lwe_dimension
    samples = []
    for msg in range(msg_modulus - 1, -1, -1):
        sk = keygen(1000 + msg, n)
        pts = np.full(NB_TESTS, msg * delta, dtype=np.uint64)
        cts = encrypt(2000 + msg, sk, pts, params.lwe_modular_std_dev)
        dec = decrypt(sk, cts)
        rounding = (dec & np.uint64(delta >> 1)) << np.uint64(1)
        assert np.all(((dec + rounding) // np.uint64(delta)) % np.uint64(msg_modulus) == msg)
        samples.append(torus_modular_diff(pts, dec))
    return variance(np.concatenate(samples))


def _check(measured):
    from tfhe_mi355.parameters import TEST_PARAMS_4_BITS_NATIVE_U64 as P

    expected = P.lwe_modular_std_dev ** 2
    assert abs(expected - measured) < RELATIVE_TOLERANCE * expected, (measured, expected)


def test_lwe_encryption_noise_distribution_engine_client():
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import TEST_PARAMS_4_BITS_NATIVE_U64 as P

    _check(_encryption_noise(client.lwe_encrypt, client.lwe_decrypt,
                             lambda seed, n: client.gen_binary_key(seed, 1, n), P))


def test_lwe_encryption_noise_distribution_oracle(orc):
    from tfhe_mi355.parameters import TEST_PARAMS_4_BITS_NATIVE_U64 as P

    _check(_encryption_noise(orc.lwe_encrypt, orc.lwe_decrypt, lambda seed, n: orc.binary_key(seed, 1, n), P))


@pytest.mark.parametrize("N", [32, 64, 512, 2048])
def test_exact_product_karatsuba_equals_schoolbook(orc, N):
    rng = np.random.default_rng(N)
    a = rng.integers(0, 2 ** 64, N, dtype=np.uint64)
    b = rng.integers(0, 2 ** 64, N, dtype=np.uint64)
    acc = rng.integers(0, 2 ** 64, N, dtype=np.uint64)
    assert np.array_equal(orc.negacyclic_mul_add_exact(a, b, acc), acc + orc.negacyclic_mul(a, b))


@pytest.fixture(scope="module")
def small_keys(orc):
    """2_2 GLWE parameters with a 16-dimensional input key (exact PBS in well under a second)."""
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS

    p = PARAM_MESSAGE_2_CARRY_2_KS_PBS.with_(lwe_dimension=16, name="2_2_n16")
    lwe_sk = orc.binary_key(21, 1, 16)
    glwe_sk = orc.binary_key(21, 2, 2048)
    bsk = orc.gen_bsk(22, lwe_sk, glwe_sk, 1, 2048, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev, threads=8)
    return p, lwe_sk, glwe_sk, bsk


def test_exact_pbs_decrypts(orc, small_keys):
    p, lwe_sk, glwe_sk, bsk = small_keys
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (3 * x + 1) % 16)
    msgs = np.arange(16, dtype=np.uint64)
    cts = orc.lwe_encrypt(23, lwe_sk, msgs * np.uint64(p.delta), p.lwe_modular_std_dev)
    out = orc.exact_pbs(bsk, 16, 1, 2048, p.pbs_base_log, p.pbs_level, cts, acc)
    d = orc.lwe_decrypt(glwe_sk, out)
    dec = ((d + ((d & np.uint64(p.delta >> 1)) << np.uint64(1))) // np.uint64(p.delta)) % np.uint64(16)
    assert np.array_equal(dec, (3 * msgs + 1) % 16)


def test_fft_oracle_single_cmux_within_reference_tolerance(orc, small_keys):
    """One CMUX (a single nonzero mask element) from a random accumulator: the FFT oracle's
    accumulator (bit-identical to the GPU's) vs the exact one, every coefficient."""
    p, lwe_sk, glwe_sk, bsk = small_keys
    rng = np.random.default_rng(5)
    acc = rng.integers(0, 2 ** 64, 2 * 2048, dtype=np.uint64)
    cts = np.zeros((8, 17), dtype=np.uint64)
    for c in range(8):
        cts[c, c] = rng.integers(1, 2 ** 64, dtype=np.uint64)
        cts[c, 16] = rng.integers(0, 2 ** 64, dtype=np.uint64)
    fb = orc.FourierBsk(bsk, 16, 1, 2048, p.pbs_base_log, p.pbs_level)
    got = fb.blind_rotate(cts, acc, threads=8)
    exact = orc.exact_pbs(bsk, 16, 1, 2048, p.pbs_base_log, p.pbs_level, cts, acc, glwe_out=True)
    dist = modular_distance(got, exact)
    tol = external_product_tolerance(p)
    assert int(dist.max()) <= tol, (int(dist.max()).bit_length(), tol.bit_length())
