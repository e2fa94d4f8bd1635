"""Oracle pinning (CPU): the restatement against the reference's own known-answer tests and
tolerances.  No GPU needed.

  decomposer KATs        core_crypto/commons/math/decomposition/decomposer.rs:95-96, term.rs:48,144
  f64 -> i64 twiddles    core_crypto/fft_impl/fft64/math/fft/tests.rs:244-300
  FFT product tolerance  fft/tests.rs:82-222  (threshold 2^(64-(52-int_bits-log2 N)))
  FFT round trip         fft/tests.rs:9-80    (error < 2^(64-50))
  PBS round trip         core_crypto/algorithms/test/lwe_programmable_bootstrapping.rs:70-166
  keyswitch round trip   core_crypto/algorithms/test/lwe_keyswitch.rs
"""
import numpy as np
import pytest

from conftest import decode


def test_decomposer_closest_representable_kat(orc):
    # u32 KAT (decomposer.rs:95-96) evaluated in the top 32 bits of a u64
    assert orc.closest_representable(1_340_987_234 << 32, 4, 3) >> 32 == 1_341_128_704


def test_decomposer_term_kat(orc):
    # term.rs:48 / :144 -- first term of decompose(2^19) (u32, base 2^4, 3 levels) is 1 and
    # recomposes to 1048576 = 1 << (32 - 4*3)
    terms = orc.decompose((2 ** 19) << 32, 4, 3)
    assert terms[0] == 1
    assert (terms[0] << (32 - 4 * 3)) == 1048576


@pytest.mark.parametrize("base_log,level", [(23, 1), (15, 2), (3, 5), (3, 7), (7, 2), (4, 3), (21, 1)])
def test_decomposition_recomposes_and_is_balanced(orc, base_log, level):
    rng = np.random.default_rng(base_log * 100 + level)
    for x in rng.integers(0, 2 ** 64, 200, dtype=np.uint64):
        x = int(x)
        digits = orc.decompose(x, base_log, level)
        half = 1 << (base_log - 1)
        total = 0
        for l, d in enumerate(digits):  # digits[0] is level `level` (least significant)
            ds = d - (1 << 64) if d >= (1 << 63) else d
            assert -half <= ds <= half
            lvl = level - l
            total += ds << (64 - base_log * lvl)
        assert total % (1 << 64) == orc.closest_representable(x, base_log, level)


def test_f64_to_i64_bit_twiddles(orc):
    for x in [0.0, -0.0, 37.1242161, -37.1242161, 0.1, -0.1, 1.0, -1.0, 0.9, -0.9, 2.0, -2.0, 1e-310,
              -1e-310, 2.0 ** 62, -(2.0 ** 62), 1.1 * 2.0 ** 62, 1.1 * -(2.0 ** 62), -(2.0 ** 63)]:
        assert orc.f64_to_i64(x) == int(x)


def test_pbs_modulus_switch(orc):
    # fast_pbs_modulus_switch may return 2N (common.rs:18-25)
    assert orc.pbs_modulus_switch(0, 11) == 0
    assert orc.pbs_modulus_switch((1 << 64) - 1, 11) == 4096
    assert orc.pbs_modulus_switch(1 << 63, 11) == 2048
    assert orc.pbs_modulus_switch((1 << 52) - 1, 11) == 1  # rounds half up


def _digit_reversed_index(M, radices):
    """frequency index of each position of the DIF output (DESIGN.md FFT spec)."""
    idx = np.zeros(M, dtype=np.int64)
    for p in range(M):
        rem, m, k, scale = p, M, 0, 1
        for R in radices:
            m //= R
            c = rem // m
            rem -= c * m
            k += c * scale
            scale *= R
        idx[p] = k
    return idx


@pytest.mark.parametrize("M,radices", [(1024, [16, 16, 4]), (512, [8, 8, 8]), (16384, [16, 16, 16, 4]),
                                       (64, [16, 4]), (2048, [2, 16, 16, 4]), (4096, [4, 16, 16, 4]),
                                       (8192, [8, 16, 16, 4])])
def test_complex_fft_matches_dft(orc, M, radices):
    rng = np.random.default_rng(M)
    z = rng.standard_normal(M) + 1j * rng.standard_normal(M)
    got = orc.fft_complex(z)
    ref = np.fft.fft(z)[_digit_reversed_index(M, radices)]
    assert np.max(np.abs(got - ref)) < 1e-11 * np.sqrt(M) * np.max(np.abs(ref))
    back = orc.fft_complex(got, inverse=True) / M
    assert np.max(np.abs(back - z)) < 1e-12 * np.sqrt(M) * np.max(np.abs(z))


@pytest.mark.parametrize("log_n", list(range(5, 15)))
def test_fft_product_within_reference_tolerance(orc, log_n):
    N = 1 << log_n
    rng = np.random.default_rng(log_n)
    int_bits = 16
    trials = 3 if N <= 4096 else 1
    for _ in range(trials):
        a = rng.integers(0, 2 ** 64, N, dtype=np.uint64)
        b = rng.integers(0, 2 ** 64, N, dtype=np.uint64) >> np.uint64(64 - int_bits)
        got = orc.fft_product(a, b)
        exact = orc.negacyclic_mul(a, b)
        diff = (got - exact).view(np.int64).astype(np.float64)
        threshold = 2.0 ** (64 - (52 - int_bits - log_n))
        assert np.max(np.abs(diff)) <= threshold


@pytest.mark.parametrize("log_n", list(range(5, 16)))
def test_fft_roundtrip(orc, log_n):
    N = 1 << log_n
    a = np.random.default_rng(log_n + 100).integers(0, 2 ** 64, N, dtype=np.uint64)
    rt = orc.fft_roundtrip(a)
    assert np.max(np.abs((rt - a).view(np.int64).astype(np.float64))) < 2.0 ** 14


def test_oracle_pbs_round_trip_2_2(orc, keys_2_2):
    """lwe_encrypt_pbs_decrypt_custom_mod at TEST_PARAMS_4_BITS_NATIVE_U64 (= 2_2 crypto params):
    every message 0..15, identity LUT, decode(decrypt(PBS(ct))) == msg."""
    p = keys_2_2.params
    delta = (1 << 63) // 16
    acc = orc.fill_accumulator(p.polynomial_size, p.glwe_dimension, 4, 4, lambda x: x)
    msgs = np.repeat(np.arange(16, dtype=np.uint64), 2)
    cts = orc.lwe_encrypt(21, keys_2_2.lwe_sk, msgs * np.uint64(delta), p.lwe_modular_std_dev)
    out = keys_2_2.fbsk.pbs(cts, acc, threads=8)
    dec = decode(orc.lwe_decrypt(keys_2_2.glwe_sk, out), delta) % 16
    assert np.array_equal(dec, msgs)


def test_oracle_pbs_round_trip_manticore(orc, keys_manticore):
    """N=1024, L=2 (fork's MANTICORE_PARAMETERS, gadget/parameters/mod.rs:224-235)."""
    p = keys_manticore.params
    delta = (1 << 63) // 4
    acc = orc.fill_accumulator(p.polynomial_size, p.glwe_dimension, 2, 2, lambda x: (x + 1) % 4)
    msgs = np.arange(4, dtype=np.uint64)
    cts = orc.lwe_encrypt(22, keys_manticore.lwe_sk, msgs * np.uint64(delta), p.lwe_modular_std_dev)
    out = keys_manticore.fbsk.pbs(cts, acc, threads=4)
    dec = decode(orc.lwe_decrypt(keys_manticore.glwe_sk, out), delta) % 4
    assert np.array_equal(dec, (msgs + 1) % 4)


@pytest.mark.parametrize("N", [1024, 2048, 32768])
def test_position_frequency_map(orc, N):
    """FFT output position P holds frequency pos_freq(P): the transform of e_1 is W^f(P)."""
    M = N // 2
    f = orc.pos_freq(N)
    assert np.array_equal(np.sort(f), np.arange(M))
    z = np.zeros(M, dtype=np.complex128)
    z[1] = 1.0
    out = orc.fft_complex(z)
    assert np.allclose(out, np.exp(-2j * np.pi * f / M), atol=1e-12)


@pytest.mark.parametrize("N", [1024, 2048])
def test_monomial_spectrum_closed_form(orc, N):
    """Multi-bit keybundle monomials (incomplete_monomial_forward_as_integer, fft/mod.rs:407-445):
    the closed form i^q twist[r] equals the transform of X^d for d in [0, 2N]."""
    M = N // 2
    ds = [0, 1, 2, 3, M - 1, M, M + 1, N - 1, N, N + 1, N + M, 2 * N - 1, 2 * N]
    ds += [int(d) for d in np.random.default_rng(N).integers(0, 2 * N + 1, 20)]
    for d in ds:
        x = np.zeros(N, dtype=np.uint64)
        dm = d % (2 * N)
        if dm < N:
            x[dm] = 1
        else:
            x[dm - N] = np.uint64(2 ** 64 - 1)
        ref = orc.fft_forward_integer(x)
        got = orc.mono_spectrum(N, d)
        assert np.max(np.abs(ref - got)) < 1e-9, d
        assert np.allclose(np.abs(got), 1.0, atol=1e-15)


def test_oracle_multi_bit_pbs_round_trip(orc, keys_mb):
    """multi_bit_programmable_bootstrap_lwe_ciphertext (lwe_multi_bit_programmable_bootstrapping.rs:
    1035-1128) at PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS, deterministic group order:
    decode(decrypt(PBS(ct))) == f(msg) for every message (test/lwe_multi_bit_programmable_bootstrapping.rs)."""
    p = keys_mb.params
    delta = (1 << 63) // 16
    acc = orc.fill_accumulator(p.polynomial_size, p.glwe_dimension, 4, 4, lambda x: (3 * x + 1) % 16)
    msgs = np.arange(16, dtype=np.uint64)
    cts = orc.lwe_encrypt(24, keys_mb.lwe_sk, msgs * np.uint64(delta), p.lwe_modular_std_dev)
    out = keys_mb.fbsk.pbs(cts, acc, threads=8)
    dec = decode(orc.lwe_decrypt(keys_mb.glwe_sk, out), delta) % 16
    assert np.array_equal(dec, (3 * msgs + 1) % 16)


def test_oracle_keyswitch_round_trip(orc, keys_2_2):
    p = keys_2_2.params
    delta = (1 << 63) // 16
    msgs = np.arange(16, dtype=np.uint64)
    big = orc.lwe_encrypt(23, keys_2_2.glwe_sk, msgs * np.uint64(delta), p.glwe_modular_std_dev)
    small = orc.keyswitch(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
    dec = decode(orc.lwe_decrypt(keys_2_2.lwe_sk, small), delta) % 16
    assert np.array_equal(dec, msgs)


@pytest.mark.parametrize("beta", [23, 21, 15, 10])
def test_single_level_digit_shortcut_matches_decomposer(orc, beta):
    """The HIP kernels' L=1 digit shortcut (pbs_common.h DigitL1):
    ((x_hi + ((2^beta - 1) << (31 - beta))) >> (32 - beta)) - (2^(beta-1) - 1), and the bfe form
    bfe((x_hi >> (31 - beta)) + 2^beta - 1, 1, beta) - (2^(beta-1) - 1) it replaced, must equal the
    SignedDecomposer digit (decomposer.rs:99-153, iter.rs:134-141)."""
    rng = np.random.default_rng(beta)
    xs = [int(x) for x in rng.integers(0, 2 ** 64, 3000, dtype=np.uint64)]
    # rounding ties and overflow edges: values around multiples of 2^(63-beta)
    for k in [0, 1, 2, (1 << beta) - 1, 1 << beta, (1 << (beta - 1)), (1 << (beta - 1)) + 1, (1 << (beta + 1)) - 1]:
        for d in [-1, 0, 1]:
            xs.append(((k << (63 - beta)) + d) % (1 << 64))
    mask = (1 << beta) - 1
    h = (1 << (beta - 1)) - 1
    for x in xs:
        hi = x >> 32
        t = ((hi >> (31 - beta)) + mask) & 0xFFFFFFFF
        d = ((t >> 1) & mask) - h
        d_shift = (((hi + (mask << (31 - beta))) & 0xFFFFFFFF) >> (32 - beta)) - h
        ref = orc.decompose(x, beta, 1)[0]
        ref = ref - (1 << 64) if ref >= (1 << 63) else ref
        assert d == ref, (hex(x), d, ref)
        assert d_shift == ref, (hex(x), d_shift, ref)


def test_exact_multi_bit_pbs_vs_fft_oracle(orc):
    """The FFT-free multi-bit PBS (exact standard-domain keybundles, exact external products)
    against the FFT oracle's multi-bit PBS: with ONE group (n = g) both start from the same
    accumulator and digits, so every output coefficient must agree within the reference FFT
    product tolerance (fft/tests.rs:166-172) times the 2^g GGSWs a keybundle sums; with several
    groups the two decrypt identically."""
    from noise_tools import external_product_tolerance, modular_distance
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS as MB

    g, N = MB.grouping_factor, MB.polynomial_size
    for n, seed in ((g, 61), (4 * g, 62)):
        p = MB.with_(lwe_dimension=n)
        lwe_sk = orc.binary_key(seed, 1, n)
        glwe_sk = orc.binary_key(seed, 2, N)
        bsk = orc.gen_mb_bsk(seed, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, g, p.glwe_modular_std_dev,
                             threads=8)
        fb = orc.MultiBitFourierBsk(bsk, n, 1, N, p.pbs_base_log, p.pbs_level, g)
        acc = orc.fill_accumulator(N, 1, 4, 4, lambda x: (x + 1) % 16)
        msgs = np.arange(16) % 16
        cts = orc.lwe_encrypt(seed + 1, lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
        fft = fb.pbs(cts, acc, threads=8)
        exact = orc.exact_mb_pbs(bsk, n, 1, N, p.pbs_base_log, p.pbs_level, g, cts, acc, threads=8)
        for out in (fft, exact):
            assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, out), p.delta) % 16, (msgs + 1) % 16)
        if n == g:
            worst = int(modular_distance(fft, exact).max())
            assert 0 < worst <= (1 << g) * external_product_tolerance(p)
