"""The GPU PBS against the FFT-FREE exact oracle (oracle/pbs_oracle.c 'FFT-free exact PBS':
blind rotation bootstrap.rs:243-344 and external product ggsw.rs:477-598 with exact negacyclic
products over Z/2^64 from the standard-domain BSK).  This pins the engine to reference semantics
independently of the FFT DAG the engine and the FFT oracle share.

1. One CMUX at the real shapes (2_2 with its full n = 742 key, MANTICORE N = 1024 L = 2, 4_4
   N = 32768 L = 2): from the same accumulator the decomposition digits are identical, so every
   output coefficient must be within the reference's FFT product tolerance (fft/tests.rs:166-172,
   2^(64-(52-int_bits-log2 N)) per product, int_bits = base_log - 1 for the signed digits) summed
   over the (k+1)L products of an output column.
2. Whole bootstraps: once an FFT rounding moves a coefficient across a digit boundary the two
   computations take different (equally valid) digit paths, so coefficients are no longer
   comparable; what must hold is that every output decrypts identically and that the output
   noise distribution matches the exact one (port of noise_distribution/lwe_encryption_noise.rs:
   variance within 1/16), up to the extra variance the reference's own FFT tolerance admits
   (n CMUXes x (1 + kN/2) coefficient errors of variance <= T^2/3 each in the phase).  The
   measured excess is predicted by the single-CMUX error: excess = n (1 + kN/2) rms^2 (the FFT
   noise term of TFHE, which the reference's concrete-fft path carries too); the test checks it
   within a factor 2 (n = 64, 2048 samples; n = 742, 1024 samples).
"""
import numpy as np
import pytest

from conftest import decode
from noise_tools import RELATIVE_TOLERANCE, external_product_tolerance, modular_distance, torus_modular_diff, variance

pytestmark = pytest.mark.gpu

THREADS = 16


def _single_cmux_inputs(n, N, k, count, seed):
    rng = np.random.default_rng(seed)
    acc = rng.integers(0, 2 ** 64, (k + 1) * N, dtype=np.uint64)       # a random accumulator
    cts = np.zeros((count, n + 1), dtype=np.uint64)
    pos = rng.choice(n, count, replace=False)
    for c in range(count):                                              # ONE nonzero mask element
        cts[c, pos[c]] = rng.integers(1, 2 ** 64, dtype=np.uint64)
        cts[c, n] = rng.integers(0, 2 ** 64, dtype=np.uint64)
    return acc, cts


def _engine(params, bsk):
    from tfhe_mi355 import Engine

    e = Engine(params, 0)
    e.upload_bootstrap_key(bsk)
    return e


def _check_single_cmux(orc, params, bsk, glwe_out, seed, count=12):
    p = params
    n, N, k = p.lwe_dimension, p.polynomial_size, p.glwe_dimension
    acc, cts = _single_cmux_inputs(n, N, k, count, seed)
    eng = _engine(p, bsk)
    got = eng.blind_rotate(cts, acc) if glwe_out else eng.programmable_bootstrap(cts, acc)
    exact = orc.exact_pbs(bsk, n, k, N, p.pbs_base_log, p.pbs_level, cts, acc, threads=THREADS, glwe_out=glwe_out)
    eng.close()
    dist = modular_distance(got, exact)
    tol = external_product_tolerance(p)
    worst = int(dist.max())
    print(f"{p.name}: max |GPU - exact| = 2^{np.log2(max(worst, 1)):.1f}, tolerance 2^{tol.bit_length() - 1}")
    assert worst <= tol
    assert worst > 0  # the FFT path is not secretly exact arithmetic
    return float(np.sqrt(np.mean((dist.astype(np.float64) / 2.0 ** 64) ** 2)))


def test_single_cmux_2_2_full_key_within_reference_fft_tolerance(orc, keys_2_2):
    _check_single_cmux(orc, keys_2_2.params, keys_2_2.bsk, True, 41)


def test_single_cmux_manticore_within_reference_fft_tolerance(orc, keys_manticore):
    _check_single_cmux(orc, keys_manticore.params, keys_manticore.bsk, True, 42)


def test_single_cmux_4_4_n32768_within_reference_fft_tolerance(orc):
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import PARAM_MESSAGE_4_CARRY_4_KS_PBS

    p = PARAM_MESSAGE_4_CARRY_4_KS_PBS.with_(lwe_dimension=4)
    lwe_sk = client.gen_binary_key(43, 1, 4)
    glwe_sk = client.gen_binary_key(43, 2, p.big_lwe_dimension)
    bsk = client.gen_bootstrap_key(44, lwe_sk, glwe_sk, 1, p.polynomial_size, p.pbs_base_log, p.pbs_level,
                                   p.glwe_modular_std_dev)
    _check_single_cmux(orc, p, bsk, False, 45, count=4)   # sample-extracted (no glwe_out at N = 32768)


@pytest.mark.parametrize("name", ["PARAM_MESSAGE_1_CARRY_4_KS_PBS",    # N = 4096, L = 2 (top radix 2)
                                  "PARAM_MESSAGE_3_CARRY_3_KS_PBS",    # N = 8192, L = 2 (top radix 4)
                                  "PARAM_MESSAGE_1_CARRY_6_KS_PBS"])   # N = 16384, L = 3 (64-bit digits)
def test_single_cmux_split_within_reference_fft_tolerance(orc, name):
    """The split CMUX (pbs_large.hip, [R | 16, 16, 4] DAG) against the exact product, one CMUX."""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import SHORTINT_ALL

    p = SHORTINT_ALL[name].with_(lwe_dimension=4)
    lwe_sk = client.gen_binary_key(46, 1, 4)
    glwe_sk = client.gen_binary_key(46, 2, p.big_lwe_dimension)
    bsk = client.gen_bootstrap_key(47, lwe_sk, glwe_sk, 1, p.polynomial_size, p.pbs_base_log, p.pbs_level,
                                   p.glwe_modular_std_dev)
    _check_single_cmux(orc, p, bsk, False, 48, count=4)


def test_single_group_multibit_n8192_within_reference_fft_tolerance(orc):
    """Multi-bit g = 3 at N = 8192, L = 2 (PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3, the paired
    sub-block kernel): one group against the exact keybundle and external product."""
    from tfhe_mi355 import Engine, client
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS as MB

    g, N = MB.grouping_factor, MB.polynomial_size
    p = MB.with_(lwe_dimension=g)
    lwe_sk = client.gen_binary_key(73, 1, g)
    glwe_sk = client.gen_binary_key(73, 2, N)
    bsk = client.gen_multi_bit_bootstrap_key(74, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, g,
                                             p.glwe_modular_std_dev, threads=THREADS)
    rng = np.random.default_rng(75)
    acc = rng.integers(0, 2 ** 64, 2 * N, dtype=np.uint64)
    cts = rng.integers(0, 2 ** 64, (6, g + 1), dtype=np.uint64)
    eng = Engine(p, 0)
    eng.upload_bootstrap_key(bsk)
    got = eng.programmable_bootstrap(cts, acc)
    eng.close()
    exact = orc.exact_mb_pbs(bsk, g, 1, N, p.pbs_base_log, p.pbs_level, g, cts, acc, threads=THREADS)
    tol = (1 << g) * external_product_tolerance(p)
    worst = int(modular_distance(got, exact).max())
    print(f"multi-bit N={N} g={g}: max |GPU - exact| = 2^{np.log2(max(worst, 1)):.1f}, tolerance 2^{tol.bit_length() - 1}")
    assert 0 < worst <= tol


def _noise(orc, glwe_sk, out, msgs, delta):
    ph = orc.lwe_decrypt(glwe_sk, out)
    return torus_modular_diff(ph, np.asarray(msgs, dtype=np.uint64) * np.uint64(delta)), ph


def _compare_noise(orc, p, lwe_sk, glwe_sk, bsk, B, seed, rel_tol, band):
    rms = _check_single_cmux(orc, p, bsk, True, seed + 1, count=8)   # FFT error of one CMUX, this key
    eng = _engine(p, bsk)
    msgs = np.random.default_rng(seed).integers(0, 16, B).astype(np.uint64)
    cts = orc.lwe_encrypt(seed, lwe_sk, msgs * np.uint64(p.delta), p.lwe_modular_std_dev)
    acc = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: x)
    got = eng.programmable_bootstrap(cts, acc)
    eng.close()
    exact = orc.exact_pbs(bsk, p.lwe_dimension, 1, p.polynomial_size, p.pbs_base_log, p.pbs_level, cts, acc,
                          threads=THREADS)
    e_gpu, ph_gpu = _noise(orc, glwe_sk, got, msgs, p.delta)
    e_exact, ph_exact = _noise(orc, glwe_sk, exact, msgs, p.delta)
    assert np.array_equal(decode(ph_gpu, p.delta) % 16, msgs)
    assert np.array_equal(decode(ph_exact, p.delta) % 16, msgs)
    v_gpu, v_exact = variance(e_gpu), variance(e_exact)
    v_diff = variance(e_gpu - e_exact)
    T = external_product_tolerance(p) / 2.0 ** 64
    fft_var_bound = p.lwe_dimension * (1 + p.big_lwe_dimension / 2) * T * T / 3
    predicted = p.lwe_dimension * (1 + p.big_lwe_dimension / 2) * rms * rms
    print(f"{p.name} n={p.lwe_dimension} B={B}: var GPU 2^{np.log2(v_gpu):.2f}, exact 2^{np.log2(v_exact):.2f}, "
          f"var(GPU - exact) 2^{np.log2(v_diff):.2f}, reference-tolerance bound 2^{np.log2(fft_var_bound):.2f}, "
          f"excess 2^{np.log2(max(v_gpu - v_exact, 1e-300)):.2f} predicted 2^{np.log2(predicted):.2f}")
    assert v_gpu > (1 - rel_tol) * v_exact
    assert v_gpu < (1 + rel_tol) * v_exact + fft_var_bound
    assert v_diff < fft_var_bound
    excess = v_gpu - v_exact
    assert predicted / band < excess < predicted * band
    return v_gpu, v_exact


def test_pbs_noise_distribution_reduced_n_vs_exact(orc):
    """2_2 GLWE parameters with a 64-dimensional input key, 2048 bootstraps."""
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS

    p = PARAM_MESSAGE_2_CARRY_2_KS_PBS.with_(lwe_dimension=64, name="2_2_n64")
    lwe_sk = orc.binary_key(51, 1, 64)
    glwe_sk = orc.binary_key(51, 2, 2048)
    bsk = orc.gen_bsk(52, lwe_sk, glwe_sk, 1, 2048, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev,
                      threads=THREADS)
    _compare_noise(orc, p, lwe_sk, glwe_sk, bsk, 2048, 53, RELATIVE_TOLERANCE, 2.0)


def test_pbs_noise_full_2_2_vs_exact(orc, keys_2_2):
    """The full PARAM_MESSAGE_2_CARRY_2 bootstrap (n = 742) on 1024 ciphertexts: every output decrypts
    like the exact one and the variances agree within 1/10.  The excess v_GPU - v_exact is the
    difference of two independent sample variances (the digit paths diverge, so the two output
    noises are uncorrelated): at B samples its standard error is about 2.6 v / sqrt(B) -- 0.27 v at
    B = 96, where a first run measured 0.19 v against the predicted 0.65 v (1.7 sigma), 0.08 v at
    B = 1024, which the factor-2 band holds."""
    k = keys_2_2
    _compare_noise(orc, k.params, k.lwe_sk, k.glwe_sk, k.bsk, 1024, 54, 0.1, 2.0)


def test_single_group_multibit_within_reference_fft_tolerance(orc):
    """Multi-bit g = 3 (BASELINE config 5 parameters) with ONE group: the GPU's fused keybundle +
    external product against the exact standard-domain keybundle and exact external product
    (orc.exact_mb_pbs).  Same accumulator and digits on both sides, so each accumulator
    coefficient must be within the reference FFT tolerance times the 2^g GGSWs a keybundle sums."""
    from tfhe_mi355 import Engine
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS as MB

    g, N = MB.grouping_factor, MB.polynomial_size
    p = MB.with_(lwe_dimension=g)
    lwe_sk = orc.binary_key(71, 1, g)
    glwe_sk = orc.binary_key(71, 2, N)
    bsk = orc.gen_mb_bsk(71, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, g, p.glwe_modular_std_dev,
                         threads=THREADS)
    rng = np.random.default_rng(72)
    acc = rng.integers(0, 2 ** 64, 2 * N, dtype=np.uint64)
    cts = rng.integers(0, 2 ** 64, (16, g + 1), dtype=np.uint64)
    cts[0, :g] = 0  # every selector's monomial is X^0
    eng = Engine(p, 0)
    eng.upload_bootstrap_key(bsk)
    got = eng.blind_rotate(cts, acc)
    got_lwe = eng.programmable_bootstrap(cts, acc)
    eng.close()
    exact = orc.exact_mb_pbs(bsk, g, 1, N, p.pbs_base_log, p.pbs_level, g, cts, acc, threads=THREADS, glwe_out=True)
    exact_lwe = orc.exact_mb_pbs(bsk, g, 1, N, p.pbs_base_log, p.pbs_level, g, cts, acc, threads=THREADS)
    tol = (1 << g) * external_product_tolerance(p)
    for a, b in ((got, exact), (got_lwe, exact_lwe)):
        worst = int(modular_distance(a, b).max())
        print(f"multi-bit g={g}: max |GPU - exact| = 2^{np.log2(max(worst, 1)):.1f}, tolerance 2^{tol.bit_length() - 1}")
        assert 0 < worst <= tol
