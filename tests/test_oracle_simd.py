"""The CPU baseline's SIMD build of the oracle PBS (oracle/pbs_simd.c: W ciphertexts per SIMD
register) is bit-identical to the scalar oracle (oracle/pbs_oracle.c) -- the baseline leg of
bench.py times the same computation the parity tests check."""
import numpy as np
import pytest


@pytest.mark.parametrize("variant", ["v3", "v4"])
def test_simd_pbs_bit_identical_to_oracle(orc, variant):
    import ctypes
    import os

    if variant == "v4" and orc.simd_variant() != "v4":
        pytest.skip("host has no AVX-512")
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS

    p = PARAM_MESSAGE_2_CARRY_2_KS_PBS.with_(lwe_dimension=12)
    N = p.polynomial_size
    lwe_sk = orc.binary_key(7, 1, p.lwe_dimension)
    glwe_sk = orc.binary_key(7, 2, N)
    bsk = orc.gen_bsk(8, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev, threads=8)
    fb = orc.FourierBsk(bsk, p.lwe_dimension, 1, N, p.pbs_base_log, p.pbs_level)
    luts = np.stack([orc.fill_accumulator(N, 1, 4, 4, f) for f in (lambda x: x, lambda x: (3 * x + 1) % 16)])
    rng = np.random.default_rng(3)
    cts = rng.integers(0, 2 ** 64, (11, p.lwe_dimension + 1), dtype=np.uint64)  # 11: ragged lane tail
    cts[0, :p.lwe_dimension] = 0          # every CMUX of this one is a rotation by 0
    cts[1, p.lwe_dimension] = np.uint64((1 << 64) - 1)
    idx = (np.arange(11) % 2).astype(np.uint32)
    exp = fb.pbs(cts, luts, lut_idx=idx, threads=4)
    # load the requested variant explicitly (the wrapper picks by cpu flags)
    orc.build()
    L = ctypes.CDLL(os.path.join(os.path.dirname(orc.__file__), f"libpbs_simd_{variant}.so"))
    L.simd_pbs_batch.restype = ctypes.c_int
    f = fb.fourier()
    out = np.zeros_like(exp)
    u64p, u32p, f64p = orc.u64p, orc.u32p, orc.f64p
    rc = L.simd_pbs_batch(f.ctypes.data_as(f64p), ctypes.c_int(p.lwe_dimension), ctypes.c_int(1), ctypes.c_int(N),
                          ctypes.c_int(p.pbs_base_log), ctypes.c_int(p.pbs_level), cts.ctypes.data_as(u64p),
                          out.ctypes.data_as(u64p), luts.ctypes.data_as(u64p), idx.ctypes.data_as(u32p),
                          ctypes.c_size_t(11), ctypes.c_int(3))
    assert rc == 0
    assert np.array_equal(out, exp), f"{np.count_nonzero(out != exp)} words differ"
    if variant == orc.simd_variant():
        assert np.array_equal(fb.pbs_simd(cts, luts, lut_idx=idx, threads=2), exp)


def test_simd_keyswitch_bit_identical_to_oracle(orc, keys_2_2):
    p = keys_2_2.params
    rng = np.random.default_rng(4)
    cts = rng.integers(0, 2 ** 64, (5, p.big_lwe_dimension + 1), dtype=np.uint64)
    exp = orc.keyswitch(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, cts)
    got = orc.keyswitch_simd(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, cts)
    assert np.array_equal(got, exp)


def test_simd_multibit_pbs_bit_identical_to_oracle(orc):
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS as MB

    g, N, n = MB.grouping_factor, MB.polynomial_size, 9
    p = MB.with_(lwe_dimension=n)
    lwe_sk = orc.binary_key(9, 1, n)
    glwe_sk = orc.binary_key(9, 2, N)
    bsk = orc.gen_mb_bsk(9, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, g, p.glwe_modular_std_dev, threads=8)
    fb = orc.MultiBitFourierBsk(bsk, n, 1, N, p.pbs_base_log, p.pbs_level, g)
    acc = orc.fill_accumulator(N, 1, 4, 4, lambda x: (5 * x) % 16)
    rng = np.random.default_rng(10)
    cts = rng.integers(0, 2 ** 64, (11, n + 1), dtype=np.uint64)  # ragged lane tail
    cts[0, :n] = 0
    exp = fb.pbs(cts, acc, threads=4)
    assert np.array_equal(fb.pbs_simd(cts, acc, threads=3), exp)


def test_oracle_engine_simd_mode_matches_scalar(orc, keys_2_2):
    """bench.py's FheUint32-multiply CPU leg runs OracleEngine(simd=True): same words as the scalar engine."""
    p = keys_2_2.params
    acc = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: (x * x) % 16)
    rng = np.random.default_rng(11)
    cts = rng.integers(0, 2 ** 64, (9, p.big_lwe_dimension + 1), dtype=np.uint64)
    outs = []
    for simd in (False, True):
        eng = orc.OracleEngine(p, threads=4, simd=simd)
        eng.upload_bootstrap_key(keys_2_2.bsk)
        eng.upload_keyswitch_key(keys_2_2.ksk)
        outs.append(eng.keyswitch_programmable_bootstrap(cts, acc))
    assert np.array_equal(outs[0], outs[1])
