"""GPU seeded-key decompression against the oracle, bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device_to_host(ptr, nbytes):
    import ctypes

    import torch  # noqa: F401  (loads libamdhip64)

    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(nbytes // 8, dtype=np.uint64)
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0
    return out


@pytest.mark.parametrize("words", [1, 2, 3, 64, 1001, 100003])
def test_gpu_mask_stream_matches_oracle(orc, words):
    from tfhe_mi355 import Engine
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    eng = Engine(P, 0)
    for seed in (0, 0x0123456789ABCDEF_FEDCBA9876543210, (1 << 128) - 1):
        assert np.array_equal(eng.csprng_mask_words(seed, words), orc.seeded_mask_words(seed, 0, words))


@pytest.mark.parametrize("name", ["PARAM_MESSAGE_2_CARRY_2_KS_PBS", "MANTICORE_PARAMETERS",
                                  "PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS",
                                  "GADGET_AES_PARAMETERS_40"])
def test_seeded_bsk_upload_equals_decompressed_key(orc, name):
    """Seeded upload (GPU decompression + Fourier conversion) == standard upload of the oracle's
    decompression of the same bodies (random bodies: decompression is key-agnostic)."""
    from tfhe_mi355 import Engine
    from tfhe_mi355.parameters import ALL

    P = ALL[name].with_(lwe_dimension=6)
    g = P.grouping_factor
    n_ggsw = (P.lwe_dimension // g) << g if g else P.lwe_dimension
    k, N = P.glwe_dimension, P.polynomial_size
    rng = np.random.default_rng(1)
    bodies = rng.integers(0, 2 ** 64, n_ggsw * P.pbs_level * (k + 1) * N, dtype=np.uint64)
    seed = 0x1234_5678_9ABC_DEF0_0FED_CBA9_8765_4321
    std = orc.decompress_seeded_bsk(seed, bodies, n_ggsw, P.pbs_level, k, N)
    a, b = Engine(P, 0), Engine(P, 0)
    a.upload_bootstrap_key(std)
    b.upload_seeded_bootstrap_key(bodies, seed)
    fa, fb = _device_to_host(*a.fourier_bootstrap_key()), _device_to_host(*b.fourier_bootstrap_key())
    assert np.array_equal(fa, fb)


def test_seeded_ksk_upload_and_end_to_end(orc):
    """Seeded KSK on device == oracle decompression; seeded BSK + KSK bootstrap correctly."""
    from tfhe_mi355 import Engine, client, fill_accumulator
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    lwe_sk = client.gen_binary_key(8, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(8, 2, P.big_lwe_dimension)
    bseed, kseed = 0xB5EED, 0xC5EED << 64 | 7
    bb = client.gen_seeded_bootstrap_key(1, bseed, lwe_sk, glwe_sk, 1, P.polynomial_size, P.pbs_base_log,
                                         P.pbs_level, P.glwe_modular_std_dev)
    kb = client.gen_seeded_keyswitch_key(2, kseed, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    eng = Engine(P, 0)
    eng.upload_seeded_bootstrap_key(bb, bseed)
    eng.upload_seeded_keyswitch_key(kb, kseed)
    ksk = _device_to_host(*eng.keyswitch_key_device())
    assert np.array_equal(ksk, orc.decompress_seeded_ksk(kseed, kb, P.big_lwe_dimension, P.ks_level,
                                                         P.lwe_dimension))
    msgs = np.arange(64, dtype=np.uint64) % 16
    cts = client.lwe_encrypt(4, glwe_sk, msgs * np.uint64(P.delta), P.glwe_modular_std_dev)
    out = eng.keyswitch_programmable_bootstrap(cts, fill_accumulator(P, lambda x: (3 * x + 1) % 16))
    dec = client.decode(client.lwe_decrypt(glwe_sk, out), P.delta) % 16
    assert np.array_equal(dec, (3 * msgs + 1) % 16)
