"""Serialized server keys onto the GPU: a CompressedServerKey decompresses into the
same engine keys as the seeded uploads, and a ServerKey's Fourier BSK (natural DFT order, the
oracle's transform) lands in the engine layout so that its bootstraps are bit-exact with the
oracle's.  Keys are written by tfhe_mi355.serialization (byte layout pinned by
tests/test_serialization.py); parity unpinned against real tfhe-rs bytes (none in the reference)."""
import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu


def _device_words(ptr, nbytes):
    import ctypes

    import torch  # noqa: F401  (loads libamdhip64)

    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(nbytes // 8, dtype=np.uint64)
    assert hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 2) == 0
    return out


def test_compressed_server_key_decompress_and_bootstrap():
    """2_2: seeded keys from the engine's client side, serialized, decompressed on the GPU: the
    resident keys equal the seeded uploads' and the bootstraps decrypt."""
    from tfhe_mi355 import Engine, client, fill_accumulator, serialization, shortint
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    lwe_sk = client.gen_binary_key(21, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(21, 2, P.big_lwe_dimension)
    bseed, kseed = (0xB5 << 64) | 0x5EED, 0xC0FFEE
    bb = client.gen_seeded_bootstrap_key(1, bseed, lwe_sk, glwe_sk, P.glwe_dimension, P.polynomial_size,
                                         P.pbs_base_log, P.pbs_level, P.glwe_modular_std_dev)
    kb = client.gen_seeded_keyswitch_key(2, kseed, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    data = serialization.serialize_compressed_server_key(P, kb, kseed, bb, bseed)

    sks = shortint.CompressedServerKey.deserialize(data).decompress(0)
    assert sks.parameters == P
    ref = Engine(P, 0)
    ref.upload_seeded_bootstrap_key(bb, bseed)
    ref.upload_seeded_keyswitch_key(kb, kseed)
    assert np.array_equal(_device_words(*sks.engine.fourier_bootstrap_key()), _device_words(*ref.fourier_bootstrap_key()))
    assert np.array_equal(_device_words(*sks.engine.keyswitch_key_device()), _device_words(*ref.keyswitch_key_device()))

    msgs = np.arange(48, dtype=np.uint64) % 16
    cts = client.lwe_encrypt(4, glwe_sk, msgs * np.uint64(P.delta), P.glwe_modular_std_dev)
    out = sks.engine.keyswitch_programmable_bootstrap(cts, fill_accumulator(P, lambda x: (5 * x + 2) % 16))
    assert np.array_equal(decode(client.lwe_decrypt(glwe_sk, out), P.delta) % 16, (5 * msgs + 2) % 16)


def test_compressed_multi_bit_server_key_equals_seeded_upload():
    """Multi-bit (ShortintCompressedBootstrappingKey::MultiBit): random bodies (decompression is
    key-agnostic) -> the same resident keys as the seeded uploads."""
    from tfhe_mi355 import Engine, serialization, shortint
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS as P0

    P = P0.with_(lwe_dimension=12)
    rng = np.random.default_rng(7)
    ggsw = (P.lwe_dimension // 3) << 3
    bb = rng.integers(0, 2 ** 64, ggsw * P.pbs_level * 2 * P.polynomial_size, dtype=np.uint64)
    kb = rng.integers(0, 2 ** 64, P.big_lwe_dimension * P.ks_level, dtype=np.uint64)
    data = serialization.serialize_compressed_server_key(P, kb, 3, bb, 4, deterministic_execution=True)
    ck = shortint.CompressedServerKey.deserialize(data)
    assert ck.info.grouping_factor == 3 and ck.info.deterministic_execution
    sks = ck.decompress(0, parameters=P)
    ref = Engine(P, 0)
    ref.upload_seeded_bootstrap_key(bb, 4)
    ref.upload_seeded_keyswitch_key(kb, 3)
    assert np.array_equal(_device_words(*sks.engine.fourier_bootstrap_key()), _device_words(*ref.fourier_bootstrap_key()))
    assert np.array_equal(_device_words(*sks.engine.keyswitch_key_device()), _device_words(*ref.keyswitch_key_device()))


def test_compressed_server_key_wrong_context_is_rejected():
    from tfhe_mi355 import Engine, serialization
    from tfhe_mi355.parameters import MANTICORE_PARAMETERS, PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    kb = np.zeros(P.big_lwe_dimension * P.ks_level, dtype=np.uint64)
    bb = np.zeros(P.lwe_dimension * P.pbs_level * 2 * P.polynomial_size, dtype=np.uint64)
    data = serialization.serialize_compressed_server_key(P, kb, 1, bb, 2)
    eng = Engine(MANTICORE_PARAMETERS, 0)
    with pytest.raises(Exception, match="context was created with"):
        eng.upload_compressed_server_key(data)


@pytest.mark.parametrize("which", ["2_2", "mb_g3", "1_1", "1_0", "1_2"])
def test_server_key_fourier_ingestion_bit_exact_vs_oracle(orc, keys_2_2, keys_mb, which):
    """The oracle's Fourier BSK, serialized in natural DFT order (position P -> frequency
    pos_freq(P)), ingested through tfhe_mi355_server_key_upload: every bootstrap equals the
    oracle's bit for bit, and the resident key equals the GPU's own conversion of the standard key.
    1_1 (N = 512, k = 3), 1_0 (N = 256, k = 5) and 1_2 (N = 1024, k = 2) cover the small-N
    layouts of WaveFft<256> / <128> / <512>."""
    from conftest import KeySet
    from tfhe_mi355 import Engine, fill_accumulator, serialization, shortint
    from tfhe_mi355 import parameters as PS

    small = {"1_1": (PS.PARAM_MESSAGE_1_CARRY_1_KS_PBS, 31), "1_0": (PS.PARAM_MESSAGE_1_CARRY_0_KS_PBS, 32),
             "1_2": (PS.PARAM_MESSAGE_1_CARRY_2_KS_PBS, 33)}
    if which in small:
        k = KeySet(orc, small[which][0], seed=small[which][1])
    else:
        k = keys_2_2 if which == "2_2" else keys_mb
    P = k.params
    p = P.message_modulus * P.carry_modulus
    M = P.polynomial_size // 2
    four = k.fbsk.fourier().reshape(-1, M)                  # position order, reference scale
    natural = np.empty_like(four)
    natural[:, orc.pos_freq(P.polynomial_size)] = four
    data = serialization.serialize_server_key(P, k.ksk, natural)
    sks = shortint.ServerKey.deserialize(data, 0)
    ref = Engine(P, 0)
    ref.upload_bootstrap_key(k.bsk)
    assert np.array_equal(_device_words(*sks.engine.fourier_bootstrap_key()), _device_words(*ref.fourier_bootstrap_key()))

    rng = np.random.default_rng(3)
    msgs = rng.integers(0, p, 24).astype(np.uint64)
    cts = orc.lwe_encrypt(9, k.lwe_sk, msgs * np.uint64(P.delta), P.lwe_modular_std_dev)
    acc = orc.fill_accumulator(P.polynomial_size, P.glwe_dimension, P.message_modulus, P.carry_modulus,
                               lambda x: (x * x) % p)
    got = sks.engine.programmable_bootstrap(cts, acc)
    assert np.array_equal(got, k.fbsk.pbs(cts, acc, threads=16))
    assert np.array_equal(decode(orc.lwe_decrypt(k.glwe_sk, got), P.delta) % p, (msgs * msgs) % p)
