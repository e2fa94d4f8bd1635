"""The core_crypto mirror (tfhe_mi355/core_crypto.py) the way the reference tests its own entry
points: test/lwe_programmable_bootstrapping.rs:70-166 (every message of the 2_2 space through
programmable_bootstrap_lwe_ciphertext, decrypting to f(m)), test/lwe_multi_bit_programmable_
bootstrapping.rs and test/lwe_keyswitch.rs (keyswitch round trip) -- plus bit-exactness with the
oracle and the reference's dimension assertions (lwe_programmable_bootstrapping.rs:1088-1102,
lwe_keyswitch.rs:106-141) as ValueError."""
import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu


def test_programmable_bootstrap_every_message(orc, keys_2_2):
    from tfhe_mi355 import core_crypto as cc

    k, P = keys_2_2, keys_2_2.params
    fbsk = cc.convert_standard_lwe_bootstrap_key_to_fourier(k.bsk, P)
    assert (fbsk.input_lwe_dimension, fbsk.output_lwe_dimension, fbsk.glwe_size) == (742, 2048, 2)
    acc = orc.fill_accumulator(P.polynomial_size, 1, 4, 4, lambda x: (7 * x + 3) % 16)
    msgs = np.repeat(np.arange(15, -1, -1, dtype=np.uint64), 4)  # msg = 15 .. 0, several encryptions each
    cts = orc.lwe_encrypt(31, k.lwe_sk, msgs * np.uint64(P.delta), P.lwe_modular_std_dev)
    outs = np.zeros((msgs.size, P.big_lwe_dimension + 1), dtype=np.uint64)
    for i in range(msgs.size):   # one ciphertext per call, as the reference's loop
        cc.programmable_bootstrap_lwe_ciphertext(cts[i], outs[i], acc, fbsk)
    assert np.array_equal(decode(orc.lwe_decrypt(k.glwe_sk, outs), P.delta) % 16, (7 * msgs + 3) % 16)
    assert np.array_equal(outs, k.fbsk.pbs(cts, acc, threads=16))
    assert np.array_equal(cc.programmable_bootstrap_lwe_ciphertext_batch(cts, acc, fbsk), outs)
    with pytest.raises(ValueError, match="input LweDimension"):
        cc.programmable_bootstrap_lwe_ciphertext(cts[0][:-1], outs[0], acc, fbsk)
    with pytest.raises(ValueError, match="output LweDimension"):
        cc.programmable_bootstrap_lwe_ciphertext(cts[0], outs[0][:-1], acc, fbsk)
    with pytest.raises(ValueError, match="multi-bit"):
        cc.multi_bit_programmable_bootstrap_lwe_ciphertext(cts[0], outs[0], acc, fbsk)


def test_multi_bit_programmable_bootstrap(orc, keys_mb):
    from tfhe_mi355 import core_crypto as cc

    k, P = keys_mb, keys_mb.params
    bsk = cc.convert_standard_lwe_bootstrap_key_to_fourier(k.bsk, P)
    acc = orc.fill_accumulator(P.polynomial_size, 1, 4, 4, lambda x: (x + 5) % 16)
    msgs = np.arange(16, dtype=np.uint64)
    cts = orc.lwe_encrypt(32, k.lwe_sk, msgs * np.uint64(P.delta), P.lwe_modular_std_dev)
    outs = np.zeros((16, P.big_lwe_dimension + 1), dtype=np.uint64)
    again = np.zeros_like(outs)
    for i in range(16):  # run twice for determinism, as lwe_multi_bit_programmable_bootstrapping.rs:9-10
        cc.multi_bit_programmable_bootstrap_lwe_ciphertext(cts[i], outs[i], acc, bsk, thread_count=7)
        cc.multi_bit_programmable_bootstrap_lwe_ciphertext(cts[i], again[i], acc, bsk, thread_count=7)
    assert np.array_equal(outs, again)
    assert np.array_equal(decode(orc.lwe_decrypt(k.glwe_sk, outs), P.delta) % 16, (msgs + 5) % 16)
    assert np.array_equal(outs, k.fbsk.pbs(cts, acc, threads=16))


def test_keyswitch_round_trip(orc, keys_2_2):
    from tfhe_mi355 import core_crypto as cc

    k, P = keys_2_2, keys_2_2.params
    ksk = cc.upload_keyswitch_key(k.ksk, P)
    assert (ksk.input_key_lwe_dimension, ksk.output_key_lwe_dimension) == (2048, 742)
    msgs = np.arange(16, dtype=np.uint64)
    big = orc.lwe_encrypt(33, k.glwe_sk, msgs * np.uint64(P.delta), P.glwe_modular_std_dev)
    small = np.zeros((16, P.lwe_dimension + 1), dtype=np.uint64)
    for i in range(16):
        cc.keyswitch_lwe_ciphertext(ksk, big[i], small[i])
    assert np.array_equal(decode(orc.lwe_decrypt(k.lwe_sk, small), P.delta) % 16, msgs)
    exp = orc.keyswitch(k.ksk, P.big_lwe_dimension, P.lwe_dimension, P.ks_base_log, P.ks_level, big)
    assert np.array_equal(small, exp)
    assert np.array_equal(cc.keyswitch_lwe_ciphertext_batch(ksk, big), exp)
    with pytest.raises(ValueError, match="input"):
        cc.keyswitch_lwe_ciphertext(ksk, big[0][:-1], small[0])
    with pytest.raises(ValueError, match="output"):
        cc.keyswitch_lwe_ciphertext(ksk, big[0], small[0][:-1])
