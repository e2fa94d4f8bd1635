"""The core_crypto mirror (tfhe_mi355/core_crypto.py) driven the way the reference's own
core_crypto tests drive the CPU functions it replaces:

  lwe_encrypt_pbs_decrypt_custom_mod            algorithms/test/lwe_programmable_bootstrapping.rs:70-164
  lwe_encrypt_multi_bit_pbs_decrypt_custom_mod  algorithms/test/lwe_multi_bit_programmable_bootstrapping.rs:74-170
  lwe_encrypt_ks_decrypt_custom_mod             algorithms/test/lwe_keyswitch.rs:8-100

Every message of the 4-bit space, one ciphertext per call into a caller-owned output, decrypted
and decoded (the reference's assertion), and here also bit-exact against the oracle.  The CPU
tests check the mirror's argument checks (the reference asserts on mismatched dimensions,
lwe_programmable_bootstrapping.rs:1088-1102, lwe_keyswitch.rs:106-141) without a GPU.
"""
from types import SimpleNamespace

import numpy as np
import pytest

from conftest import decode

NB_TESTS = 10        # lwe_programmable_bootstrapping.rs / lwe_keyswitch.rs
NB_TESTS_LIGHT = 5   # lwe_multi_bit_programmable_bootstrapping.rs:10 (each run twice for determinism)


def _stub_engine(n=742, big_dim=2048, grouping=0):
    params = SimpleNamespace(lwe_dimension=n, polynomial_size=big_dim, glwe_dimension=1, grouping_factor=grouping)
    return SimpleNamespace(n=n, big_dim=big_dim, params=params)


def test_mirror_reports_the_key_dimensions():
    from tfhe_mi355 import core_crypto as cc

    f = cc.FourierLweBootstrapKey(_stub_engine())
    assert (f.input_lwe_dimension, f.output_lwe_dimension, f.polynomial_size, f.glwe_size) == (742, 2048, 2048, 2)
    k = cc.LweKeyswitchKey(_stub_engine())
    assert (k.input_key_lwe_dimension, k.output_key_lwe_dimension) == (2048, 742)


def test_mirror_rejects_mismatched_dimensions_before_any_device_call():
    from tfhe_mi355 import core_crypto as cc

    f = cc.FourierLweBootstrapKey(_stub_engine())
    acc = np.zeros((2, 2048), dtype=np.uint64)
    with pytest.raises(ValueError, match="input LweDimension"):
        cc.programmable_bootstrap_lwe_ciphertext(np.zeros(742, np.uint64), np.zeros(2049, np.uint64), acc, f)
    with pytest.raises(ValueError, match="output LweDimension"):
        cc.programmable_bootstrap_lwe_ciphertext(np.zeros(743, np.uint64), np.zeros(2048, np.uint64), acc, f)
    with pytest.raises(ValueError, match="multi-bit key"):
        cc.multi_bit_programmable_bootstrap_lwe_ciphertext(np.zeros(743, np.uint64), np.zeros(2049, np.uint64),
                                                           acc, f)
    k = cc.LweKeyswitchKey(_stub_engine())
    with pytest.raises(ValueError, match="input LweDimension"):
        cc.keyswitch_lwe_ciphertext(k, np.zeros(743, np.uint64), np.zeros(743, np.uint64))
    with pytest.raises(ValueError, match="output LweDimension"):
        cc.keyswitch_lwe_ciphertext(k, np.zeros(2049, np.uint64), np.zeros(2049, np.uint64))


def _accumulator(orc, p):
    # generate_accumulator(N, k + 1, msg_modulus = 16, delta = 2^63 / 16, f = id) is shortint's
    # box over message x carry = 4 x 4 at this delta
    return orc.fill_accumulator(p.polynomial_size, p.glwe_dimension, 4, 4, lambda x: x)


@pytest.mark.gpu
def test_lwe_encrypt_pbs_decrypt_custom_mod(orc, keys_2_2):
    from tfhe_mi355 import core_crypto as cc
    from tfhe_mi355.parameters import TEST_PARAMS_4_BITS_NATIVE_U64 as P

    fbsk = cc.convert_standard_lwe_bootstrap_key_to_fourier(keys_2_2.bsk, P, device=0)
    acc = _accumulator(orc, P)
    msgs = np.repeat(np.arange(15, -1, -1), NB_TESTS)  # msg = 15 .. 0, NB_TESTS each
    cts = orc.lwe_encrypt(201, keys_2_2.lwe_sk, msgs.astype(np.uint64) * np.uint64(P.delta), P.lwe_modular_std_dev)
    outs = np.empty((msgs.size, fbsk.output_lwe_dimension + 1), dtype=np.uint64)
    for t in range(msgs.size):
        out = np.zeros(fbsk.output_lwe_dimension + 1, dtype=np.uint64)
        cc.programmable_bootstrap_lwe_ciphertext(cts[t], out, acc, fbsk)
        outs[t] = out
    assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.glwe_sk, outs), P.delta) % 16, msgs)
    assert np.array_equal(outs, keys_2_2.fbsk.pbs(cts, acc, threads=8))


@pytest.mark.gpu
def test_lwe_encrypt_multi_bit_pbs_decrypt_custom_mod(orc, keys_mb):
    from tfhe_mi355 import core_crypto as cc

    p = keys_mb.params
    fbsk = cc.convert_standard_lwe_bootstrap_key_to_fourier(keys_mb.bsk, p, device=0)
    acc = _accumulator(orc, p)
    msgs = np.repeat(np.arange(15, -1, -1), NB_TESTS_LIGHT)
    cts = orc.lwe_encrypt(202, keys_mb.lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    outs = np.empty((msgs.size, fbsk.output_lwe_dimension + 1), dtype=np.uint64)
    for t in range(msgs.size):
        first = np.zeros(fbsk.output_lwe_dimension + 1, dtype=np.uint64)
        second = np.zeros_like(first)
        cc.multi_bit_programmable_bootstrap_lwe_ciphertext(cts[t], first, acc, fbsk, thread_count=5)
        cc.multi_bit_programmable_bootstrap_lwe_ciphertext(cts[t], second, acc, fbsk, thread_count=5)
        assert np.array_equal(first, second)  # the reference's determinism check
        outs[t] = first
    assert np.array_equal(decode(orc.lwe_decrypt(keys_mb.glwe_sk, outs), p.delta) % 16, msgs)
    sample = np.arange(0, msgs.size, 7)
    assert np.array_equal(outs[sample], keys_mb.fbsk.pbs(cts[sample], acc, threads=8))


@pytest.mark.gpu
def test_lwe_encrypt_ks_decrypt_custom_mod(orc, keys_2_2):
    from tfhe_mi355 import core_crypto as cc
    from tfhe_mi355.parameters import TEST_PARAMS_4_BITS_NATIVE_U64 as P

    ksk = cc.upload_keyswitch_key(keys_2_2.ksk, P, device=0)
    msgs = np.repeat(np.arange(15, -1, -1), NB_TESTS)
    cts = orc.lwe_encrypt(203, keys_2_2.glwe_sk, msgs.astype(np.uint64) * np.uint64(P.delta),
                          P.glwe_modular_std_dev)
    outs = np.empty((msgs.size, ksk.output_key_lwe_dimension + 1), dtype=np.uint64)
    for t in range(msgs.size):
        out = np.zeros(ksk.output_key_lwe_dimension + 1, dtype=np.uint64)
        cc.keyswitch_lwe_ciphertext(ksk, cts[t], out)
        outs[t] = out
    assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.lwe_sk, outs), P.delta) % 16, msgs)
    assert np.array_equal(outs, cc.keyswitch_lwe_ciphertext_batch(ksk, cts))
    assert np.array_equal(outs, orc.keyswitch(keys_2_2.ksk, ksk.input_key_lwe_dimension, ksk.output_key_lwe_dimension,
                                              P.ks_base_log, P.ks_level, cts))
