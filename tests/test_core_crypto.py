"""The core_crypto mirror (tfhe_mi355/core_crypto.py) without a GPU: the key dimensions it reports
and its argument checks, which fire before any device call (the reference asserts on mismatched
dimensions, lwe_programmable_bootstrapping.rs:1088-1102, lwe_keyswitch.rs:106-141).  The GPU side
is tests/test_core_crypto_gpu.py.
"""
from types import SimpleNamespace

import numpy as np
import pytest


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
