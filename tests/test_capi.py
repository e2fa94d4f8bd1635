"""C ABI checks that need no GPU: the engine library loads, exports every symbol that
include/tfhe_mi355.h declares, its ctypes signatures agree with the header, and its host-only
logic (LUT construction, client-side key generation) agrees with the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, decode, gpu_available

HEADER = os.path.join(ROOT, "include", "tfhe_mi355.h")


def header_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(tfhe_mi355_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from tfhe_mi355 import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_signatures_cover_header():
    from tfhe_mi355 import _lib

    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert bound == set(header_symbols())
    txt = open(HEADER).read()
    for name, _, args in _lib.SIGNATURES:
        m = re.search(name + r"\s*\(([^)]*)\)", txt)
        decl = m.group(1).strip()
        n_decl = 0 if decl in ("", "void") else decl.count(",") + 1
        assert n_decl == len(args), name


def test_fill_accumulator_matches_oracle(orc, params_2_2):
    from tfhe_mi355 import fill_accumulator

    for f in [lambda x: x, lambda x: (x * x) % 4, lambda x: x // 4, lambda x: 0]:
        got = fill_accumulator(params_2_2, f)
        exp = orc.fill_accumulator(2048, 1, 4, 4, f)
        assert np.array_equal(got, exp)


def test_parameter_sets_match_reference_constants():
    from tfhe_mi355 import parameters as P

    p = P.PARAM_MESSAGE_2_CARRY_2_KS_PBS
    assert (p.lwe_dimension, p.glwe_dimension, p.polynomial_size, p.pbs_base_log, p.pbs_level,
            p.ks_base_log, p.ks_level) == (742, 1, 2048, 23, 1, 3, 5)
    q = P.PARAM_MESSAGE_4_CARRY_4_KS_PBS
    assert (q.lwe_dimension, q.polynomial_size, q.pbs_base_log, q.pbs_level, q.ks_level) == (996, 32768, 15, 2, 7)
    mb = P.PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS
    assert (mb.lwe_dimension, mb.grouping_factor, mb.pbs_base_log, mb.ks_base_log, mb.ks_level) == (888, 3, 21, 7, 2)


def test_client_bootstrap_key_is_valid_for_the_oracle(orc, params_2_2):
    """The engine's client-side BSK/KSK generator produces keys the oracle bootstraps with."""
    from tfhe_mi355 import client

    p = params_2_2
    lwe_sk = client.gen_binary_key(5, 1, p.lwe_dimension)
    glwe_sk = client.gen_binary_key(5, 2, p.big_lwe_dimension)
    assert set(np.unique(lwe_sk)) <= {0, 1} and 0.4 < lwe_sk.mean() < 0.6
    bsk = client.gen_bootstrap_key(5, lwe_sk, glwe_sk, 1, 2048, 23, 1, p.glwe_modular_std_dev, threads=8)
    fb = orc.FourierBsk(bsk, p.lwe_dimension, 1, 2048, 23, 1)
    delta = p.delta
    msgs = np.array([0, 3, 7, 12], dtype=np.uint64)
    cts = client.lwe_encrypt(9, lwe_sk, msgs * np.uint64(delta), p.lwe_modular_std_dev)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: x)
    out = fb.pbs(cts, acc, threads=4)
    assert np.array_equal(decode(client.lwe_decrypt(glwe_sk, out), delta) % 16, msgs)
    ksk = client.gen_keyswitch_key(6, glwe_sk, lwe_sk, 3, 5, p.lwe_modular_std_dev)
    big = client.lwe_encrypt(10, glwe_sk, msgs * np.uint64(delta), p.glwe_modular_std_dev)
    small = orc.keyswitch(ksk, 2048, 742, 3, 5, big)
    assert np.array_equal(decode(client.lwe_decrypt(lwe_sk, small), delta) % 16, msgs)


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU failure path")
def test_context_create_without_gpu_fails_loudly(params_2_2):
    from tfhe_mi355 import Engine, EngineError

    with pytest.raises(EngineError):
        Engine(params_2_2, 0)


def test_unsupported_parameters_are_rejected(params_2_2):
    from tfhe_mi355 import Engine, EngineError

    with pytest.raises(EngineError, match="polynomial_size"):
        Engine(params_2_2.with_(polynomial_size=3000), 0)


def test_client_multi_bit_bootstrap_key_is_valid_for_the_oracle(orc):
    """tfhe_mi355_client_gen_multi_bit_bootstrap_key (combine_key_bits layout) bootstraps
    correctly through the oracle's multi-bit PBS."""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS as p

    lwe_sk = client.gen_binary_key(7, 1, p.lwe_dimension)
    glwe_sk = client.gen_binary_key(7, 2, p.big_lwe_dimension)
    bsk = client.gen_multi_bit_bootstrap_key(7, lwe_sk, glwe_sk, 1, 2048, p.pbs_base_log, 1, 2,
                                             p.glwe_modular_std_dev, threads=8)
    assert bsk.size == (p.lwe_dimension // 2) * 4 * 4 * 2048
    fb = orc.MultiBitFourierBsk(bsk, p.lwe_dimension, 1, 2048, p.pbs_base_log, 1, 2)
    msgs = np.array([1, 6, 11, 15], dtype=np.uint64)
    cts = client.lwe_encrypt(9, lwe_sk, msgs * np.uint64(p.delta), p.lwe_modular_std_dev)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 5) % 16)
    out = fb.pbs(cts, acc, threads=4)
    assert np.array_equal(decode(client.lwe_decrypt(glwe_sk, out), p.delta) % 16, (msgs + 5) % 16)


def test_unsupported_multi_bit_parameters_are_rejected():
    from tfhe_mi355 import Engine, EngineError
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS as mb

    with pytest.raises(EngineError, match="multi-bit"):
        Engine(mb.with_(grouping_factor=5), 0)
    with pytest.raises(EngineError, match="multiple of grouping_factor"):
        Engine(mb.with_(lwe_dimension=889), 0)



@pytest.mark.parametrize("N,base_log,level,ok", [
    (8192, 15, 2, True),     # PARAM_MESSAGE_3_CARRY_3 (split CMUX, int16 digit packing)
    (8192, 16, 2, False),    # a digit of +2^15 would wrap in int16
    (32768, 16, 2, False),   # grouped N = 32768 path: 32-bit decomposition needs beta * L <= 30
    (32768, 11, 3, True),    # PARAM_MESSAGE_1_CARRY_7 (64-bit decomposition, 33 bits)
    (4096, 22, 1, True),     # one level: no packing
])
def test_context_create_validates_split_decomposition(N, base_log, level, ok):
    """tfhe_mi355_context_create checks the decomposition before touching the GPU (capi.cpp):
    base_log > 15 with more than one level is rejected at N >= 4096."""
    from tfhe_mi355 import _lib
    from tfhe_mi355._lib import TfheMi355Parameters, vp

    p = TfheMi355Parameters(800, 1, N, base_log, level, 3, 6, 4, 4, 0)
    h = vp()
    lib = _lib.load()
    rc = lib.tfhe_mi355_context_create(ctypes.byref(p), 0, ctypes.byref(h))
    msg = lib.tfhe_mi355_last_error().decode()
    if ok:
        # valid parameters get past validation: on a CPU box the first HIP call then fails
        if rc == 0:
            lib.tfhe_mi355_context_destroy(h)
        else:
            assert "decomposition" not in msg and "base_log" not in msg, msg
    else:
        assert rc == 1 and not h.value and "base_log" in msg, msg
