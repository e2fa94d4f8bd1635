"""GPU parity tests for the multi-bit PBS: the HIP engine through
its C ABI against the oracle's deterministic multi-bit PBS
(lwe_multi_bit_programmable_bootstrapping.rs:548-828, 1035-1128) on the same inputs.

Bar: bit-exact u64 outputs; decryption round trips at the full batch.
"""
import numpy as np
import pytest

from conftest import KeySet, decode

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine_mb(keys_mb):
    from tfhe_mi355 import Engine

    eng = Engine(keys_mb.params, 0)
    eng.upload_bootstrap_key(keys_mb.bsk)
    eng.upload_keyswitch_key(keys_mb.ksk)
    return eng


def _cts(orc, keys, msgs, seed):
    p = keys.params
    return orc.lwe_encrypt(seed, keys.lwe_sk, np.asarray(msgs, dtype=np.uint64) * np.uint64(p.delta),
                           p.lwe_modular_std_dev)


def test_multi_bit_pbs_bit_exact_vs_oracle_g3(orc, keys_mb, engine_mb):
    p = keys_mb.params
    fs = [lambda x: x, lambda x: (x * x) % 16, lambda x: (7 * x + 2) % 16]
    luts = np.stack([orc.fill_accumulator(2048, 1, 4, 4, f) for f in fs])
    msgs = np.arange(40) % 16
    idx = (np.arange(40) * 5) % 3
    cts = _cts(orc, keys_mb, msgs, 201)
    exp = keys_mb.fbsk.pbs(cts, luts, lut_idx=idx, threads=8)
    got = engine_mb.programmable_bootstrap(cts, luts, lut_indexes=idx)
    assert got.shape == exp.shape == (40, 2049)
    assert np.array_equal(got, exp), f"{np.count_nonzero(got != exp)} words differ"
    dec = decode(orc.lwe_decrypt(keys_mb.glwe_sk, got), p.delta) % 16
    assert all(dec[i] == fs[idx[i]](msgs[i]) for i in range(40))


def test_multi_bit_pbs_edge_inputs_bit_exact(orc, keys_mb, engine_mb):
    """Monomial degrees 0, N and 2N (modulus switch allows 2N), zero groups, all-ones masks."""
    n = keys_mb.params.lwe_dimension
    rng = np.random.default_rng(17)
    cts = rng.integers(0, 2 ** 64, (6, n + 1), dtype=np.uint64)
    cts[0, n] = np.uint64((1 << 64) - 1)   # b~ = 2N
    cts[1, :n] = 0                         # every keybundle = GGSW_0 + sum GGSW_sel
    cts[2, :n] = np.uint64((1 << 64) - 1)  # every a~ = 2N, sums wrap
    cts[3, : n // 2] = np.uint64(1 << 63)  # a~ = N
    cts[4, 0::3] = 0                       # one zero element per group
    cts[5, n] = 0
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (3 * x + 1) % 16)
    exp = keys_mb.fbsk.pbs(cts, acc, threads=6)
    got = engine_mb.programmable_bootstrap(cts, acc)
    assert np.array_equal(got, exp)


def test_multi_bit_keyswitch_pbs_bit_exact(orc, keys_mb, engine_mb):
    """shortint KS -> multi-bit PBS (PBSOrder::KeyswitchBootstrap) at the GROUP_3 parameters."""
    p = keys_mb.params
    msgs = np.arange(16)
    big = orc.lwe_encrypt(202, keys_mb.glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                          p.glwe_modular_std_dev)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 3) % 16)
    small = orc.keyswitch(keys_mb.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
    exp = keys_mb.fbsk.pbs(small, acc, threads=8)
    got = engine_mb.keyswitch_programmable_bootstrap(big, acc)
    assert np.array_equal(got, exp)
    assert np.array_equal(decode(orc.lwe_decrypt(keys_mb.glwe_sk, got), p.delta) % 16, (msgs + 3) % 16)


def test_multi_bit_pbs_bit_exact_g2(orc):
    from tfhe_mi355 import Engine
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS

    keys = KeySet(orc, PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS, seed=6)
    eng = Engine(keys.params, 0)
    eng.upload_bootstrap_key(keys.bsk)
    msgs = np.arange(16)
    cts = _cts(orc, keys, msgs, 203)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: 15 - x)
    exp = keys.fbsk.pbs(cts, acc, threads=8)
    got = eng.programmable_bootstrap(cts, acc)
    assert np.array_equal(got, exp)
    assert np.array_equal(decode(orc.lwe_decrypt(keys.glwe_sk, got), keys.params.delta) % 16, 15 - msgs)


def test_multi_bit_full_batch_decrypts(orc, keys_mb, engine_mb):
    """BASELINE config 5 batch (4096 per GPU): every output decrypts to f(m)."""
    p = keys_mb.params
    rng = np.random.default_rng(5)
    msgs = rng.integers(0, 16, 4096)
    cts = _cts(orc, keys_mb, msgs, 204)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x * 5 + 1) % 16)
    got = engine_mb.programmable_bootstrap(cts, acc)
    dec = decode(orc.lwe_decrypt(keys_mb.glwe_sk, got), p.delta) % 16
    assert np.array_equal(dec, (msgs * 5 + 1) % 16)
    # spot-check a sample of the batch bit-exactly against the oracle
    sel = np.arange(0, 4096, 512)
    assert np.array_equal(got[sel], keys_mb.fbsk.pbs(cts[sel], acc, threads=8))


@pytest.mark.parametrize("name", ["PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_2_KS_PBS",
                                  "PARAM_MULTI_BIT_MESSAGE_1_CARRY_1_GROUP_3_KS_PBS"])
def test_multi_bit_k3_sets_bit_exact(orc, name):
    """The N = 512, k = 3 multi-bit sets (multi_bit.rs:96,154; per-ciphertext keybundle kernel):
    KS -> PBS bit-exact against the oracle at n = 6, per-ciphertext LUTs, edge inputs, and the
    full-n set decrypting to f(m)."""
    from tfhe_mi355 import Engine, client
    from tfhe_mi355.parameters import MULTI_BIT_ALL

    for n in (6, None):
        p = MULTI_BIT_ALL[name] if n is None else MULTI_BIT_ALL[name].with_(lwe_dimension=n)
        N, k, g, space = p.polynomial_size, p.glwe_dimension, p.grouping_factor, p.message_modulus * p.carry_modulus
        lwe_sk = client.gen_binary_key(121, 1, p.lwe_dimension)
        glwe_sk = client.gen_binary_key(121, 2, p.big_lwe_dimension)
        bsk = client.gen_multi_bit_bootstrap_key(122, lwe_sk, glwe_sk, k, N, p.pbs_base_log, p.pbs_level, g,
                                                 p.glwe_modular_std_dev, threads=8)
        ksk = client.gen_keyswitch_key(123, glwe_sk, lwe_sk, p.ks_base_log, p.ks_level, p.lwe_modular_std_dev)
        eng = Engine(p, 0)
        eng.upload_bootstrap_key(bsk)
        eng.upload_keyswitch_key(ksk)
        fs = [lambda x: (x + 1) % space, lambda x: (3 * x) % space]
        luts = np.stack([orc.fill_accumulator(N, k, p.message_modulus, p.carry_modulus, f) for f in fs])
        msgs = np.arange(8) % space
        idx = (np.arange(8) % 2).astype(np.uint32)
        big = orc.lwe_encrypt(124, glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.glwe_modular_std_dev)
        out = eng.keyswitch_programmable_bootstrap(big, luts, lut_indexes=idx)
        assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, out), p.delta) % space,
                              [fs[i](m) for i, m in zip(idx, msgs)])
        if n is not None:
            fb = orc.MultiBitFourierBsk(bsk, p.lwe_dimension, k, N, p.pbs_base_log, p.pbs_level, g)
            small = orc.keyswitch(ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
            assert np.array_equal(out, fb.pbs(small, luts, lut_idx=idx, threads=8)), f"{name}: KS -> PBS differs"
            edge = np.random.default_rng(12).integers(0, 2 ** 64, (3, p.lwe_dimension + 1), dtype=np.uint64)
            edge[0, :-1] = 0
            edge[1, :-1] = np.uint64(1 << 63)
            assert np.array_equal(eng.programmable_bootstrap(edge, luts[1]), fb.pbs(edge, luts[1], threads=3))
