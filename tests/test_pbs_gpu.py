"""GPU parity tests: the HIP engine (through its C ABI) against the oracle on the same inputs.

Bar: bit-exact u64 outputs (PBS, KS, KS->PBS, PBS->KS), plus decryption round trips at the
reference's test shapes and at BASELINE.json's full batch (size-independent properties).
"""
import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine_2_2(keys_2_2):
    from tfhe_mi355 import Engine

    eng = Engine(keys_2_2.params, 0)
    eng.upload_bootstrap_key(keys_2_2.bsk)
    eng.upload_keyswitch_key(keys_2_2.ksk)
    return eng


def _small_cts(orc, keys, msgs, seed, delta):
    return orc.lwe_encrypt(seed, keys.lwe_sk, np.asarray(msgs, dtype=np.uint64) * np.uint64(delta),
                           keys.params.lwe_modular_std_dev)


def test_pbs_bit_exact_vs_oracle_2_2(orc, keys_2_2, engine_2_2):
    p = keys_2_2.params
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: x)
    msgs = np.arange(32) % 16
    cts = _small_cts(orc, keys_2_2, msgs, 101, p.delta)
    exp = keys_2_2.fbsk.pbs(cts, acc, threads=8)
    got = engine_2_2.programmable_bootstrap(cts, acc)
    assert got.shape == exp.shape
    assert np.array_equal(got, exp), f"{np.count_nonzero(got != exp)} words differ"
    assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.glwe_sk, got), p.delta) % 16, msgs)


def test_pbs_multi_lut_indexes_bit_exact(orc, keys_2_2, engine_2_2):
    p = keys_2_2.params
    fs = [lambda x: x, lambda x: (x * x) % 16, lambda x: (3 * x + 1) % 16, lambda x: 15 - x]
    luts = np.stack([orc.fill_accumulator(2048, 1, 4, 4, f) for f in fs])
    msgs = np.arange(24) % 16
    idx = (np.arange(24) * 7) % 4
    cts = _small_cts(orc, keys_2_2, msgs, 102, p.delta)
    exp = keys_2_2.fbsk.pbs(cts, luts, lut_idx=idx, threads=8)
    got = engine_2_2.programmable_bootstrap(cts, luts, lut_indexes=idx)
    assert np.array_equal(got, exp)
    dec = decode(orc.lwe_decrypt(keys_2_2.glwe_sk, got), p.delta) % 16
    assert all(dec[i] == fs[idx[i]](msgs[i]) for i in range(24))


def test_pbs_edge_inputs_bit_exact(orc, keys_2_2, engine_2_2):
    """modulus-switched body/mask at 0, N, 2N (common.rs:18-25 allows 2N), zero mask entries
    (skipped CMUX, bootstrap.rs:285), trivial-looking inputs."""
    n = keys_2_2.params.lwe_dimension
    rng = np.random.default_rng(7)
    cts = rng.integers(0, 2 ** 64, (6, n + 1), dtype=np.uint64)
    cts[0, n] = np.uint64((1 << 64) - 1)   # b~ = 2N
    cts[1, n] = np.uint64(1 << 63)         # b~ = N
    cts[2, n] = 0
    cts[3, : n // 2] = 0                   # half of the CMUXes skipped
    cts[4, :n] = 0                         # every CMUX skipped
    cts[5, :n] = np.uint64((1 << 64) - 1)  # every a~ = 2N
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (5 * x + 3) % 16)
    exp = keys_2_2.fbsk.pbs(cts, acc, threads=6)
    got = engine_2_2.programmable_bootstrap(cts, acc)
    assert np.array_equal(got, exp)


def test_pbs_empty_and_single_batch(orc, keys_2_2, engine_2_2):
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: x)
    out = engine_2_2.programmable_bootstrap(np.zeros((0, 743), dtype=np.uint64), acc)
    assert out.shape == (0, 2049)
    ct = _small_cts(orc, keys_2_2, [9], 103, keys_2_2.params.delta)
    assert np.array_equal(engine_2_2.programmable_bootstrap(ct, acc), keys_2_2.fbsk.pbs(ct, acc, threads=1))


def test_keyswitch_bit_exact_vs_oracle(orc, keys_2_2, engine_2_2):
    p = keys_2_2.params
    msgs = np.arange(100) % 16
    big = orc.lwe_encrypt(104, keys_2_2.glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                          p.glwe_modular_std_dev)
    exp = orc.keyswitch(keys_2_2.ksk, 2048, 742, 3, 5, big)
    got = engine_2_2.keyswitch(big)
    assert np.array_equal(got, exp)
    assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.lwe_sk, got), p.delta) % 16, msgs)
    rnd = np.random.default_rng(3).integers(0, 2 ** 64, (70, 2049), dtype=np.uint64)  # ragged tile
    assert np.array_equal(engine_2_2.keyswitch(rnd), orc.keyswitch(keys_2_2.ksk, 2048, 742, 3, 5, rnd))


@pytest.mark.parametrize("count", [1, 2, 63, 64, 65, 200])
def test_keyswitch_split_k_counts_bit_exact(orc, keys_2_2, engine_2_2, count):
    """Small batches split the MFMA keyswitch's K over workgroups and sum the partial products
    with 64-bit atomics (keyswitch.hip): every count around the 64-row tile, random rows."""
    rnd = np.random.default_rng(40 + count).integers(0, 2 ** 64, (count, 2049), dtype=np.uint64)
    assert np.array_equal(engine_2_2.keyswitch(rnd), orc.keyswitch(keys_2_2.ksk, 2048, 742, 3, 5, rnd))


def test_keyswitch_programmable_bootstrap_shortint_order(orc, keys_2_2, engine_2_2):
    """PBSOrder::KeyswitchBootstrap (server_key/mod.rs:783-857): big-key in, big-key out."""
    p = keys_2_2.params
    msgs = np.arange(16)
    big = orc.lwe_encrypt(105, keys_2_2.glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                          p.glwe_modular_std_dev)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x * x) % 4)
    exp = keys_2_2.fbsk.pbs(orc.keyswitch(keys_2_2.ksk, 2048, 742, 3, 5, big), acc, threads=8)
    got = engine_2_2.keyswitch_programmable_bootstrap(big, acc)
    assert np.array_equal(got, exp)
    assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.glwe_sk, got), p.delta) % 16, (msgs * msgs) % 4)


def test_programmable_bootstrap_keyswitch_order(orc, keys_2_2, engine_2_2):
    p = keys_2_2.params
    msgs = np.arange(16)
    cts = _small_cts(orc, keys_2_2, msgs, 106, p.delta)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 5) % 16)
    exp = orc.keyswitch(keys_2_2.ksk, 2048, 742, 3, 5, keys_2_2.fbsk.pbs(cts, acc, threads=8))
    got = engine_2_2.programmable_bootstrap_keyswitch(cts, acc)
    assert np.array_equal(got, exp)


def test_manticore_n1024_two_levels_bit_exact(orc, keys_manticore):
    from tfhe_mi355 import Engine

    p = keys_manticore.params
    eng = Engine(p, 0)
    eng.upload_bootstrap_key(keys_manticore.bsk)
    delta = (1 << 63) // 4
    acc = orc.fill_accumulator(1024, 1, 2, 2, lambda x: (x + 1) % 4)
    msgs = np.arange(16) % 4
    cts = orc.lwe_encrypt(107, keys_manticore.lwe_sk, msgs.astype(np.uint64) * np.uint64(delta),
                          p.lwe_modular_std_dev)
    exp = keys_manticore.fbsk.pbs(cts, acc, threads=8)
    got = eng.programmable_bootstrap(cts, acc)
    assert np.array_equal(got, exp)
    assert np.array_equal(decode(orc.lwe_decrypt(keys_manticore.glwe_sk, got), delta) % 4, (msgs + 1) % 4)


def test_async_device_api_matches_sync(orc, keys_2_2, engine_2_2):
    import torch

    p = keys_2_2.params
    msgs = np.arange(40) % 16
    cts = _small_cts(orc, keys_2_2, msgs, 108, p.delta)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: x)
    d_in = torch.from_numpy(cts.view(np.int64)).cuda()
    d_out = torch.zeros((40, 2049), dtype=torch.int64, device="cuda")
    d_lut = torch.from_numpy(acc.view(np.int64)).cuda()
    engine_2_2.programmable_bootstrap_async(d_in, d_out, d_lut, 1, 40)
    torch.cuda.synchronize()
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), engine_2_2.programmable_bootstrap(cts, acc))


def test_full_batch_4096_decrypts_and_is_deterministic(orc, keys_2_2, engine_2_2):
    """BASELINE config 2 (4096 independent PBS, identity LUT): every output decrypts to its input
    and two runs are bit-identical; a sample is checked bit-exact against the oracle."""
    p = keys_2_2.params
    B = 4096
    msgs = np.random.default_rng(2).integers(0, 16, B)
    cts = _small_cts(orc, keys_2_2, msgs, 2, p.delta)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: x)
    out1 = engine_2_2.programmable_bootstrap(cts, acc)
    out2 = engine_2_2.programmable_bootstrap(cts, acc)
    assert np.array_equal(out1, out2)
    assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.glwe_sk, out1), p.delta) % 16, msgs)
    sample = np.arange(0, B, 257)
    assert np.array_equal(out1[sample], keys_2_2.fbsk.pbs(cts[sample], acc, threads=8))


def test_shortint_api_end_to_end():
    """shortint gen_keys + apply_lookup_table (server_key/mod.rs:383-476 doc examples)."""
    from tfhe_mi355 import shortint
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS

    ck, sk = shortint.gen_keys(PARAM_MESSAGE_2_CARRY_2_KS_PBS, seed=3)
    ct = ck.encrypt(3)
    acc = sk.generate_lookup_table(lambda x: x ** 2 % 4)
    assert ck.decrypt(sk.apply_lookup_table(ct, acc)) == 1
    acc3 = sk.generate_msg_lookup_table(lambda x: x * x * x, 4)
    assert ck.decrypt(sk.apply_lookup_table(ct, acc3)) == 3
    cts = ck.encrypt_many(range(4))
    res = sk.apply_lookup_table_batch(cts, [acc, acc3, acc, acc3])
    assert [ck.decrypt(c) for c in res] == [0, 1, 0, 3]
    triv = sk.create_trivial(2)
    sk.apply_lookup_table_assign(triv, acc)
    assert ck.decrypt(triv) == 0


def test_pinned_host_buffers_direct_dma(orc, keys_2_2, engine_2_2):
    """Page-locked caller buffers (tfhe_mi355_host_alloc) take the direct-DMA path of the
    host-pointer entry points: same outputs as pageable buffers, over several pipeline chunks and
    a ragged last chunk, for PBS and KS->PBS."""
    from tfhe_mi355 import pinned_empty

    p = keys_2_2.params
    B = 2500  # > 2 chunks of 1024 with a ragged tail
    msgs = np.random.default_rng(11).integers(0, 16, B)
    cts = _small_cts(orc, keys_2_2, msgs, 11, p.delta)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 3) % 16)
    exp = engine_2_2.programmable_bootstrap(cts, acc)
    p_in = pinned_empty(cts.shape)
    p_in[...] = cts
    p_out = pinned_empty(exp.shape)
    p_out[...] = 0
    got = engine_2_2.programmable_bootstrap(p_in, acc, out=p_out)
    assert got is p_out
    assert np.array_equal(p_out, exp)
    # pinned input, pageable output and the reverse
    assert np.array_equal(engine_2_2.programmable_bootstrap(p_in, acc), exp)
    assert np.array_equal(engine_2_2.programmable_bootstrap(cts, acc, out=pinned_empty(exp.shape)), exp)
    big = orc.lwe_encrypt(12, keys_2_2.glwe_sk, msgs[:300].astype(np.uint64) * np.uint64(p.delta),
                          p.glwe_modular_std_dev)
    pb = pinned_empty(big.shape)
    pb[...] = big
    assert np.array_equal(engine_2_2.keyswitch_programmable_bootstrap(pb, acc, out=pinned_empty(big.shape)),
                          engine_2_2.keyswitch_programmable_bootstrap(big, acc))
