"""The latency kernel (csrc/pbs_latency.hip: one ciphertext per 8-wave workgroup, batches of at
most TFHE_MI355_LATENCY_MAX = 256 ciphertexts at N = 2048, k = 1, L = 1) against the throughput
kernel (pbs_classic_kernel, larger batches) and the oracle: bit-identical u64 outputs on the same
inputs, LUT indexes, edge bodies/masks, blind rotation without extraction, and the KS -> PBS call.
Same DAG as the oracle, so every row must be equal, not merely decrypt equal."""
import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu

SMALL, BIG = 200, 300   # <= 256 rows: latency kernel; > 256: throughput kernel


@pytest.fixture(scope="module")
def eng(keys_2_2):
    from tfhe_mi355 import Engine

    e = Engine(keys_2_2.params, 0)
    e.upload_bootstrap_key(keys_2_2.bsk)
    e.upload_keyswitch_key(keys_2_2.ksk)
    return e


def _edge_batch(keys, rows, seed):
    n = keys.params.lwe_dimension
    rng = np.random.default_rng(seed)
    cts = rng.integers(0, 2 ** 64, (rows, n + 1), dtype=np.uint64)
    cts[0, n] = np.uint64((1 << 64) - 1)   # b~ = 2N
    cts[1, n] = np.uint64(1 << 63)         # b~ = N
    cts[2, n] = 0
    cts[3, : n // 2] = 0                   # half the CMUXes are rotations by 0
    cts[4, :n] = 0
    cts[5, :n] = np.uint64((1 << 64) - 1)  # every a~ = 2N
    cts[6, :n] = np.uint64(1 << 63)        # every a~ = N
    return cts


def test_latency_equals_throughput_kernel_and_oracle(orc, keys_2_2, eng):
    fs = [lambda x: x, lambda x: (x * x) % 16, lambda x: (7 * x + 3) % 16]
    luts = np.stack([orc.fill_accumulator(2048, 1, 4, 4, f) for f in fs])
    cts = _edge_batch(keys_2_2, BIG, 41)
    idx = (np.arange(BIG) * 5 % 3).astype(np.uint32)
    thr = eng.programmable_bootstrap(cts, luts, lut_indexes=idx)               # throughput kernel
    lat = eng.programmable_bootstrap(cts[:SMALL], luts, lut_indexes=idx[:SMALL])  # latency kernel
    assert np.array_equal(lat, thr[:SMALL]), f"{np.count_nonzero(lat != thr[:SMALL])} words differ"
    sub = np.r_[0:8, 190:200]
    exp = keys_2_2.fbsk.pbs(cts[sub], luts, lut_idx=idx[sub], threads=16)
    assert np.array_equal(lat[sub], exp)


def test_latency_single_and_odd_counts_decrypt(orc, keys_2_2, eng):
    p = keys_2_2.params
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (3 * x + 1) % 16)
    for count in (1, 2, 7, 64, 255, 256):
        msgs = (np.arange(count) * 11) % 16
        cts = orc.lwe_encrypt(500 + count, keys_2_2.lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                              p.lwe_modular_std_dev)
        got = eng.programmable_bootstrap(cts, acc)
        assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.glwe_sk, got), p.delta) % 16, (3 * msgs + 1) % 16)
        if count <= 2:
            assert np.array_equal(got, keys_2_2.fbsk.pbs(cts, acc, threads=2))


def test_latency_blind_rotate_equals_throughput(orc, keys_2_2, eng):
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: 15 - x)
    cts = _edge_batch(keys_2_2, BIG, 43)
    thr = eng.blind_rotate(cts, acc)
    lat = eng.blind_rotate(cts[:SMALL], acc)
    assert np.array_equal(lat, thr[:SMALL])


def test_latency_keyswitch_pbs_equals_throughput(orc, keys_2_2, eng):
    p = keys_2_2.params
    msgs = np.arange(BIG) % 16
    big = orc.lwe_encrypt(45, keys_2_2.glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.glwe_modular_std_dev)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 5) % 16)
    thr = eng.keyswitch_programmable_bootstrap(big, acc)
    lat = eng.keyswitch_programmable_bootstrap(big[:SMALL], acc)
    assert np.array_equal(lat, thr[:SMALL])
    assert np.array_equal(decode(orc.lwe_decrypt(keys_2_2.glwe_sk, lat), p.delta) % 16, (msgs[:SMALL] + 5) % 16)
