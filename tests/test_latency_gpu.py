"""The latency kernel (csrc/pbs_latency.hip: one ciphertext per 8-wave workgroup, batches of up to
three passes of one ciphertext per CU -- 768 rows on 256 CUs -- at N = 2048, k = 1, L = 1) against the throughput
kernel (pbs_classic_kernel, larger batches) and the oracle: bit-identical u64 outputs on the same
inputs, LUT indexes, edge bodies/masks, blind rotation without extraction, and the KS -> PBS call.
Same DAG as the oracle, so every row must be equal, not merely decrypt equal."""
import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu

SMALL, BIG = 200, 1100   # <= 3 x CUs rows: latency kernel; > 1024: throughput kernel (persistent grid)


def _ran(eng, f):
    """f()'s result and the kernel families it launched (the engine's kernel timer): the row counts
    above assume a device of 200 .. 366 CUs, so every test also checks the kernel that ran."""
    eng.kernel_timing(1)
    out = f()
    ran = set(eng.kernel_times())
    eng.kernel_timing(0)
    return out, ran


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
    thr, ran = _ran(eng, lambda: eng.programmable_bootstrap(cts, luts, lut_indexes=idx))  # throughput kernel
    assert "pbs_classic_kernel" in ran, ran  # (the host pipeline's ragged last chunk may take the latency kernel)
    lat, ran = _ran(eng, lambda: eng.programmable_bootstrap(cts[:SMALL], luts, lut_indexes=idx[:SMALL]))
    assert ran == {"pbs_latency_kernel"}, ran
    assert np.array_equal(lat, thr[:SMALL]), f"{np.count_nonzero(lat != thr[:SMALL])} words differ"
    sub = np.r_[0:8, 190:200]
    exp = keys_2_2.fbsk.pbs(cts[sub], luts, lut_idx=idx[sub], threads=16)
    assert np.array_equal(lat[sub], exp)


def test_latency_single_and_odd_counts_decrypt(orc, keys_2_2, eng):
    p = keys_2_2.params
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (3 * x + 1) % 16)
    for count in (1, 2, 7, 64, 255, 256, 257, 700):  # 257 and 700: two and three latency passes
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


# ---- multi-bit latency kernel (pbs_mb_latency_kernel: N = 2048, k = 1, L = 1, g = 2 / 3) ----

@pytest.fixture(scope="module")
def mb_keys(orc, keys_mb):
    """g = 3 (BASELINE config 5's set, full n = 888) and g = 2 (n reduced to 96: the kernel does not
    depend on n beyond the group count)."""
    from conftest import KeySet
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS as P2

    return {3: keys_mb, 2: KeySet(orc, P2.with_(lwe_dimension=96), seed=71)}


@pytest.mark.parametrize("g", [3, 2])
def test_mb_latency_equals_throughput_kernel_and_oracle(orc, mb_keys, g):
    """The same rows through the latency kernel (a batch of 200) and the slot-split throughput
    kernel (inside a batch of 1100), edge bodies and masks, three LUTs: every word equal; a sample of
    rows equal to the oracle's deterministic multi-bit PBS."""
    from tfhe_mi355 import Engine

    keys = mb_keys[g]
    e = Engine(keys.params, 0)
    e.upload_bootstrap_key(keys.bsk)
    fs = [lambda x: x, lambda x: (x * x) % 16, lambda x: (7 * x + 3) % 16]
    luts = np.stack([orc.fill_accumulator(2048, 1, 4, 4, f) for f in fs])
    cts = _edge_batch(keys, BIG, 47 + g)
    idx = (np.arange(BIG) * 5 % 3).astype(np.uint32)
    thr, ran = _ran(e, lambda: e.programmable_bootstrap(cts, luts, lut_indexes=idx))
    assert "pbs_multibit" in ran, ran
    lat, ran = _ran(e, lambda: e.programmable_bootstrap(cts[:SMALL], luts, lut_indexes=idx[:SMALL]))
    assert ran == {"pbs_mb_latency_kernel"}, ran
    assert np.array_equal(lat, thr[:SMALL]), f"{np.count_nonzero(lat != thr[:SMALL])} words differ"
    sub = np.r_[0:7, 199:200]
    exp = keys.fbsk.pbs(cts[sub], luts, lut_idx=idx[sub], threads=16)
    assert np.array_equal(lat[sub], exp)
    # one ciphertext (the reference's per-call pattern) and glwe output (blind rotation)
    assert np.array_equal(e.programmable_bootstrap(cts[5:6], luts[1]), e.programmable_bootstrap(cts[:BIG], luts[1])[5:6])
    br_thr = e.blind_rotate(cts, luts[2])
    assert np.array_equal(e.blind_rotate(cts[:SMALL], luts[2]), br_thr[:SMALL])
    e.close()


def test_mb_latency_decrypts_at_every_small_count(orc, mb_keys):
    keys = mb_keys[3]
    p = keys.params
    from tfhe_mi355 import Engine

    e = Engine(p, 0)
    e.upload_bootstrap_key(keys.bsk)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (5 * x + 2) % 16)
    for count in (1, 3, 64, 256):
        msgs = (np.arange(count) * 7) % 16
        cts = orc.lwe_encrypt(600 + count, keys.lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                              p.lwe_modular_std_dev)
        got = e.programmable_bootstrap(cts, acc)
        assert np.array_equal(decode(orc.lwe_decrypt(keys.glwe_sk, got), p.delta) % 16, (5 * msgs + 2) % 16)
    e.close()
