"""Multi-device contexts (tfhe_mi355_context_create_devices, SURVEY.md 8b `device_mask`): one
process reaching several GPUs through ONE context, as the reference's one process reaches its rayon
pool (shortint/engine/mod.rs:23-25; radix_parallel/mul.rs:347-407 -> shortint/server_key/mod.rs:
783-857).  The box has one GPU, so the shards are listed on device 0 more than once ({0, 0}, {0, 0,
0}): keys are replicated by device copies (and, forced, through a one-rank RCCL broadcast), batches
split over the shards' streams, small calls and submits spread over their coalescers.  Bar: every
output bit-identical to the single-device context (itself bit-exact vs the oracle in the other
tests); the 8-GPU case (RCCL over xGMI between distinct devices) is not measurable on this box.
"""
import os

import numpy as np
import pytest

from conftest import KeySet, decode

pytestmark = pytest.mark.gpu


def _engines(params, devices):
    from tfhe_mi355 import Engine

    return Engine(params, 0), Engine(params, devices=devices)


def _upload(engs, keys, ksk=True):
    for e in engs:
        e.upload_bootstrap_key(keys.bsk)
        if ksk:
            e.upload_keyswitch_key(keys.ksk)


@pytest.fixture(scope="module")
def small_2_2(orc, params_2_2):
    return KeySet(orc, params_2_2.with_(lwe_dimension=96), seed=61)


def _cts(orc, keys, count, seed, big=False):
    p = keys.params
    rng = np.random.default_rng(seed)
    msgs = rng.integers(0, p.message_modulus * p.carry_modulus, count).astype(np.uint64)
    sk = keys.glwe_sk if big else keys.lwe_sk
    std = p.glwe_modular_std_dev if big else p.lwe_modular_std_dev
    return msgs, orc.lwe_encrypt(seed, sk, msgs * np.uint64(p.delta), std)


def test_context_reports_its_shards(params_2_2):
    from tfhe_mi355 import Engine
    from tfhe_mi355._lib import EngineError

    e = Engine(params_2_2, devices=[0, 0, 0])
    assert e.device_ordinals() == [0, 0, 0]
    assert Engine(params_2_2, devices=[0]).device_ordinals() == [0]
    import ctypes

    from tfhe_mi355 import _lib

    sub, dev = ctypes.c_void_p(), ctypes.c_int(-1)
    _lib.call("tfhe_mi355_context_device_context", e._h, 1, ctypes.byref(sub), ctypes.byref(dev))
    assert sub.value and dev.value == 0
    with pytest.raises(EngineError, match="multi-device"):
        _lib.call("tfhe_mi355_context_destroy", sub)  # owned by the multi-device context
    with pytest.raises(EngineError, match="out of range"):
        _lib.call("tfhe_mi355_context_device_context", e._h, 3, ctypes.byref(sub), ctypes.byref(dev))
    with pytest.raises(EngineError, match="not visible"):
        Engine(params_2_2, devices=[0, 4096])
    e.close()


@pytest.mark.parametrize("replicate", ["auto", "rccl"])
def test_pbs_and_ks_pbs_bit_exact_vs_single_device(orc, small_2_2, replicate, monkeypatch):
    """Batched PBS / KS->PBS / PBS->KS / KS (split over 2 shards, ragged), a count-1 call (coalesced
    on one shard), every row identical to the single-device context; keys replicated by device copy
    or (forced) a one-rank RCCL broadcast into the second shard."""
    monkeypatch.setenv("TFHE_MI355_REPLICATE", replicate)
    keys = small_2_2
    p = keys.params
    single, multi = _engines(p, [0, 0])
    _upload((single, multi), keys)
    luts = np.stack([orc.fill_accumulator(p.polynomial_size, 1, 4, 4, f)
                     for f in (lambda x: x, lambda x: (3 * x + 1) % 16)])
    msgs, small = _cts(orc, keys, 301, 5)
    idx = (np.arange(301) % 3 == 0).astype(np.uint32)
    a = single.programmable_bootstrap(small, luts, idx)
    b = multi.programmable_bootstrap(small, luts, idx)
    assert np.array_equal(a, b)
    want = np.where(idx == 1, (3 * msgs + 1) % 16, msgs)
    assert np.array_equal(decode(orc.lwe_decrypt(keys.glwe_sk, b), p.delta) % 16, want)
    assert np.array_equal(multi.programmable_bootstrap(small[:1], luts), single.programmable_bootstrap(small[:1], luts))
    _, big = _cts(orc, keys, 133, 6, big=True)
    assert np.array_equal(multi.keyswitch_programmable_bootstrap(big, luts[1]),
                          single.keyswitch_programmable_bootstrap(big, luts[1]))
    assert np.array_equal(multi.keyswitch(big), single.keyswitch(big))
    assert np.array_equal(multi.programmable_bootstrap_keyswitch(small[:97], luts[0]),
                          single.programmable_bootstrap_keyswitch(small[:97], luts[0]))
    assert np.array_equal(multi.blind_rotate(small[:70], luts), single.blind_rotate(small[:70], luts))
    multi.close()
    single.close()


def test_submit_wait_spread_over_shards(orc, small_2_2):
    """64 count-1 requests of each op in flight on a 3-shard context (round robin over the shards'
    coalescers): each equal to the single-device batched call."""
    keys = small_2_2
    p = keys.params
    single, multi = _engines(p, [0, 0, 0])
    _upload((single, multi), keys)
    lut = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: (x * x) % 16)
    _, small = _cts(orc, keys, 64, 7)
    _, big = _cts(orc, keys, 64, 8, big=True)
    reqs = []
    for i in range(64):
        reqs.append(("pbs", i, multi.submit("pbs", small[i:i + 1], lut)))
        reqs.append(("ks_pbs", i, multi.submit("ks_pbs", big[i:i + 1], lut)))
        reqs.append(("ks", i, multi.submit("ks", big[i:i + 1])))
    want = {"pbs": single.programmable_bootstrap(small, lut), "ks_pbs": single.keyswitch_programmable_bootstrap(big, lut),
            "ks": single.keyswitch(big)}
    for op, i, r in reqs:
        assert np.array_equal(r.wait()[0], want[op][i]), (op, i)
    st = multi.coalesce_stats()
    assert st["rows"] >= 192 and st["batches"] >= 3
    multi.close()
    single.close()


def test_multi_bit_split_bit_exact(orc, keys_mb):
    """Multi-bit g = 3 (config 5) over 2 shards: identical to the single-device context."""
    p = keys_mb.params
    single, multi = _engines(p, [0, 0])
    _upload((single, multi), keys_mb, ksk=False)
    lut = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: (5 * x + 2) % 16)
    msgs, small = _cts(orc, keys_mb, 257, 9)
    got = multi.programmable_bootstrap(small, lut)
    assert np.array_equal(got, single.programmable_bootstrap(small, lut))
    assert np.array_equal(decode(orc.lwe_decrypt(keys_mb.glwe_sk, got), p.delta) % 16, (5 * msgs + 2) % 16)
    multi.close()
    single.close()


def test_large_4_4_chunked_split_bit_exact(orc):
    """4_4 (N = 32768, the chunked split-CMUX path) over 2 shards, 150 ciphertexts = one 128-chunk +
    ragged on shard 0's 75 and 75 on shard 1: identical to the single-device context."""
    from test_large_gpu import LargeKeys
    from tfhe_mi355.parameters import PARAM_MESSAGE_4_CARRY_4_KS_PBS

    keys = LargeKeys(orc, PARAM_MESSAGE_4_CARRY_4_KS_PBS.with_(lwe_dimension=16), 41)
    p = keys.params
    single, multi = _engines(p, [0, 0])
    for e in (single, multi):
        e.upload_bootstrap_key(keys.bsk)
    msgs = np.random.default_rng(3).integers(0, 256, 150)
    cts = keys.encrypt(orc, msgs, 77)
    acc = orc.fill_accumulator(p.polynomial_size, 1, 16, 16, lambda x: (x * 7 + 3) % 256)
    got = multi.programmable_bootstrap(cts, acc)
    assert np.array_equal(got, single.programmable_bootstrap(cts, acc))
    assert np.array_equal(decode(orc.lwe_decrypt(keys.glwe_sk, got), p.delta) % 256, (msgs * 7 + 3) % 256)
    multi.close()
    single.close()


def test_two_phase_fourier_upload_replicates_on_set_ready(orc, small_2_2):
    """The _fourier / _set_ready pair on a multi-device context: the caller fills the FIRST device's
    buffer, _set_ready replicates it to the other shards (a PBS before any key fails), and every
    shard then bootstraps like the single-device context."""
    import ctypes

    import torch
    from tfhe_mi355._lib import EngineError

    keys = small_2_2
    p = keys.params
    from tfhe_mi355 import Engine

    single = Engine(p, 0)
    single.upload_bootstrap_key(keys.bsk)
    multi = Engine(p, devices=[0, 0, 0])
    lut = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: x)
    _, small = _cts(orc, keys, 90, 10)
    with pytest.raises(EngineError, match="not uploaded"):
        multi.programmable_bootstrap(small, lut)
    ptr, nbytes = single.fourier_bootstrap_key()
    mptr, mbytes = multi.fourier_bootstrap_key()
    assert mbytes == nbytes
    hip = ctypes.CDLL("libamdhip64.so")
    tmp = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    assert hip.hipMemcpy(ctypes.c_void_p(tmp.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 3) == 0
    assert hip.hipMemcpy(ctypes.c_void_p(mptr), ctypes.c_void_p(tmp.data_ptr()), ctypes.c_size_t(nbytes), 3) == 0
    multi.fourier_bootstrap_key_set_ready()
    assert np.array_equal(multi.programmable_bootstrap(small, lut), single.programmable_bootstrap(small, lut))
    multi.close()
    single.close()


def _hip_get_device():
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    d = ctypes.c_int(-1)
    assert hip.hipGetDevice(ctypes.byref(d)) == 0
    return d.value


def test_caller_device_unchanged_and_replication_reported(orc, small_2_2, monkeypatch):
    """Every entry point leaves the calling thread's current HIP device as it found it (create_devices,
    uploads with replication, a batched split call, a coalesced call, destroy); the context reports
    how the keys were replicated: device copies for {0, 0} in auto mode, the (forced) one-rank RCCL
    broadcast with TFHE_MI355_REPLICATE=rccl."""
    keys = small_2_2
    p = keys.params
    from tfhe_mi355 import Engine

    before = _hip_get_device()
    for mode, want in (("auto", "device_copy"), ("rccl", "rccl"), ("copy", "device_copy")):
        monkeypatch.setenv("TFHE_MI355_REPLICATE", mode)
        multi = Engine(p, devices=[0, 0])
        assert _hip_get_device() == before
        assert multi.replication() == ("none", "")
        _upload((multi,), keys)
        assert _hip_get_device() == before
        assert multi.replication()[0] == want, mode
        lut = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: x)
        msgs, small = _cts(orc, keys, 40, 12)
        got = multi.programmable_bootstrap(small, lut)
        assert np.array_equal(decode(orc.lwe_decrypt(keys.glwe_sk, got), p.delta) % 16, msgs)
        multi.programmable_bootstrap(small[:1], lut)
        assert _hip_get_device() == before
        multi.close()
        assert _hip_get_device() == before
    assert Engine(p, 0).replication() == ("none", "")


def test_failed_replication_leaves_every_shard_not_uploaded(orc, small_2_2, monkeypatch):
    """a key upload whose replication fails leaves the key part not uploaded on EVERY
    shard (shard 0 included, though it holds the new key), so batched, split, coalesced and submitted
    calls all fail with 'not uploaded' rather than succeeding only where they land on shard 0; a
    later successful upload restores every shard."""
    from tfhe_mi355._lib import EngineError

    keys = small_2_2
    p = keys.params
    single, multi = _engines(p, [0, 0, 0])
    _upload((single,), keys)
    lut = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: x)
    _, small = _cts(orc, keys, 64, 13)
    monkeypatch.setenv("TFHE_MI355_REPLICATE", "fail")
    with pytest.raises(EngineError, match="test hook"):
        multi.upload_bootstrap_key(keys.bsk)
    with pytest.raises(EngineError, match="not uploaded"):
        multi.programmable_bootstrap(small, lut)  # split over the shards
    for i in range(3):  # round robin: every shard's coalescer refuses
        with pytest.raises(EngineError, match="not uploaded"):
            multi.programmable_bootstrap(small[i:i + 1], lut)
        with pytest.raises(EngineError, match="not uploaded"):
            multi.submit("pbs", small[i:i + 1], lut).wait()
    monkeypatch.setenv("TFHE_MI355_REPLICATE", "auto")
    multi.upload_bootstrap_key(keys.bsk)
    assert np.array_equal(multi.programmable_bootstrap(small, lut), single.programmable_bootstrap(small, lut))
    for i in range(3):
        assert np.array_equal(multi.programmable_bootstrap(small[i:i + 1], lut)[0],
                              single.programmable_bootstrap(small[i:i + 1], lut)[0])
    multi.close()
    single.close()


def test_key_buffer_hand_out_marks_every_shard_not_ready(orc, small_2_2):
    """handing out the first device's key buffer (bootstrap_key_fourier /
    keyswitch_key_device) on a multi-device context marks that key part not uploaded everywhere until
    _set_ready replicates the rewritten buffer; the other key part is unaffected."""
    from tfhe_mi355._lib import EngineError

    keys = small_2_2
    p = keys.params
    single, multi = _engines(p, [0, 0])
    _upload((single, multi), keys)
    lut = orc.fill_accumulator(p.polynomial_size, 1, 4, 4, lambda x: (x + 1) % 16)
    _, small = _cts(orc, keys, 50, 14)
    _, big = _cts(orc, keys, 50, 15, big=True)
    multi.fourier_bootstrap_key()
    with pytest.raises(EngineError, match="not uploaded"):
        multi.programmable_bootstrap(small, lut)
    assert np.array_equal(multi.keyswitch(big), single.keyswitch(big))  # the KSK still serves
    multi.fourier_bootstrap_key_set_ready()  # the buffer was not changed: the old key, replicated
    assert np.array_equal(multi.programmable_bootstrap(small, lut), single.programmable_bootstrap(small, lut))
    multi.keyswitch_key_device()
    with pytest.raises(EngineError, match="not uploaded"):
        multi.keyswitch(big)
    multi.keyswitch_key_set_ready()
    assert np.array_equal(multi.keyswitch_programmable_bootstrap(big, lut),
                          single.keyswitch_programmable_bootstrap(big, lut))
    multi.close()
    single.close()
