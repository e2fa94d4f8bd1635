"""GPU tests of the C ABI's runtime contract (include/tfhe_mi355.h conventions):

* concurrent _async callers sharing one context on different streams, each with its own
  caller-provided scratch, get exactly the synchronous results (reference: rayon workers sharing
  one server key, shortint/engine/mod.rs:23-25);
* keys ingested through the device (_async) forms are complete for the very next call on any
  stream, and bit-identical to host uploads;
* the host-pointer entry points' chunked two-lane pipeline returns the same bits as one device
  launch for batches spanning several chunks, with per-ciphertext LUTs;
* _async LUT indexes past lut_count are clamped (no out-of-bounds read);
* the whole FheUint32 multiply DAG captured into one hipGraph replays bit-identically.
"""
import threading

import numpy as np
import pytest

from conftest import decode

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(keys_2_2):
    from tfhe_mi355 import Engine

    e = Engine(keys_2_2.params, 0)
    e.upload_bootstrap_key(keys_2_2.bsk)
    e.upload_keyswitch_key(keys_2_2.ksk)
    return e


def _big_cts(orc, keys, msgs, seed):
    p = keys.params
    return orc.lwe_encrypt(seed, keys.glwe_sk, np.asarray(msgs, dtype=np.uint64) * np.uint64(p.delta),
                           p.glwe_modular_std_dev)


def test_two_threads_two_streams_match_sync(orc, keys_2_2, eng):
    import torch

    p = keys_2_2.params
    fs = [lambda x: x, lambda x: (5 * x + 3) % 16]
    accs = [orc.fill_accumulator(2048, 1, 4, 4, f) for f in fs]
    msgs = [np.arange(300) % 16, (np.arange(300) * 3) % 16]
    cts = [_big_cts(orc, keys_2_2, m, 500 + i) for i, m in enumerate(msgs)]
    exp = [eng.keyswitch_programmable_bootstrap(c, a) for c, a in zip(cts, accs)]
    dev = torch.device("cuda", 0)
    results = [None, None]
    errors = []

    def worker(i):
        try:
            s = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(s):
                d_in = torch.from_numpy(cts[i].view(np.int64)).to(dev)
                d_lut = torch.from_numpy(accs[i].view(np.int64)).to(dev)
                d_out = torch.zeros_like(d_in)
                scratch = torch.empty(eng.ks_pbs_scratch_bytes(300), dtype=torch.uint8, device=dev)
                for _ in range(3):   # overlap the other thread's launches
                    eng.keyswitch_programmable_bootstrap_async(d_in, d_out, d_lut, 1, 300, scratch, stream=s)
                s.synchronize()
                results[i] = d_out.cpu().numpy().view(np.uint64)
        except Exception as ex:  # pragma: no cover - reported below
            errors.append(ex)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    for i in range(2):
        assert np.array_equal(results[i], exp[i]), f"stream {i}: {np.count_nonzero(results[i] != exp[i])} words differ"
        dec = decode(orc.lwe_decrypt(keys_2_2.glwe_sk, results[i]), p.delta) % 16
        assert np.array_equal(dec, [fs[i](m) for m in msgs[i]])


def test_async_scratch_too_small_is_an_error(keys_2_2, eng):
    import torch

    from tfhe_mi355._lib import EngineError

    d_in = torch.zeros((64, 2049), dtype=torch.int64, device="cuda")
    d_out = torch.zeros_like(d_in)
    d_lut = torch.zeros(4096, dtype=torch.int64, device="cuda")
    small = torch.empty(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(EngineError, match="scratch"):
        eng.keyswitch_programmable_bootstrap_async(d_in, d_out, d_lut, 1, 64, small)


def test_device_key_ingestion_is_complete_and_bit_identical(orc, keys_2_2, eng):
    """convert_bootstrap_key_async / keyswitch_key_upload_async on torch's stream, then at once a
    synchronous call (on the context's own stream): same bits as the host-uploaded keys."""
    import torch

    from tfhe_mi355 import Engine

    p = keys_2_2.params
    e2 = Engine(p, 0)
    d_bsk = torch.from_numpy(keys_2_2.bsk.view(np.int64)).cuda()
    d_ksk = torch.from_numpy(keys_2_2.ksk.view(np.int64)).cuda()
    e2.convert_bootstrap_key_device(d_bsk, d_bsk.numel())
    e2.upload_keyswitch_key_device(d_ksk, d_ksk.numel())
    del d_bsk, d_ksk
    msgs = np.arange(64) % 16
    cts = _big_cts(orc, keys_2_2, msgs, 510)
    acc = orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 7) % 16)
    got = e2.keyswitch_programmable_bootstrap(cts, acc)
    assert np.array_equal(got, eng.keyswitch_programmable_bootstrap(cts, acc))
    e2.close()


def test_host_pipeline_multi_chunk_matches_device_launch(orc, keys_2_2, eng):
    """2500 ciphertexts = chunks of 1024, 1024, 452 over two lanes, with per-ciphertext LUTs."""
    import torch

    p = keys_2_2.params
    B = 2500
    fs = [lambda x: x, lambda x: (x * x) % 16, lambda x: 15 - x]
    luts = np.stack([orc.fill_accumulator(2048, 1, 4, 4, f) for f in fs])
    rng = np.random.default_rng(11)
    msgs = rng.integers(0, 16, B)
    idx = rng.integers(0, 3, B).astype(np.uint32)
    cts = orc.lwe_encrypt(511, keys_2_2.lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    got = eng.programmable_bootstrap(cts, luts, lut_indexes=idx)
    d_in = torch.from_numpy(cts.view(np.int64)).cuda()
    d_out = torch.zeros((B, 2049), dtype=torch.int64, device="cuda")
    d_luts = torch.from_numpy(luts.view(np.int64)).cuda()
    d_idx = torch.from_numpy(idx.view(np.int32)).cuda()
    eng.programmable_bootstrap_async(d_in, d_out, d_luts, 3, B, d_lut_indexes=d_idx)
    torch.cuda.synchronize()
    assert np.array_equal(got, d_out.cpu().numpy().view(np.uint64))
    dec = decode(orc.lwe_decrypt(keys_2_2.glwe_sk, got), p.delta) % 16
    assert all(dec[i] == fs[idx[i]](msgs[i]) for i in range(0, B, 7))
    # KS -> PBS through the same pipeline (scratch per lane)
    big = _big_cts(orc, keys_2_2, msgs[:1500], 512)
    ks_pbs = eng.keyswitch_programmable_bootstrap(big, luts[0])
    dec = decode(orc.lwe_decrypt(keys_2_2.glwe_sk, ks_pbs), p.delta) % 16
    assert np.array_equal(dec, msgs[:1500])


def test_async_lut_index_out_of_range_is_clamped(orc, keys_2_2, eng):
    import torch

    p = keys_2_2.params
    luts = np.stack([orc.fill_accumulator(2048, 1, 4, 4, f) for f in (lambda x: x, lambda x: 15 - x)])
    msgs = np.arange(8) % 16
    cts = orc.lwe_encrypt(513, keys_2_2.lwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.lwe_modular_std_dev)
    d_in = torch.from_numpy(cts.view(np.int64)).cuda()
    d_out = torch.zeros((8, 2049), dtype=torch.int64, device="cuda")
    d_luts = torch.from_numpy(luts.view(np.int64)).cuda()
    d_idx = torch.tensor([1, 7, 1000, 2, 1, 99, 3, 1 << 30], dtype=torch.int32, device="cuda")
    eng.programmable_bootstrap_async(d_in, d_out, d_luts, 2, 8, d_lut_indexes=d_idx)
    torch.cuda.synchronize()
    exp = eng.programmable_bootstrap(cts, luts, lut_indexes=np.ones(8, dtype=np.uint32))
    assert np.array_equal(d_out.cpu().numpy().view(np.uint64), exp)


def test_fheuint32_mul_dag_as_one_hipgraph(keys_2_2):
    """integer mul_parallelized captured once (every layer's LUT stack and index array cached on the
    device by the eager warm-up) and replayed: same bits as the eager run, products decrypt."""
    import torch

    from tfhe_mi355 import Engine, integer, shortint

    p = keys_2_2.params
    ck = shortint.ClientKey(p, 7)
    e = Engine(p, 0)
    from tfhe_mi355 import client

    e.upload_bootstrap_key(client.gen_bootstrap_key(8, ck.small_lwe_secret_key, ck.glwe_secret_key, 1, 2048,
                                                    p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev))
    e.upload_keyswitch_key(client.gen_keyswitch_key(9, ck.large_lwe_secret_key, ck.small_lwe_secret_key,
                                                    p.ks_base_log, p.ks_level, p.lwe_modular_std_dev))
    sks = integer.ServerKey(shortint.ServerKey(None, engine=e, parameters=p))
    cks = integer.ClientKey(ck, 16)
    rng = np.random.default_rng(4)
    a = rng.integers(0, 2 ** 32, 8, dtype=np.uint64)
    b = rng.integers(0, 2 ** 32, 8, dtype=np.uint64)
    ca, cb = sks.to_device(cks.encrypt(a)), sks.to_device(cks.encrypt(b))
    eager = sks.mul_parallelized(ca, cb)
    torch.cuda.synchronize()
    eager_bits = eager.data.cpu().numpy().copy()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = sks.mul_parallelized(ca, cb)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.data.cpu().numpy(), eager_bits)
    assert np.array_equal(cks.decrypt(out), (a * b) % np.uint64(1 << 32))
    e.close()
