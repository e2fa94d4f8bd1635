"""The drop-in under the reference's own calling pattern: one ciphertext per call, from many
threads at once (shortint keyswitch_programmable_bootstrap_assign, shortint/server_key/mod.rs:
783-857, called from rayon workers per block, integer/server_key/radix_parallel/mul.rs:347-407).

Small host-pointer calls on one context are coalesced into batches (capi.cpp "request
coalescing"): every caller must still get exactly its own rows -- bit-exact against the oracle's
keyswitch + PBS of the same ciphertext with the same LUT -- whatever the batch it landed in, with
different LUTs per caller (deduplicated by buffer), per-row LUT indexes and different ops
interleaved.
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


def _run_threads(n, fn):
    errors = []

    def wrap(i):
        try:
            fn(i)
        except Exception as ex:  # pragma: no cover - reported below
            errors.append(repr(ex))

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a caller never returned"
    assert not errors, errors[:3]


def test_16_threads_x_64_single_ciphertext_ks_pbs_bit_exact(orc, keys_2_2, eng):
    p = keys_2_2.params
    T, C = 16, 64
    fs = [lambda x, a=a: (a * x + 1) % 16 for a in (1, 3, 5, 7)]
    accs = [orc.fill_accumulator(2048, 1, 4, 4, f) for f in fs]   # 4 LUT buffers shared by 16 threads
    msgs = (np.arange(T * C) * 7) % 16
    cts = orc.lwe_encrypt(901, keys_2_2.glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                          p.glwe_modular_std_dev)
    out = np.zeros((T * C, p.big_lwe_dimension + 1), dtype=np.uint64)

    def worker(t):
        for c in range(C):
            i = t * C + c
            out[i:i + 1] = eng.keyswitch_programmable_bootstrap(cts[i:i + 1], accs[t % 4])

    _run_threads(T, worker)
    small = orc.keyswitch(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, cts)
    for a in range(4):
        rows = np.nonzero((np.arange(T * C) // C) % 4 == a)[0]
        exp = keys_2_2.fbsk.pbs(small[rows], accs[a], threads=16)
        bad = np.nonzero(np.any(out[rows] != exp, axis=1))[0]
        assert bad.size == 0, f"LUT {a}: {bad.size} of {rows.size} single-ciphertext calls differ from the oracle"
        dec = decode(orc.lwe_decrypt(keys_2_2.glwe_sk, out[rows]), p.delta) % 16
        assert np.array_equal(dec, [fs[a](m) for m in msgs[rows]])


def test_lone_caller_runs_directly_and_exactly(orc, keys_2_2):
    """One blocking caller at a time on a fresh context: every call runs at once on the calling
    thread (capi.cpp coalesced_call: a batch of its own, never counted in flight), with the same
    rows as the oracle; KS+PBS with two LUTs and a per-row index through the same path."""
    from tfhe_mi355 import Engine

    p = keys_2_2.params
    e = Engine(p, 0)
    e.upload_bootstrap_key(keys_2_2.bsk)
    e.upload_keyswitch_key(keys_2_2.ksk)
    accs = np.stack([orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 3) % 16),
                     orc.fill_accumulator(2048, 1, 4, 4, lambda x: (5 * x) % 16)])
    msgs = np.arange(6) % 16
    big = orc.lwe_encrypt(905, keys_2_2.glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                          p.glwe_modular_std_dev)
    small = orc.keyswitch(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
    e.coalesce_stats(reset=True)
    for i in range(6):
        idx = np.array([i % 2], dtype=np.uint32)
        got = e.keyswitch_programmable_bootstrap(big[i:i + 1], accs, lut_indexes=idx)
        assert np.array_equal(got, keys_2_2.fbsk.pbs(small[i:i + 1], accs[i % 2], threads=1))
        got = e.programmable_bootstrap(small[i:i + 1], accs[0])
        assert np.array_equal(got, keys_2_2.fbsk.pbs(small[i:i + 1], accs[0], threads=1))
    st = e.coalesce_stats()
    assert st["batches"] == 12 and st["rows"] == 12 and st["max_in_flight"] == 0, st


def test_mixed_ops_counts_and_lut_indexes_coalesce_exactly(orc, keys_2_2, eng):
    """Concurrent PBS, KS+PBS and KS calls of 1-5 ciphertexts, some with two LUTs and per-row
    indexes: each result equals the oracle's result of the same call made alone."""
    p = keys_2_2.params
    accs = np.stack([orc.fill_accumulator(2048, 1, 4, 4, lambda x: x),
                     orc.fill_accumulator(2048, 1, 4, 4, lambda x: 15 - x)])
    rng = np.random.default_rng(5)
    jobs = []
    for j in range(96):
        cnt = int(rng.integers(1, 6))
        msgs = rng.integers(0, 16, cnt).astype(np.uint64)
        big = orc.lwe_encrypt(1000 + j, keys_2_2.glwe_sk, msgs * np.uint64(p.delta), p.glwe_modular_std_dev)
        op = ("pbs", "ks_pbs", "ks")[j % 3]
        idx = rng.integers(0, 2, cnt).astype(np.uint32) if j % 2 else None
        jobs.append((op, big, idx))
    small_all = [orc.keyswitch(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, b)
                 for _, b, _ in jobs]

    def call(op, big, small, idx):
        luts = accs if idx is not None else accs[0]
        if op == "pbs":
            return eng.programmable_bootstrap(small, luts, idx)
        if op == "ks_pbs":
            return eng.keyswitch_programmable_bootstrap(big, luts, idx)
        return eng.keyswitch(big)

    got = [None] * len(jobs)

    def worker(t):
        for j in range(t, len(jobs), 12):
            op, big, idx = jobs[j]
            got[j] = call(op, big, small_all[j], idx)

    _run_threads(12, worker)
    # the oracle's result of each call on its own
    for j, (op, big, idx) in enumerate(jobs):
        if op == "ks":
            exp = small_all[j]
        else:
            luts = accs if idx is not None else accs[0]
            exp = keys_2_2.fbsk.pbs(small_all[j], luts, lut_idx=idx, threads=8)
        assert np.array_equal(got[j], exp), f"job {j} ({op}, {big.shape[0]} cts, idx={idx is not None}) differs"


@pytest.mark.parametrize("name", ["PARAM_MESSAGE_3_CARRY_3_KS_PBS",                     # digits-fed split CMUX
                                  "PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS",   # multi-bit paired kernel
                                  "PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS"])  # multi-bit N = 2048
def test_coalesced_single_calls_on_the_other_kernels(orc, name):
    """8 threads x 6 one-ciphertext KS+PBS calls through the coalescer at a large-N and the
    multi-bit shapes (reduced n): each caller's rows equal the same ciphertexts' rows from one
    batched call (which the parity tests pin to the oracle) and decrypt to f(m)."""
    from tfhe_mi355 import Engine, client
    from tfhe_mi355.parameters import ALL

    p = ALL[name].with_(lwe_dimension=6)
    N, k, g = p.polynomial_size, p.glwe_dimension, p.grouping_factor
    space = p.message_modulus * p.carry_modulus
    lwe_sk = client.gen_binary_key(131, 1, p.lwe_dimension)
    glwe_sk = client.gen_binary_key(131, 2, p.big_lwe_dimension)
    if g:
        bsk = client.gen_multi_bit_bootstrap_key(132, lwe_sk, glwe_sk, k, N, p.pbs_base_log, p.pbs_level, g,
                                                 p.glwe_modular_std_dev, threads=8)
    else:
        bsk = client.gen_bootstrap_key(132, lwe_sk, glwe_sk, k, N, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev)
    ksk = client.gen_keyswitch_key(133, glwe_sk, lwe_sk, p.ks_base_log, p.ks_level, p.lwe_modular_std_dev)
    e = Engine(p, 0)
    e.upload_bootstrap_key(bsk)
    e.upload_keyswitch_key(ksk)
    T, C = 8, 6
    acc = orc.fill_accumulator(N, k, p.message_modulus, p.carry_modulus, lambda x: (x + 3) % space)
    msgs = (np.arange(T * C) * 5) % space
    big = orc.lwe_encrypt(134, glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta), p.glwe_modular_std_dev)
    ref = e.keyswitch_programmable_bootstrap(big, acc)
    out = np.zeros_like(ref)

    def worker(t):
        for c in range(C):
            i = t * C + c
            out[i] = e.keyswitch_programmable_bootstrap(big[i:i + 1], acc)[0]

    _run_threads(T, worker)
    e.close()
    assert np.array_equal(out, ref)
    assert np.array_equal(decode(orc.lwe_decrypt(glwe_sk, out), p.delta) % space, (msgs + 3) % space)


def test_submit_wait_many_in_flight_from_one_thread(orc, keys_2_2, eng):
    """tfhe_mi355_submit / tfhe_mi355_wait: one thread keeps 256 one-ciphertext requests of the
    four ops in flight, then waits for all of them; each result equals the oracle's result of
    the same call made alone."""
    p = keys_2_2.params
    accs = np.stack([orc.fill_accumulator(2048, 1, 4, 4, lambda x: (x + 1) % 16),
                     orc.fill_accumulator(2048, 1, 4, 4, lambda x: (3 * x) % 16)])
    R = 256
    msgs = (np.arange(R) * 11) % 16
    big = orc.lwe_encrypt(977, keys_2_2.glwe_sk, msgs.astype(np.uint64) * np.uint64(p.delta),
                          p.glwe_modular_std_dev)
    small = orc.keyswitch(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, big)
    ops = ("ks_pbs", "pbs", "ks", "pbs_ks")
    reqs = []
    for i in range(R):
        op = ops[i % 4]
        src = big[i:i + 1] if op in ("ks_pbs", "ks") else small[i:i + 1]
        if op == "ks":
            reqs.append(eng.submit(op, src))
        else:
            reqs.append(eng.submit(op, src, accs, np.array([i % 2], dtype=np.uint32)))
    got = [r.wait() for r in reqs]
    with pytest.raises(RuntimeError):
        reqs[0].wait()
    pbs = keys_2_2.fbsk.pbs(small, accs, lut_idx=(np.arange(R) % 2).astype(np.uint32), threads=16)
    pbs_ks = orc.keyswitch(keys_2_2.ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log, p.ks_level, pbs)
    for i in range(R):
        exp = {"ks_pbs": pbs, "pbs": pbs, "ks": small, "pbs_ks": pbs_ks}[ops[i % 4]][i:i + 1]
        assert np.array_equal(got[i], exp), f"request {i} ({ops[i % 4]}) differs from the oracle"
    dec = decode(orc.lwe_decrypt(keys_2_2.glwe_sk, pbs), p.delta) % 16
    assert np.array_equal(dec, np.where(np.arange(R) % 2 == 0, (msgs + 1) % 16, (3 * msgs) % 16))
    st = eng.coalesce_stats()
    assert st["rows"] >= R


def test_submit_rejects_bad_requests(eng):
    from tfhe_mi355 import _lib

    with pytest.raises((_lib.EngineError, ValueError)):
        eng.submit("pbs", np.zeros((2000, eng.n + 1), dtype=np.uint64), np.zeros(eng.glwe_len, dtype=np.uint64))
    with pytest.raises(KeyError):
        eng.submit("nope", np.zeros((1, eng.n + 1), dtype=np.uint64))


_SMALL_BATCH_CHILD = r'''
import sys, threading
import numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[1] + "/tfhe-rs-odd_amd"]
from tfhe_mi355 import Engine, client, fill_accumulator
from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P0
P = P0.with_(lwe_dimension=32)
lsk = client.gen_binary_key(1, 1, P.lwe_dimension)
gsk = client.gen_binary_key(1, 2, P.big_lwe_dimension)
eng = Engine(P, 0)
eng.upload_bootstrap_key(client.gen_bootstrap_key(2, lsk, gsk, 1, P.polynomial_size, P.pbs_base_log,
                                                  P.pbs_level, P.glwe_modular_std_dev))
acc = fill_accumulator(P, lambda x: (x + 1) % 16)
msgs = np.arange(64, dtype=np.uint64) % 16
cts = client.lwe_encrypt(3, lsk, msgs * np.uint64(P.delta), P.lwe_modular_std_dev)
ref = eng.programmable_bootstrap(cts, acc)            # 64 rows: above the clamped max count
outs = [None] * 8
def call(i):
    outs[i] = eng.programmable_bootstrap(cts[8 * i: 8 * i + 8], acc)   # coalesced, 8 per call
ts = [threading.Thread(target=call, args=(i,)) for i in range(8)]
[t.start() for t in ts]; [t.join() for t in ts]
assert np.array_equal(np.concatenate(outs), ref), "coalesced rows differ"
dec = client.decode(client.lwe_decrypt(gsk, ref), P.delta) % np.uint64(16)
assert np.array_equal(dec, (msgs + 1) % 16), dec
st = eng.coalesce_stats()
assert st["rows"] == 64 and max(1, st["batches"]) >= 4, st   # batches of <= 16 rows
print("OK", st)
'''


def test_coalesce_batch_smaller_than_max_count_is_safe():
    """TFHE_MI355_COALESCE_BATCH (16) below TFHE_MI355_COALESCE_MAX_COUNT (64): the max count is
    clamped to the batch, so a 64-row call takes the pipelined path instead of overflowing the
    batch staging, and 8-row calls are coalesced into batches of at most 16 rows."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TFHE_MI355_COALESCE_BATCH="16", TFHE_MI355_COALESCE_MAX_COUNT="64")
    r = subprocess.run([sys.executable, "-c", _SMALL_BATCH_CHILD, root], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr[-2000:]
