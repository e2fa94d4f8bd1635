"""Integer radix multiplication DAG (radix_parallel/mul.rs:300-414,
add.rs:206-960) on the CPU: the batched host orchestration run against the oracle engine
(test infrastructure), checked by decryption (a * b mod 2^32) and by its PBS count."""
import numpy as np
import pytest

from conftest import OracleEngine


def _keys(seed, engine):
    from tfhe_mi355 import integer, shortint
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    ck = shortint.ClientKey(P, seed)
    sk = shortint.ServerKey(ck, engine=engine)
    return integer.ClientKey(ck, 16), integer.ServerKey(sk)


def test_blockshift_and_trivial_pbs_host_logic():
    """blockshift (radix/scalar_mul.rs:345-355) and the trivial PBS shortcut on the host."""
    from tfhe_mi355 import integer
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P
    from tfhe_mi355.shortint import NOISE_NOMINAL, NOISE_ZERO

    class _NoEngine:
        def upload_bootstrap_key(self, bsk):
            pass

        def upload_keyswitch_key(self, ksk):
            pass

    from tfhe_mi355 import shortint

    sk = integer.ServerKey(shortint.ServerKey(None, engine=_NoEngine(), parameters=P))
    rb = integer.RadixBatch(np.arange(2 * 4 * 3, dtype=np.uint64).reshape(2, 4, 3), [3, 2, 1, 3],
                            [NOISE_NOMINAL] * 4)
    sh = sk.blockshift(rb, 1)
    assert sh.degree == [0, 3, 2, 1] and sh.noise[0] == NOISE_ZERO
    assert np.array_equal(sh.data[:, 1:, :], rb.data[:, :3, :])
    # trivial PBS of a trivial block holding 2: f(2) * delta
    sk.lwe_size = 3
    z = sk.create_trivial_zero(2, 1)
    z.data[:, 0, -1] = np.uint64(2 * P.delta)
    z.degree[0] = 2
    lut = sk.shortint.generate_lookup_table(lambda x: (x + 1) % 4)
    sk._trivial_pbs(z, 0, lut)
    assert np.all(z.data[:, 0, -1] == np.uint64(3 * P.delta))


@pytest.mark.timeout(600)
def test_fheuint32_mul_dag_with_oracle_engine():
    """FheUint32 multiply (16 blocks of 2_2) through the batched DAG with the oracle behind the
    engine API: decrypts to a * b mod 2^32; the DAG issues the reference's PBS count."""
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    cks, sks = _keys(3, OracleEngine(P, threads=8))
    a = np.array([0xDEADBEEF, 123456789], dtype=np.uint64)
    b = np.array([0x12345678, 4294967295], dtype=np.uint64)
    ca, cb = cks.encrypt(a), cks.encrypt(b)
    out = sks.mul_parallelized(ca, cb)
    assert np.array_equal(cks.decrypt(out), (a * b) % np.uint64(1 << 32))
    # 136 + 120 bivariate products; sum rounds; final extraction + Hillis-Steele add
    assert sks.pbs_count % 2 == 0
    per_mul = sks.pbs_count // 2
    assert 256 < per_mul < 700, per_mul


def test_device_table_cache_is_bounded_and_pins_captured_entries():
    """the layer-table cache is an LRU of bounded size; entries used while a hipGraph
    is captured are never evicted (the graph reads their device memory on every replay)."""
    from tfhe_mi355.integer import _BoundedCache

    capturing = [False]
    c = _BoundedCache(3, lambda: capturing[0])
    for k in range(5):
        c.put(k, k * 10)
    assert len(c) == 3 and c.get(0) is None and c.get(1) is None and c.get(4) == 40
    c.get(2)                      # 2 becomes most recent: 3 is evicted next
    c.put(5, 50)
    assert c.get(3) is None and c.get(2) == 20
    capturing[0] = True
    assert c.get(4) == 40         # touched during capture: pinned
    c.put(6, 60)                  # created during capture: pinned
    capturing[0] = False
    for k in range(100, 110):
        c.put(k, k)
    assert c.get(4) == 40 and c.get(6) == 60 and c.get(5) is None
