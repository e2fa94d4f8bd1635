"""GPU parity for the integer radix multiplication DAG (BASELINE config 4):
the same batched DAG run with the GPU engine and with the oracle engine must give bit-identical
radix ciphertexts, and decrypt to a * b mod 2^32."""
import numpy as np
import pytest

from conftest import OracleEngine

pytestmark = pytest.mark.gpu


def _keys(seed, engine=None):
    from tfhe_mi355 import integer, shortint
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    ck = shortint.ClientKey(P, seed)
    sk = shortint.ServerKey(ck, engine=engine)
    return integer.ClientKey(ck, 16), integer.ServerKey(sk)


@pytest.mark.timeout(600)
def test_fheuint32_mul_bit_exact_vs_oracle_dag():
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P

    cks, gpu = _keys(5)
    _, cpu = _keys(5, OracleEngine(P, threads=16))
    a = np.array([0xFFFFFFFF, 0x80000001, 7], dtype=np.uint64)
    b = np.array([0xFFFFFFFF, 3, 0x0F0F0F0F], dtype=np.uint64)
    ca, cb = cks.encrypt(a), cks.encrypt(b)
    g = gpu.to_host(gpu.mul_parallelized(ca, cb))   # device-resident DAG (lwe_ops kernels)
    c = cpu.mul_parallelized(ca, cb)                 # host numpy DAG, oracle engine
    assert gpu.pbs_count == cpu.pbs_count
    assert g.degree == c.degree and g.noise == c.noise
    assert np.array_equal(g.data, c.data), f"{np.count_nonzero(g.data != c.data)} words differ"
    assert np.array_equal(cks.decrypt(g), (a * b) % np.uint64(1 << 32))


def test_fheuint32_mul_batch_decrypts():
    cks, gpu = _keys(6)
    rng = np.random.default_rng(4)
    a = rng.integers(0, 2 ** 32, 64, dtype=np.uint64)
    b = rng.integers(0, 2 ** 32, 64, dtype=np.uint64)
    out = gpu.mul_parallelized(cks.encrypt(a), cks.encrypt(b))
    assert np.array_equal(cks.decrypt(out), (a * b) % np.uint64(1 << 32))
