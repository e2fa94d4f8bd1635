"""Shared test fixtures.  `gpu` marks tests that need an MI355X (run with -m gpu on the GPU box).

Keys for parity tests come from the oracle (oracle/, test infrastructure) and are handed to the
HIP engine through its C ABI as standard-domain u64 keys, exactly as a Rust caller would.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-odd_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O

    O.build()
    return O


class KeySet:
    """Oracle-generated key material for one parameter set."""

    def __init__(self, O, params, seed):
        p = params
        self.params = p
        self.seed = seed
        self.lwe_sk = O.binary_key(seed, 1, p.lwe_dimension)
        self.glwe_sk = O.binary_key(seed, 2, p.glwe_dimension * p.polynomial_size)
        if p.grouping_factor:
            self.bsk = O.gen_mb_bsk(seed, self.lwe_sk, self.glwe_sk, p.glwe_dimension, p.polynomial_size,
                                    p.pbs_base_log, p.pbs_level, p.grouping_factor,
                                    p.glwe_modular_std_dev, threads=8)
            self.fbsk = O.MultiBitFourierBsk(self.bsk, p.lwe_dimension, p.glwe_dimension,
                                             p.polynomial_size, p.pbs_base_log, p.pbs_level,
                                             p.grouping_factor)
        else:
            self.bsk = O.gen_bsk(seed, self.lwe_sk, self.glwe_sk, p.glwe_dimension, p.polynomial_size,
                                 p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev, threads=8)
            self.fbsk = O.FourierBsk(self.bsk, p.lwe_dimension, p.glwe_dimension, p.polynomial_size,
                                     p.pbs_base_log, p.pbs_level)
        self._ksk = None
        self._O = O

    @property
    def ksk(self):
        if self._ksk is None:
            p = self.params
            self._ksk = self._O.gen_ksk(self.seed + 1, self.glwe_sk, self.lwe_sk, p.ks_base_log, p.ks_level,
                                        p.lwe_modular_std_dev)
        return self._ksk


@pytest.fixture(scope="session")
def params_2_2():
    from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS

    return PARAM_MESSAGE_2_CARRY_2_KS_PBS


@pytest.fixture(scope="session")
def keys_2_2(orc, params_2_2):
    return KeySet(orc, params_2_2, seed=0)


@pytest.fixture(scope="session")
def keys_manticore(orc):
    from tfhe_mi355.parameters import MANTICORE_PARAMETERS

    return KeySet(orc, MANTICORE_PARAMETERS, seed=11)


@pytest.fixture(scope="session")
def keys_mb(orc):
    from tfhe_mi355.parameters import PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS

    return KeySet(orc, PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS, seed=5)


def decode(pts, delta):
    d = np.asarray(pts, dtype=np.uint64)
    rounding = (d & np.uint64(delta >> 1)) << np.uint64(1)
    return (d + rounding) // np.uint64(delta)


from oracle.oracle import OracleEngine  # noqa: E402,F401  (re-exported for the tests)
