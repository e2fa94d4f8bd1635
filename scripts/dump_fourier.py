"""Debug helper: dump the engine's Fourier BSK and the oracle's (engine layout) for a small key."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-odd_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as O  # noqa: E402
from test_large_gpu import _device_to_host, engine_position  # noqa: E402
from tfhe_mi355 import Engine, client  # noqa: E402
from tfhe_mi355.parameters import PARAM_MESSAGE_4_CARRY_4_KS_PBS  # noqa: E402

N = 32768
p = PARAM_MESSAGE_4_CARRY_4_KS_PBS.with_(lwe_dimension=2)
lwe_sk = client.gen_binary_key(3, 1, 2)
glwe_sk = client.gen_binary_key(3, 2, N)
bsk = client.gen_bootstrap_key(4, lwe_sk, glwe_sk, 1, N, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev)
eng = Engine(p, 0)
eng.upload_bootstrap_key(bsk)
ptr, nbytes = eng.fourier_bootstrap_key()
got = _device_to_host(ptr, nbytes).view(np.complex128).reshape(-1, N // 2)
exp = O.FourierBsk(bsk, 2, 1, N, p.pbs_base_log, p.pbs_level).fourier().reshape(-1, N // 2)
exp = np.ascontiguousarray(exp[:, engine_position(N)])
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/fourier_got.npy", got[:2])
np.save("gpurun_out/fourier_exp.npy", exp[:2])
np.save("gpurun_out/bsk_polys.npy", bsk[: 2 * N])
print("saved")
