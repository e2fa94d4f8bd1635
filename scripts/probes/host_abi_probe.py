"""Where the pageable host-pointer PBS call spends its time (2_2, 4096 ciphertexts): fresh output
array per call vs a reused (already faulted-in) one vs page-locked buffers, and the host chunk."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tfhe-rs-odd_amd"))
if os.environ.get("PROBE_TORCH"):  # the bench's process state: torch's HIP context first
    import torch

    _t = torch.zeros(1 << 20, device="cuda")
    torch.cuda.synchronize()
from tfhe_mi355 import Engine, client, fill_accumulator, pinned_empty  # noqa: E402
from tfhe_mi355.parameters import PARAM_MESSAGE_2_CARRY_2_KS_PBS as P  # noqa: E402

eng = Engine(P, 0)
lwe_sk = client.gen_binary_key(1, 1, P.lwe_dimension)
glwe_sk = client.gen_binary_key(1, 2, P.big_lwe_dimension)
bsk = client.gen_bootstrap_key(2, lwe_sk, glwe_sk, P.glwe_dimension, P.polynomial_size, P.pbs_base_log,
                               P.pbs_level, P.glwe_modular_std_dev)
eng.upload_bootstrap_key(bsk)
B = 4096
msgs = np.random.default_rng(0).integers(0, 4, B).astype(np.uint64)
cts = client.lwe_encrypt(3, lwe_sk, msgs * np.uint64(P.delta), P.lwe_modular_std_dev)
acc = fill_accumulator(P, lambda x: x)
eng.programmable_bootstrap(cts, acc)


def rate(f, reps=4):
    f()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    return B * reps / (time.perf_counter() - t)


reuse = np.empty((B, P.big_lwe_dimension + 1), dtype=np.uint64)
p_in = pinned_empty(cts.shape)
p_in[...] = cts
p_out = pinned_empty(reuse.shape)
res = {
    "fresh_out": rate(lambda: eng.programmable_bootstrap(cts, acc)),
    "reused_out": rate(lambda: eng.programmable_bootstrap(cts, acc, out=reuse)),
    "pinned": rate(lambda: eng.programmable_bootstrap(p_in, acc, out=p_out)),
    "pinned_in_reused_out": rate(lambda: eng.programmable_bootstrap(p_in, acc, out=reuse)),
}
t = time.perf_counter()
for _ in range(4):
    np.empty_like(reuse).fill(1)
res["numpy_fresh_fill_GBps"] = 4 * reuse.nbytes / (time.perf_counter() - t) / 1e9
print("torch" if os.environ.get("PROBE_TORCH") else "plain", os.environ.get("TFHE_MI355_HOST_CHUNK", "default"), os.environ.get("TFHE_MI355_COPY_THREADS", "8"),
      {k: round(v, 1) for k, v in res.items()}, flush=True)
