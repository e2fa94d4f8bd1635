"""Timeline of small KS+PBS calls through the host-pointer ABI (run under rocprofv3 --kernel-trace to
see each call's kernels and the gaps between them).  Prints the median wall time of one call per
count.

usage: single_call_probe.py [reps] [counts]     env PROBE_PARAMS = parameter set (default 2_2)
  e.g. PROBE_PARAMS=PARAM_MESSAGE_3_CARRY_3_KS_PBS python3 scripts/single_call_probe.py 10 1,64
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-odd_amd")]


def main():
    from tfhe_mi355 import Engine, client, fill_accumulator
    from tfhe_mi355.parameters import ALL

    P = ALL[os.environ.get("PROBE_PARAMS", "PARAM_MESSAGE_2_CARRY_2_KS_PBS")]
    lwe_sk = client.gen_binary_key(3, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(3, 2, P.big_lwe_dimension)
    if P.grouping_factor:
        bsk = client.gen_multi_bit_bootstrap_key(4, lwe_sk, glwe_sk, P.glwe_dimension, P.polynomial_size,
                                                 P.pbs_base_log, P.pbs_level, P.grouping_factor,
                                                 P.glwe_modular_std_dev)
    else:
        bsk = client.gen_bootstrap_key(4, lwe_sk, glwe_sk, P.glwe_dimension, P.polynomial_size, P.pbs_base_log,
                                       P.pbs_level, P.glwe_modular_std_dev)
    ksk = client.gen_keyswitch_key(6, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    eng = Engine(P, 0)
    eng.upload_bootstrap_key(bsk)
    eng.upload_keyswitch_key(ksk)
    acc = fill_accumulator(P, lambda x: x)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    counts = [int(c) for c in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1]
    msg = P.message_modulus * P.carry_modulus
    res = {"params": P.name}
    for cnt in counts:
        msgs = (np.arange(cnt) % msg).astype(np.uint64)
        big = client.lwe_encrypt(5, glwe_sk, msgs * np.uint64(P.delta), P.glwe_modular_std_dev)
        f = eng.keyswitch_programmable_bootstrap
        f(big, acc)
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            out = f(big, acc)
            ts.append(time.perf_counter() - t)
        dec = client.decode(client.lwe_decrypt(glwe_sk, out), P.delta) % np.uint64(msg)
        res[str(cnt)] = {"median_ms": 1e3 * float(np.median(ts)), "min_ms": 1e3 * min(ts),
                         "ok": int(np.count_nonzero(dec == msgs)), "of": cnt}
        if os.environ.get("PROBE_STAMPS") == "1":  # a QUAD_STAMPS build: phase stamps of CMUX 200
            res[str(cnt)]["stamps_w0"] = [int(v) for v in out[0, 2:14]]
            res[str(cnt)]["stamps_w4"] = [int(v) for v in out[0, 15:27]]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
