"""Generate tests/golden/pbs_golden.json: seeded inputs -> SHA-256 of the oracle's outputs.

The reference ships no golden vectors (every reference test is OS-seeded), so the
fixtures pin the oracle (C restatement, oracle/pbs_oracle.c) to itself across rounds and give
the GPU tests a committed, oracle-free target.  Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-odd_amd")]

CASES = [
    # name, parameter set, key seed, lwe_dimension override, messages, lut multiplier/offset
    ("classic_2_2", "PARAM_MESSAGE_2_CARRY_2_KS_PBS", 100, None, [0, 5, 10, 15], (3, 1)),
    ("classic_manticore", "MANTICORE_PARAMETERS", 101, None, [0, 1, 2, 3], (1, 1)),
    ("multibit_g3", "PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS", 102, None, [2, 9], (5, 0)),
    ("large_4_4_n16", "PARAM_MESSAGE_4_CARRY_4_KS_PBS", 103, 16, [7, 200], (1, 3)),
    # split CMUX (round 3): N = 8192 L = 2 (the reference's 121 ms set), N = 16384 L = 3 (64-bit
    # decomposition of 33 bits), multi-bit at N = 8192 (keybundle in the paired sub-block kernel)
    ("split_3_3_n8", "PARAM_MESSAGE_3_CARRY_3_KS_PBS", 104, 8, [5, 60], (3, 7)),
    ("split_1_6_n6", "PARAM_MESSAGE_1_CARRY_6_KS_PBS", 105, 6, [1, 100], (1, 1)),
    ("multibit_3_3_g3_n6", "PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS", 106, 6, [3, 44], (2, 5)),
    # round 5: the on-chip CMUX's other shapes, N = 4096 L = 2 and N = 8192 L = 1 (base 2^22)
    ("split_1_4_n8", "PARAM_MESSAGE_1_CARRY_4_KS_PBS", 107, 8, [3, 30], (5, 2)),
    ("split_6_0_n8", "PARAM_MESSAGE_6_CARRY_0_KS_PBS", 108, 8, [9, 50], (3, 4)),
]


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


def inputs(O, name, pname, seed, n_override, msgs, lut):
    """Keys, ciphertexts and LUT of one case (shared by the generator and the tests)."""
    from tfhe_mi355 import client
    from tfhe_mi355.parameters import ALL

    p = ALL[pname]
    if n_override:
        p = p.with_(lwe_dimension=n_override)
    N, k = p.polynomial_size, p.glwe_dimension
    if N > 4096:   # schoolbook oracle keygen is too slow at N >= 8192: engine client keygen
        lwe_sk = client.gen_binary_key(seed, 1, p.lwe_dimension)
        glwe_sk = client.gen_binary_key(seed, 2, k * N)
        if p.grouping_factor:
            bsk = client.gen_multi_bit_bootstrap_key(seed + 1, lwe_sk, glwe_sk, k, N, p.pbs_base_log, p.pbs_level,
                                                     p.grouping_factor, p.glwe_modular_std_dev, threads=8)
        else:
            bsk = client.gen_bootstrap_key(seed + 1, lwe_sk, glwe_sk, k, N, p.pbs_base_log, p.pbs_level,
                                           p.glwe_modular_std_dev)
    else:
        lwe_sk = O.binary_key(seed, 1, p.lwe_dimension)
        glwe_sk = O.binary_key(seed, 2, k * N)
        if p.grouping_factor:
            bsk = O.gen_mb_bsk(seed, lwe_sk, glwe_sk, k, N, p.pbs_base_log, p.pbs_level, p.grouping_factor,
                               p.glwe_modular_std_dev)
        else:
            bsk = O.gen_bsk(seed, lwe_sk, glwe_sk, k, N, p.pbs_base_log, p.pbs_level, p.glwe_modular_std_dev)
    delta = p.delta
    space = p.message_modulus * p.carry_modulus
    cts = O.lwe_encrypt(seed + 7, lwe_sk, np.asarray(msgs, dtype=np.uint64) * np.uint64(delta),
                        p.lwe_modular_std_dev)
    a, b = lut
    acc = O.fill_accumulator(N, k, p.message_modulus, p.carry_modulus, lambda x: (a * x + b) % space)
    return p, lwe_sk, glwe_sk, bsk, cts, acc


def main():
    from oracle import oracle as O

    O.build()
    out = []
    for name, pname, seed, n_override, msgs, lut in CASES:
        p, lwe_sk, glwe_sk, bsk, cts, acc = inputs(O, name, pname, seed, n_override, msgs, lut)
        if p.grouping_factor:
            fb = O.MultiBitFourierBsk(bsk, p.lwe_dimension, p.glwe_dimension, p.polynomial_size,
                                      p.pbs_base_log, p.pbs_level, p.grouping_factor)
        else:
            fb = O.FourierBsk(bsk, p.lwe_dimension, p.glwe_dimension, p.polynomial_size, p.pbs_base_log,
                              p.pbs_level)
        res = fb.pbs(cts, acc, threads=8)
        space = p.message_modulus * p.carry_modulus
        raw = O.lwe_decrypt(glwe_sk, res)
        dec = ((raw + ((raw & np.uint64(p.delta >> 1)) << np.uint64(1))) // np.uint64(p.delta)) % np.uint64(space)
        out.append({"name": name, "parameters": pname, "lwe_dimension": p.lwe_dimension, "key_seed": seed,
                    "messages": msgs, "lut": list(lut), "decrypted": [int(x) for x in dec],
                    "input_sha256": digest(cts), "output_sha256": digest(res),
                    "output_head": [str(int(x)) for x in res[0, :4]]})
        print(name, out[-1]["decrypted"])
    with open(os.path.join(HERE, "pbs_golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": out}, f, indent=1)


if __name__ == "__main__":
    main()
