"""Single-ciphertext calling pattern probe: T native callers of the count = 1
host ABI through the request coalescer, with the coalescer's own counters (batches, rows per
batch, batches in flight, batch wall time).  Run under different TFHE_MI355_COALESCE_* settings:
    python scripts/single_ct_probe.py [--params 2_2] [--callers 16 64 256] [--windows 1x256 16x64]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-odd_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", default="2_2")
    ap.add_argument("--callers", type=int, nargs="+", default=[1, 16, 64, 256])
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--windows", nargs="+", default=["1x256", "16x64"],
                    help="submit/wait legs: THREADSxIN_FLIGHT_PER_THREAD")
    args = ap.parse_args()
    from tfhe_mi355 import client, fill_accumulator
    from tfhe_mi355.parameters import ALL

    pname = bench.PARAMS[args.params][0]
    P = ALL[pname]
    with_ks = args.params in bench.WITH_KS
    ns = argparse.Namespace(seed=1)
    import torch

    R = bench.Ranks(torch.device("cuda", 0), None)
    eng, lwe_sk, glwe_sk, bsk, ksk, _ = bench.make_keys(ns, P, R, with_ks)
    msgs = np.random.default_rng(2).integers(0, P.message_modulus * P.carry_modulus, 1024).astype(np.uint64)
    key, std = (glwe_sk, P.glwe_modular_std_dev) if with_ks else (lwe_sk, P.lwe_modular_std_dev)
    cts = client.lwe_encrypt(3, key, msgs * np.uint64(P.delta), std)
    acc = fill_accumulator(P, lambda x: x)
    env = {k: v for k, v in os.environ.items() if k.startswith("TFHE_MI355_COALESCE")}
    res = bench.single_ct_rates(eng, cts, acc, with_ks, 1.0, secs=args.seconds, callers=tuple(args.callers),
                               submit_windows=tuple(tuple(int(v) for v in w.split("x")) for w in args.windows))
    print(json.dumps({"params": args.params, "env": env, "single_ct": res}))


if __name__ == "__main__":
    main()
