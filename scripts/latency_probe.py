"""Device time of one async PBS launch at 2_2 for a range of batch sizes (HIP events on the launch
stream), to place the latency/throughput kernel switch (TFHE_MI355_LATENCY_MAX, capi.cpp).
Run it twice, with TFHE_MI355_LATENCY_MAX=0 (throughput kernel only) and =4096 (latency kernel
for every count), and compare.  Prints one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-odd_amd")]


def main():
    import torch

    from tfhe_mi355 import Engine, client, fill_accumulator
    from tfhe_mi355.parameters import ALL

    # LAT_PARAMS: the parameter set (default 2_2; e.g. PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS)
    P = ALL[os.environ.get("LAT_PARAMS", "PARAM_MESSAGE_2_CARRY_2_KS_PBS")]

    counts = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "1,16,64,128,256,384,512,768,1024").split(",")]
    lwe_sk = client.gen_binary_key(3, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(3, 2, P.big_lwe_dimension)
    if P.grouping_factor:
        bsk = client.gen_multi_bit_bootstrap_key(4, lwe_sk, glwe_sk, 1, P.polynomial_size, P.pbs_base_log,
                                                 P.pbs_level, P.grouping_factor, P.glwe_modular_std_dev)
    else:
        bsk = client.gen_bootstrap_key(4, lwe_sk, glwe_sk, 1, P.polynomial_size, P.pbs_base_log, P.pbs_level,
                                       P.glwe_modular_std_dev)
    eng = Engine(P, 0)
    eng.upload_bootstrap_key(bsk)
    C = max(counts)
    msgs = np.arange(C, dtype=np.uint64) % 16
    cts = client.lwe_encrypt(5, lwe_sk, msgs * np.uint64(P.delta), P.lwe_modular_std_dev)
    acc = fill_accumulator(P, lambda x: x)
    d_in = torch.from_numpy(cts.view(np.int64)).cuda()
    d_out = torch.zeros((C, P.big_lwe_dimension + 1), dtype=torch.int64, device="cuda")
    d_lut = torch.from_numpy(acc.view(np.int64)).cuda()
    stamps = os.environ.get("LAT_STAMPS") == "1"   # a LAT_STAMPS=1 build (TFHE_MI355_LIB)
    scratch = torch.zeros(max(eng.pbs_scratch_bytes(C), 1 << 16), dtype=torch.uint8, device="cuda")
    res = {"params": P.name if hasattr(P, "name") else str(P.polynomial_size), "latency_max_env": os.environ.get("TFHE_MI355_LATENCY_MAX"), "ms": {}}
    for c in counts:
        eng.programmable_bootstrap_async(d_in, d_out, d_lut, 1, c, d_scratch=scratch)
        torch.cuda.synchronize()
        reps = 3 if c > 256 else 5
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for s, e in evs:
            s.record()
            eng.programmable_bootstrap_async(d_in, d_out, d_lut, 1, c, d_scratch=scratch)
            e.record()
        torch.cuda.synchronize()
        ms = float(np.median([s.elapsed_time(e) for s, e in evs]))
        out = d_out[:c].cpu().numpy().view(np.uint64)
        dec = client.decode(client.lwe_decrypt(glwe_sk, out), P.delta) % np.uint64(16)
        res["ms"][c] = {"ms": ms, "pbs_per_s": c / ms * 1e3, "decrypt_ok": int(np.count_nonzero(dec == msgs[:c]))}
        if stamps and c <= 256:
            st = scratch[: 2 * 8 * 12 * 8].cpu().numpy().view(np.uint64).reshape(2, 8, 12).astype(np.int64)
            d = np.diff(st[:, :, :11], axis=2)            # per phase, cycles
            res["ms"][c]["phase_cycles_row0"] = np.median(d[0], axis=0).tolist()
            res["ms"][c]["phase_cycles_row1"] = np.median(d[1], axis=0).tolist()
            res["ms"][c]["cmux_cycles"] = float(np.median(st[0, 1:, 0] - st[0, :-1, 0]))
        print(c, res["ms"][c], file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
