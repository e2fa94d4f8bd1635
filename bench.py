#!/usr/bin/env python3
"""bench.py -- programmable bootstraps/sec at PARAM_MESSAGE_2_CARRY_2 on 1/2/4/8 MI355X.

BASELINE.json metric "programmable bootstraps/sec (PARAM_MESSAGE_2_CARRY_2) at 1/2/4/8 MI355X",
workload = BASELINE config 2: a batch of 4096 independent classic PBS per GPU, identity LUT
(PARAM_MESSAGE_2_CARRY_2_KS_PBS: n=742, k=1, N=2048, L=1, base 2^23).  One step = one PBS
launch over the GPU's batch (blind rotation + sample extraction), inputs resident in HBM.

Multi-GPU (weak scaling): one process per GPU launched by torch.distributed.run; the standard
BSK is generated once on rank 0 and broadcast ONCE over RCCL (xGMI), each rank converts it to
the Fourier domain on its own GPU, then each rank bootstraps its own batch -- no collective in
the timed loop except the bracketing barriers.  value = sum of PBS over ranks / max wall time.

Also printed: roofline of the dominant kernel (pbs_classic_kernel) -- BSK-streaming HBM model
 with the FP64 fraction beside it -- and the CPU baseline (oracle C restatement,
1 PBS per thread, rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-odd_amd"))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 vector (= matrix) spec, SURVEY.md 8d


PARAMS = {  # --params choice -> (parameter set name, workload text, kernel name)
    "2_2": ("PARAM_MESSAGE_2_CARRY_2_KS_PBS",
            "BASELINE config 2: batch of 4096 independent classic PBS per GPU, identity LUT",
            "pbs_classic_kernel<2048,1,1>"),
    "mb3": ("PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS",
            "BASELINE config 5: batch of 4096 independent multi-bit (grouping 3) PBS per GPU, identity LUT",
            "pbs_multibit_kernel<2048,1,1,3>"),
    "4_4": ("PARAM_MESSAGE_4_CARRY_4_KS_PBS",
            "BASELINE config 3: shortint apply_lookup_table (keyswitch -> PBS) at N=32768 per GPU batch",
            "large_top_fwd_kernel<1,2> + large_sub_kernel<1,2> + large_top_inv_kernel<1> (+ ks_mfma_kernel)"),
    "mul32": ("PARAM_MESSAGE_2_CARRY_2_KS_PBS",
              "BASELINE config 4: FheUint32 multiply (16-block radix DAG, radix_parallel/mul.rs), "
              "K independent pairs per GPU, every DAG layer one batched KS+PBS launch",
              "pbs_classic_kernel<2048,1,1> + keyswitch_kernel"),
    "mb2": ("PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS",
            "batch of 4096 independent multi-bit (grouping 2) PBS per GPU, identity LUT",
            "pbs_multibit_kernel<2048,1,1,2>"),
    # the fork's gadget parameter sets (gadget/parameters/mod.rs), same PBS workload
    "manticore": ("MANTICORE_PARAMETERS",
                  "batch of 4096 independent classic PBS per GPU at the fork's MANTICORE_PARAMETERS",
                  "pbs_classic_kernel<1024,1,2>"),
    "ascon": ("GADGET_ASCON_PARAMETERS_40",
              "batch of 4096 independent classic PBS per GPU at the fork's ASCON_PARAMETERS_40",
              "pbs_classic_kernel<1024,2,3>"),
    "simon": ("GADGET_SIMON_PARAMETERS_40",
              "batch of 4096 independent classic PBS per GPU at the fork's SIMON_PARAMETERS_40",
              "pbs_classic_kernel<512,3,2>"),
    "tfhelib": ("GADGET_TFHE_LIB_PARAMETERS",
                "batch of 4096 independent classic PBS per GPU at the fork's TFHE_LIB_PARAMETERS",
                "pbs_classic_kernel<1024,2,1>"),
    "aes40": ("GADGET_AES_PARAMETERS_40",
              "batch of 4096 independent classic PBS per GPU at the fork's AES_PARAMETERS_40",
              "pbs_classic_kernel<512,3,4>"),
    "sha3": ("GADGET_SHA3_PARAMETERS_40",
             "batch of 4096 independent classic PBS per GPU at the fork's SHA3_PARAMETERS_40",
             "pbs_classic_kernel<256,5,1>"),
}


def ggsw_count(p) -> int:
    g = p.grouping_factor
    return (p.lwe_dimension // g) << g if g else p.lwe_dimension


def pbs_algorithmic_bytes(p) -> int:
    """SURVEY.md 8d BSK-streaming model: |BSK_fourier| + 8(n+1) + 8(kN+1) + 8(k+1)N
    (multi-bit: (n/g) 2^g GGSWs in the BSK)."""
    M = p.polynomial_size // 2
    k1 = p.glwe_dimension + 1
    fbsk = ggsw_count(p) * p.pbs_level * k1 * k1 * M * 16
    return fbsk + 8 * (p.lwe_dimension + 1) + 8 * (p.glwe_dimension * p.polynomial_size + 1) + 8 * k1 * p.polynomial_size


def pbs_flops(p) -> float:
    """per CMUX ((k+1)L + (k+1)) (5 M log2 M + 6 M) + (k+1)^2 L M 8, times n.
    Multi-bit: the same external product per group of g, plus the keybundle's (2^g - 1)
    complex FMAs (8 flop) per GGSW element, times n/g."""
    M = p.polynomial_size // 2
    k1 = p.glwe_dimension + 1
    per = (k1 * p.pbs_level + k1) * (5 * M * math.log2(M) + 6 * M) + k1 * k1 * p.pbs_level * M * 8
    g = p.grouping_factor
    if g:
        per += ((1 << g) - 1) * k1 * k1 * p.pbs_level * M * 8
        return per * (p.lwe_dimension // g)
    return per * p.lwe_dimension


def load_pmc_traffic(batch: int, tag: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json,
    FETCH_SIZE doubled per MI355X_MICROARCH.md 'HBM' + WRITE_SIZE), scaled to this batch."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json" if tag == "2_2" else f"pmc_traffic_{tag}.json")
    try:
        d = json.load(open(path))
        return float(d["hbm_bytes_per_pbs"]) * batch
    except Exception:
        return None


def cpu_baseline(params, bsk, cts, acc, threads: int, ksk=None):
    """Oracle (C restatement of the reference fft64 PBS) on the host cores, one PBS per thread,
    as the reference's pbs_throughput bench (benches/core_crypto/pbs_bench.rs:430-549).
    With `ksk` (config 3) each ciphertext is keyswitched first (threads split the batch)."""
    sys.path.insert(0, ROOT)
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O

    p = params

    def ks(batch):
        if ksk is None:
            return batch
        parts = np.array_split(batch, min(threads, batch.shape[0]))
        with ThreadPoolExecutor(len(parts)) as ex:
            outs = list(ex.map(lambda c: O.keyswitch(ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log,
                                                     p.ks_level, c), parts))
        return np.concatenate(outs)

    O.build()
    if params.grouping_factor:
        fb = O.MultiBitFourierBsk(bsk, params.lwe_dimension, params.glwe_dimension, params.polynomial_size,
                                  params.pbs_base_log, params.pbs_level, params.grouping_factor)
    else:
        fb = O.FourierBsk(bsk, params.lwe_dimension, params.glwe_dimension, params.polynomial_size,
                          params.pbs_base_log, params.pbs_level)
    t = time.perf_counter()
    fb.pbs(ks(cts[:1]), acc, threads=1)
    t1 = time.perf_counter() - t
    count = max(threads, int(round(15.0 / max(t1, 1e-3))))
    count = min(((count + threads - 1) // threads) * threads, cts.shape[0])
    t = time.perf_counter()
    fb.pbs(ks(cts[:count]), acc, threads=threads)
    wall = time.perf_counter() - t
    return {
        "value": count / wall,
        "unit": "PBS/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{count} {'KS+' if ksk is not None else ''}PBS of the same {params.name} batch, oracle C "
                   f"restatement of the reference fft64 PBS, 1 PBS per thread on {threads} threads ({wall:.1f} s wall); "
                   f"single-thread latency {t1 * 1e3:.1f} ms/PBS (reference published "
                   f"{'811 ms' if p.polynomial_size == 32768 else '16.6 ms'} KS+PBS at "
                   f"{'4_4' if p.polynomial_size == 32768 else '2_2'} on Xeon 8375C AVX-512, benchmarks.md:42)"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0, help="ciphertexts per GPU per step (default 4096; 1024 at 4_4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--params", choices=sorted(PARAMS), default="2_2",
                    help="2_2 = the BASELINE metric; mb3/mb2 = multi-bit PBS (config 5)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from tfhe_mi355 import Engine, client, fill_accumulator
    from tfhe_mi355.distributed import broadcast_u64, env_rank_world
    from tfhe_mi355.parameters import ALL

    pname, workload, kname = PARAMS[args.params]
    P = ALL[pname]

    rank, world, local = env_rank_world()
    # one process per GPU; on a box with fewer GPUs than ranks (a rehearsal of the multi-rank
    # path, BENCH_DIST_BACKEND=gloo) ranks share devices round-robin
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)

    def barrier():
        if world > 1:
            t = torch.ones(1, device=device)
            dist.all_reduce(t)
        torch.cuda.synchronize()

    if args.params == "mul32":
        return run_mul32(args, P, workload, kname, rank, world, local, device, barrier)
    B = args.batch or (1024 if args.params == "4_4" else 4096)
    with_ks = args.params == "4_4"   # config 3 is the shortint KS -> PBS
    msg_space = P.message_modulus * P.carry_modulus
    eng = Engine(P, local)
    # secret keys: derived from the seed on every rank (cheap); the BSK once on rank 0
    lwe_sk = client.gen_binary_key(args.seed, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(args.seed, 2, P.big_lwe_dimension)
    bsk_len = ggsw_count(P) * P.pbs_level * (P.glwe_dimension + 1) ** 2 * P.polynomial_size
    bsk = None
    t_key = time.perf_counter()
    if rank == 0:
        if P.grouping_factor:
            bsk = client.gen_multi_bit_bootstrap_key(args.seed + 100, lwe_sk, glwe_sk, P.glwe_dimension,
                                                     P.polynomial_size, P.pbs_base_log, P.pbs_level,
                                                     P.grouping_factor, P.glwe_modular_std_dev)
        else:
            bsk = client.gen_bootstrap_key(args.seed + 100, lwe_sk, glwe_sk, P.glwe_dimension,
                                           P.polynomial_size, P.pbs_base_log, P.pbs_level,
                                           P.glwe_modular_std_dev)
    t_gen = time.perf_counter() - t_key
    t_bc = time.perf_counter()
    d_bsk = broadcast_u64(bsk, bsk_len, 0, device)  # one RCCL broadcast (48.6 MB at 2_2)
    torch.cuda.synchronize()
    t_bc = time.perf_counter() - t_bc
    eng.convert_bootstrap_key_device(d_bsk, bsk_len)
    torch.cuda.synchronize()
    del d_bsk
    if with_ks:
        ksk_len = P.big_lwe_dimension * P.ks_level * (P.lwe_dimension + 1)
        ksk = None
        if rank == 0:
            ksk = client.gen_keyswitch_key(args.seed + 200, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level,
                                           P.lwe_modular_std_dev)
        d_ksk = broadcast_u64(ksk, ksk_len, 0, device)
        eng.upload_keyswitch_key_device(d_ksk, ksk_len)
        torch.cuda.synchronize()
        del d_ksk
    else:
        ksk = None

    rng = np.random.default_rng(args.seed * 1000 + rank)
    msgs = rng.integers(0, msg_space, B).astype(np.uint64)
    if with_ks:
        cts = client.lwe_encrypt(args.seed * 1000 + rank, glwe_sk, msgs * np.uint64(P.delta),
                                 P.glwe_modular_std_dev)
    else:
        cts = client.lwe_encrypt(args.seed * 1000 + rank, lwe_sk, msgs * np.uint64(P.delta),
                                 P.lwe_modular_std_dev)
    acc = fill_accumulator(P, lambda x: x)
    d_in = torch.from_numpy(cts.view(np.int64)).to(device)
    d_out = torch.zeros((B, P.big_lwe_dimension + 1), dtype=torch.int64, device=device)
    d_lut = torch.from_numpy(acc.view(np.int64)).to(device)
    stream = torch.cuda.current_stream()
    if with_ks:
        d_scratch = torch.empty(eng.ks_pbs_scratch_bytes(B), dtype=torch.uint8, device=device)

    def step():
        if with_ks:
            eng.keyswitch_programmable_bootstrap_async(d_in, d_out, d_lut, 1, B, d_scratch, stream=stream)
        else:
            eng.programmable_bootstrap_async(d_in, d_out, d_lut, 1, B, stream=stream)

    for _ in range(args.warmup):
        step()
    barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record(stream)
        step()
        e.record(stream)
    barrier()
    wall = time.perf_counter() - t0
    kernel_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    tt = torch.tensor([wall], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    wall_max = float(tt.item())

    # correctness of this rank's outputs (decrypt with the big key)
    out = d_out.cpu().numpy().view(np.uint64)
    dec = client.decode(client.lwe_decrypt(glwe_sk, out), P.delta) % np.uint64(msg_space)
    ok = int(np.count_nonzero(dec == msgs))
    okt = torch.tensor([ok, B], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(okt)

    if rank == 0:
        total = world * B * args.steps
        value = total / wall_max
        per_launch_bytes = pbs_algorithmic_bytes(P) * B
        achieved = per_launch_bytes / (kernel_ms * 1e-3) / 1e9
        flops = pbs_flops(P) * B / (kernel_ms * 1e-3) / 1e12
        line = {
            "metric": ("programmable bootstraps/sec (PARAM_MESSAGE_2_CARRY_2) at 1/2/4/8 MI355X"
                       if args.params == "2_2" else f"programmable bootstraps/sec ({pname}) at 1/2/4/8 MI355X"),
            "value": value,
            "unit": "PBS/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded LWE encryptions of uniform 4-bit messages; keys from the engine's client-side keygen)",
            "config": {
                "workload": workload,
                "parameters": (f"{pname} (n={P.lwe_dimension}, k={P.glwe_dimension}, N={P.polynomial_size}, "
                               f"pbs 2^{P.pbs_base_log} x {P.pbs_level}"
                               + (f", grouping {P.grouping_factor})" if P.grouping_factor else ")")),
                "batch_per_gpu": B,
                "global_batch": world * B,
                "parallelism": f"dp{world} (batch shards, BSK replicated by one RCCL broadcast)",
            },
            "roofline": {
                "bound": "hbm",
                "model": (f"BSK-streaming (SURVEY.md 8d): {pbs_algorithmic_bytes(P):,} B per PBS; "
                          "frac > 1 would mean reuse beyond streaming"),
                "kernel": kname,
                "kernel_ms": kernel_ms,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": load_pmc_traffic(B, args.params),
                "fp64": {"achieved": flops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": flops / FP64_PEAK_TFLOPS,
                         "flop_per_pbs": pbs_flops(P)},
            },
            "check": {"decrypted_ok": int(okt[0].item()), "of": int(okt[1].item())},
            "setup": {"bsk_keygen_s": t_gen, "bsk_broadcast_s": t_bc},
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(P, bsk, cts, acc, threads, ksk)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_mul32(args, P, workload, kname, rank, world, local, device, barrier):
    """Config 4: K FheUint32 multiplies per GPU per step through the batched integer DAG
    (tfhe_mi355.integer); value = multiplies/s over all ranks."""
    import torch
    import torch.distributed as dist

    from tfhe_mi355 import Engine, client, integer, shortint
    from tfhe_mi355.distributed import broadcast_u64

    K = args.batch or 256
    ck = shortint.ClientKey(P, args.seed)
    eng = Engine(P, local)
    bsk_len = ggsw_count(P) * P.pbs_level * (P.glwe_dimension + 1) ** 2 * P.polynomial_size
    ksk_len = P.big_lwe_dimension * P.ks_level * (P.lwe_dimension + 1)
    bsk = ksk = None
    if rank == 0:
        bsk = client.gen_bootstrap_key(args.seed + 100, ck.small_lwe_secret_key, ck.glwe_secret_key,
                                       P.glwe_dimension, P.polynomial_size, P.pbs_base_log, P.pbs_level,
                                       P.glwe_modular_std_dev)
        ksk = client.gen_keyswitch_key(args.seed + 200, ck.large_lwe_secret_key, ck.small_lwe_secret_key,
                                       P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    d = broadcast_u64(bsk, bsk_len, 0, device)
    eng.convert_bootstrap_key_device(d, bsk_len)
    d = broadcast_u64(ksk, ksk_len, 0, device)
    eng.upload_keyswitch_key_device(d, ksk_len)
    torch.cuda.synchronize()
    del d
    sks = integer.ServerKey(shortint.ServerKey(None, engine=eng, parameters=P))
    cks = integer.ClientKey(ck, 16)
    rng = np.random.default_rng(args.seed * 1000 + rank)
    a = rng.integers(0, 2 ** 32, K, dtype=np.uint64)
    b = rng.integers(0, 2 ** 32, K, dtype=np.uint64)
    ca, cb = cks.encrypt(a), cks.encrypt(b)
    ca_d, cb_d = sks.to_device(ca), sks.to_device(cb)   # operands resident in HBM

    out = None
    for _ in range(args.warmup):
        out = sks.mul_parallelized(ca_d, cb_d)
    barrier()
    pbs0, l0 = sks.pbs_count, sks.launches
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = sks.mul_parallelized(ca_d, cb_d)
    barrier()
    wall = time.perf_counter() - t0
    pbs_per_mul = (sks.pbs_count - pbs0) / (args.steps * K)
    launches = (sks.launches - l0) / args.steps
    tt = torch.tensor([wall], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    wall_max = float(tt.item())
    ok = int(np.count_nonzero(cks.decrypt(out) == (a * b) % np.uint64(1 << 32)))
    okt = torch.tensor([ok, K], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(okt)
    if rank == 0:
        muls = world * K * args.steps
        pbs_rate = muls * pbs_per_mul / wall_max
        line = {
            "metric": "FheUint32 multiplies/sec (PARAM_MESSAGE_2_CARRY_2 radix, 16 blocks) at 1/2/4/8 MI355X",
            "value": muls / wall_max,
            "unit": "mul/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (uniform u32 operand pairs, seeded encryptions)",
            "config": {"workload": workload, "parameters": P.name, "pairs_per_gpu": K,
                       "global_pairs": world * K, "pbs_per_multiply": pbs_per_mul,
                       "launches_per_multiply_batch": launches,
                       "parallelism": f"dp{world} (whole multiplies sharded, keys broadcast once)"},
            "pbs_per_sec": pbs_rate,
            "roofline": {"bound": "hbm", "kernel": kname,
                         "achieved": pbs_rate * pbs_algorithmic_bytes(P) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": pbs_rate * pbs_algorithmic_bytes(P) / 1e9 / HBM_PEAK_GBS,
                         "traffic": None,
                         "model": "BSK-streaming bytes per PBS x PBS/s of the whole DAG (host orchestration included)"},
            "check": {"decrypted_ok": int(okt[0].item()), "of": int(okt[1].item())},
        }
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, ROOT)
            from oracle.oracle import OracleEngine  # oracle behind the engine API (test infrastructure)

            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            oe = OracleEngine(P, threads=threads)
            oe.upload_bootstrap_key(bsk)
            oe.upload_keyswitch_key(ksk)
            csk = integer.ServerKey(shortint.ServerKey(None, engine=oe, parameters=P))
            t = time.perf_counter()
            csk.mul_parallelized(RadixSlice(ca, 2), RadixSlice(cb, 2))
            cw = time.perf_counter() - t
            line["cpu_baseline"] = {
                "value": 2 / cw, "unit": "mul/s", "cores": threads, "kind": "port",
                "sample": (f"2 FheUint32 multiplies through the same DAG with the oracle C restatement behind "
                           f"the engine API, {threads} threads ({cw:.1f} s); reference published 333 ms/mul "
                           f"on a 128-vCPU m6i.metal (benchmarks.md:17)"),
            }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def RadixSlice(rb, n):
    from tfhe_mi355.integer import RadixBatch

    return RadixBatch(rb.data[:n].copy(), list(rb.degree), list(rb.noise))


if __name__ == "__main__":
    main()
