#!/usr/bin/env python3
"""bench.py -- programmable bootstraps/sec at PARAM_MESSAGE_2_CARRY_2 on 1/2/4/8 MI355X.

BASELINE.json metric "programmable bootstraps/sec (PARAM_MESSAGE_2_CARRY_2) at 1/2/4/8 MI355X",
workload = BASELINE config 2: a batch of 4096 independent classic PBS per GPU, identity LUT
(PARAM_MESSAGE_2_CARRY_2_KS_PBS: n=742, k=1, N=2048, L=1, base 2^23).  One step = one PBS
launch over the GPU's batch (blind rotation + sample extraction), inputs resident in HBM.
Model: the reference's throughput bench, tfhe/benches/core_crypto/pbs_bench.rs:430-549.

Multi-GPU (weak scaling): one process per GPU.  `python bench.py --gpus N` with no
WORLD_SIZE in the environment starts `python -m torch.distributed.run --nproc-per-node N bench.py
...` as a child process (before anything touches the GPU) and exits with its return code; the
driver may also launch the ranks itself.  The global batch (N x the per-GPU batch) is split into
contiguous shards (`shard_range`); the standard BSK is generated once on rank 0 and broadcast
ONCE over RCCL (xGMI); each rank converts it to the Fourier domain on its own GPU and bootstraps
its shard -- no collective in the timed loop except the bracketing barriers.  value = sum of PBS
over ranks / max wall time over ranks.

The JSON line also carries the roofline of the dominant kernel (FP64-VALU bound; its duration from
the engine's per-kernel HIP-event timer on the launch stream -- DESIGN.md 6), the measured traffic
and issue counters of that same kernel from the committed per-kernel rocprofv3 PMC summaries
(profiles/r03_pmc_*.json), the rates of the host-pointer C ABI (PCIe-inclusive, and the
reference's one-ciphertext-per-call pattern from native threads; never `value`) and the CPU
baseline (oracle C restatement, 1 PBS per thread on the host's CPU share, rank 0, N = 1 only).
The default run also measures the other BASELINE configurations (`other_workloads`), at N > 1
on every rank of the job.

`--launch-selftest` runs the rank/shard/aggregation code with a stub step on the CPU (gloo), so
that the multi-rank path is testable without a GPU (tests/test_bench_launch.py).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-odd_amd"))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
# measured ceiling of a streaming kernel (2 reads : 1 write, 16-byte lanes) whose 96-255 MiB working
# set stays in the Infinity Cache: 6.5-7.0 TB/s; 5.0-5.6 TB/s from HBM (768 MiB)
# (scripts/probes/mall_stream_probe.hip, profiles/r03_mall_stream_probe.log)
MALL_STREAM_GBS = 6970.0
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 vector (= matrix) spec, SURVEY.md 8d


PARAMS = {  # --params choice -> (parameter set name, workload text, kernel name)
    "2_2": ("PARAM_MESSAGE_2_CARRY_2_KS_PBS",
            "BASELINE config 2: batch of 4096 independent classic PBS per GPU, identity LUT",
            "pbs_classic_kernel<2048,1,1>"),
    "2_2ks": ("PARAM_MESSAGE_2_CARRY_2_KS_PBS",
              "shortint keyswitch -> PBS (apply_lookup_table, shortint/server_key/mod.rs:783-857) over a batch "
              "of 4096 big-key ciphertexts per GPU, identity LUT; the reference publishes 16.6 ms per KS+PBS "
              "(benchmarks.md:42)",
              "pbs_classic_kernel<2048,1,1> (+ ks_digits_kernel + ks_mfma_kernel)"),
    "mb3": ("PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_3_KS_PBS",
            "BASELINE config 5: batch of 4096 independent multi-bit (grouping 3) PBS per GPU, identity LUT",
            "pbs_multibit_shared_kernel<2048,1,1,3>"),
    "4_4": ("PARAM_MESSAGE_4_CARRY_4_KS_PBS",
            "BASELINE config 3: shortint apply_lookup_table (keyswitch -> PBS) at N=32768 per GPU batch",
            "large_group_cmux_kernel (+ large_digits_kernel + large_top_inv_kernel<1> per CMUX, ks_mfma_kernel)"),
    "mul32": ("PARAM_MESSAGE_2_CARRY_2_KS_PBS",
              "BASELINE config 4: FheUint32 multiply (16-block radix DAG, radix_parallel/mul.rs), "
              "K independent pairs per GPU, every DAG layer one batched KS+PBS launch, the whole DAG "
              "replayed as one hipGraph",
              "pbs_classic_kernel<2048,1,1> + ks_mfma_kernel"),
    "mb2": ("PARAM_MULTI_BIT_MESSAGE_2_CARRY_2_GROUP_2_KS_PBS",
            "batch of 4096 independent multi-bit (grouping 2) PBS per GPU, identity LUT",
            "pbs_multibit_shared_kernel<2048,1,1,2>"),
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



def mb_digits_on() -> bool:
    """The multi-bit pair kernel reads packed digits (pbs_large.hip mb_dig) unless switched off."""
    return all(os.environ.get(v, "1") != "0" for v in ("TFHE_MI355_MB_DIGITS", "TFHE_MI355_MB_FUSED", "TFHE_MI355_MB_PAIR2"))


def _split_params():
    """`--params m_c`: every shortint KS_PBS set at N = 4096 ... 32768 (the split CMUX, pbs_large.hip)
    as a shortint apply_lookup_table (KS -> PBS) batch; 4_4 keeps its grouped-CMUX entry above."""
    sys.path.insert(0, os.path.join(ROOT, "tfhe-rs-odd_amd"))
    from tfhe_mi355.parameters import SHORTINT_ALL, SHORTINT_SOURCE_LINE

    out = {}
    for name, p in SHORTINT_ALL.items():
        if p.polynomial_size < 4096 or not name.endswith("_KS_PBS"):
            continue
        tag = f"{p.message_modulus.bit_length() - 1}_{p.carry_modulus.bit_length() - 1}"
        if tag == "4_4":
            continue
        out[tag] = (name, f"shortint apply_lookup_table (keyswitch -> PBS) at {name} (shortint/parameters/mod.rs:"
                          f"{SHORTINT_SOURCE_LINE[name]}), N={p.polynomial_size}, batch per GPU; the reference publishes "
                          + ("121 ms per KS+PBS at 3_3 (benchmarks.md:42)" if tag == "3_3" else "no number for this set"),
                    (f"onchip_cmux_kernel<{p.polynomial_size},"
                     f"{'true' if p.pbs_level * p.pbs_base_log <= 30 else 'false'},{p.pbs_level}> "
                     "(the whole blind rotation per workgroup, ks_mfma_kernel)"
                     if p.pbs_level <= 2 and p.polynomial_size in (4096, 8192) and os.environ.get("TFHE_MI355_ONCHIP", "1") != "0"
                     else f"large_dsub_kernel<{p.polynomial_size}> (+ split_digits/large_top_inv per CMUX, ks_mfma_kernel)"
                     if p.pbs_level == 2 and p.polynomial_size <= 8192 else
                     f"large_sub_kernel<{p.polynomial_size},1,{p.pbs_level}> (+ large_top_fwd/top_inv per CMUX, "
                     "ks_mfma_kernel)"))
    # the multi-bit sets at N = 8192 (shortint/parameters/multi_bit.rs:134-153, 192-210): the split
    # CMUX with the keybundle built inside large_sub_kernel, one CMUX per group of g
    from tfhe_mi355.parameters import MULTI_BIT_ALL

    for g, line in ((2, 134), (3, 192)):
        name = f"PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_{g}_KS_PBS"
        p = MULTI_BIT_ALL[name]
        out[f"mb3_3g{g}"] = (name, f"shortint apply_lookup_table (keyswitch -> multi-bit PBS, grouping {g}) at {name} "
                                   f"(shortint/parameters/multi_bit.rs:{line}), N={p.polynomial_size}, batch per GPU; "
                                   "the reference publishes no number for this set",
                             (f"large_mb_pair2_kernel<{p.polynomial_size},{g},{'true' if mb_digits_on() else 'false'}> "
                              "(+ large_mb_inv_fwd per group: packed "
                              "digits in, twist + top DIF in the pair kernel; ks_mfma_kernel)" if os.environ.get("TFHE_MI355_MB_PAIR2", "1") != "0" else
                              f"large_pair_sub_kernel<{p.polynomial_size},1,{p.pbs_level},{g},1> (+ large_top_fwd/top_inv "
                              "per group, ks_mfma_kernel)"))
    return out


PARAMS.update(_split_params())
SPLIT_TAGS = {t for t, v in PARAMS.items()
              if v[2].startswith(("large_sub_kernel", "large_pair_sub_kernel", "large_mb_pair2_kernel", "large_dsub_kernel",
                                  "onchip_cmux_kernel"))}
WITH_KS = {"4_4", "2_2ks"} | SPLIT_TAGS


# ---------------------------------------------------------------------------------------------
# models

def ggsw_count(p) -> int:
    g = p.grouping_factor
    return (p.lwe_dimension // g) << g if g else p.lwe_dimension


def fourier_bsk_bytes(p) -> int:
    M = p.polynomial_size // 2
    k1 = p.glwe_dimension + 1
    return ggsw_count(p) * p.pbs_level * k1 * k1 * M * 16


def io_bytes(p, with_ks: bool) -> int:
    """Per ciphertext: LWE in (big key when keyswitched first) + LWE out."""
    big = p.glwe_dimension * p.polynomial_size + 1
    return 8 * ((big if with_ks else p.lwe_dimension + 1) + big)


def pbs_streaming_bytes(p) -> int:
    """BSK-streaming model: |BSK_fourier| + 8(n+1) + 8(kN+1) + 8(k+1)N (every PBS reads the whole
    key once; multi-bit: (n/g) 2^g GGSWs)."""
    return fourier_bsk_bytes(p) + io_bytes(p, False) + 8 * (p.glwe_dimension + 1) * p.polynomial_size


def pbs_min_unique_bytes(p, batch: int, with_ks: bool) -> float:
    """Minimal unique bytes per PBS at batch B: |BSK|/B (+ |KSK|/B) + in + out + LUT/B."""
    b = fourier_bsk_bytes(p) + 8 * (p.glwe_dimension + 1) * p.polynomial_size
    if with_ks:
        b += 8 * p.glwe_dimension * p.polynomial_size * p.ks_level * (p.lwe_dimension + 1)
    return b / batch + io_bytes(p, with_ks)


def pbs_flops(p) -> float:
    """Per CMUX ((k+1)L + (k+1)) (5 M log2 M + 6 M) + (k+1)^2 L M 8, times n.  Multi-bit: the same
    external product per group of g, plus the keybundle's (2^g - 1) complex FMAs (8 flop) per
    GGSW element, times n/g."""
    M = p.polynomial_size // 2
    k1 = p.glwe_dimension + 1
    per = (k1 * p.pbs_level + k1) * (5 * M * math.log2(M) + 6 * M) + k1 * k1 * p.pbs_level * M * 8
    g = p.grouping_factor
    if g:
        per += ((1 << g) - 1) * k1 * k1 * p.pbs_level * M * 8
        return per * (p.lwe_dimension // g)
    return per * p.lwe_dimension


PMC_ALIAS = {"mul32": "2_2ks"}  # the multiply DAG runs the 2_2 KS+PBS kernels: per-PBS traffic of that workload
PMC_ROUNDS = ("r06b", "r06", "r05", "r04", "r03")  # newest committed PMC summary first (kernels unchanged since are still described by it)

# dominant kernel of each workload: (kernel-timer family, rocprofv3 name normalised as
# scripts/pmc_workload.py does).  Its average duration comes from the engine's HIP-event timer
# on the launch stream (tfhe_mi355_kernel_timing_*), its counters from the PMC file.
DOMINANT = {
    "2_2": ("pbs_classic_kernel", "pbs_classic_kernel<2048,1,1>"),
    "2_2ks": ("pbs_classic_kernel", "pbs_classic_kernel<2048,1,1>"),
    "mul32": ("pbs_classic_kernel", "pbs_classic_kernel<2048,1,1>"),
    "mb3": ("pbs_multibit", "pbs_multibit_shared_kernel<2048,1,1,3>"),
    "mb2": ("pbs_multibit", "pbs_multibit_shared_kernel<2048,1,1,2>"),
    "4_4": ("large_group_cmux_kernel", "large_group_cmux_kernel"),
    "manticore": ("pbs_classic_kernel", "pbs_classic_kernel<1024,1,2>"),
    "ascon": ("pbs_classic_kernel", "pbs_classic_kernel<1024,2,3>"),
    "simon": ("pbs_classic_kernel", "pbs_classic_kernel<512,3,2>"),
    "tfhelib": ("pbs_classic_kernel", "pbs_classic_kernel<1024,2,1>"),
    "aes40": ("pbs_classic_kernel", "pbs_classic_kernel<512,3,4>"),
    "sha3": ("pbs_classic_kernel", "pbs_classic_kernel<256,5,1>"),
}
DOMINANT.update({t: (PARAMS[t][2].split("<")[0], PARAMS[t][2].split(" ")[0]) for t in SPLIT_TAGS})


def pmc_entry(by_kernel: dict, kernel: str):
    """The entry of `kernel` in a per-kernel PMC summary: its exact normalised rocprofv3 name, else
    (a timer family name without template arguments) the one instantiation of that family."""
    if kernel in by_kernel:
        return by_kernel[kernel]
    if "<" not in kernel:
        hits = [v for k, v in by_kernel.items() if k == kernel or k.startswith(kernel + "<")]
        if len(hits) == 1:
            return hits[0]
    return None


def load_pmc(tag: str, kernel: str):
    """The committed rocprofv3 PMC summary of this workload (scripts/pmc_workload.sh ->
    profiles/r04_pmc_<tag>.json, else r03) and its entry for `kernel`.  A file without an entry for the
    kernel the bench times is refused (returns the reason instead): counters of another kernel
    are not evidence for this one."""
    for rnd in PMC_ROUNDS:
        name = f"{rnd}_pmc_{PMC_ALIAS.get(tag, tag)}.json"
        path = os.path.join(ROOT, "profiles", name)
        if os.path.exists(path):
            break
    else:
        return None, f"no PMC summary profiles/{PMC_ROUNDS[0]}_pmc_{PMC_ALIAS.get(tag, tag)}.json"
    d = json.load(open(path))
    e = pmc_entry(d.get("by_kernel") or {}, kernel)
    if e is None:
        return None, (f"refused: profiles/{name} holds counters for {sorted(d.get('by_kernel') or {})}, "
                      f"not for the timed kernel {kernel}")
    e = dict(e)
    e.pop("sq_counters_sum", None)
    e["_file"] = f"profiles/{name}"
    e["_all"] = d.get("by_kernel")
    return e, None


def large_group_flops(p) -> float:
    """FP64 flop of large_group_cmux_kernel per ciphertext and CMUX (k = 1, L = 2):
    twist of the (k+1)L digit polynomials (6 flop per point), their whole forward FFTs (the top
    radix-16 share and the 1024-point sub-FFTs: 5 M log2 M each), the MAC ((k+1)^2 L M 8) and the
    (k+1) inverse sub-FFTs (5 M log2(1024) each; the top DIT stage runs in large_top_inv)."""
    M = p.polynomial_size // 2
    k1, L = p.glwe_dimension + 1, p.pbs_level
    return (k1 * L * (6 * M + 5 * M * math.log2(M)) + k1 * k1 * L * M * 8 + k1 * 5 * M * 10)


def split_sub_flops(p) -> float:
    """FP64 flop of large_sub_kernel per ciphertext and CMUX (split CMUX, pbs_large.hip): the
    1024-point forward sub-FFTs of the (k+1)L digit polynomials (5 M log2(1024) each, M = R 1024),
    the MAC ((k+1)^2 L M 8) and the (k+1) inverse sub-FFTs; the top radix-R stages and the twist run
    in large_top_fwd / large_top_inv."""
    M = p.polynomial_size // 2
    k1, L = p.glwe_dimension + 1, p.pbs_level
    g = p.grouping_factor
    # multi-bit: one launch per group of g, the keybundle's (2^g - 1) monomial-weighted GGSW sums
    # (8 flop per element, as pbs_flops) built in the same kernel
    kb = ((1 << g) - 1) * k1 * k1 * L * M * 8 if g else 0
    return k1 * L * 5 * M * 10 + k1 * k1 * L * M * 8 + k1 * 5 * M * 10 + kb


def split_dsub_flops(p) -> float:
    """FP64 flop of large_dsub_kernel per ciphertext and CMUX (digits-fed split CMUX, L = 2): the
    twist (6 M) and top radix-R stage (5 M log2 R) of the (k+1)L digit polynomials -- counted once,
    as the algorithm needs them, although each of the R sub-block workgroups recomputes its share --
    plus large_sub_kernel's sub-FFTs and MAC."""
    M = p.polynomial_size // 2
    R = M // 1024
    k1, L = p.glwe_dimension + 1, p.pbs_level
    return k1 * L * (6 * M + 5 * M * math.log2(R)) + split_sub_flops(p)


def split_chunk(p, units: int) -> int:
    """Ciphertexts per pass of the split CMUX (capi.cpp large_chunk)."""
    if p.polynomial_size >= 32768:
        return min(units, 128)
    if p.grouping_factor:
        return min(units, 1024)
    M, k1 = p.polynomial_size // 2, p.glwe_dimension + 1
    per = k1 * p.polynomial_size * 8 + p.pbs_level * k1 * M * 16
    return min(units, min(1024, max(64, (200 << 20) // per // 64 * 64)))


def large_memory_model(p):
    """Bytes per ciphertext and CMUX of the two memory kernels of the N = 32768 grouped CMUX
    (DESIGN.md 5.3): large_digits reads the accumulator rows (twice: self and rotated) and writes
    the packed digits; large_top_inv reads U and the accumulator and writes the accumulator."""
    M, N = p.polynomial_size // 2, p.polynomial_size
    k1 = p.glwe_dimension + 1
    return {"large_digits_kernel": 2 * k1 * N * 8 + k1 * M * 8,
            "large_top_inv_kernel": k1 * M * 16 + 2 * k1 * N * 8}


def roofline(tag, p, units_per_launch: int, step_ms: float, kname: str, with_ks: bool, ktimes: dict | None):
    """Roofline object of the DOMINANT kernel (FP64-VALU bound for every PBS kernel here: DESIGN.md
    5): achieved = its algorithmic flop per launch / its average launch duration from the engine's
    HIP-event timer on the launch stream; traffic and VALU issue from the PMC entry of that same
    kernel.  The whole step's FP64 rate and the HBM/fabric byte models sit beside it."""
    fam, pmc_name = DOMINANT.get(tag, ("pbs_classic_kernel", kname))
    steps_flop = pbs_flops(p) * units_per_launch
    fp64_step = steps_flop / (step_ms * 1e-3) / 1e12
    # the on-chip CMUX runs every CMUX of the batch in one launch: the whole-PBS flop model per launch
    large = p.polynomial_size > 2048 and fam != "onchip_cmux_kernel"
    grouped = p.polynomial_size == 32768 and p.pbs_level == 2 and p.glwe_dimension == 1
    chunk = split_chunk(p, units_per_launch) if large else units_per_launch
    kt = (ktimes or {}).get(fam)
    if kt:
        kernel_ms, timed = kt
        kernel_src = f"engine HIP-event timer on the launch stream, {timed} timed launches"
    else:  # one launch per step (or a replayed graph): the step's own events
        kernel_ms, timed = step_ms, None
        kernel_src = "HIP events around the whole step on the launch stream (no per-kernel timer)"
    # digits-fed kernels (the twist + top radix-R share inside): large_dsub, and the multi-bit pair kernel
    # unless TFHE_MI355_MB_DIGITS=0 / TFHE_MI355_MB_FUSED=0
    dsub = large and (fam == "large_dsub_kernel" or (fam == "large_mb_pair2_kernel" and mb_digits_on()))
    flop_launch = ((large_group_flops(p) if grouped else split_dsub_flops(p) if dsub else split_sub_flops(p)) * chunk
                   if large else steps_flop)
    fp64 = flop_launch / (kernel_ms * 1e-3) / 1e12
    if tag == "mul32":
        pmc, why = None, ("the multiply DAG replays the 2_2 KS+PBS kernels in one hipGraph: their per-kernel "
                          "counters are those of the 2_2ks line")
    else:
        pmc, why = load_pmc(tag, pmc_name)
    traffic = pmc.get("hbm_bytes_per_dispatch") if pmc else None
    r = {"bound": "fp64-valu", "achieved": fp64, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
         "frac": fp64 / FP64_PEAK_TFLOPS, "traffic": traffic,
         "kernel": pmc_name, "kernel_ms": kernel_ms, "kernel_ms_source": kernel_src,
         "flop_per_launch": flop_launch,
         "units_per_launch": chunk,
         "model": ((f"large_group_cmux_kernel FP64 flop per ciphertext and CMUX {large_group_flops(p):,.0f} "
                    f"(twist, forward FFTs incl. the top radix-16 share, MAC, inverse sub-FFTs) x {chunk} ciphertexts "
                    f"per launch / its average launch duration") if grouped else
                   (f"{fam} FP64 flop per ciphertext and {'group' if p.grouping_factor else 'CMUX'} "
                    f"{(split_dsub_flops(p) if dsub else split_sub_flops(p)):,.0f} ("
                    f"{'twist and top radix-R share, ' if dsub else ''}1024-point forward and inverse sub-FFTs, MAC"
                    f"{', keybundle' if p.grouping_factor else ''}) x {chunk} ciphertexts per launch / its average "
                    f"launch duration") if large else
                   (f"FP64 flop model (SURVEY.md 8d): {pbs_flops(p):,.0f} flop per PBS x {units_per_launch} PBS per "
                    f"launch / the kernel's average launch duration")),
         "traffic_note": ("L2<->fabric bytes per launch of this kernel (2 FETCH_SIZE + WRITE_SIZE, gfx950 correction; "
                          "Infinity-Cache hits included)" if pmc else why),
         "whole_step": {"fp64_tflops": fp64_step, "frac": fp64_step / FP64_PEAK_TFLOPS, "step_ms": step_ms,
                        "flop_per_pbs": pbs_flops(p),
                        "note": "PBS flop model x PBS per step / step time" + (
                            " (keyswitch included in the time, its int8 MFMA work not counted)" if with_ks else "")}}
    if pmc:
        r["valu_issue"] = {k: pmc.get(k) for k in ("sq_active_inst_valu_per_wave_cycle", "avg_waves_per_simd",
                                                   "valu_busy", "sq_wait_inst_any_per_wave_cycle",
                                                   "sq_wait_any_per_wave_cycle", "lds_bank_conflict_frac",
                                                   "l2_hit_rate") if pmc.get(k) is not None}
        r["valu_issue"]["source"] = pmc["_file"]
        r["valu_issue"]["note"] = ("per-wave-cycle fractions x avg_waves_per_simd = share of SIMD issue cycles; "
                                   "valu_busy = the same over GRBM_GUI_ACTIVE x 1024 SIMDs (scripts/pmc_workload.py)")
    stream_b = pbs_streaming_bytes(p) + (io_bytes(p, True) - io_bytes(p, False) if with_ks else 0)
    secs = step_ms * 1e-3
    r["hbm"] = {"streaming_model_bytes_per_pbs": stream_b,
                "streaming_model_GBps": stream_b * units_per_launch / secs / 1e9,
                "min_unique_bytes_per_pbs": pbs_min_unique_bytes(p, units_per_launch, with_ks),
                "note": "BSK-streaming model (SURVEY.md 8d) over the whole step; >8 TB/s means on-chip reuse"}
    if grouped and ktimes:
        mem = {}
        for kn, b in large_memory_model(p).items():
            t = ktimes.get(kn)
            if not t:
                continue
            e = pmc_entry((pmc or {}).get("_all") or {}, kn) or {}
            ach = b * chunk / (t[0] * 1e-3) / 1e9
            mem[kn] = {"bound": "fabric (L2 <-> Infinity Cache / HBM)", "model_bytes_per_launch": b * chunk,
                       "kernel_ms": t[0], "achieved_GBps": ach, "frac_of_hbm_peak": ach / HBM_PEAK_GBS,
                       "frac_of_mall_stream_ceiling": ach / MALL_STREAM_GBS,
                       "pmc_bytes_per_launch": e.get("hbm_bytes_per_dispatch")}
        r["memory_kernels"] = mem
        r["memory_kernels_note"] = (f"per-CMUX memory kernels on a chunk of {chunk}: the chunk's accumulators, digits "
                                    "and sub-block outputs (~1.5 MiB per ciphertext) stay in the 256 MB Infinity Cache, "
                                    "so these byte rates are fabric rates, not DRAM rates (MI355X_MICROARCH.md 'HBM'); "
                                    "a streaming probe with a cache-resident working set tops out at 6.97 TB/s "
                                    "(profiles/r03_mall_stream_probe.log)")
    if ktimes:
        r["kernel_times_ms"] = {k: v[0] for k, v in ktimes.items()}
    return r


# ---------------------------------------------------------------------------------------------
# host / CPU baseline

def cpu_share() -> int:
    """Threads the CPU baseline may use: the process's affinity set, capped by OMP_NUM_THREADS
    (the GPU box exports its per-GPU CPU share there: 16)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(aff, cap) if cap > 0 else aff)


def host_info() -> dict:
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = None
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(params, bsk, cts, acc, threads: int, ksk=None):
    """The oracle's PBS (C restatement of the reference fft64 PBS) on the host cores, as the
    reference's pbs_throughput bench (benches/core_crypto/pbs_bench.rs:430-549: independent
    ciphertexts over all threads), through oracle/pbs_simd.c: W ciphertexts per SIMD register
    (AVX-512: 8, AVX2: 4), every lane the oracle's exact operation sequence (classic and
    multi-bit, bit-identical: tests/test_oracle_simd.py).  With `ksk`
    each ciphertext is keyswitched first (scalar oracle keyswitch, threads split the batch)."""
    sys.path.insert(0, ROOT)
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O

    p = params

    def ks(batch):
        if ksk is None:
            return batch
        parts = np.array_split(batch, min(threads, batch.shape[0]))
        with ThreadPoolExecutor(len(parts)) as ex:
            outs = list(ex.map(lambda c: O.keyswitch_simd(ksk, p.big_lwe_dimension, p.lwe_dimension, p.ks_base_log,
                                                          p.ks_level, c), parts))
        return np.concatenate(outs)

    O.build()
    if params.grouping_factor:
        fb = O.MultiBitFourierBsk(bsk, params.lwe_dimension, params.glwe_dimension, params.polynomial_size,
                                  params.pbs_base_log, params.pbs_level, params.grouping_factor)
    else:
        fb = O.FourierBsk(bsk, params.lwe_dimension, params.glwe_dimension, params.polynomial_size,
                          params.pbs_base_log, params.pbs_level)
    lanes = O.simd_lib().simd_width()
    run = fb.pbs_simd
    how = (f"oracle/pbs_simd.c: {lanes} ciphertexts per {'AVX-512' if lanes == 8 else 'AVX2'} register, each lane "
           f"the oracle's exact op sequence (bit-identical), {lanes} PBS per thread step")
    run(ks(cts[:lanes]), acc, threads=1)  # warm (page-in, tables)
    t = time.perf_counter()
    run(ks(cts[:lanes]), acc, threads=1)
    t1 = (time.perf_counter() - t) / lanes
    # about 15 s of CPU work in total, rounded to whole rounds of `threads` x `lanes`
    step = threads * lanes
    count = max(step, int(round(15.0 / max(t1, 1e-3))))
    count = min(((count + step - 1) // step) * step, cts.shape[0])
    t = time.perf_counter()
    run(ks(cts[:count]), acc, threads=threads)
    wall = time.perf_counter() - t
    ref = "811 ms" if p.polynomial_size == 32768 else "16.6 ms"
    label = "4_4" if p.polynomial_size == 32768 else "2_2"
    h = host_info()
    kp = "KS+" if ksk is not None else ""
    return {
        "value": count / wall,
        "unit": "KS+PBS/s" if ksk is not None else "PBS/s",
        "cores": threads,
        "kind": "port",
        "host": h,
        "single_thread_ms": t1 * 1e3,
        "lanes_per_thread": lanes,
        "sample": (f"{count} {kp}PBS of the same {params.name} batch, {how}, on {threads} threads = this process's "
                   f"CPU share ({wall:.1f} s wall) on {h['cpu_model']} (nproc {h['nproc']}); single-thread "
                   f"{t1 * 1e3:.1f} ms per {kp}PBS (throughput per core) against the reference's published {ref} "
                   f"KS+PBS latency at {label} (Xeon 8375C, concrete-fft AVX-512 within one FFT, "
                   f"benchmarks.md:42)"),
    }


# ---------------------------------------------------------------------------------------------
# ranks

def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """--gpus N without a launcher: start N ranks with torch.distributed.run as a child process
    (nothing in this process has touched the GPU) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# The other BASELINE configurations measured beside the headline by the default run:
# (entry name, --params, extra options).  `4_4_full` is config 3 at its stated size (65,536
# ciphertexts in one call, a GLOBAL batch: split over the ranks at N > 1, i.e. strong scaling for
# that entry), warmed up on its first 1024 ciphertexts.
# `callers`: the entry also measures the reference's calling pattern (one ciphertext per blocking
# call from 1 / 64 / 256 native threads, and 256 submitted requests from one thread), every row
# checked against a batched call (bench.py --callers-only).
OTHER_WORKLOADS = (
    ("2_2ks", "2_2ks", {"steps": 3, "callers": True}),
    ("mb3", "mb3", {"steps": 3, "callers": True}),
    ("mb2", "mb2", {"steps": 3}),
    ("4_4", "4_4", {"steps": 3}),
    ("mul32", "mul32", {"steps": 2}),
    ("4_4_full", "4_4", {"steps": 1, "global_batch": 65536, "warmup_batch": 1024}),
    ("3_3", "3_3", {"steps": 3, "callers": True}),
    ("mb3_3g3", "mb3_3g3", {"steps": 3, "callers": True}),
    # the other on-chip CMUX shapes: N = 4096 L = 2 (two ciphertexts per workgroup)
    # and N = 8192 L = 1
    ("1_4", "1_4", {"steps": 3}),
    ("6_0", "6_0", {"steps": 3}),
)
# Wall-clock budget of one such workload (keys, warm-up, steps, checks).  N = 1: the child's
# subprocess timeout; N > 1: a per-rank watchdog (below).  BENCH_WORKLOAD_BUDGET_S overrides.
WORKLOAD_BUDGET_S = 420.0


def workload_budget() -> float:
    return float(os.environ.get("BENCH_WORKLOAD_BUDGET_S", WORKLOAD_BUDGET_S))


def callers_summary(host_abi: dict | None) -> dict | None:
    """Compact form of host_abi.single_ct: calls/s at 1 / 16 / 64 / 256 blocking callers and of the
    submitted windows, with the total of rows that differed from the batched call."""
    sct = (host_abi or {}).get("single_ct")
    if not sct:
        return None
    out = {f"callers_{t}": round(v["value"], 1) for t, v in sct.get("callers", {}).items()}
    out.update({f"submit_{w}": round(v["value"], 1) for w, v in sct.get("submit_wait", {}).items()})
    if "64" in sct.get("callers", {}):
        out["callers_64_frac_of_batched"] = round(sct["callers"]["64"]["frac_of_batched_device_rate"], 3)
    out["mismatching_rows"] = int(sum(v["mismatching_rows"] + v["failed_calls"]
                                      for grp in ("callers", "submit_wait") for v in sct.get(grp, {}).values()))
    return out


def summarize(line: dict) -> dict:
    rl = line.get("roofline") or {}
    out = {"value": line["value"], "unit": line["unit"], "ms_per_step": line["ms_per_step"],
           "steps": line["steps"], "n_gpus": line["n_gpus"], "world_size": line.get("world_size"),
           "scaling": line.get("scaling"), "workload": line["config"]["workload"],
           "batch": line["config"].get("global_batch", line["config"].get("global_pairs")),
           "kernel": rl.get("kernel"), "bound": rl.get("bound"), "frac": rl.get("frac"),
           "check": line.get("check"), "setup": line.get("setup"),
           "single_call_latency_ms": line.get("single_call_latency_ms")}
    cs = callers_summary(line.get("host_abi"))
    if cs:
        out["callers"] = cs
    if "ctx_devices" in line:
        out["ctx_devices"] = line["ctx_devices"]
    return out


def compact_summary(line: dict) -> dict:
    """One short entry per workload (value, roofline frac, one-call latency, 1 / 64 / 256 blocking
    callers, 256 submitted, rows that differed), printed as the LAST key of the JSON line and on
    stderr, so that a tail of the output keeps every configuration's numbers."""
    def one(e):
        c = e.get("callers") or {}
        pairs = (("v", round(e["value"], 1) if e.get("value") is not None else None),
                 ("frac", round(e["frac"], 3) if e.get("frac") is not None else None),
                 ("lat_ms", round(e["single_call_latency_ms"], 2) if e.get("single_call_latency_ms") is not None
                  else None),
                 ("c1", c.get("callers_1")), ("c64", c.get("callers_64")), ("c256", c.get("callers_256")),
                 ("s1x256", c.get("submit_1x256")), ("bad", c.get("mismatching_rows")))
        return {k: v for k, v in pairs if v is not None}
    out = {"2_2": one(summarize(line))}
    for k, v in (line.get("other_workloads") or {}).items():
        out[k] = one(v) if "error" not in v else {"error": str(v["error"])[:80]}
    return out


def _child_args(args, params, opts) -> list:
    a = ["--params", params, "--steps", str(opts["steps"]), "--warmup", str(opts.get("warmup", 1)),
         "--no-cpu-baseline", "--seed", str(args.seed)]
    a += ["--callers-only"] if opts.get("callers") else ["--no-host-abi"]
    if opts.get("global_batch"):
        a += ["--global-batch", str(opts["global_batch"])]
    if opts.get("warmup_batch"):
        a += ["--warmup-batch", str(opts["warmup_batch"])]
    return a


def other_workloads(args) -> dict:
    """N = 1: the other configurations, each run once as a child `bench.py --params X` BEFORE this
    process touches the GPU, so the default run also measures them under the caller's clock;
    summarised into the headline line (the headline value stays the 2_2 PBS rate).  A failed
    child is reported, not fatal."""
    res = {}
    for name, params, opts in OTHER_WORKLOADS:
        cmd = [sys.executable, os.path.abspath(__file__)] + _child_args(args, params, opts)
        t = time.perf_counter()
        budget = workload_budget()
        try:
            cp = subprocess.run(cmd, capture_output=True, text=True, timeout=budget)
            lines = [l for l in cp.stdout.splitlines() if l.startswith("{")]
            if cp.returncode != 0 or not lines:
                res[name] = {"error": f"rc={cp.returncode}: {cp.stderr.strip()[-300:]}"}
            else:
                res[name] = summarize(json.loads(lines[-1]))
        except subprocess.TimeoutExpired:
            res[name] = {"error": f"timeout after {budget:.0f} s"}
        res[name]["wall_s"] = time.perf_counter() - t
        print(f"bench.py: {name} done in {res[name]['wall_s']:.1f} s", file=sys.stderr, flush=True)
    # the one-process multi-device context on this GPU listed twice (its split / replication overhead)
    cmd = [sys.executable, os.path.abspath(__file__), "--ctx-devices", "0,0", "--steps", "3", "--warmup", "1",
           "--seed", str(args.seed)]
    t = time.perf_counter()
    try:
        cp = subprocess.run(cmd, capture_output=True, text=True, timeout=workload_budget())
        lines = [l for l in cp.stdout.splitlines() if l.startswith("{")]
        res["ctx_devices"] = (summarize(json.loads(lines[-1])) if cp.returncode == 0 and lines
                              else {"error": f"rc={cp.returncode}: {cp.stderr.strip()[-300:]}"})
    except subprocess.TimeoutExpired:
        res["ctx_devices"] = {"error": f"timeout after {workload_budget():.0f} s"}
    res["ctx_devices"]["wall_s"] = time.perf_counter() - t
    print(f"bench.py: ctx_devices done in {res['ctx_devices']['wall_s']:.1f} s", file=sys.stderr, flush=True)
    return res


def ctx_devices_ranks(args, R, emit=None) -> dict:
    """N > 1: after every per-rank workload, rank 0 alone runs the one-process multi-device context
    over all the job's devices (ctx_devices_line) while the other ranks wait on the process group's
    key-value store (no collective kernel spinning on their GPUs meanwhile).  Under the same per-rank
    watchdog as the other entries; an error is reported in the entry, not fatal."""
    import datetime
    import threading

    R.barrier()
    budget = workload_budget()
    res = {}
    store = None
    try:
        store = R.dist.distributed_c10d._get_default_store()
    except Exception:
        store = None
    t = time.perf_counter()
    if R.rank == 0:
        def over_budget():
            res["ctx_devices"] = {"error": f"over its {budget:.0f} s budget (watchdog)", "wall_s": time.perf_counter() - t}
            if emit is not None:
                emit(res)
            sys.stdout.flush()
            os._exit(3)

        dog = threading.Timer(budget, over_budget)
        dog.daemon = True
        dog.start()
        try:
            import torch

            visible = max(1, torch.cuda.device_count())
            devs = [d % visible for d in range(R.world)]  # a rehearsal with fewer GPUs lists a device twice
            a = argparse.Namespace(**vars(args))
            a.steps, a.warmup = 3, 1
            res["ctx_devices"] = summarize(ctx_devices_line(a, devs))
        except Exception as ex:  # reported, not fatal
            res["ctx_devices"] = {"error": repr(ex)[:300]}
        finally:
            dog.cancel()
        res["ctx_devices"]["wall_s"] = time.perf_counter() - t
        print(f"bench.py: ctx_devices done in {res['ctx_devices']['wall_s']:.1f} s", file=sys.stderr, flush=True)
        if store is not None:
            store.set("bench_ctx_devices_done", "1")
    elif store is not None:
        store.wait(["bench_ctx_devices_done"], datetime.timedelta(seconds=budget + 60))
    R.barrier()
    return res


def other_workloads_ranks(args, R, runner, emit=None) -> dict:
    """N > 1 (every rank of the driver's torch.distributed.run runs this): the same configurations
    in-process, one after the other on the job's process group, each a full multi-rank run
    (keys broadcast once, contiguous shards, barrier-bracketed timing, max wall over ranks), after
    the headline.  `runner(args) -> line` (rank 0) runs one workload; the CPU self-test passes a
    stub.  Device memory of one workload is released before the next.

    Each workload runs under a per-rank watchdog of workload_budget() seconds (no re-exec: a
    thread).  A rank over budget (a stuck kernel, or a collective waiting on a stuck peer -- every
    rank's watchdog then fires) marks that entry as an error; rank 0 calls `emit(res)` to print the
    merged line with what was measured so far, and every rank exits with status 3, so the job ends
    non-zero instead of stalling the whole multi-GPU run."""
    import copy
    import gc
    import threading

    res = {}
    budget = workload_budget()
    for name, params, opts in OTHER_WORKLOADS:
        a = copy.copy(args)
        a.params, a.steps, a.warmup = params, opts["steps"], opts.get("warmup", 1)
        a.no_cpu_baseline = a.no_host_abi = True
        a.global_batch = opts.get("global_batch", 0)
        a.warmup_batch = opts.get("warmup_batch", 0)
        a.batch = args.batch if args.launch_selftest else 0
        a.other = None
        t = time.perf_counter()

        def over_budget(name=name, t=t):
            res[name] = {"error": f"over its {budget:.0f} s budget on rank {R.rank} (watchdog)",
                         "wall_s": time.perf_counter() - t}
            print(f"bench.py: rank {R.rank}: {name} exceeded {budget:.0f} s; exiting", file=sys.stderr, flush=True)
            if R.rank == 0 and emit is not None:
                emit(res)
            sys.stdout.flush()
            os._exit(3)

        dog = threading.Timer(budget, over_budget)
        dog.daemon = True
        dog.start()
        try:
            line = runner(a)
        finally:
            dog.cancel()
        if R.rank == 0:
            res[name] = summarize(line)
            res[name]["wall_s"] = time.perf_counter() - t
            print(f"bench.py: {name} done in {res[name]['wall_s']:.1f} s", file=sys.stderr, flush=True)
        gc.collect()
        if R.device.type == "cuda":
            R.torch.cuda.synchronize(R.device)
            R.torch.cuda.empty_cache()
    return res


def env_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


class Ranks:
    """Process-group plumbing shared by the GPU workloads and the CPU self-test."""

    def __init__(self, device, backend: str | None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.rank, self.world, self.local = env_world()
        self.device = device
        self.backend = None
        if self.world > 1:
            self.backend = backend
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group(backend)
            assert dist.get_world_size() == self.world

    @property
    def coll_device(self):
        # gloo reduces host tensors; nccl (RCCL) device tensors
        return self.device if self.backend == "nccl" else self.torch.device("cpu")

    def barrier(self):
        if self.world > 1:
            t = self.torch.ones(1, device=self.coll_device)
            self.dist.all_reduce(t)
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)

    def max(self, x: float) -> float:
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.coll_device)
        if self.world > 1:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, xs) -> list:
        t = self.torch.tensor(list(xs), dtype=self.torch.int64, device=self.coll_device)
        if self.world > 1:
            self.dist.all_reduce(t)
        return [int(v) for v in t.tolist()]

    def gather(self, xs) -> list:
        t = self.torch.tensor(list(xs), dtype=self.torch.int64, device=self.coll_device)
        if self.world == 1:
            return [list(xs)]
        outs = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t)
        return [o.tolist() for o in outs]

    def finish(self):
        if self.world > 1:
            self.dist.barrier()
            self.dist.destroy_process_group()

    def info(self) -> dict:
        ws = self.dist.get_world_size() if self.world > 1 else 1
        return {"backend": self.backend or "none (single process)", "world_size": ws}


def aggregate(R: Ranks, units: int, wall: float, ok: int, of: int, lo: int, hi: int) -> dict:
    """Sum of units over ranks / max wall over ranks; all-reduced decrypt check; shard table."""
    wall_max = R.max(wall)
    total, ok_all, of_all = R.sum([units, ok, of])
    shards = R.gather([lo, hi])
    return {"units": total, "wall_max": wall_max, "ok": ok_all, "of": of_all, "shards": shards,
            "value": total / wall_max}


# ---------------------------------------------------------------------------------------------
# the CPU self-test of the multi-rank path

def run_selftest(args) -> int:
    import torch

    R = Ranks(torch.device("cpu"), os.environ.get("BENCH_DIST_BACKEND", "gloo"))
    line = selftest_line(args, R)
    if args.params is None and not args.no_other_workloads and R.world > 1:
        line = merge_other(line, other_workloads_ranks(args, R, lambda a: selftest_line(a, R),
                                                       emit=lambda res: print(json.dumps(merge_other(line, res)),
                                                                              flush=True)))
    if R.rank == 0:
        print(json.dumps(line), flush=True)
    R.finish()
    return 0


def selftest_line(args, R) -> dict | None:
    """One stub workload through the rank/shard/aggregation code (rank 0 gets the line)."""
    from tfhe_mi355.distributed import shard_range

    B = args.batch or 64
    G = args.global_batch or R.world * B
    lo, hi = shard_range(G, R.rank, R.world)
    msgs = np.random.default_rng(args.seed).integers(0, 16, G).astype(np.uint64)[lo:hi]
    per_step = 0.02 * (R.rank + 1)   # ranks run at different speeds: the max must win
    if args.params and args.params == os.environ.get("BENCH_SELFTEST_STALL"):
        time.sleep(3600)             # a stuck workload (tests the per-workload watchdog)

    def step():
        time.sleep(per_step)
        return msgs.copy()            # stub "PBS" with the identity LUT

    for _ in range(args.warmup):
        step()
    R.barrier()
    t0 = time.perf_counter()
    out = None
    for _ in range(args.steps):
        out = step()
    R.barrier()
    wall = time.perf_counter() - t0
    ok = int(np.count_nonzero(out == msgs))
    agg = aggregate(R, (hi - lo) * args.steps, wall, ok, hi - lo, lo, hi)
    if R.rank != 0:
        return None
    return {"metric": "launch self-test (stub step, no GPU)", "selftest": True,
            "value": agg["value"], "unit": "stub units/s", "n_gpus": R.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": agg["wall_max"] / args.steps * 1e3,
            "scaling": "strong" if args.global_batch else "weak",
            "check": {"decrypted_ok": agg["ok"], "of": agg["of"]},
            "config": {"workload": f"stub {args.params or 'headline'}", "global_batch": G, "batch_per_rank": B,
                       "shards": agg["shards"], "stub_seconds_per_step": [0.02 * (r + 1) for r in range(R.world)]},
            "units_total": agg["units"], "wall_max_s": agg["wall_max"], **R.info()}


# ---------------------------------------------------------------------------------------------
# GPU workloads

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=0, help="ciphertexts per GPU per step (default 4096; 1024 at 4_4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-abi", action="store_true", help="skip the host-pointer ABI rate")
    ap.add_argument("--callers-only", action="store_true",
                    help="host-pointer ABI: only the one-ciphertext-per-call leg (1 / 64 / 256 callers, 1 x 256 "
                         "submitted), not the batched pageable / pinned rates")
    ap.add_argument("--no-single-call", action="store_true",
                    help="skip the one-ciphertext call latency (kernel traces / PMC runs of the batch)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-other-workloads", action="store_true",
                    help="default run only: skip the other configurations measured beside the headline")
    ap.add_argument("--params", choices=sorted(PARAMS), default=None,
                    help="2_2 = the BASELINE metric; 2_2ks = KS+PBS; mb3/mb2 = multi-bit PBS (config 5)")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="exercise the rank launch / shard / aggregation path on the CPU (gloo, stub step)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="total ciphertexts over all ranks (split into contiguous shards: strong scaling)")
    ap.add_argument("--warmup-batch", type=int, default=0,
                    help="warm-up launches use only the first N ciphertexts of the rank's batch")
    ap.add_argument("--ctx-devices", default=None, metavar="LIST",
                    help="only the one-process multi-device context entry over the comma-separated device "
                         "list (the default run adds it: devices 0,0 at N = 1, 0..N-1 at N > 1)")
    args = ap.parse_args()
    if args.ctx_devices:
        print(json.dumps(ctx_devices_line(args, [int(d) for d in args.ctx_devices.split(",")])), flush=True)
        return

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}; n_gpus is taken from the world that runs")
    if args.launch_selftest:
        sys.exit(run_selftest(args))
    # the default invocation (no --params) also measures the other configurations: on one GPU as
    # child processes before this one touches the GPU, on N GPUs in-process on every rank
    default_run = args.params is None and not args.no_other_workloads
    args.other = None
    if default_run and ws == 1:
        args.other = other_workloads(args)
    args.params = args.params or "2_2"

    import torch

    _, world, local = env_world()
    # one process per GPU; on a box with fewer GPUs than ranks (a rehearsal of the multi-rank
    # path, BENCH_DIST_BACKEND=gloo) ranks share devices round-robin
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    R = Ranks(device, os.environ.get("BENCH_DIST_BACKEND", "nccl"))  # nccl = RCCL over xGMI
    line = run_workload(args, R)
    if args.other is not None:  # N = 1: measured by the child runs above
        line = merge_other(line, args.other)
    if default_run and ws > 1:
        # after the headline, so that a workload over its budget still leaves a complete line
        line = merge_other(line, other_workloads_ranks(args, R, lambda a: run_workload(a, R),
                                                       emit=lambda res: print(json.dumps(merge_other(line, res)),
                                                                              flush=True)))
        prev = dict((line or {}).get("other_workloads") or {})
        ctx = ctx_devices_ranks(args, R, emit=lambda res: print(json.dumps(merge_other(line, {**prev, **res})),
                                                                flush=True))
        line = merge_other(line, {**prev, **ctx})
    if R.rank == 0:
        if default_run:
            line["summary"] = compact_summary(line)
        print(json.dumps(line), flush=True)
        if default_run:
            print("bench.py summary: " + json.dumps(line["summary"], separators=(",", ":")), file=sys.stderr,
                  flush=True)
    R.finish()


def merge_other(line, res):
    """The headline line (rank 0) with the other configurations' entries; an entry that failed
    makes the line say so (`other_workloads_errors`)."""
    if line is None:
        return None
    out = dict(line)
    out["other_workloads"] = dict(res)
    bad = sorted(k for k, v in res.items() if "error" in v)
    if bad:
        out["other_workloads_errors"] = bad
    return out


def run_workload(args, R) -> dict | None:
    """One configuration on every rank; rank 0 returns its JSON line (others None)."""
    from tfhe_mi355.parameters import ALL

    pname, workload, kname = PARAMS[args.params]
    P = ALL[pname]
    if args.params == "mul32":
        return run_mul32(args, P, workload, kname, R)
    return run_pbs(args, P, pname, workload, kname, R)


def make_keys(args, P, R, with_ks):
    """Secret keys from the seed on every rank (cheap); BSK (and KSK) generated once on rank 0 and
    broadcast over RCCL; each rank converts its copy to the Fourier domain."""
    import torch

    from tfhe_mi355 import Engine, client
    from tfhe_mi355.distributed import broadcast_u64

    eng = Engine(P, R.device.index)
    lwe_sk = client.gen_binary_key(args.seed, 1, P.lwe_dimension)
    glwe_sk = client.gen_binary_key(args.seed, 2, P.big_lwe_dimension)
    bsk_len = ggsw_count(P) * P.pbs_level * (P.glwe_dimension + 1) ** 2 * P.polynomial_size
    bsk = ksk = None
    t = time.perf_counter()
    if R.rank == 0:
        if P.grouping_factor:
            bsk = client.gen_multi_bit_bootstrap_key(args.seed + 100, lwe_sk, glwe_sk, P.glwe_dimension,
                                                     P.polynomial_size, P.pbs_base_log, P.pbs_level,
                                                     P.grouping_factor, P.glwe_modular_std_dev)
        else:
            bsk = client.gen_bootstrap_key(args.seed + 100, lwe_sk, glwe_sk, P.glwe_dimension,
                                           P.polynomial_size, P.pbs_base_log, P.pbs_level,
                                           P.glwe_modular_std_dev)
    t_gen = time.perf_counter() - t
    t = time.perf_counter()
    d_bsk = broadcast_u64(bsk, bsk_len, 0, R.device if R.backend != "gloo" else torch.device("cpu"))
    torch.cuda.synchronize()
    t_bc = time.perf_counter() - t
    eng.convert_bootstrap_key_device(d_bsk.to(R.device), bsk_len)
    del d_bsk
    if with_ks:
        ksk_len = P.big_lwe_dimension * P.ks_level * (P.lwe_dimension + 1)
        if R.rank == 0:
            ksk = client.gen_keyswitch_key(args.seed + 200, glwe_sk, lwe_sk, P.ks_base_log, P.ks_level,
                                           P.lwe_modular_std_dev)
        t = time.perf_counter()
        d_ksk = broadcast_u64(ksk, ksk_len, 0, R.device if R.backend != "gloo" else torch.device("cpu"))
        torch.cuda.synchronize()
        t_bc_ksk = time.perf_counter() - t
        eng.upload_keyswitch_key_device(d_ksk.to(R.device), ksk_len)
        del d_ksk
    torch.cuda.synchronize()
    setup = {"bsk_keygen_s": t_gen, "bsk_broadcast_s": t_bc}
    if with_ks:
        setup["ksk_broadcast_s"] = t_bc_ksk
    return eng, lwe_sk, glwe_sk, bsk, ksk, setup


def host_abi_rate(eng, P, cts, acc, with_ks: bool, reps: int = 3) -> dict:
    """Rate of the synchronous host-pointer entry point (numpy in, numpy out: the form the Rust
    binding of INTEGRATION.md calls), chunk-pipelined through pinned staging; PCIe-inclusive."""
    f = eng.keyswitch_programmable_bootstrap if with_ks else eng.programmable_bootstrap
    f(cts, acc)
    t = time.perf_counter()
    for _ in range(reps):
        out = f(cts, acc)
    wall = time.perf_counter() - t
    B = cts.shape[0]
    mb_in, mb_out = cts.nbytes / 1e6, out.nbytes / 1e6
    # the same entry point with page-locked caller buffers (tfhe_mi355_host_alloc): DMA'd directly
    from tfhe_mi355 import pinned_empty

    p_in = pinned_empty(cts.shape)
    p_in[...] = cts
    p_out = pinned_empty(out.shape)
    f(p_in, acc, out=p_out)
    t = time.perf_counter()
    for _ in range(reps):
        f(p_in, acc, out=p_out)
    wall_p = time.perf_counter() - t
    assert np.array_equal(p_out, out), "pinned-buffer path differs from the pageable path"
    return {"value": B * reps / wall, "unit": "KS+PBS/s" if with_ks else "PBS/s", "batch": B,
            "pinned_buffers_value": B * reps / wall_p,
            "entry_point": ("tfhe_mi355_keyswitch_programmable_bootstrap" if with_ks
                            else "tfhe_mi355_programmable_bootstrap"),
            "note": (f"host numpy buffers in and out ({mb_in:.1f} MB in, {mb_out:.1f} MB out per call): `value` with "
                     "pageable buffers (two-lane chunked H2D/kernel/D2H pipeline through the engine's pinned "
                     "staging), `pinned_buffers_value` with caller buffers from tfhe_mi355_host_alloc (DMA'd "
                     "directly, same outputs); PCIe-inclusive, rank 0's GPU, not the headline value")}


# the reference's published single-thread KS+PBS latencies (tfhe/docs/getting_started/benchmarks.md:42)
REFERENCE_KS_PBS_MS = {"PARAM_MESSAGE_2_CARRY_2_KS_PBS": 16.6, "PARAM_MESSAGE_3_CARRY_3_KS_PBS": 121.0,
                       "PARAM_MESSAGE_4_CARRY_4_KS_PBS": 811.0}


def single_call_latency(eng, pname, cts, acc, with_ks: bool, secs: float = 1.5, max_reps: int = 50) -> dict:
    """Wall time of ONE synchronous count = 1 call through the host-pointer ABI, the reference's
    calling pattern (keyswitch_programmable_bootstrap_assign bootstraps one ciphertext,
    shortint/server_key/mod.rs:783-857), on an otherwise idle GPU: median over repeated calls,
    PCIe copies included.  Beside the reference's published single-thread latency where one exists."""
    f = eng.keyswitch_programmable_bootstrap if with_ks else eng.programmable_bootstrap
    x = np.ascontiguousarray(cts[:1])
    f(x, acc)
    times = []
    t_end = time.perf_counter() + secs
    while len(times) < max_reps and (len(times) < 3 or time.perf_counter() < t_end):
        t = time.perf_counter()
        f(x, acc)
        times.append(time.perf_counter() - t)
    ref = REFERENCE_KS_PBS_MS.get(pname) if with_ks else None
    return {"ms": 1e3 * float(np.median(times)), "min_ms": 1e3 * min(times), "calls": len(times),
            "op": "KS+PBS" if with_ks else "PBS",
            "entry_point": ("tfhe_mi355_keyswitch_programmable_bootstrap" if with_ks
                            else "tfhe_mi355_programmable_bootstrap"),
            "reference_single_thread_ms": ref,
            "note": "one count = 1 synchronous host-pointer call at a time (median), PCIe-inclusive"
                    + ("; reference: benchmarks.md:42, one Xeon thread" if ref else "")}


def single_ct_rates(eng, cts, acc, with_ks: bool, batched_rate: float, secs: float = 2.0,
                    callers=(1, 16, 64, 256), submit_windows=((1, 256), (16, 64))) -> dict:
    """The reference's own calling pattern through the synchronous host-pointer ABI: ONE ciphertext
    per call (keyswitch_programmable_bootstrap_assign, shortint/server_key/mod.rs:783-857), from T
    native threads at once (rayon workers, radix_parallel/mul.rs:347-407), each issuing its next
    call when the previous returns (lib/libtfhe_mi355_loadgen.so: std::threads, no GIL).  The
    engine coalesces concurrent small calls into batches.  Every output is compared
    with the same ciphertext's row from one batched call.  By Little's law T callers cannot exceed
    T / latency (`little_bound`).  `submit_wait` drives tfhe_mi355_submit / tfhe_mi355_wait
    (count = 1 per request, W requests in flight per thread)."""
    import ctypes

    from tfhe_mi355 import _lib

    lg = ctypes.CDLL(os.path.join(ROOT, "tfhe-rs-odd_amd", "lib", "libtfhe_mi355_loadgen.so"))
    lg.tfhe_mi355_loadgen_run.restype = ctypes.c_int
    n_in = min(cts.shape[0], 1024)
    x = np.ascontiguousarray(cts[:n_in])
    f = eng.keyswitch_programmable_bootstrap if with_ks else eng.programmable_bootstrap
    exp = f(x, acc)   # one batched call: the expected rows
    a = np.ascontiguousarray(acc, dtype=np.uint64)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    res = {"entry_point": ("tfhe_mi355_keyswitch_programmable_bootstrap" if with_ks
                           else "tfhe_mi355_programmable_bootstrap"), "callers": {}}
    for T in callers:
        eng.coalesce_stats(reset=True)
        calls, bad, fails = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        wall, lat = ctypes.c_double(), ctypes.c_double()
        rc = lg.tfhe_mi355_loadgen_run(
            eng._h, ctypes.c_int(1 if with_ks else 0), x.ctypes.data_as(u64p), ctypes.c_size_t(x.shape[1]),
            ctypes.c_size_t(n_in), exp.ctypes.data_as(u64p), ctypes.c_size_t(exp.shape[1]), a.ctypes.data_as(u64p),
            ctypes.c_int(T), ctypes.c_double(secs if T > 1 else secs / 2), ctypes.byref(calls), ctypes.byref(wall),
            ctypes.byref(lat), ctypes.byref(bad), ctypes.byref(fails))
        if rc != 0:
            raise _lib.EngineError("loadgen failed")
        rate = calls.value / wall.value
        res["callers"][str(T)] = {"value": rate, "frac_of_batched_device_rate": rate / batched_rate,
                                  "mean_call_latency_ms": lat.value * 1e3,
                                  "little_bound": T / lat.value if lat.value else None,
                                  "calls": calls.value, "mismatching_rows": bad.value, "failed_calls": fails.value,
                                  "coalescing": eng.coalesce_stats()}
    if "1" in res["callers"]:
        res["single_call_latency_ms"] = res["callers"]["1"]["mean_call_latency_ms"]
    # the asynchronous pair (tfhe_mi355_submit / tfhe_mi355_wait): T threads, each with W count = 1
    # requests in flight, so T * W ciphertexts can share one coalesced batch
    lg.tfhe_mi355_loadgen_submit_run.restype = ctypes.c_int
    res["submit_wait"] = {}
    for T, W in submit_windows:
        eng.coalesce_stats(reset=True)
        calls, bad, fails = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        wall, lat = ctypes.c_double(), ctypes.c_double()
        rc = lg.tfhe_mi355_loadgen_submit_run(
            eng._h, ctypes.c_int(1 if with_ks else 0), x.ctypes.data_as(u64p), ctypes.c_size_t(x.shape[1]),
            ctypes.c_size_t(n_in), exp.ctypes.data_as(u64p), ctypes.c_size_t(exp.shape[1]), a.ctypes.data_as(u64p),
            ctypes.c_int(T), ctypes.c_int(W), ctypes.c_double(secs), ctypes.byref(calls), ctypes.byref(wall),
            ctypes.byref(lat), ctypes.byref(bad), ctypes.byref(fails))
        if rc != 0:
            raise _lib.EngineError("loadgen (submit) failed")
        rate = calls.value / wall.value
        res["submit_wait"][f"{T}x{W}"] = {"threads": T, "in_flight_per_thread": W, "value": rate,
                                          "frac_of_batched_device_rate": rate / batched_rate,
                                          "mean_request_latency_ms": lat.value * 1e3, "calls": calls.value,
                                          "mismatching_rows": bad.value, "failed_calls": fails.value,
                                          "coalescing": eng.coalesce_stats()}
    res["note"] = ("T native threads (libtfhe_mi355_loadgen), closed loop, count = 1 per call, every output "
                   "compared with a batched call's row; T callers cannot exceed T / latency (little_bound); "
                   "the batched device rate is the headline step's")
    return res


CTX_DEVICES_PAIRS = 32  # FheUint32 pairs per shard of the ctx_devices entry (host radix batches)


def ctx_devices_line(args, devices: list) -> dict:
    """The one-process multi-device drop-in (tfhe_mi355_context_create_devices):
    ONE context over `devices`, driven the way a Rust caller drives it -- through the host-pointer C
    ABI, with no torch in the data path.  The reference is one process whose rayon workers call
    KS+PBS per block (shortint/engine/mod.rs:23-25, radix_parallel/mul.rs:347-407 ->
    shortint/server_key/mod.rs:783-857).  2_2 keys are uploaded once (the first device converts the
    BSK; the others receive it by ncclBroadcast over xGMI, or by device copies when a device repeats),
    then
      * `value`: classic 2_2 PBS over 4096 x S rows per call (S = shards), page-locked caller buffers
        (tfhe_mi355_host_alloc), split into contiguous shares run concurrently -- PCIe-inclusive;
      * `mul32`: BASELINE config 4 with CTX_DEVICES_PAIRS x S FheUint32 pairs through the integer
        DAG's host path (each layer ONE host-pointer KS+PBS call split over the shards);
      * sampled rows (each shard boundary, both ends) and sampled products compared bit for bit with
        a single-device context, every output decrypted."""
    from tfhe_mi355 import Engine, client, fill_accumulator, integer, pinned_empty, shortint
    from tfhe_mi355.parameters import ALL

    P = ALL["PARAM_MESSAGE_2_CARRY_2_KS_PBS"]
    S = len(devices)
    ck = shortint.ClientKey(P, args.seed)
    t = time.perf_counter()
    bsk = client.gen_bootstrap_key(args.seed + 100, ck.small_lwe_secret_key, ck.glwe_secret_key, P.glwe_dimension,
                                   P.polynomial_size, P.pbs_base_log, P.pbs_level, P.glwe_modular_std_dev)
    ksk = client.gen_keyswitch_key(args.seed + 200, ck.large_lwe_secret_key, ck.small_lwe_secret_key,
                                   P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    t_gen = time.perf_counter() - t
    single = Engine(P, devices[0])
    t = time.perf_counter()
    single.upload_bootstrap_key(bsk)
    single.upload_keyswitch_key(ksk)
    t_single = time.perf_counter() - t
    t = time.perf_counter()
    multi = Engine(P, devices=devices)
    t_create = time.perf_counter() - t
    t = time.perf_counter()
    multi.upload_bootstrap_key(bsk)
    t_bsk = time.perf_counter() - t
    t = time.perf_counter()
    multi.upload_keyswitch_key(ksk)
    t_ksk = time.perf_counter() - t
    mode, note = multi.replication()

    # classic PBS through the host-pointer ABI, split over the shards
    B = 4096 * S
    msgs = np.random.default_rng(args.seed).integers(0, 16, B).astype(np.uint64)
    cts = client.lwe_encrypt(args.seed * 1000, ck.small_lwe_secret_key, msgs * np.uint64(P.delta),
                             P.lwe_modular_std_dev)
    acc = fill_accumulator(P, lambda x: x)
    p_in = pinned_empty(cts.shape)
    p_in[...] = cts
    p_out = pinned_empty((B, P.big_lwe_dimension + 1))
    for _ in range(max(1, args.warmup)):
        multi.programmable_bootstrap(p_in, acc, out=p_out)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        multi.programmable_bootstrap(p_in, acc, out=p_out)
    wall = time.perf_counter() - t0
    out = np.array(p_out)
    dec = client.decode(client.lwe_decrypt(ck.glwe_secret_key, out), P.delta) % np.uint64(16)
    ok = int(np.count_nonzero(dec == msgs))
    bounds = sorted({min(max(B * i // S + d, 0), B - 1) for i in range(S + 1) for d in range(-16, 16)})
    idx = np.asarray(bounds)
    same = bool(np.array_equal(single.programmable_bootstrap(np.ascontiguousarray(cts[idx]), acc), out[idx]))

    # FheUint32 multiplies: the integer DAG over the multi-device context (host radix batches)
    K = CTX_DEVICES_PAIRS * S
    sks_m = integer.ServerKey(shortint.ServerKey(None, engine=multi, parameters=P))
    cks = integer.ClientKey(ck, 16)
    rng = np.random.default_rng(args.seed + 7)
    a = rng.integers(0, 2 ** 32, K, dtype=np.uint64)
    b = rng.integers(0, 2 ** 32, K, dtype=np.uint64)
    ca, cb = cks.encrypt(a), cks.encrypt(b)
    prod = sks_m.mul_parallelized(ca, cb)   # warm-up (LUT caches)
    t0 = time.perf_counter()
    msteps = max(1, min(args.steps, 2))
    for _ in range(msteps):
        prod = sks_m.mul_parallelized(ca, cb)
    mwall = time.perf_counter() - t0
    mok = int(np.count_nonzero(cks.decrypt(prod) == (a * b) % np.uint64(1 << 32)))
    sks_s = integer.ServerKey(shortint.ServerKey(None, engine=single, parameters=P))
    pick = [0, 1, K // 2, K - 1]
    ref = sks_s.mul_parallelized(sks_s.to_device(RadixSlice(_radix_rows(ca, pick), len(pick))),
                                 sks_s.to_device(RadixSlice(_radix_rows(cb, pick), len(pick))))
    msame = bool(np.array_equal(sks_s.to_host(ref).data, prod.data[pick]))
    multi.close()
    single.close()
    return {
        "metric": "programmable bootstraps/sec through ONE multi-device context (tfhe_mi355_context_create_devices), "
                  "host-pointer C ABI, PARAM_MESSAGE_2_CARRY_2",
        "value": B * args.steps / wall, "unit": "PBS/s", "n_gpus": len(set(devices)), "steps": args.steps,
        "warmup": max(1, args.warmup), "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded LWE encryptions of uniform messages)",
        "config": {"workload": (f"one context over devices {devices}: 2_2 PBS of 4096 x {S} rows per host-pointer call "
                                f"(page-locked buffers, PCIe-inclusive), and {K} FheUint32 multiplies per step "
                                "through the integer DAG's host path"),
                   "global_batch": B, "devices": devices, "shards": S},
        "check": {"decrypted_ok": ok, "of": B, "sampled_rows_equal_single_device": same,
                  "sampled_rows": len(bounds)},
        "setup": {"keygen_s": t_gen, "context_create_s": t_create, "bsk_upload_replicate_s": t_bsk,
                  "ksk_upload_replicate_s": t_ksk, "single_device_upload_s": t_single,
                  "replication": mode, "replication_note": note},
        "ctx_devices": {
            "pbs_per_s": B * args.steps / wall,
            "mul32": {"value": K * msteps / mwall, "unit": "mul/s", "pairs": K, "steps": msteps,
                      "ms_per_step": mwall / msteps * 1e3, "decrypted_ok": mok, "of": K,
                      "sampled_products_equal_single_device": msame, "sampled": len(pick)},
            "replication": mode,
            "note": ("one process, one context, every shard fed through the host-pointer ABI by the context's own "
                     "per-shard workers; host radix batches for mul32 (each DAG layer crosses PCIe), so both rates "
                     "are PCIe- and host-memory-inclusive and not comparable with the HBM-resident entries"),
        },
    }


def _radix_rows(rb, rows):
    from tfhe_mi355.integer import RadixBatch

    return RadixBatch(np.ascontiguousarray(rb.data[rows]), list(rb.degree), list(rb.noise))


def run_pbs(args, P, pname, workload, kname, R):
    import torch

    from tfhe_mi355 import client, fill_accumulator
    from tfhe_mi355.distributed import shard_range

    with_ks = args.params in WITH_KS   # config 3, the other shortint sets at N >= 4096, the 2_2 KS+PBS line
    B = args.batch or (1024 if args.params == "4_4" else 4096)
    msg_space = P.message_modulus * P.carry_modulus
    eng, lwe_sk, glwe_sk, bsk, ksk, setup = make_keys(args, P, R, with_ks)

    G = args.global_batch or R.world * B   # --global-batch: fixed total (strong scaling)
    lo, hi = shard_range(G, R.rank, R.world)
    B = hi - lo if args.global_batch else B
    msgs = np.random.default_rng(args.seed).integers(0, msg_space, G).astype(np.uint64)[lo:hi]
    key, std = (glwe_sk, P.glwe_modular_std_dev) if with_ks else (lwe_sk, P.lwe_modular_std_dev)
    cts = client.lwe_encrypt(args.seed * 1000 + R.rank, key, msgs * np.uint64(P.delta), std)
    nb = hi - lo
    acc = fill_accumulator(P, lambda x: x)
    d_in = torch.from_numpy(cts.view(np.int64)).to(R.device)
    d_out = torch.zeros((nb, P.big_lwe_dimension + 1), dtype=torch.int64, device=R.device)
    d_lut = torch.from_numpy(acc.view(np.int64)).to(R.device)
    stream = torch.cuda.current_stream()
    need = eng.ks_pbs_scratch_bytes(nb) if with_ks else eng.pbs_scratch_bytes(nb)
    d_scratch = torch.empty(max(need, 1), dtype=torch.uint8, device=R.device)

    def step(cnt=nb):
        if with_ks:
            eng.keyswitch_programmable_bootstrap_async(d_in, d_out, d_lut, 1, cnt, d_scratch, stream=stream)
        else:
            eng.programmable_bootstrap_async(d_in, d_out, d_lut, 1, cnt, stream=stream, d_scratch=d_scratch)

    for _ in range(args.warmup):
        step(min(nb, args.warmup_batch) if args.warmup_batch else nb)
    # per-kernel durations of the timed steps (HIP events on the launch stream around every launch
    # of a classic / multi-bit PBS, every 16th CMUX launch of the N = 32768 kernels)
    eng.kernel_timing(16 if P.polynomial_size > 2048 else 1)
    R.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record(stream)
        step()
        e.record(stream)
    R.barrier()
    wall = time.perf_counter() - t0
    step_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    ktimes = eng.kernel_times()
    eng.kernel_timing(0)

    out = d_out.cpu().numpy().view(np.uint64)
    dec = client.decode(client.lwe_decrypt(glwe_sk, out), P.delta) % np.uint64(msg_space)
    ok = int(np.count_nonzero(dec == msgs))
    agg = aggregate(R, nb * args.steps, wall, ok, nb, lo, hi)

    # (profiling runs skip it: its count = 1 launches would mix into the per-kernel averages)
    latency = single_call_latency(eng, pname, cts, acc, with_ks) if R.rank == 0 and not args.no_single_call else None
    host_abi = None
    if not args.no_host_abi and R.rank == 0:
        if args.callers_only:  # the reference's calling pattern only (other_workloads children)
            host_abi = {"single_ct": single_ct_rates(eng, cts, acc, with_ks, nb * args.steps / wall, secs=1.5,
                                                     callers=(1, 64, 256), submit_windows=((1, 256),))}
        else:
            host_abi = host_abi_rate(eng, P, cts, acc, with_ks)
            host_abi["single_ct"] = single_ct_rates(eng, cts, acc, with_ks, nb * args.steps / wall)

    if R.rank == 0:
        unit = "KS+PBS/s" if with_ks else "PBS/s"
        if args.params == "2_2":
            metric = "programmable bootstraps/sec (PARAM_MESSAGE_2_CARRY_2) at 1/2/4/8 MI355X"
        elif with_ks:
            metric = f"keyswitch + programmable bootstraps/sec ({pname}) at 1/2/4/8 MI355X"
        else:
            metric = f"programmable bootstraps/sec ({pname}) at 1/2/4/8 MI355X"
        line = {
            "metric": metric,
            "value": agg["value"],
            "unit": unit,
            "n_gpus": R.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": agg["wall_max"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.global_batch else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded LWE encryptions of uniform messages; keys from the engine's client-side keygen)",
            "config": {
                "workload": workload,
                "parameters": (f"{pname} (n={P.lwe_dimension}, k={P.glwe_dimension}, N={P.polynomial_size}, "
                               f"pbs 2^{P.pbs_base_log} x {P.pbs_level}"
                               + (f", ks 2^{P.ks_base_log} x {P.ks_level}" if with_ks else "")
                               + (f", grouping {P.grouping_factor})" if P.grouping_factor else ")")),
                "batch_per_gpu": B,
                "global_batch": G,
                "shards": agg["shards"],
                "parallelism": f"dp{R.world} (contiguous batch shards, BSK replicated by one RCCL broadcast)",
            },
            **R.info(),
            "roofline": roofline(args.params, P, nb, step_ms, kname, with_ks, ktimes),
            "check": {"decrypted_ok": agg["ok"], "of": agg["of"]},
            "setup": setup,
        }
        if host_abi:
            line["host_abi"] = host_abi
        if latency:
            line["single_call_latency_ms"] = latency["ms"]
            line["single_call_latency"] = latency
        if R.world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or cpu_share()
            line["cpu_baseline"] = cpu_baseline(P, bsk, cts, acc, threads, ksk)
        return line
    return None


def run_mul32(args, P, workload, kname, R):
    """Config 4: K FheUint32 multiplies per GPU per step through the batched integer DAG
    (tfhe_mi355.integer), the whole DAG captured once into a hipGraph and replayed per step;
    value = multiplies/s over all ranks."""
    import torch

    from tfhe_mi355 import Engine, client, integer, shortint
    from tfhe_mi355.distributed import broadcast_u64, shard_range

    K = args.batch or 1024  # K = 1024: every DAG layer a multiple of 1024 slots or close (2048-65536 PBS per layer at 256 pairs left partial rounds)
    ck = shortint.ClientKey(P, args.seed)
    eng = Engine(P, R.device.index)
    bsk_len = ggsw_count(P) * P.pbs_level * (P.glwe_dimension + 1) ** 2 * P.polynomial_size
    ksk_len = P.big_lwe_dimension * P.ks_level * (P.lwe_dimension + 1)
    bsk = ksk = None
    t = time.perf_counter()
    if R.rank == 0:
        bsk = client.gen_bootstrap_key(args.seed + 100, ck.small_lwe_secret_key, ck.glwe_secret_key,
                                       P.glwe_dimension, P.polynomial_size, P.pbs_base_log, P.pbs_level,
                                       P.glwe_modular_std_dev)
        ksk = client.gen_keyswitch_key(args.seed + 200, ck.large_lwe_secret_key, ck.small_lwe_secret_key,
                                       P.ks_base_log, P.ks_level, P.lwe_modular_std_dev)
    t_gen = time.perf_counter() - t
    bdev = R.device if R.backend != "gloo" else torch.device("cpu")
    t = time.perf_counter()
    d = broadcast_u64(bsk, bsk_len, 0, bdev)
    torch.cuda.synchronize()
    t_bc = time.perf_counter() - t
    eng.convert_bootstrap_key_device(d.to(R.device), bsk_len)
    t = time.perf_counter()
    d = broadcast_u64(ksk, ksk_len, 0, bdev)
    torch.cuda.synchronize()
    t_bc_ksk = time.perf_counter() - t
    eng.upload_keyswitch_key_device(d.to(R.device), ksk_len)
    torch.cuda.synchronize()
    del d
    sks = integer.ServerKey(shortint.ServerKey(None, engine=eng, parameters=P))
    cks = integer.ClientKey(ck, 16)
    G = R.world * K
    lo, hi = shard_range(G, R.rank, R.world)
    rng = np.random.default_rng(args.seed)
    a = rng.integers(0, 2 ** 32, G, dtype=np.uint64)[lo:hi]
    b = rng.integers(0, 2 ** 32, G, dtype=np.uint64)[lo:hi]
    ca, cb = cks.encrypt(a), cks.encrypt(b)
    ca_d, cb_d = sks.to_device(ca), sks.to_device(cb)   # operands resident in HBM

    # eager warm-up (fills the layer LUT caches), then capture the whole DAG once
    out = sks.mul_parallelized(ca_d, cb_d)
    torch.cuda.synchronize()
    pbs0, l0 = sks.pbs_count, sks.launches
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = sks.mul_parallelized(ca_d, cb_d)
    pbs_per_mul = (sks.pbs_count - pbs0) / (hi - lo)
    launches = sks.launches - l0
    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        graph.replay()
    R.barrier()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s, e in evs:
        s.record(stream)
        graph.replay()
        e.record(stream)
    R.barrier()
    wall = time.perf_counter() - t0
    step_ms = float(np.mean([s.elapsed_time(e) for s, e in evs]))
    ok = int(np.count_nonzero(cks.decrypt(out) == (a * b) % np.uint64(1 << 32)))
    agg = aggregate(R, (hi - lo) * args.steps, wall, ok, hi - lo, lo, hi)
    latency = None
    if R.rank == 0 and not args.no_single_call:
        # ONE multiply (the reference's published FheUint32 `*`: 333 ms on a 128-vCPU m6i.metal,
        # benchmarks.md:17): eager, every layer a small batch (<= 256 PBS: the latency kernel)
        one_a, one_b = sks.to_device(RadixSlice(ca, 1)), sks.to_device(RadixSlice(cb, 1))
        o1 = sks.mul_parallelized(one_a, one_b)
        torch.cuda.synchronize()
        times = []
        for _ in range(5):
            t = time.perf_counter()
            o1 = sks.mul_parallelized(one_a, one_b)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t)
        eager_ok = bool(cks.decrypt(o1)[0] == (int(a[0]) * int(b[0])) % (1 << 32))
        latency = {"ms": 1e3 * float(np.median(times)), "min_ms": 1e3 * min(times), "calls": len(times),
                   "op": "one FheUint32 multiply (mul_parallelized DAG, eager: 11 KS+PBS layers of <= 256 "
                         "ciphertexts on the latency kernel, plus the LWE additions)",
                   "correct": eager_ok,
                   "reference_ms": 333.0,
                   "note": "reference: FheUint32 mul, whole 128-vCPU machine (benchmarks.md:17,27)"}
        # the same one-pair DAG captured once into a hipGraph (its launch sequence does not depend on
        # the data) and replayed: the multiply without the per-layer host work
        try:
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                o1g = sks.mul_parallelized(one_a, one_b)
            g1.replay()
            torch.cuda.synchronize()
            gt = []
            for _ in range(5):
                t = time.perf_counter()
                g1.replay()
                torch.cuda.synchronize()
                gt.append(time.perf_counter() - t)
            gok = bool(cks.decrypt(o1g)[0] == (int(a[0]) * int(b[0])) % (1 << 32))
            latency["graph"] = {"ms": 1e3 * float(np.median(gt)), "min_ms": 1e3 * min(gt), "calls": len(gt),
                                "correct": gok,
                                "op": "the same one-pair DAG captured into one hipGraph and replayed (host time "
                                      "around replay + synchronize)"}
            if gok and eager_ok:
                latency["eager_ms"], latency["eager_min_ms"] = latency["ms"], latency["min_ms"]
                latency["ms"], latency["min_ms"] = latency["graph"]["ms"], latency["graph"]["min_ms"]
                latency["op"] = "one FheUint32 multiply: the one-pair DAG replayed from a hipGraph (eager in eager_ms)"
        except Exception as ex:  # capture unsupported here: the eager number stands
            latency["graph_error"] = repr(ex)[:200]
    if R.rank == 0:
        pbs_rate = agg["value"] * pbs_per_mul
        units = int(round(pbs_per_mul * (hi - lo)))
        rl = roofline("mul32", P, units, step_ms, kname, True, None)
        rl["model"] += "; the step is the whole multiply DAG (11 KS+PBS layers and the LWE additions)"
        line = {
            "metric": "FheUint32 multiplies/sec (PARAM_MESSAGE_2_CARRY_2 radix, 16 blocks) at 1/2/4/8 MI355X",
            "value": agg["value"],
            "unit": "mul/s",
            "n_gpus": R.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": agg["wall_max"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (uniform u32 operand pairs, seeded encryptions)",
            "config": {"workload": workload, "parameters": P.name, "pairs_per_gpu": K,
                       "global_pairs": G, "shards": agg["shards"], "pbs_per_multiply": pbs_per_mul,
                       "launches_per_multiply_batch": launches,
                       "parallelism": f"dp{R.world} (whole multiplies sharded, keys broadcast once)"},
            **R.info(),
            "pbs_per_sec": pbs_rate,
            "roofline": rl,
            "check": {"decrypted_ok": agg["ok"], "of": agg["of"]},
            "setup": {"keygen_s": t_gen, "bsk_broadcast_s": t_bc, "ksk_broadcast_s": t_bc_ksk},
        }
        if latency:
            line["single_call_latency_ms"] = latency["ms"]
            line["single_call_latency"] = latency
        if R.world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, ROOT)
            from oracle.oracle import OracleEngine  # oracle behind the engine API (test infrastructure)

            threads = args.cpu_threads or cpu_share()
            oe = OracleEngine(P, threads=threads, simd=True)
            oe.upload_bootstrap_key(bsk)
            oe.upload_keyswitch_key(ksk)
            csk = integer.ServerKey(shortint.ServerKey(None, engine=oe, parameters=P))
            t = time.perf_counter()
            csk.mul_parallelized(RadixSlice(ca, 2), RadixSlice(cb, 2))
            cw = time.perf_counter() - t
            line["cpu_baseline"] = {
                "value": 2 / cw, "unit": "mul/s", "cores": threads, "kind": "port", "host": host_info(),
                "sample": (f"2 FheUint32 multiplies through the same DAG with the oracle's SIMD build (pbs_simd.c, "
                           f"bit-identical) behind the engine API, {threads} threads ({cw:.1f} s); reference published 333 ms/mul "
                           f"on a 128-vCPU m6i.metal (benchmarks.md:17)"),
            }
        return line
    return None


def RadixSlice(rb, n):
    from tfhe_mi355.integer import RadixBatch

    d = rb.data[:n]
    return RadixBatch(d.copy() if isinstance(d, np.ndarray) else d.clone(), list(rb.degree), list(rb.noise))


if __name__ == "__main__":
    main()
