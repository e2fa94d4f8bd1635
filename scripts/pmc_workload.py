#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of one bench workload into profiles/r03_pmc_<tag>.json
(read by bench.py's roofline), per kernel.

For every kernel (name normalised: no return type, namespace, argument list or spaces, e.g.
`pbs_classic_kernel<2048,1,1>`) the summary holds its dispatch count and, per dispatch:
  hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: FETCH_SIZE is reported in KiB and on
    gfx950 counts half the bytes of a wide coalesced (16 B/lane) stream, so it is doubled
    (MI355X_MICROARCH.md 'HBM'); WRITE_SIZE is taken as is.  Infinity-Cache (MALL) hits count as
    fabric traffic for these counters (same guide), so this is L2<->fabric traffic, an upper bound
    on DRAM bytes;
  the SQ counters, and derived: valu_per_wave_cycle = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (x the
    resident waves per SIMD = the fraction of SIMD issue cycles with a VALU instruction),
    avg_waves_per_simd = 4 SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs), valu_busy =
    4 SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 x 1024) (SQ counters in 4-cycle units summed over
    waves; GRBM_GUI_ACTIVE summed over the 8 XCDs).
The workload totals of round 2 (all matching kernels together, per unit = per ciphertext) are kept
for comparison.

usage: pmc_workload.py --fetch DIR --write DIR --sq DIR --tag T --kernels RE --unit-kernel RE
                       --units-per-dispatch U --main-kernel RE --out FILE
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def rows(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        yield from csv.DictReader(open(f))


def norm(name: str) -> str:
    """'void tfhe_mi355::pbs_classic_kernel<2048, 1, 1>(tfhe_mi355::ClassicPbsLaunch)' ->
    'pbs_classic_kernel<2048,1,1>'"""
    n = name.split("(")[0].replace(" ", "")
    n = re.sub(r"^void", "", n)
    return n.split("::")[-1] if "<" not in n else re.sub(r"^[\w:]*::", "", n)


def per_dispatch(d):
    """{dispatch id: (normalised kernel name, {counter: value summed over the dispatch's records})}"""
    out = {}
    for r in rows(d):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        name, c = out.setdefault(key, (norm(r["Kernel_Name"]), collections.Counter()))
        c[r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def derive(c: collections.Counter) -> dict:
    r = {}
    if c.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                  "SQ_WAIT_INST_LDS", "SQ_INSTS_VALU"):
            if k in c:
                r[f"{k.lower()}_per_wave_cycle"] = c[k] / c["SQ_WAVE_CYCLES"]
    if c.get("GRBM_GUI_ACTIVE"):
        cycles = c["GRBM_GUI_ACTIVE"] / 8
        if c.get("SQ_ACTIVE_INST_VALU"):
            r["valu_busy"] = 4 * c["SQ_ACTIVE_INST_VALU"] / (cycles * 1024)
        if c.get("SQ_WAVE_CYCLES"):
            r["avg_waves_per_simd"] = 4 * c["SQ_WAVE_CYCLES"] / (cycles * 1024)
    if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c:
        r["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    hit, miss = c.get("TCC_HIT_sum", c.get("TCC_HIT")), c.get("TCC_MISS_sum", c.get("TCC_MISS"))
    if hit is not None and miss is not None and hit + miss > 0:
        r["l2_hit_rate"] = hit / (hit + miss)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq")
    ap.add_argument("--extra", action="append", default=[], help="more counter passes (SQ LDS, TCC hit/miss)")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernels", required=True)
    ap.add_argument("--unit-kernel", required=True)
    ap.add_argument("--units-per-dispatch", type=float, required=True)
    ap.add_argument("--main-kernel", required=True)
    ap.add_argument("--note", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    kre, ure, mre = re.compile(a.kernels), re.compile(a.unit_kernel), re.compile(a.main_kernel)

    by = collections.defaultdict(lambda: {"dispatches": {}, "counters": collections.Counter()})
    units = {}
    for tag, d, counter in (("fetch", a.fetch, "FETCH_SIZE"), ("write", a.write, "WRITE_SIZE")):
        tot, u = 0.0, 0
        for name, c in per_dispatch(d).values():
            if kre.search(name):
                tot += c[counter]
                k = by[name]
                k["counters"][counter] += c[counter]
                k["dispatches"][tag] = k["dispatches"].get(tag, 0) + 1
            if ure.search(name):
                u += 1
        units[tag] = (tot, u * a.units_per_dispatch)
    for i, d in enumerate(([a.sq] if a.sq else []) + a.extra):
        tag = "sq" if i == 0 and a.sq else f"extra{i}"
        for name, c in per_dispatch(d).values():
            if kre.search(name):
                k = by[name]
                k["counters"].update(c)
                k["dispatches"][tag] = k["dispatches"].get(tag, 0) + 1

    kernels = {}
    for name, k in sorted(by.items()):
        c, disp = k["counters"], k["dispatches"]
        e = {"dispatches": disp}
        if disp.get("fetch"):
            e["fetch_bytes_per_dispatch"] = 2 * c["FETCH_SIZE"] * 1024 / disp["fetch"]
        if disp.get("write"):
            e["write_bytes_per_dispatch"] = c["WRITE_SIZE"] * 1024 / disp["write"]
        if "fetch_bytes_per_dispatch" in e and "write_bytes_per_dispatch" in e:
            e["hbm_bytes_per_dispatch"] = e["fetch_bytes_per_dispatch"] + e["write_bytes_per_dispatch"]
        sq = {kk: v for kk, v in c.items() if kk.startswith(("SQ_", "GRBM_", "TCC_"))}
        if sq:
            e["sq_counters_sum"] = sq
            e.update(derive(collections.Counter(sq)))
        kernels[name] = e

    (fetch, uf), (write, uw) = units["fetch"], units["write"]
    main_names = [n for n in kernels if mre.search(n)]
    res = {"tag": a.tag, "kernels_re": a.kernels, "note": a.note,
           "main_kernels": main_names,
           "method": ("per dispatch: 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction; "
                      "L2<->fabric bytes, Infinity-Cache hits included); SQ counters from a separate pass"),
           "by_kernel": kernels,
           "workload_bytes_per_unit": (2 * fetch * 1024 / uf + write * 1024 / uw) if uf and uw else None,
           "units_counted": [uf, uw]}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({"tag": a.tag, "main_kernels": main_names,
                      "by_kernel": {n: {kk: v for kk, v in e.items() if not isinstance(v, dict)}
                                    for n, e in kernels.items()}}, indent=1))


if __name__ == "__main__":
    main()
