#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc passes of one bench workload into profiles/r02_pmc_<tag>.json
(read by bench.py's roofline).

HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 summed over the dispatches whose kernel name
matches --kernels: FETCH_SIZE is reported in KiB and on gfx950 counts half the bytes of a wide
coalesced (16 B/lane) stream, so it is doubled (MI355X_MICROARCH.md 'HBM'); WRITE_SIZE is taken
as is.  Infinity-Cache hits are counted as fabric traffic by these counters (same guide), so this
is L2<->fabric traffic, an upper bound on HBM bytes.  Units = dispatches of --unit-kernel x
--units-per-dispatch.

valu_busy = 4 * SQ_ACTIVE_INST_VALU / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs): the fraction of every
SIMD's cycles with a VALU instruction issued, over the dispatches of --main-kernel (SQ counters
in 4-cycle units summed over waves; GRBM_GUI_ACTIVE summed over the 8 XCDs).

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


def per_dispatch(d):
    """{dispatch id: (kernel name, {counter: value summed over the dispatch's records})}"""
    out = {}
    for r in rows(d):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        name, c = out.setdefault(key, (r["Kernel_Name"], collections.Counter()))
        c[r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernels", required=True)
    ap.add_argument("--unit-kernel", required=True)
    ap.add_argument("--units-per-dispatch", type=float, required=True)
    ap.add_argument("--main-kernel", required=True)
    ap.add_argument("--note", default="")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    kre, ure, mre = re.compile(a.kernels), re.compile(a.unit_kernel), re.compile(a.main_kernel)

    def traffic(d, counter):
        tot, units, per_kernel = 0.0, 0, collections.Counter()
        for name, c in per_dispatch(d).values():
            if kre.search(name):
                tot += c[counter]
                per_kernel[name.split("(")[0]] += c[counter]
            if ure.search(name):
                units += 1
        return tot, units, per_kernel

    fetch, u1, pk_f = traffic(a.fetch, "FETCH_SIZE")
    write, u2, pk_w = traffic(a.write, "WRITE_SIZE")
    units_f, units_w = u1 * a.units_per_dispatch, u2 * a.units_per_dispatch
    res = {"tag": a.tag, "kernels": a.kernels, "note": a.note,
           "method": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per unit (gfx950 FETCH_SIZE half-count correction)",
           "fetch_bytes_per_unit": 2 * fetch * 1024 / units_f if units_f else None,
           "write_bytes_per_unit": write * 1024 / units_w if units_w else None,
           "units_counted": [units_f, units_w],
           "fetch_kib_by_kernel": dict(pk_f), "write_kib_by_kernel": dict(pk_w)}
    if units_f and units_w:
        res["hbm_bytes_per_unit"] = res["fetch_bytes_per_unit"] + res["write_bytes_per_unit"]
    if a.sq:
        agg, n = collections.Counter(), 0
        for name, c in per_dispatch(a.sq).values():
            if mre.search(name):
                agg.update(c)
                n += 1
        res["sq_dispatches"] = n
        res["sq_counters_sum"] = dict(agg)
        if agg.get("GRBM_GUI_ACTIVE") and agg.get("SQ_ACTIVE_INST_VALU"):
            cycles = agg["GRBM_GUI_ACTIVE"] / 8
            res["valu_busy"] = 4 * agg["SQ_ACTIVE_INST_VALU"] / (cycles * 1024)
            res["avg_waves_per_simd"] = 4 * agg.get("SQ_WAVE_CYCLES", 0) / (cycles * 1024)
        if agg.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if k in agg:
                    res[f"{k.lower()}_per_wave_cycle"] = agg[k] / agg["SQ_WAVE_CYCLES"]
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if not isinstance(v, dict)}, indent=1))


if __name__ == "__main__":
    main()
