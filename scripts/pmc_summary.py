#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes of bench.py into profiles/pmc_traffic.json.

HBM bytes per launch of the dominant kernel = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024:
FETCH_SIZE is reported in KiB and, on gfx950, reads exactly half the bytes of a wide coalesced
(16 B/lane) stream (MI355X_MICROARCH.md 'HBM'; the GGSW stream is 16 B/lane double2 loads), so it
is doubled; WRITE_SIZE is exact for 16-B streaming stores and is taken as is (the LWE outputs are
8-B stores: uncalibrated, they are ~1.4% of the traffic).

usage: pmc_summary.py <fetch_dir> <write_dir> [<sq_dir>] --batch B --kernel SUBSTR --out FILE
"""
import argparse
import collections
import csv
import glob
import json
import os


def counters(d, kernel):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--kernel", default="pbs_classic_kernel")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    vals, n = {}, {}
    for d in a.dirs:
        v, c = counters(d, a.kernel)
        vals.update(v)
        n.update(c)
    fetch = vals.get("FETCH_SIZE")
    write = vals.get("WRITE_SIZE")
    res = {"kernel": a.kernel, "batch": a.batch, "dispatches_per_counter": n, "counters_avg_per_dispatch": vals}
    if fetch is not None and write is not None:
        hbm = 2 * fetch * 1024 + write * 1024
        res["hbm_bytes_per_launch"] = hbm
        res["hbm_bytes_per_pbs"] = hbm / a.batch
        res["method"] = "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)"
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
