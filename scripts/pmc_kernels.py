#!/usr/bin/env python3
"""Per-kernel average duration and PMC counters from rocprofv3 csv directories.

usage: pmc_kernels.py TRACE_DIR PMC_DIR... [--match SUBSTR]
HBM bytes per launch = (2 FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE half-count correction).
"""
import collections
import csv
import glob
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
    args = [a for a in args if a != match]
    for r in csv.DictReader(open(glob.glob(args[0] + "/*kernel_stats.csv")[0])):
        if match in r["Name"]:
            print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg {float(r['AverageNs']) / 1e3:9.2f} us  {float(r['Percentage']):5.1f}%")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in args[1:]:
        for f in glob.glob(d + "/*counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        if match not in k:
            continue
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        line = " ".join(f"{c}={v:.3g}" for c, v in sorted(avg.items()))
        hbm = (2 * avg.get("FETCH_SIZE", 0) + avg.get("WRITE_SIZE", 0)) * 1024
        print(f"{k:60s} HBM {hbm / 1e6:8.1f} MB/launch  {line}")


if __name__ == "__main__":
    main()
