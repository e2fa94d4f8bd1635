#!/usr/bin/env python3
"""Launch gaps of a rocprofv3 --kernel-trace CSV: per kernel name, count, mean duration, and the
mean idle time between a dispatch's start and the end of the previous dispatch on the same queue
(gap), plus the share of wall time (first start .. last end) the GPU spent with no kernel running.

usage: trace_gaps.py kernel_trace.csv [name-regex]
"""
import collections
import csv
import re
import sys


def main():
    path = sys.argv[1]
    rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Name")
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "")))
    rows.sort()
    if rx:
        rows = [r for r in rows if rx.search(r[2])]
    if not rows:
        print("no dispatches")
        return
    busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    for s, e, _, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = max(r[1] for r in rows) - rows[0][0]
    print(f"dispatches {len(rows)}  wall {wall / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(wall - busy) / wall:.1%}")
    stat = collections.defaultdict(lambda: [0, 0, 0, 0])
    prev_end = {}
    for s, e, name, q in rows:
        st = stat[name[:90]]
        st[0] += 1
        st[1] += e - s
        if q in prev_end:
            st[2] += max(0, s - prev_end[q])
            st[3] += 1
        prev_end[q] = e
    for name, (n, dur, gap, ng) in sorted(stat.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:7d}  dur {dur / n / 1e3:9.2f} us  gap-before {gap / max(ng, 1) / 1e3:8.2f} us  {name}")
    # the busiest kernel's mean duration over ten consecutive slices of its dispatches (drift over
    # the run: clocks, caches)
    top = max(stat.items(), key=lambda kv: kv[1][1])[0]
    durs = [e - s for s, e, name, _ in rows if name[:90] == top]
    k = max(1, len(durs) // 10)
    print("deciles (us):", " ".join(f"{sum(durs[i:i + k]) / len(durs[i:i + k]) / 1e3:.1f}"
                                    for i in range(0, len(durs), k)))


if __name__ == "__main__":
    main()
