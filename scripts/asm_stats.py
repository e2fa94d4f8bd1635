#!/usr/bin/env python3
"""Instruction mix of the hottest loop of a kernel in a hipcc -save-temps .s file.

usage: asm_stats.py file.s kernel_substring
Finds the kernel, then the backward branch with the largest span (the CMUX loop), and counts
the instructions between its target label and the branch.
"""
import collections
import re
import sys


def main():
    path, kname = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r'^(\S*' + re.escape(kname) + r'\S*):', s, re.M)
    start = m.start()
    end = s.index('.Lfunc_end', start)
    lines = s[start:end].split('\n')
    labels = {}
    for i, l in enumerate(lines):
        mm = re.match(r'^(\.LBB\w+):', l)
        if mm:
            labels[mm.group(1)] = i
    best = None
    for i, l in enumerate(lines):
        mm = re.match(r'\s+s_cbranch_\w+\s+(\.LBB\w+)', l) or re.match(r'\s+s_branch\s+(\.LBB\w+)', l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            span = i - labels[mm.group(1)]
            if best is None or span > best[0]:
                best = (span, labels[mm.group(1)], i)
    _, a, b = best
    c = collections.Counter()
    for l in lines[a:b + 1]:
        mm = re.match(r'\s+([vsdgb]\w*_\w+|buffer_\w+|scratch_\w+)', l)
        if mm and not l.strip().startswith(';'):
            c[mm.group(1)] += 1
    valu = sum(v for k, v in c.items() if k.startswith('v_'))
    f64 = sum(v for k, v in c.items() if k.startswith('v_') and 'f64' in k)
    print(f"loop lines {a}-{b}: VALU {valu} (f64 {f64}), LDS {sum(v for k, v in c.items() if k.startswith('ds_'))}, "
          f"VMEM {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_', 'scratch_')))}, "
          f"SALU {sum(v for k, v in c.items() if k.startswith('s_'))}")
    for k, v in c.most_common(40):
        print(f"  {k:32s} {v}")


if __name__ == "__main__":
    main()
