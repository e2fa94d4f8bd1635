#!/usr/bin/env python3
"""List profiles/* files that DESIGN.md / README.md / INTEGRATION.md do not name (review item 7).
A name may be written with brace alternatives (r06_pmc_{2_2,mb3}.json), a * glob, or an _a/_b/..
suffix family written as name_{a,b}.  usage: check_profiles_cited.py [--delete]"""
import fnmatch
import itertools
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def expand(tok):
    m = re.search(r"\{([^{}]*)\}", tok)
    if not m:
        return [tok]
    return list(itertools.chain.from_iterable(expand(tok[:m.start()] + alt + tok[m.end():]) for alt in m.group(1).split(",")))


def main():
    text = "".join(open(os.path.join(ROOT, f)).read() for f in ("DESIGN.md", "README.md", "INTEGRATION.md")
                   if os.path.exists(os.path.join(ROOT, f)))
    toks = set(re.findall(r"[A-Za-z0-9_.*{},<>-]*r0\d[a-z]*_[A-Za-z0-9_.*{},-]+", text))
    pats = set()
    for t in toks:
        t = t.split("/")[-1].strip(".,;:)")
        for e in expand(t):
            pats.add(e)
            if "." not in e.split("_")[-1]:
                pats.add(e + "*")  # a stem: every extension
    files = sorted(os.listdir(os.path.join(ROOT, "profiles")))
    unc = [f for f in files if not any(fnmatch.fnmatch(f, p) or f.startswith(p.rstrip("*") + ".") for p in pats)]
    for f in unc:
        print(f)
    print(f"{len(unc)} of {len(files)} profiles/ files not named", file=sys.stderr)
    if "--delete" in sys.argv:
        for f in unc:
            os.remove(os.path.join(ROOT, "profiles", f))


if __name__ == "__main__":
    main()
