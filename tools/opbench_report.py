#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of tools/opbench.py: per case, per kernel,
mean/min duration (µs) over the iterations after the first quarter."""
import csv
import sys
from collections import defaultdict


def main(trace, cases_file):
    names = [l.strip() for l in open(cases_file) if l.strip()]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], None
    for r in rows:
        if "k_argsort" in r["Kernel_Name"]:
            cur = []
            groups.append(cur)
            continue
        if cur is not None:
            cur.append(r)
    for name, g in zip(names, groups):
        per = defaultdict(list)
        for r in g:
            kn = r["Kernel_Name"]
            kn = kn[:90]
            per[kn].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
        print(f"== {name}")
        for kn, ds in per.items():
            tail = ds[len(ds) // 4:] or ds
            print(f"   {sum(tail) / len(tail):8.2f} us  min {min(tail):7.2f}  n={len(ds):4d}  {kn}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
