#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc CSVs (one or more files).

usage: python tools/sq_summary.py gpurun_out/pmc_base/run_counter_collection.csv [...]"""
import collections
import csv
import sys

for path in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "fmcw::" not in name:
            continue
        acc[name.split("fmcw::", 1)[1].split("(", 1)[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(path)
    for k, d in acc.items():
        print("  ", k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
