#!/usr/bin/env python3
"""Per-wave PMC summary of one kernel from rocprofv3 counter_collection.csv files.
usage: pmc_summary.py KERNEL_SUBSTR file.csv [file.csv ...]"""
import collections
import csv
import sys

kern = sys.argv[1]
for path in sys.argv[2:]:
    acc = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        if kern not in r.get("Kernel_Name", ""):
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
    waves = acc.get("SQ_WAVES", 0) or 1
    print(path)
    for k in sorted(acc):
        per = f"  per wave {acc[k] / waves:10.1f}" if "SQ_" in k and k != "SQ_WAVES" else ""
        print(f"  {k:22s} {acc[k] / max(1, n[k]):16.1f} per dispatch{per}")
