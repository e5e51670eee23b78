#!/usr/bin/env python3
"""Per-dispatch, per-wave SQ counters of one kernel from a rocprofv3 counter_collection.csv
(e.g. `rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python3 scripts/tick_times.py`): one line per
launch (= per tick for the band kernels), counters divided by SQ_WAVES; cycle counters are in
quad-cycles (MI355X_MICROARCH.md), printed as such.
usage: pmc_per_dispatch.py KERNEL_SUBSTR counter_collection.csv"""
import collections
import csv
import sys


def main():
    kern, path = sys.argv[1], sys.argv[2]
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if kern not in r.get("Kernel_Name", ""):
            continue
        d = per.setdefault(int(r["Dispatch_Id"]), collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
    names = None
    for i, (disp, d) in enumerate(sorted(per.items())):
        waves = d.get("SQ_WAVES", 0) or 1
        if names is None:
            names = [k for k in sorted(d) if k != "SQ_WAVES"]
            print("launch  waves     " + "  ".join(f"{k[3:]:>14s}" for k in names) + "   (per wave)")
        print(f"{i:6d} {int(waves):8d}  " + "  ".join(f"{d[k] / waves:14.1f}" for k in names))


if __name__ == "__main__":
    main()
