#!/usr/bin/env python3
"""Average PMC counter values per dispatch of the kernels whose name contains a substring, over
the rocprofv3 --pmc output directories under <dir> (a/, b/, ...).

    python3 tools/pmc_summary.py <dir> <kernel substring>
"""
import collections
import csv
import glob
import os
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    for f in sorted(glob.glob(os.path.join(d, "*", "*counter_collection.csv"))):
        agg, n = collections.defaultdict(float), collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add(r["Dispatch_Id"])
        for k, v in sorted(agg.items()):
            print(f"{os.path.basename(os.path.dirname(f))} {k:32s} {v / len(n[k]):16.1f}  ({len(n[k])} dispatches)")


if __name__ == "__main__":
    main()
