#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 --pmc counter_collection.csv files (one dir per pass)."""
import csv
import re
import sys
from collections import defaultdict


def summarize(paths):
    tot = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for p in paths:
        for row in csv.DictReader(open(p)):
            m = re.search(r"(\w+_kernel)(<\w+>)?", row["Kernel_Name"])
            k = m.group(0) if m else row["Kernel_Name"][:24]
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
            calls[k].add(row["Dispatch_Id"])
    return tot, calls


if __name__ == "__main__":
    tot, calls = summarize(sys.argv[1:])
    for k, d in sorted(tot.items()):
        n = len(calls[k])
        print("%-28s dispatches=%d  " % (k[:28], n) + "  ".join("%s=%.4g" % (c, v / n) for c, v in sorted(d.items())))
