#!/usr/bin/env python3
"""Copy/kernel overlap from a rocprofv3 --kernel-trace --memory-copy-trace run.

For the scan kernels (tsg::...), reports how much of their execution time runs
while a host->device copy is in flight, and the busy spans of each engine.
Usage: tools/overlap_report.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv>
"""
import csv
import glob
import json
import os
import sys


def spans(path, pred):
    out = []
    for r in csv.DictReader(open(path)):
        if pred(r):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out)


def union_len(iv):
    tot, cur = 0, None
    for a, b in sorted(iv):
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def intersect(a_iv, b_iv):
    out = []
    j = 0
    b_iv = sorted(b_iv)
    for a0, a1 in sorted(a_iv):
        for b0, b1 in b_iv:
            lo, hi = max(a0, b0), min(a1, b1)
            if lo < hi:
                out.append((lo, hi))
    return out


def main(d):
    kt = glob.glob(os.path.join(d, "*_kernel_trace.csv"))[0]
    mt = glob.glob(os.path.join(d, "*_memory_copy_trace.csv"))[0]
    kern = spans(kt, lambda r: "tsg::" in r["Kernel_Name"])
    h2d = spans(mt, lambda r: r["Direction"].endswith("HOST_TO_DEVICE"))
    # chunk copies: 1-40 ms (a 1-GiB chunk at ~56 GB/s is ~19 ms; the bench's 4-GB H2D probe and
    # small table uploads are excluded)
    big = [s for s in h2d if 1_000_000 < s[1] - s[0] < 40_000_000]
    k_busy = union_len(kern)
    c_busy = union_len(big)
    both = union_len(intersect(kern, big))
    t0 = min(s[0] for s in kern + big)
    t1 = max(s[1] for s in kern + big)
    print(json.dumps({"trace": d, "kernels": len(kern), "chunk_copies": len(big),
                      "kernel_busy_ms": round(k_busy / 1e6, 3), "copy_busy_ms": round(c_busy / 1e6, 3),
                      "kernel_time_under_copy_ms": round(both / 1e6, 3),
                      "kernel_overlap_frac": round(both / k_busy, 3) if k_busy else None,
                      "span_ms": round((t1 - t0) / 1e6, 3)}))


if __name__ == "__main__":
    main(sys.argv[1])
