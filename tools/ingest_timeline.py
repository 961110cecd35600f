#!/usr/bin/env python3
"""Copy timeline of an ingest run (rocprofv3 --kernel-trace --memory-copy-trace, CSV).

For the large host->device copies (the staging chunks of GpuEngine::RunHost) it reports
how busy the copy engine was over the leg, the gaps between consecutive chunk copies and
what the GPU ran in each gap (kernel names by total time), so a pipeline stall shows as
a gap with the stage that caused it.
Usage: tools/ingest_timeline.py <trace dir> [--min-mb 64] [--last-s 3.0]
"""
import argparse
import csv
import re
import glob
import os
from collections import defaultdict


def rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True):
        out += list(csv.DictReader(open(p)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-mb", type=float, default=64.0, help="copies at least this large are chunk copies")
    ap.add_argument("--last-s", type=float, default=0.0, help="only the last N seconds of the trace (0: all)")
    a = ap.parse_args()
    cp = rows(a.dir, "memory_copy_trace.csv")
    kt = rows(a.dir, "kernel_trace.csv")
    if not cp:
        raise SystemExit("no memory_copy_trace.csv under %s" % a.dir)
    print("copy columns:", list(cp[0].keys()))
    size_key = next((k for k in cp[0] if k.lower() in ("bytes", "size", "copy_bytes")), None)
    h2d = []
    for r in cp:
        d = r.get("Direction", "") + r.get("Kind", "")
        if "HOST_TO_DEVICE" not in d.upper():
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nb = int(r[size_key]) if size_key else None
        h2d.append((s, e, nb))
    h2d.sort()
    t_end = max(e for _, e, _ in h2d)
    if a.last_s > 0:
        h2d = [x for x in h2d if x[0] >= t_end - a.last_s * 1e9]
    big = [x for x in h2d if (x[2] or 0) >= a.min_mb * 1e6 or (x[2] is None and x[1] - x[0] > a.min_mb * 1e6 / 60e3)]
    if not big:
        raise SystemExit("no large copies")
    span = big[-1][1] - big[0][0]
    busy = sum(e - s for s, e, _ in big)
    print("large H2D copies: %d over %.1f ms, copy engine busy %.1f ms (%.3f)" % (len(big), span / 1e6, busy / 1e6,
                                                                                 busy / span))
    if big[0][2]:
        tot = sum(nb for _, _, nb in big)
        print("bytes %.2f GB, %.1f GB/s while copying, %.1f GB/s over the span" % (tot / 1e9, tot / busy, tot / span))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", r.get("Name", "?"))) for r in kt]
    ks.sort()
    gaps = []
    for (s0, e0, _), (s1, e1, _) in zip(big, big[1:]):
        if s1 > e0:
            gaps.append((e0, s1))
    print("gaps between chunk copies: %d, total %.1f ms" % (len(gaps), sum(b - a for a, b in gaps) / 1e6))
    show = sorted(sorted(gaps, key=lambda g: -(g[1] - g[0]))[:16])  # the largest, in time order
    for ga, gb in show:
        by = defaultdict(float)
        for s, e, n in ks:
            if e > ga and s < gb:
                m = re.findall(r"(\w+)(?:<[^()]*>)?\(", n)
                by[m[0] if m else n[:40]] += (min(e, gb) - max(s, ga)) / 1e6
        top = sorted(by.items(), key=lambda kv: -kv[1])[:4]
        print("  gap %.3f ms at +%.1f ms: %s" % ((gb - ga) / 1e6, (ga - big[0][0]) / 1e6,
                                               ", ".join("%s %.3f" % kv for kv in top) or "(no kernels)"))


if __name__ == "__main__":
    main()
