#!/usr/bin/env python3
"""GPU idle gaps of a traced run and the host calls behind them (tuning aid).

  rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d DIR -o run --output-format csv -- python3 bench.py ...
  python tools/drain_trace.py DIR [--min-us 100]

For every gap in the union of the GPU's kernels and copies longer than
--min-us, prints the op that ended it, the HIP call that enqueued that op (by
correlation id) and when that call ran relative to the gap: a call that began
after the gap opened means the GPU waited for the host to submit; one that
ended before it means the op waited on the device (a dependency or a barrier).
"""
import argparse
import collections
import csv
import glob
import os


def load(d, name):
    fs = glob.glob(os.path.join(d, "**", "*%s.csv" % name), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=100.0)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    ops = []
    for r in load(a.dir, "kernel_trace"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-36:],
                    r["Correlation_Id"], r.get("Stream_Id", "")))
    for r in load(a.dir, "memory_copy_trace"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", ""),
                    r["Correlation_Id"], r.get("Stream_Id", "")))
    api = {r["Correlation_Id"]: r for r in load(a.dir, "hip_api_trace")}
    calls = collections.defaultdict(list)  # thread -> its HIP calls
    for r in api.values():
        calls[r["Thread_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]))
    for v in calls.values():
        v.sort()
    ops.sort()
    if not ops:
        raise SystemExit("no kernel / copy records under %s" % a.dir)
    t0 = ops[0][0]
    cur = ops[0][1]
    gaps = []
    for s, e, n, cid, st in ops[1:]:
        if s - cur > a.min_us * 1e3:
            gaps.append((cur, s, n, cid, st))
        cur = max(cur, e)
    busy_idle = sum(g[1] - g[0] for g in gaps)
    print("ops %d, span %.2f ms, idle in gaps > %.0f us: %.2f ms in %d gaps" %
          (len(ops), (cur - t0) / 1e6, a.min_us, busy_idle / 1e6, len(gaps)))
    for g0, g1, n, cid, st in gaps[:a.top]:
        r = api.get(cid)
        if r is None:
            print("%10.3f ms gap %7.3f ms -> %-36s stream %s (no HIP call)" % ((g0 - t0) / 1e6, (g1 - g0) / 1e6, n, st))
            continue
        cs, ce = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        # what the enqueuing thread did during the gap (its longest calls)
        during = [c for c in calls[r["Thread_Id"]] if c[1] > g0 and c[0] < cs]
        during.sort(key=lambda c: c[0] - c[1])
        busy = ", ".join("%s %.2f" % (c[2], (c[1] - c[0]) / 1e6) for c in during[:3])
        print("%10.3f ms gap %7.3f ms -> %-36s stream %s by %s on thread %s: call at gap%+.3f ms (ended %+.3f)%s" %
              ((g0 - t0) / 1e6, (g1 - g0) / 1e6, n, st, r["Function"], r["Thread_Id"], (cs - g0) / 1e6,
               (ce - g0) / 1e6, "; before it: " + busy if busy else ""))


if __name__ == "__main__":
    main()
