#!/usr/bin/env python3
"""FETCH_SIZE (rocprofv3 --pmc) -> HBM bytes per launch of a kernel, with the gfx950
correction of /opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of
wide streaming reads: x2).  Writes profiles/traffic_<tag>.json for bench.py's roofline.traffic.

  python tools/pmc_traffic.py gpurun_out/pmc_<tag> --gb 20 --kernel filter_kernel --out profiles/traffic_r01.json
"""
import argparse
import collections
import csv
import glob
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gb", type=float, required=True)
    ap.add_argument("--kernel", default="filter_kernel")
    ap.add_argument("--out", required=True)
    ap.add_argument("--csv-out", default=None, help="per-kernel summary CSV")
    ap.add_argument("--workload", default="c2", help="bench workload id the pass ran (bench.py matches it)")
    ap.add_argument("--note", default="")
    args = ap.parse_args()
    per = collections.defaultdict(list)
    for f in glob.glob(args.dir + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != "FETCH_SIZE":
                continue
            per[(r["Kernel_Name"], r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
    by_kernel = collections.defaultdict(list)
    for (k, _), vals in per.items():
        by_kernel[k].append(sum(vals))  # per dispatch (summed over XCD instances)
    rows = []
    for k, v in sorted(by_kernel.items()):
        kb = sum(v) / len(v)
        rows.append((k, len(v), kb, kb * 1024, kb * 1024 * 2))
    if args.csv_out:
        with open(args.csv_out, "w") as fo:
            fo.write("kernel,counter,dispatches,avg_value_KB,avg_bytes_raw,avg_bytes_x2_gfx950\n")
            for k, n, kb, raw, x2 in rows:
                fo.write('"%s",FETCH_SIZE,%d,%.3f,%.0f,%.0f\n' % (k, n, kb, raw, x2))
    hit = [r for r in rows if args.kernel in r[0]]
    if not hit:
        raise SystemExit("no FETCH_SIZE rows for " + args.kernel)
    k, n, kb, raw, x2 = hit[0]
    # the whole GPU phase of one scan: every tsg kernel, each averaged per dispatch
    phase = {r[0]: round(r[4]) for r in rows if "tsg::" in r[0]}
    json.dump({"workload": args.workload, "gb": args.gb, "kernel": k, "dispatches": n,
               "bytes_per_launch": round(x2), "k1_bytes_per_launch": round(x2),
               "phase_bytes_per_scan": sum(phase.values()), "phase_kernels_bytes": phase,
               "fetch_size_kb": kb,
               "correction": "x2 (gfx950 FETCH_SIZE counts half of wide streaming reads); calibrated for K1's "
                             "16-B/lane stream, an upper bound for the other kernels' gathers",
               "note": args.note},
              open(args.out, "w"), indent=1)
    print(json.dumps(json.load(open(args.out))))


if __name__ == "__main__":
    main()
