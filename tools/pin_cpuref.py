#!/usr/bin/env python3
"""Pin tsg_cpuref_scan against the Python oracle at size (TEST INFRASTRUCTURE, CPU only).

The GPU-vs-cpuref every-file diffs (bench.py `gpu_vs_cpuref_all_files`,
tests/test_gpu_bench_corpus.py) prove the GPU path equals tsg_cpuref_scan
(oracle/native/host_hooks.cpp), which links the product's own Go-semantics
regex engine (goregex.cpp).  This script closes that loop independently of
goregex.cpp: every file of a generated corpus is scanned by the pure-Python
oracle (oracle/secret_scanner.py + oracle/goregexp.py, pinned by the
reference's scanner_test.go goldens) in a process pool and compared field for
field (Secret dicts: RuleID, Category, Severity, Title, StartLine, EndLine,
Code lines, Match, Offset) with tsg_cpuref_scan's result for the same file.

Workloads: c2 -- the bench's C2 generator (seed corpus.SEED, 5 % CRLF files
stripped as the bench's resident leg does) cut at --mb; c3f -- the
tests' C3f corpus (2,000 generated rules, 5 % bare class-run rules).
Reference: pkg/fanal/secret/scanner.go:102-148, 377-558.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(args):
    idx, ap, op, pp, cfg_path = args
    from oracle import secret_scanner as osc
    arena = np.load(ap, mmap_mode="r")
    offs = np.load(op)
    paths = np.load(pp)
    sc = osc.new_scanner(osc.parse_config(cfg_path) if cfg_path else None)
    out = {}
    for i in idx:
        b = arena[int(offs[i]):int(offs[i + 1])].tobytes()
        p = paths[i * 64:(i + 1) * 64].tobytes().split(b"\0", 1)[0].decode()
        out[i] = sc.scan(p, b)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["c2", "c3f"], default="c2")
    ap.add_argument("--mb", type=float, default=1000)
    ap.add_argument("--procs", type=int, default=max(1, (os.cpu_count() or 2) - 2))
    ap.add_argument("--out", default=None, help="JSON summary path")
    args = ap.parse_args()
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    from tests.test_gpu_bench_corpus import _cpuref
    cfg_path = None
    tmp = tempfile.mkdtemp(prefix="pin_")
    t0 = time.time()
    if args.workload == "c2":
        C = corpus.generate(int(args.mb * 1e6), seed=corpus.SEED, crlf_share=0.05)
        C = C.stripped()
    else:
        y, samples = corpus.c3_rules(fullscan_share=0.05)
        cfg_path = os.path.join(tmp, "trivy-secret.yaml")
        with open(cfg_path, "w") as f:
            f.write(y)
        C = corpus.generate_c3(int(args.mb * 1e6), samples, seed=corpus.SEED + 17, secrets_per_byte=1.0 / 16384)
    print("corpus: %d files, %.1f MB (%.0f s)" % (C.n_files, C.n_bytes / 1e6, time.time() - t0), flush=True)
    t1 = time.time()
    ref = _cpuref(C, n_threads=args.procs, cfg_path=cfg_path)
    print("tsg_cpuref_scan: %.1f s" % (time.time() - t1), flush=True)
    n = C.n_files
    apath, opath, ppath = (os.path.join(tmp, x) for x in ("arena.npy", "offs.npy", "paths.npy"))
    np.save(apath, C.arena[:int(C.offsets[n])])
    np.save(opath, C.offsets[:n + 1])
    np.save(ppath, C.path_buf[:n * 64])
    sizes = np.diff(C.offsets.astype(np.int64))
    order = [int(i) for i in np.argsort(-sizes, kind="stable")]  # largest first, spread over the workers
    chunks = [order[k::args.procs * 8] for k in range(args.procs * 8)]
    t2 = time.time()
    want = {}
    ctx = mp.get_context("spawn")
    with ctx.Pool(args.procs) as pool:
        for k, part in enumerate(pool.imap_unordered(_worker, [(ch, apath, opath, ppath, cfg_path) for ch in chunks])):
            want.update(part)
            print("oracle: %d/%d chunks, %d files, %.0f s" % (k + 1, len(chunks), len(want), time.time() - t2),
                  flush=True)
    t_oracle = time.time() - t2
    bad, first, n_find, n_find_files = 0, None, 0, 0
    got = ref.secrets([C.path(i) for i in range(n)], lo=0)
    for i in range(n):
        w = want[i]
        g = got[i].to_dict()
        k = len(w["Findings"] or [])
        n_find += k
        n_find_files += k > 0
        if g != w:
            bad += 1
            if first is None:
                first = i
    summary = {"workload": args.workload, "files": n, "bytes": int(C.n_bytes), "findings": n_find,
               "files_with_findings": n_find_files, "mismatches": bad,
               "first_mismatch": C.path(first) if first is not None else None,
               "oracle_s": round(t_oracle, 1), "oracle_procs": args.procs,
               "oracle_MBps_per_proc": round(C.n_bytes / 1e6 / t_oracle / args.procs, 3),
               "reference": "oracle/secret_scanner.py (Python restatement of scanner.go, pinned by the reference's "
                            "goldens) vs oracle/native/host_hooks.cpp tsg_cpuref_scan, every file"}
    print(json.dumps(summary), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(summary, f, indent=1)
    for x in (apath, opath, ppath):
        os.remove(x)
    if cfg_path:
        os.remove(cfg_path)
    os.rmdir(tmp)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
