#!/usr/bin/env python3
"""Time the native FS walk (tsg_collector_add_fs: FS.Walk + Required + reads into the
arena) on host cores, no scan -- the c1fs workload's host side.

Writes a c1fs-style source tree (--gb of the C1/C2 generator's files) under /dev/shm,
walks it into 256-MiB batches with a host-only scanner from the oracle library (no GPU
needed) and prints seconds per full walk.  SPROF=/tmp/x.prof samples the walks' CPU time
(tools/sprof).
"""
import argparse
import ctypes
import os
import shutil
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import hostlib  # noqa: E402
from trivy_amd import corpus  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--arena-mb", type=int, default=256)
    ap.add_argument("--root", default=None, help="an existing tree (default: written under /dev/shm, removed after)")
    a = ap.parse_args()
    import bench
    from trivy_amd.analyzer import AnalyzerOptions, SecretAnalyzer, SecretScannerOption
    from trivy_amd.analyzer.secret import Collector
    from trivy_amd.walker import FS, Option, _CFsAddStats
    root, made = a.root, False
    if root is None:
        root, made = "/dev/shm/tsg-fswalk-%d" % os.getpid(), True
        C0 = corpus.generate(int(a.gb * 1e9), seed=corpus.SEED, crlf_share=0.05)
        bench.write_tree(C0, root)
        del C0
    try:
        L = hostlib.lib()
        an = SecretAnalyzer(lib=L, host_only=True)
        an.Init(AnalyzerOptions(SecretScannerOption("")))
        col = Collector(an, a.arena_mb << 20, True)
        sp = None
        if os.environ.get("SPROF"):
            sp = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sprof", "sprof.so"))
            sp.sprof_start(4000)
        for _ in range(a.reps):
            w = FS().Walk(root, Option(), lib=L)
            st = _CFsAddStats()
            t0 = time.time()
            files = nbytes = 0
            while True:
                rc = L.tsg_collector_add_fs(col._h, w._h, ctypes.byref(st))
                if rc < 0:
                    raise SystemExit(hostlib.last_error())
                files += col.files()
                col.reset()
                if rc == 0:
                    break
            dt = time.time() - t0
            print("fs walk %.3f s  files %d  %s" % (dt, files, {n: getattr(st, n) for n, _ in st._fields_}), flush=True)
        if sp is not None:
            print("sprof samples", sp.sprof_stop(os.environ["SPROF"].encode()))
    finally:
        if made:
            shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
