#!/usr/bin/env python3
"""Time the native tar walk (tsg_collector_add_tar) on host cores, no scan.

Generates a C4-style layer (--gb of file data), walks it into 256-MiB batches
with a host-only scanner from the oracle library (no GPU needed) and prints
seconds per full walk.  By default the arena gets the bytes as read (the bench's
C4 GPU pre-transform mode); --host-transform packs them transformed.  TSG_WALK_DEBUG=1 adds the per-phase split.
"""
import argparse
import os
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
    ap.add_argument("--host-transform", action="store_true",
                    help="CR strip / printable extraction while packing (default: bytes as read, as C4's GPU mode)")
    a = ap.parse_args()
    layer = corpus.generate_layer(int(a.gb * 1e9))
    from trivy_amd.analyzer import AnalyzerOptions, SecretAnalyzer, SecretScannerOption
    from trivy_amd.analyzer.secret import Collector, _CTarStats
    an = SecretAnalyzer(lib=hostlib.lib(), host_only=True)
    an.Init(AnalyzerOptions(SecretScannerOption("")))
    col = Collector(an, a.arena_mb << 20, not a.host_transform)
    sp = None
    if os.environ.get("SPROF"):  # tools/sprof: sample the walks' CPU time
        import ctypes
        sp = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sprof", "sprof.so"))
        sp.sprof_start(4000)
    for rep in range(a.reps):
        t0 = time.time()
        cur, files, st = 0, 0, _CTarStats()
        while True:
            r, cur = col.add_tar(layer, cur, st)
            files += col.files()
            col.reset()
            if r == 0:
                break
        dt = time.time() - t0
        print("walk %.3f s  %.2f GB/s layer  files %d" % (dt, layer.size / dt / 1e9, files))
    if sp is not None:
        print("sprof samples", sp.sprof_stop(os.environ["SPROF"].encode()))


if __name__ == "__main__":
    main()
