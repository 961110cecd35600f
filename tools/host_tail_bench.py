#!/usr/bin/env python3
"""Time the exact host pass on CPU over candidates dumped from a GPU run.

  gpurun ... TSG_DUMP_CANDS=gpurun_out/cands_4g.bin python bench.py --gb 4 --steps 1 --warmup 0
  python tools/host_tail_bench.py gpurun_out/cands_4g.bin --gb 4 [--threads 8] [--reps 3]
"""
import argparse
import ctypes as c
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trivy_amd import _lib, corpus  # noqa: E402
from trivy_amd.secret import builtin_allow_rules, builtin_rules  # noqa: E402
from trivy_amd.secret.scanner import CGlobal, _CBatch, _CStats  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cands")
    ap.add_argument("--gb", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from oracle import hostlib
    L = hostlib.lib()
    cand = np.fromfile(args.cands, dtype=np.uint8)
    n_c = len(cand) // 40
    t = time.time()
    C = corpus.generate(int(args.gb * 1e9))
    print("corpus %.1f s, %d files, %d candidates" % (time.time() - t, C.n_files, n_c), flush=True)
    cg = CGlobal(builtin_rules(), builtin_allow_rules(), [])
    b = _CBatch(C.n_files, C.arena.ctypes.data, C.offsets.ctypes.data, None, None, C.path_ptrs.ctypes.data,
                None, None)
    for _ in range(args.reps):
        h = c.c_void_p()
        t = time.time()
        rc = L.tsg_debug_host_tail_cands(c.byref(cg.g), c.byref(b), cand.ctypes.data, n_c, c.byref(h))
        t1 = time.time()
        if rc != 0:
            raise SystemExit(hostlib.last_error())
        s = _CStats()
        L.tsg_result_stats(h, c.byref(s))
        L.tsg_result_free(h)
        t2 = time.time()
        print("tail %.1f ms (allow %.1f, exact %.1f) free %.1f ms, findings %d" %
              ((t1 - t) * 1e3, s.ms_host_allow_path, s.ms_host_exact, (t2 - t1) * 1e3, s.findings), flush=True)


if __name__ == "__main__":
    main()
