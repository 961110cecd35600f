#!/usr/bin/env python3
"""Drive tools/zcopy.so: zero-copy kernel reads of registered host memory vs hipMemcpyAsync
(tuning aid for a C4 gather from the page-locked layer buffer).  python tools/zcopy.py [--gb 4]"""
import argparse
import ctypes as c
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=4.0)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime loaded the usual way)
    L = c.CDLL(os.path.join(ROOT, "tools", "zcopy.so"))
    L.zcopy_run.argtypes = [c.c_void_p, c.c_uint64, c.c_int, c.c_int, c.c_uint32, c.c_int, c.POINTER(c.c_float),
                            c.POINTER(c.c_float)]
    n = int(a.gb * 1e9) // 4096 * 4096
    buf = np.ones(n + 4096 * 2, dtype=np.uint8)
    base = buf.ctypes.data
    p = (base + 4095) & ~4095
    for mode, grid, off, name in [(0, 0, 0, "hipMemcpyAsync"), (1, 1024, 0, "kernel u1 g1024"),
                                  (2, 1024, 0, "kernel u4 g1024"), (3, 1024, 0, "kernel u8 g1024"),
                                  (2, 4096, 0, "kernel u4 g4096"), (3, 4096, 0, "kernel u8 g4096"),
                                  (2, 2048, 4, "kernel u4 g2048 off4"), (3, 2048, 0, "kernel u8 g2048")]:
        ms, gb = c.c_float(), c.c_float()
        rc = L.zcopy_run(p, n, mode, grid, off, 3, c.byref(ms), c.byref(gb))
        print("%-24s rc=%d %8.2f ms %7.2f GB/s" % (name, rc, ms.value, gb.value), flush=True)
        if rc:
            raise SystemExit(rc)


if __name__ == "__main__":
    main()
