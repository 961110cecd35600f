#!/usr/bin/env python3
"""Drive tools/k1x.so (K1 design experiments, tuning aid): builtin reach table +
the C2 corpus in HBM, every variant timed with HIP events; prints a table.

  python tools/k1x.py [--gb 20] [--reps 5] [--only i,j,...]
"""
import argparse
import ctypes as c
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gb", type=float, default=20.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import numpy as np
    import torch
    from tests.filter_model import FilterModel
    from trivy_amd import corpus
    from trivy_amd.secret import builtin_rules

    fm = FilterModel(builtin_rules())
    assert fm.n_words == 4, fm.n_words
    L = c.CDLL(os.path.join(ROOT, "tools", "k1x.so"))
    L.k1x_name.restype = c.c_char_p
    L.k1x_run.argtypes = [c.c_int, c.c_void_p, c.c_uint64, c.c_void_p, c.c_void_p, c.c_int, c.c_int,
                          c.POINTER(c.c_float)]
    C = corpus.generate(int(a.gb * 1e9))
    dev = torch.device("cuda", 0)
    arena = torch.from_numpy(C.arena).to(dev)
    reach = torch.from_numpy(np.ascontiguousarray(fm.reach.astype(np.uint32)).view(np.int32)).to(dev)
    out = torch.zeros(16, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    n = C.n_bytes
    only = {int(x) for x in a.only.split(",") if x}
    for v in range(L.k1x_count()):
        if only and v not in only:
            continue
        ms = c.c_float()
        rc = L.k1x_run(v, arena.data_ptr(), n, reach.data_ptr(), out.data_ptr(), a.grid, a.reps, c.byref(ms))
        if rc:
            print("variant %d failed: %d" % (v, rc), flush=True)
            sys.exit(1)
        o = out.cpu().numpy().view(np.uint32)
        print("%2d %-28s %8.3f ms %7.3f TB/s  flagged %10d  nl %10d" % (
            v, L.k1x_name(v).decode(), ms.value, n / (ms.value * 1e-3) / 1e12, o[1], o[2]), flush=True)


if __name__ == "__main__":
    main()
