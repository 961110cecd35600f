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
    ap.add_argument("--rec", type=int, default=64, help="record size of the dump (40 / 48: older builds)")
    ap.add_argument("--hints", action="store_true", help="fill Candidate::nl_back on the host first")
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c3f"],
                    help="corpus / rules of the dump (bench.py --workload; rank 0 seed)")
    ap.add_argument("--crlf", type=float, default=None,
                    help="c2: CRLF share of the generated files, stripped as the bench's resident leg does "
                         "(default 0.05, the bench's default)")
    args = ap.parse_args()
    from oracle import hostlib
    L = hostlib.lib()
    cand = np.fromfile(args.cands, dtype=np.uint8)
    if args.rec != 64:  # dumps from before Candidate::nl_back (40 B) / nl_fwd (48 B): those hints unknown
        rec = args.rec
        if True:
            old = cand.reshape(-1, rec)
            cand = np.full((len(old), 64), 0xFF, dtype=np.uint8)
            cand[:, :rec] = old
            cand[:, 60:64] = 0
            cand = cand.reshape(-1)
    n_c = len(cand) // 64
    t = time.time()
    rules = builtin_rules()
    if args.workload == "c2":
        crlf = 0.05 if args.crlf is None else args.crlf
        C = corpus.generate(int(args.gb * 1e9), crlf_share=crlf)
        if crlf > 0:
            C = C.stripped()
    else:
        import tempfile
        from trivy_amd.secret import ParseConfig
        y, samples = corpus.c3_rules(fullscan_share=0.05 if args.workload == "c3f" else 0.0)
        with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
            f.write(y)
        rules = rules + list(ParseConfig(f.name).CustomRules)
        os.remove(f.name)
        C = corpus.generate_c3(int(args.gb * 1e9), samples, seed=corpus.SEED)
    if args.hints:  # fill nl_back as the finalize kernel does (last three '\n' before wlo)
        rec = cand.reshape(-1, 64)
        file = rec[:, 0:4].copy().view(np.uint32).ravel()
        wlo = rec[:, 8:16].copy().view(np.int64).ravel()
        back = np.full((n_c, 3), 0xFFFFFFFF, dtype=np.uint32)
        fwd = np.full((n_c, 3), 0xFFFFFFFF, dtype=np.uint32)
        for i in range(n_c):
            fs, fe = int(C.offsets[file[i]]), int(C.offsets[file[i] + 1])
            w = fs + int(wlo[i])
            lo = max(fs, w - (1 << 20))
            nl = np.flatnonzero(C.arena[lo:w] == 10)[-3:][::-1]
            for k, x in enumerate(nl):
                back[i, k] = w - (lo + int(x))
            if lo == fs:
                back[i, len(nl):] = 0xFFFFFFFE
            hi = min(fe, w + (1 << 20))
            nl = np.flatnonzero(C.arena[w:hi] == 10)[:3]
            for k, x in enumerate(nl):
                fwd[i, k] = int(x)
            if hi == fe:
                fwd[i, len(nl):] = 0xFFFFFFFE
        rec[:, 36:48] = back.view(np.uint8).reshape(-1, 12)
        rec[:, 48:60] = fwd.view(np.uint8).reshape(-1, 12)
        print("hints filled %.1f s" % (time.time() - t), flush=True)
    print("corpus %.1f s, %d files, %d candidates" % (time.time() - t, C.n_files, n_c), flush=True)
    cg = CGlobal(rules, builtin_allow_rules(), [])
    b = _CBatch(C.n_files, C.arena.ctypes.data, C.offsets.ctypes.data, None, None, C.path_ptrs.ctypes.data,
                None, None)
    sp = None
    if os.environ.get("SPROF"):  # tools/sprof: sample the reps' CPU time
        sp = c.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "sprof", "sprof.so"))
        sp.sprof_start(int(os.environ.get("SPROF_US", "4000")))
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

    if sp is not None:
        print("sprof samples", sp.sprof_stop(os.environ["SPROF"].encode()))


if __name__ == "__main__":
    main()
