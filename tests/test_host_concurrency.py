"""Host-side concurrency of the exact tail (CPU; the sanitizer runs drive this file).

The tail's worker pool (parallel.h), concurrent scans on one scanner and the
reference CPU algorithm's file fan-out must give the sequential results.
tools/sanitize.sh runs these (and the host-tail / analyzer / allow-path tests)
against ASan+UBSan and TSan builds of the host library.
"""
import ctypes as c
import os
import threading
from pathlib import Path

import numpy as np

from oracle import hostlib
from tests.corpus import make_corpus
from trivy_amd.secret import NewScanner
from trivy_amd.secret.scanner import ScanResult, _CBatch, _declare

ROOT = Path(__file__).resolve().parent.parent


def _batch(files):
    contents = [b for _, b in files]
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in contents])
    arena = np.frombuffer(b"".join(contents) + b"\0" * 64, dtype=np.uint8)
    pb = [p.encode() for p, _ in files]
    parr = (c.c_char_p * len(pb))(*pb)
    plen = np.array([len(p) for p in pb], dtype=np.uint64)
    keep = (arena, offs, parr, plen)
    return keep, _CBatch(len(files), arena.ctypes.data, offs.ctypes.data, None, None,
                         c.cast(parr, c.c_void_p).value, plen.ctypes.data, None)


def _cpuref(sc, batch, threads):
    L = hostlib.lib()
    h = c.c_void_p()
    assert L.tsg_cpuref_scan(c.byref(sc._cg.g), c.byref(batch), threads, c.byref(h)) == 0, hostlib.last_error()
    return ScanResult(sc, h).raw()


def test_cpuref_threads_agree():
    L = hostlib.lib()
    _declare(L)
    sc = NewScanner(None, lib=L, host_only=True)
    files = [(p, b.replace(b"\r", b"")) for p, b in make_corpus(71, 120)]
    keep, batch = _batch(files)
    one = _cpuref(sc, batch, 1)
    assert _cpuref(sc, batch, 8) == one
    assert sum(len(f["findings"]) for f in one) > 5


def test_concurrent_host_tails():
    """Several threads running the reference scan on one scanner at once (shared pool)."""
    L = hostlib.lib()
    _declare(L)
    sc = NewScanner(None, lib=L, host_only=True)
    batches = [_batch([(p, b.replace(b"\r", b"")) for p, b in make_corpus(80 + k, 60)]) for k in range(4)]
    want = [_cpuref(sc, b, 1) for _, b in batches]
    got = [None] * len(batches)

    def run(i):
        got[i] = _cpuref(sc, batches[i][1], 4)
    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(batches))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert got == want


def test_submit_without_gpu_reports_error():
    """tsg_scan_submit / tsg_scan_wait on a host-only scanner: the scan thread fails cleanly."""
    L = hostlib.lib()
    _declare(L)
    sc = NewScanner(None, lib=L, host_only=True)
    files = [(p, b) for p, b in make_corpus(90, 10)]
    contents = [b for _, b in files]
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in contents])
    arena = np.frombuffer(b"".join(contents) + b"\0" * 64, dtype=np.uint8)
    pend = [sc.scan_arena_async(arena, offs, [p for p, _ in files]) for _ in range(3)]
    for p in pend:
        try:
            p.wait()
        except RuntimeError as e:
            assert "no GPU engine" in str(e)
        else:
            raise AssertionError("scan without a GPU engine succeeded")


def _budget_child(q, cpus, env):
    import os
    os.environ.pop("TSG_POOL_SHARE", None)
    os.environ.pop("LOCAL_WORLD_SIZE", None)
    os.environ.update(env)
    os.sched_setaffinity(0, cpus)
    from trivy_amd import _lib
    q.put(_lib.lib().tsg_debug_pool_budget())


def _budget(cpus, **env):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_budget_child, args=(q, cpus, env))
    p.start()
    v = q.get(timeout=120)
    p.join(60)
    return v


def test_pool_budget_follows_affinity_and_ranks():
    """HostPool's default size (parallel.h PoolBudget): the affinity mask, split over the ranks
    sharing it (LOCAL_WORLD_SIZE spread over the node, or TSG_POOL_SHARE), minus the reserve --
    not the whole container per process (8 ranks would otherwise oversubscribe 8x)."""
    import os
    online = os.cpu_count()
    allc = sorted(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass

    def want(aff, share, ranks):
        c = aff / share
        if quota:
            c = min(c, quota / ranks)
        c = max(1, int(c))
        return max(1, c - (4 if c >= 16 else max(1, c // 4)))

    four = set(allc[:4])
    assert _budget(four) == want(4, 1, 1)
    assert _budget(four, TSG_POOL_SHARE="2") == want(4, 2, 2)
    if len(allc) == online and online >= 8:
        # 2 ranks on all CPUs: each gets half
        assert _budget(set(allc), LOCAL_WORLD_SIZE="2") == want(online, 2, 2)
        # 8 ranks, this one bound to half the CPUs: ~4 ranks share the half
        half = set(allc[:online // 2])
        assert _budget(half, LOCAL_WORLD_SIZE="8") == want(online // 2, max(1, 8 * (online // 2) / online), 8)
    assert _budget({allc[0]}) == 1


def test_result_json_range_then_whole():
    """tsg_result_json_range keeps its own buffer: a range read first must not become what
    tsg_result_json returns for the whole batch (a bench/test full_diff followed by secrets())."""
    L = hostlib.lib()
    sc = NewScanner(None, lib=L, host_only=True)
    files = [(p, b.replace(b"\r", b"")) for p, b in make_corpus(61, 200)]
    keep, batch = _batch(files)
    h = c.c_void_p()
    assert L.tsg_cpuref_scan(c.byref(sc._cg.g), c.byref(batch), 4, c.byref(h)) == 0
    r = ScanResult(sc, h)
    tail = r.raw(150, 200)
    whole = r.raw()
    assert len(whole) == len(files) and whole[150:200] == tail
    assert r.raw(0, 10) == whole[:10] and r.raw() == whole


def test_pool_spare_workers_take_wide_jobs_only():
    """Concurrent ordinary ParallelFor jobs (pipelined scans' exact passes, allow-path passes) share the
    pool's steady workers: at most steady + callers threads run their bodies at once, however many jobs
    overlap; wide jobs (the walks, the drain) may also use the spare workers.  Run in a fresh process so
    the pool is built from the env given here."""
    import subprocess
    import sys
    code = ("import ctypes as c\nfrom oracle import hostlib\nL = hostlib.lib()\n"
            "L.tsg_debug_pool_peak.argtypes = [c.c_int, c.c_uint64, c.c_int, c.c_int, c.POINTER(c.c_int), "
            "c.POINTER(c.c_int)]\n"
            "s, w = c.c_int(), c.c_int()\n"
            "for wide in (0, 1):\n"
            "    print(L.tsg_debug_pool_peak(3, 600, 300, wide, c.byref(s), c.byref(w)), s.value, w.value)\n")
    env = dict(os.environ, TSG_POOL_THREADS="4", TSG_POOL_SPARE="3")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=str(ROOT), check=True, capture_output=True,
                         text=True, timeout=120).stdout.split("\n")
    narrow, wide = [list(map(int, l.split())) for l in out[:2]]
    assert narrow[1:] == [4, 7] and wide[1:] == [4, 7]
    assert narrow[0] <= 4 + 3, narrow
    assert wide[0] >= 4 + 3 + 1, wide  # the spare workers did join the wide jobs
