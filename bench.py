#!/usr/bin/env python3
"""Secret-scanning throughput on MI355X (BASELINE.json metric: GB/s secret-scanned).

Workload (configs[1]): builtin ruleset (87 rules) over a synthetic mixed-text
corpus of --gb GB per GPU (default 20), generated deterministically on the host
(seed 0x5EC2E7), copied once into HBM.  A "step" is one full
Scan of that corpus: K1 streaming prefilter + confirm, the careful pass over fold-rune files,
K2 NFA verify, full-scan tasks and
the exact host pass (windowed Go-regexp, allow/exclude, censoring, findings,
sort).  Inputs are resident in HBM when the timed region starts; findings
come out as C++ structs (types.Secret equivalents).

Multi-GPU (torchrun, one rank per GPU): files shard by content, each rank owns
its own --gb GB shard (weak scaling); no data-path collective.  Timing uses a
barrier + torch.cuda.synchronize() on both sides and the max over ranks.

--workload selects the BASELINE config measured (default c2 = configs[1], the
headline): c3 = configs[2] (2,000 generated custom rules appended to the
builtins, C2-style corpus with their samples planted); c4 = configs[3] (an
uncompressed image layer of millions of small files resident in host memory:
native tar walk + Required + CR strip / printable extraction into double-
buffered pinned arenas, H2D, kernels, exact tail -- the batching/arena packing
path; value counts the input bytes of the files analyzed).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _cpu_sample_worker(args):
    idx, arena_path, offs_path, paths_path, cfg_path = args
    import numpy as np
    from oracle import secret_scanner as osc
    arena = np.load(arena_path, mmap_mode="r")
    offs = np.load(offs_path)
    paths = np.load(paths_path)
    sc = osc.new_scanner(osc.parse_config(cfg_path) if cfg_path else None)
    nb = 0
    nf = 0
    res = {}
    for i in idx:
        b = arena[int(offs[i]):int(offs[i + 1])].tobytes()
        p = paths[i * 64:(i + 1) * 64].tobytes().split(b"\0", 1)[0].decode()
        r = sc.scan(p, b)
        nb += len(b)
        nf += len(r["Findings"] or [])
        res[i] = r
    return nb, nf, res


def _first_files(C, sample_bytes):
    n = 0
    while n < C.n_files and int(C.offsets[n + 1]) <= sample_bytes:
        n += 1
    return max(n, 1)


def oracle_sample(C, sample_bytes, cores, tmpdir, cfg_path=None):
    """The Python oracle (pinned by the reference's golden tests) on the first files: the parity reference."""
    import multiprocessing as mp
    import numpy as np
    n = _first_files(C, sample_bytes)
    end = int(C.offsets[n])
    ap = os.path.join(tmpdir, "cpu_arena.npy")
    op = os.path.join(tmpdir, "cpu_offs.npy")
    pp = os.path.join(tmpdir, "cpu_paths.npy")
    np.save(ap, C.arena[:end])
    np.save(op, C.offsets[:n + 1])
    np.save(pp, C.path_buf[:n * 64])
    chunks = [list(range(k, n, cores)) for k in range(cores)]  # interleave files over workers for balance
    ctx = mp.get_context("spawn")
    t0 = time.time()
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_sample_worker, [(ch, ap, op, pp, cfg_path) for ch in chunks])
    dt = time.time() - t0
    want = {}
    for r in res:
        want.update(r[2])
    for f in (ap, op, pp):
        os.remove(f)
    return want, dt


def full_diff(gpu_res, cpu_res, n, chunk=4096):
    """Every file [0, n) of two results compared byte for byte (their JSON text, findings and
    Code lines included); returns (mismatching files, first mismatching index or None)."""
    bad, first = 0, None
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        a, b = gpu_res.raw_text(lo, hi), cpu_res.raw_text(lo, hi)
        if a == b:
            continue
        ja, jb = json.loads(a.decode("ascii")), json.loads(b.decode("ascii"))
        for i, (x, y) in enumerate(zip(ja, jb)):
            if x != y:
                bad += 1
                first = lo + i if first is None else first
    return bad, first


def cpu_baseline(C, sample_bytes, threads, cfg_path, want, gpu_res=None):
    """C++ restatement of the reference CPU algorithm (oracle/native/host_hooks.cpp tsg_cpuref_scan:
    scanner.go:377-463 -- per file and rule bytes.ToLower + Contains, whole-file Go-regexp FindAll,
    the same tail) on the first files of the corpus, timed on `threads` host threads per entry.
    The restated reference is itself checked against the Python oracle on the oracle's sample
    (`want`), and the GPU's findings (`gpu_res`, the timed run) are diffed against it on every
    file of the sample."""
    import ctypes as c
    import numpy as np
    from oracle import hostlib
    import trivy_amd.secret as secret
    from trivy_amd.secret.scanner import ScanResult, _CBatch, _CStats
    L = hostlib.lib()
    sc = secret.NewScanner(secret.ParseConfig(cfg_path) if cfg_path else None, lib=L, host_only=True)
    n = _first_files(C, sample_bytes)
    offs = np.ascontiguousarray(C.offsets[:n + 1])
    batch = _CBatch(n, C.arena.ctypes.data, offs.ctypes.data, None, None, C.path_ptrs.ctypes.data, None, None)
    runs, res = [], None
    for T in threads:
        h = c.c_void_p()
        t0 = time.time()
        if L.tsg_cpuref_scan(c.byref(sc._cg.g), c.byref(batch), int(T), c.byref(h)) != 0:
            raise RuntimeError("tsg_cpuref_scan: %s" % hostlib.last_error())
        dt = time.time() - t0
        st = _CStats()
        L.tsg_result_stats(h, c.byref(st))
        runs.append({"threads": int(T), "value": round(int(offs[-1]) / dt / 1e9, 6), "s": round(dt, 2),
                     "findings": int(st.findings)})
        if res is None:
            res = ScanResult(sc, h)
        else:
            L.tsg_result_free(h)
    nw = len(want)
    got = res.secrets([C.path(i) for i in range(nw)], lo=0)
    bad = sum(1 for i in range(nw) if got[i].to_dict() != want[i])
    full = None
    if gpu_res is not None:
        t0 = time.time()
        nbad, first = full_diff(gpu_res, res, n)
        full = {"files": n, "bytes": int(offs[-1]), "findings": runs[0]["findings"], "mismatches": nbad,
                "first_mismatch": C.path(first) if first is not None else None, "s": round(time.time() - t0, 2),
                "reference": "tsg_cpuref_scan (restated reference CPU algorithm), itself 0-mismatch vs the "
                             "Python oracle on the first %d files" % nw if bad == 0 else "tsg_cpuref_scan"}
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": runs[0]["value"], "unit": "GB/s", "cores": runs[0]["threads"],
            "kind": "port (restated reference CPU algorithm, C++)",
            "sample": "first %d files (%.1f MB) of the same corpus, tsg_cpuref_scan (oracle/native/host_hooks.cpp: "
                      "scanner.go:377-463 per file and rule -- bytes.ToLower + Contains gate, whole-file "
                      "Go-regexp FindAll with the product's Go-semantics engine, same tail); %d findings"
                      % (n, int(offs[-1]) / 1e6, runs[0]["findings"]),
            "runs": runs, "cpu_model": cpu_model,
            "parity_vs_oracle": {"files": nw, "mismatches": bad}, "gpu_vs_cpuref_all_files": full}


def measure_h2d(dev, gb=4.0):
    """Pinned host -> HBM copy rate on this box (hipMemcpyAsync through torch), GB/s: the
    practical H2D ceiling the ingest-inclusive rate is compared with."""
    import torch
    n = int(gb * 1e9)
    src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 0.0
    for _ in range(3):
        e0.record()
        dst.copy_(src, non_blocking=True)
        e1.record()
        e1.synchronize()
        best = max(best, n / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del src, dst
    return round(best, 2)


def measure_h2d_from(host, dev_index, gb=4.0):
    """H2D rate from `host` itself (a registered numpy buffer: the ingest leg's source), GB/s: one
    1-GiB hipMemcpyAsync at a time (as the engine's copier issues them) into a device buffer,
    through the HIP runtime directly (torch does not know the buffer is page-locked)."""
    import ctypes as c
    hip = c.CDLL("libamdhip64.so")
    n = min(int(gb * 1e9), host.nbytes) // (1 << 30) * (1 << 30)
    if n == 0:
        return None
    d = c.c_void_p()
    s = c.c_void_p()
    if hip.hipSetDevice(dev_index) != 0 or hip.hipMalloc(c.byref(d), c.c_size_t(1 << 30)) != 0:
        return None
    hip.hipStreamCreate(c.byref(s))
    best = 0.0
    try:
        for _ in range(3):
            t0 = time.perf_counter()
            for off in range(0, n, 1 << 30):
                hip.hipMemcpyAsync(d, c.c_void_p(host.ctypes.data + off), c.c_size_t(1 << 30), 1, s)
            hip.hipStreamSynchronize(s)
            best = max(best, n / (time.perf_counter() - t0) / 1e9)
    finally:
        hip.hipStreamDestroy(s)
        hip.hipFree(d)
    return round(best, 2)


def parity_block(C, last_result, want):
    """Findings of the GPU's last timed step vs the oracle, file by file (sample files)."""
    n = len(want)
    got = last_result.secrets([C.path(i) for i in range(n)], lo=0)
    bad = [i for i in range(n) if got[i].to_dict() != want[i]]
    return {"files": n, "findings": sum(len(w["Findings"] or []) for w in want.values()),
            "mismatches": len(bad), "first_mismatch": (C.path(bad[0]) if bad else None),
            "reference": "oracle/secret_scanner.py (scanner.go:377-463 restated, pinned by the reference's "
                         "golden tests)"}


PEAK_HBM = 8000.0  # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)
# kernels of one scan's GPU phase: (name, tsg_stats field); they add up to ms_gpu_total (+ buffer clears)
KERNELS = [("chunk_map_kernel", "ms_chunkmap_kernel"), ("filter_kernel (K1)", "ms_scan_kernel"),
           ("confirm_kernel (K2)", "ms_confirm_kernel"), ("fold_kernel", "ms_careful_kernel"),
           ("verify_hits_kernel (follow check + NFA) + fullscan_kernel", "ms_nfa_kernel"),
           ("finalize_kernel", "ms_finalize_kernel"),
           ("xform kernels (c4 GPU pre-transform: lengths, scan, compaction)", "ms_xform_kernel")]

WORKLOADS = {
    # (description, GB per GPU, CPU-baseline sample MB, oracle parity sample MB)
    "c2": ("builtin ruleset (87 rules) over a %g GB synthetic mixed-text corpus per MI355X (BASELINE configs[1])",
           20.0, 1000.0, 24.0),  # CPU baseline: BASELINE configs[0] (C1), 1 GB of the same generator
    "c5": ("%g GB per MI355X per step (1 TB over 8 GPUs) streamed host->HBM from a page-locked pool of "
           "mean-64-KiB files re-emitted with distinct ids, builtin rules (BASELINE configs[4])", 125.0, 64.0, 24.0),
    "c3": ("2,000 generated custom rules (trivy-secret.yaml) + 87 builtins over a %g GB synthetic corpus per "
           "MI355X (BASELINE configs[2])", 8.0, 2.0, 0.4),
    "c3u": ("C3 variant: 2,000 generated custom rules of which ~10 %% have no literal anchor (keyword-gated "
            "full scan) + 87 builtins over a %g GB synthetic corpus per MI355X (BASELINE configs[2], VERDICT r01 #7)",
            8.0, 2.0, 0.4),
    "c3f": ("C3 variant: 2,000 generated custom rules of which ~5 %% are bare class runs ((?i)[a-z0-9/+]{32..48}, "
            "keyword-gated, no literal or rare class run: fullscan_kernel) + 87 builtins over a %g GB synthetic corpus "
            "per MI355X (BASELINE configs[2], VERDICT r02 #6)", 8.0, 2.0, 0.4),
    "c1fs": ("`trivy fs` over a %g GB synthetic source tree on tmpfs (the C1/C2 generator's files and paths): "
             "FS.Walk + Required + reads straight into double-buffered pinned arenas + GPU pre-transform + scan "
             "(BASELINE configs[0] end to end on the GPU; SURVEY §8(f)1)", 1.0, 1000.0, 2.0),
    "c4": ("image layer scan: %g GB of small files (median 1.5 KiB) in a synthetic uncompressed tar layer per "
           "MI355X, native walk + arena packing + scan (BASELINE configs[3])", 12.0, 120.0, 2.0),
}


def write_tree(C, root):
    """The corpus as files under root (tmpfs): its generator paths, contents as generated."""
    import shutil
    if os.path.exists(root):
        shutil.rmtree(root)
    os.makedirs(root)
    made = set()
    for i in range(C.n_files):
        rel = C.path(i)
        d = os.path.dirname(rel)
        if d not in made:
            os.makedirs(os.path.join(root, d), exist_ok=True)
            made.add(d)
        with open(os.path.join(root, rel), "wb") as f:
            f.write(C.arena[int(C.offsets[i]):int(C.offsets[i + 1])])


def _cpuref_prepared(rels, datas, bins, threads):
    """tsg_cpuref_scan (the restated reference CPU scan, C++) over prepared ScanArgs -- paths,
    transformed contents, Binary flags -- once per entry of `threads`; returns (runs, the first
    run's ScanResult)."""
    import ctypes as c
    import numpy as np
    from oracle import hostlib
    import trivy_amd.secret as secret
    from trivy_amd.secret.scanner import ScanResult, _CBatch, _CStats
    offs = np.zeros(len(datas) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in datas])
    arena = np.frombuffer(b"".join(datas) + b"\0" * 64, dtype=np.uint8)
    pb = [r.encode("utf-8", "surrogateescape") for r in rels]
    parr = (c.c_char_p * max(1, len(pb)))(*pb)
    plen = np.array([len(x) for x in pb], dtype=np.uint64)
    barr = np.array(bins, dtype=np.uint8) if bins is not None else None
    L = hostlib.lib()
    sc = secret.NewScanner(None, lib=L, host_only=True)
    batch = _CBatch(len(datas), arena.ctypes.data, offs.ctypes.data, None, None, c.cast(parr, c.c_void_p).value,
                    plen.ctypes.data, barr.ctypes.data if barr is not None else None)
    runs, res = [], None
    for T in threads:
        h = c.c_void_p()
        t0 = time.time()
        if L.tsg_cpuref_scan(c.byref(sc._cg.g), c.byref(batch), int(T), c.byref(h)) != 0:
            raise RuntimeError(hostlib.last_error())
        dt = time.time() - t0
        st = _CStats()
        L.tsg_result_stats(h, c.byref(st))
        runs.append({"threads": int(T), "scan_s": round(dt, 3), "findings": int(st.findings)})
        if res is None:
            res = ScanResult(sc, h)
        else:
            L.tsg_result_free(h)
    return runs, res


def _diff_secrets(got, res, rels):
    """GPU AnalysisResult secrets vs the restated reference's, in AnalysisResult.Sort order."""
    want = [s for s in res.secrets(rels) if s.Findings]
    want.sort(key=lambda s: s.FilePath.encode("utf-8", "surrogateescape"))
    for s_ in want:
        s_.Findings.sort(key=lambda f: (f.RuleID.encode(), f.StartLine))
    got = sorted(got, key=lambda s: s.FilePath.encode("utf-8", "surrogateescape"))
    for s_ in got:
        s_.Findings.sort(key=lambda f: (f.RuleID.encode(), f.StartLine))
    bad = sum(1 for x, y in zip(got, want) if x.to_dict() != y.to_dict()) + abs(len(got) - len(want))
    return {"files": len(rels), "secrets": len(want), "findings": sum(len(s.Findings) for s in want),
            "mismatches": bad}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def oracle_vs_gpu(a, rels, datas, bins, gpu_result, max_bytes):
    """The Python oracle (oracle/secret_scanner.py, pinned by the reference's golden tests) on the
    first files of a prepared analyzer sample vs the GPU's findings for the same files (the
    AnalysisResult of the timed path's analyzer): the line's parity block.  Findings compare as
    their JSON dicts, each file's in (RuleID, StartLine) order (AnalysisResult.Sort)."""
    gpu = {}
    for s_ in gpu_result.Secrets:
        gpu[s_.FilePath] = s_.to_dict()

    def key(f):
        return (f["RuleID"], f["StartLine"])
    n = bad = nf = used = 0
    first = None
    for rel, data, b in zip(rels, datas, bins):
        if n and used + len(data) > max_bytes:
            break
        want = sorted(a.scanner.scan(rel, data, b)["Findings"] or [], key=key)
        got = sorted((gpu.get(rel) or {}).get("Findings") or [], key=key)
        n += 1
        used += len(data)
        nf += len(want)
        if want != got:
            bad += 1
            first = rel if first is None else first
    return {"files": n, "bytes": used, "findings": nf, "mismatches": bad, "first_mismatch": first,
            "reference": "oracle/secret_scanner.py (scanner.go:377-463 restated, pinned by the reference's "
                         "golden tests) on the first files of the CPU-baseline sample, after the restated "
                         "analyzer steps (oracle/analyzer.py)"}


def cpu_baseline_fs(root, cores, gpu_result=None, parity_bytes=0):
    """The same tree through the reference's CPU path, restated: FS.Walk + Required in Python
    (oracle/analyzer.py walk_fs / required, os.scandir order), each file read and CR-stripped,
    then tsg_cpuref_scan (the restated reference CPU scan, C++) on `cores` threads and on 5
    (--parallel's default); end to end GB/s of the files analyzed.  With gpu_result
    (AnalyzeFS's secrets), every file's findings are compared with it."""
    from oracle import analyzer as oan
    t0 = time.time()
    a = oan.SecretAnalyzer("")
    rels, datas, bins, nbytes = [], [], [], 0
    for rel, size in oan.walk_fs(root):
        if not a.required(rel, size):
            continue
        with open(os.path.join(root, rel), "rb") as f:
            b = f.read()
        args = a.prepare(rel, root, b)
        if args is None:
            continue
        rels.append(args[0])
        datas.append(args[1])
        bins.append(args[2])
        nbytes += len(b)
    t_walk = time.time() - t0
    runs, res = _cpuref_prepared(rels, datas, bins, [cores, 5])
    for r in runs:
        r["value"] = round(nbytes / (t_walk + r["scan_s"]) / 1e9, 6)
    out = {"value": runs[0]["value"], "unit": "GB/s", "cores": cores,
           "kind": "port (restated reference CPU path: Python FS.Walk + Required + ReadAll/CR strip, "
                   "C++ tsg_cpuref_scan)",
           "sample": "the whole %.1f MB tree (%d files analyzed): walk+read %.1f s, scan %.1f s on %d threads"
                     % (nbytes / 1e6, len(datas), t_walk, runs[0]["scan_s"], cores),
           "runs": runs, "cpu_model": _cpu_model()}
    if gpu_result is not None:
        out["gpu_vs_cpuref_all_files"] = _diff_secrets(gpu_result.Secrets, res, rels)
        if parity_bytes:
            out["parity"] = oracle_vs_gpu(a, rels, datas, bins, gpu_result, parity_bytes)
    return out


def cpu_baseline_layer_cpp(layer, cores, gpu_result=None, parity_bytes=0):
    """A layer sample through the reference's CPU path, restated: LayerTar.Walk + Required +
    ReadAll / CR strip / ExtractPrintableBytes in Python (oracle/analyzer.py walk_layer_tar,
    tarfile), then tsg_cpuref_scan (C++) on `cores` threads and on 5; GB/s of the files
    analyzed.  With gpu_result (AnalyzeLayer over the same sample), every file compared."""
    from oracle import analyzer as oan
    t0 = time.time()
    files, _, _ = oan.walk_layer_tar(layer.tobytes())
    a = oan.SecretAnalyzer("")
    rels, datas, bins, nbytes = [], [], [], 0
    for fp, size, content in files:
        if not a.required(fp, size):
            continue
        args = a.prepare(fp, "", content)
        if args is None:
            continue
        rels.append(args[0])
        datas.append(args[1])
        bins.append(args[2])
        nbytes += size
    t_walk = time.time() - t0
    runs, res = _cpuref_prepared(rels, datas, bins, [cores, 5])
    for r in runs:
        r["value"] = round(nbytes / (t_walk + r["scan_s"]) / 1e9, 6)
    out = {"value": runs[0]["value"], "unit": "GB/s", "cores": cores,
           "kind": "port (restated reference CPU path: Python LayerTar.Walk + Required + transforms, "
                   "C++ tsg_cpuref_scan)",
           "sample": "a %.1f MB layer of the same generator (%d files analyzed, %.1f MB): walk+read %.1f s, "
                     "scan %.1f s on %d threads" % (layer.size / 1e6, len(datas), nbytes / 1e6, t_walk,
                                                    runs[0]["scan_s"], cores),
           "runs": runs, "cpu_model": _cpu_model()}
    if gpu_result is not None:
        out["gpu_vs_cpuref_all_files"] = _diff_secrets(gpu_result.Secrets, res, rels)
        if parity_bytes:
            out["parity"] = oracle_vs_gpu(a, rels, datas, bins, gpu_result, parity_bytes)
    return out


def _cgroup_cpu():
    """cgroup v2 cpu.stat counters and cpu.max quota of this container, or None."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            st = {k: int(v) for k, v in (ln.split() for ln in f if len(ln.split()) == 2)}
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        st["quota_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
        return st
    except (OSError, ValueError):
        return None


def _thread_cpu():
    """CPU seconds of this process: per live thread name, and the process total
    (threads that exited in between, e.g. the per-scan tsg-scan / tsg-allow
    threads, only show in the total)."""
    tck = os.sysconf("SC_CLK_TCK")
    by = {}
    try:
        for tid in os.listdir("/proc/self/task"):
            try:
                with open("/proc/self/task/%s/stat" % tid) as f:
                    st = f.read()
            except OSError:
                continue
            name = st[st.index("(") + 1:st.rindex(")")]
            fl = st[st.rindex(")") + 2:].split()
            by[name] = by.get(name, 0.0) + (int(fl[11]) + int(fl[12])) / tck
        with open("/proc/self/stat") as f:
            st = f.read()
        fl = st[st.rindex(")") + 2:].split()
        return by, (int(fl[11]) + int(fl[12])) / tck
    except (OSError, ValueError, IndexError):
        return None


def _bind_numa(device):
    """Bind the process to the CPUs of the GPU's NUMA node before the corpus
    and the host pool exist: the host pass reads the arena with cold misses,
    and a remote node adds its latency to each (None where sysfs says nothing)."""
    import torch
    try:
        p = torch.cuda.get_device_properties(device)
        dev = "/sys/bus/pci/devices/%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        with open(dev + "/numa_node") as f:
            node = int(f.read())
        if node < 0:
            return None
        with open("/sys/devices/system/node/node%d/cpulist" % node) as f:
            cpus = set()
            for part in f.read().strip().split(","):
                a, _, b = part.partition("-")
                cpus.update(range(int(a), int(b or a) + 1))
        os.sched_setaffinity(0, cpus & os.sched_getaffinity(0) or cpus)
        return node
    except (OSError, ValueError, AttributeError):
        return None


def _launch_ranks(argv, n):
    """--gpus N (N > 1) without a torchrun environment: start the N rank processes of this same
    command through torch.distributed.run (one rank per GPU, LOCAL_RANK = device) and return
    their exit code.  Runs before anything in this process touches the GPU (a child process,
    never an exec); the ranks print the one JSON line (rank 0)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def _dry_run(args, rank, world):
    """--dry-run (CPU, gloo): the launcher's rank / world plumbing, the barrier-bracketed timing with
    the max over ranks, and the rank-0 findings gather (shard.gather_records) on synthetic records --
    no GPU, no corpus.  Prints the bench's JSON shape with n_gpus = the world that ran."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from trivy_amd import shard
    if world > 1:
        dist.init_process_group("gloo")
    rng = np.random.default_rng(rank)
    dt = 0.0
    for _ in range(args.steps):
        if world > 1:
            dist.barrier()
        t0 = time.time()
        rec = np.zeros(64, dtype=[("file", "<u4"), ("rule", "<u4"), ("start_line", "<i8"), ("end_line", "<i8"),
                                  ("digest", "<u8")])
        rec["file"] = rng.integers(0, 1000, 64)
        rec["rule"] = rng.integers(0, 3, 64)
        rec["start_line"] = rng.integers(1, 100, 64)
        dt += time.time() - t0
    gathered = None
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        paths = np.array([b"r%d/f%04d" % (rank, f) for f in rec["file"]])
        merged = shard.gather_records(rec, paths, ["a", "b", "c"])
        if merged is not None:
            gathered = {"findings": int(len(merged["records"])), "ranks": int(len(set(merged["ranks"].tolist())))}
    if rank == 0:
        if world != args.gpus:
            sys.exit("--gpus %d but %d ranks ran" % (args.gpus, world))
        print(json.dumps({"metric": "dry run (no GPU)", "value": 0.0, "unit": "GB/s", "n_gpus": world,
                          "steps": args.steps, "warmup": 0, "ms_per_step": round(dt / max(1, args.steps) * 1e3, 4),
                          "scaling": "weak", "gather": gathered}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node: one rank per GPU.  Under torchrun (WORLD_SIZE set) it must equal the "
                         "world size; without it, N > 1 starts the N ranks itself (torch.distributed.run)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only (tests): the rank / world plumbing, timing and gather on synthetic records")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 50 for c2: a depth-3 pipeline's fill and drain are then a few %% of the "
                         "timed region, as in a long scan job; 10 for the other workloads)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 3 for c2, 2 otherwise)")
    ap.add_argument("--warmup-s", type=float, default=None,
                    help="then more untimed steps until this many seconds have passed (default: 10 for c2 when "
                         "--warmup is not given, else 0 -- an explicit --warmup is honoured as given): on some "
                         "boxes the kernels ran 5-7 %% slower for the first minute or two of GPU load; the JSON "
                         "reports the warm-up steps actually run and warmup_s")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--gb", type=float, default=None, help="corpus size per GPU (GB = 1e9 B)")
    ap.add_argument("--cpu-sample-mb", type=float, default=None, help="CPU-baseline sample (first files)")
    ap.add_argument("--parity-mb", type=float, default=None, help="oracle parity sample (first files)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--depth", type=int, default=None,
                    help="scans in flight (pipelined submission); default 4, c3f 8 (its exact host pass is the "
                         "bound: 773 / 755 / 670 GB/s at depth 8 / 6 / 4, profiles/r06/c3f/depth/)")
    ap.add_argument("--crlf", type=float, default=0.05,
                    help="c2: share of CRLF files (SURVEY §8(d)); stripped while packing the HBM arena")
    ap.add_argument("--numa", choices=["gpu", "off"], default="gpu",
                    help="gpu: bind this rank's threads (and so its first-touch host memory) to the GPU's NUMA "
                         "node, as numactl --cpunodebind would")
    ap.add_argument("--ingest", action="store_true",
                    help="c2/c3: host-resident corpus (page-locked), H2D inside the timed region")
    ap.add_argument("--ingest-steps", type=int, default=3,
                    help="c2 resident runs: steps of the extra ingest-inclusive leg (0: skip)")
    ap.add_argument("--arena-mb", type=int, default=256, help="c4: collector arena size")
    ap.add_argument("--layers", type=int, default=1,
                    help="c4: the step's bytes as an image of this many layers (sizes 34/26/20/12/8 %% ... of "
                         "--gb), inspected by --layer-parallel concurrent walks into the one engine "
                         "(AnalyzeLayers, image.go:202-235); 1 = one layer (AnalyzeLayer)")
    ap.add_argument("--layer-parallel", type=int, default=3, help="c4 with --layers > 1: concurrent layer walks")
    ap.add_argument("--collectors", type=int, default=None,
                    help="c4/c1fs: collectors filled in turn (collectors - 1 scans in flight during a walk); "
                         "default c4 6, c1fs 3")
    ap.add_argument("--transform", choices=["gpu", "host", "gather"], default="gather",
                    help="c4: gather (default): GPU pre-transform and no arena copy at all -- the GPU gathers each "
                         "batch's files from the layer (page-locked and device-mapped once before timing, as a "
                         "pinned layer-buffer pool would hold it); gpu: the walk copies the bytes as read into the "
                         "pinned arena and the GPU transforms them; host: the walk's threads transform while "
                         "copying")
    ap.add_argument("--pool-gb", type=float, default=64.0, help="c5: page-locked host pool size")
    ap.add_argument("--calib-mb", type=float, default=16.0,
                    help="rule compiler calibration sample: the first MB of the corpus (as a scan job would hand "
                         "the scanner its first batch; tsg_compile_options) -- 0: the static byte prior only")
    ap.add_argument("--traffic-file", default=None,
                    help="PMC traffic summary (default: the newest profiles/traffic_rNN_<workload>.json, c2: traffic_rNN.json)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 50 if args.workload == "c2" else 10
    if args.depth is None:
        args.depth = 8 if args.workload == "c3f" else 4
    if args.collectors is None:  # c4: 6 (39.5-41.8 vs 37.6-38.1 GB/s with 3, profiles/r06/c4)
        args.collectors = 6 if args.workload == "c4" else 3
    if args.warmup_s is None:  # only when the warm-up steps are not given explicitly
        args.warmup_s = 10.0 if args.workload == "c2" and args.warmup is None else 0.0
    if args.warmup is None:
        args.warmup = 3 if args.workload == "c2" else 2
    if args.traffic_file is None:  # the newest PMC pass of this workload (c2: traffic_rNN.json)
        cands = [os.path.join(ROOT, "profiles", "traffic_r%02d%s.json" % (r, "" if args.workload == "c2" else
                                                                            "_" + args.workload)) for r in range(9, 1, -1)]
        args.traffic_file = next((c for c in cands if os.path.exists(c)), cands[-1])
    wl_desc, gb_default, cpu_mb_default, parity_mb_default = WORKLOADS[args.workload]
    if args.parity_mb is None:
        args.parity_mb = parity_mb_default
    if args.gb is None:
        args.gb = gb_default
    if args.cpu_sample_mb is None:
        args.cpu_sample_mb = cpu_mb_default

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:  # N ranks, started before any GPU call
        sys.exit(_launch_ranks(sys.argv[1:], args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return _dry_run(args, rank, world)
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d (one rank per GPU)" % (args.gpus, world))

    import numpy as np
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    # one rank per GPU; on a box with fewer GPUs than ranks (a rehearsal of the N-rank path, e.g.
    # --gpus 2 on one GPU) the ranks share devices round-robin and the line says so
    n_dev = torch.cuda.device_count()  # (does not initialise the GPU)
    shared_devices = 0 < n_dev < world  # the same on every rank of the node
    local = local % n_dev if n_dev > 0 else local
    torch.cuda.set_device(local)
    numa_node = _bind_numa(local) if args.numa == "gpu" else None

    from trivy_amd import corpus, shard
    import trivy_amd.secret as secret

    tmpdir = os.environ.get("TMPDIR", "/tmp")
    cfg_path = None
    t_gen = time.time()
    C = layer = R = None
    r_crlf = r_bytes = 0  # c2: the files as read (CRLF files, bytes)
    layer_list = None  # c4 --layers > 1
    if args.workload in ("c3", "c3u", "c3f"):
        y, samples = corpus.c3_rules(unanchored_share=0.1 if args.workload == "c3u" else 0.0,
                                     fullscan_share=0.05 if args.workload == "c3f" else 0.0)
        cfg_path = os.path.join(tmpdir, "tsg-bench-c3-%d.yaml" % rank)
        with open(cfg_path, "w") as f:
            f.write(y)
        C = corpus.generate_c3(int(args.gb * 1e9), samples, seed=corpus.SEED + rank)
    elif args.workload == "c4":
        if args.layers > 1:  # an image: layers of decreasing size, the same total bytes
            w = [0.34, 0.26, 0.20, 0.12, 0.08] + [0.04] * max(0, args.layers - 5)
            w = w[:args.layers]
            layer_list = [corpus.generate_layer(int(args.gb * 1e9 * x / sum(w)), seed=corpus.SEED + rank + 1000 * k)
                          for k, x in enumerate(w)]
            layer = layer_list[0]  # (the layer-mode flag below)
        else:
            layer = corpus.generate_layer(int(args.gb * 1e9), seed=corpus.SEED + rank)
    elif args.workload == "c1fs":  # a source tree on tmpfs
        base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else tmpdir
        fs_root = os.path.join(base, "tsg-c1fs-%d-%d" % (os.getpid(), rank))
        C0 = corpus.generate(int(args.gb * 1e9), seed=corpus.SEED + rank, crlf_share=args.crlf)  # C1: 5 % CRLF
        write_tree(C0, fs_root)
        del C0
        layer = fs_root  # walked below instead of a tar layer
    elif args.workload == "c5":  # the pool, emitted `emissions` times per step through the ingest path
        pool_gb = min(args.pool_gb, args.gb)
        C = corpus.generate(int(pool_gb * 1e9), seed=corpus.SEED + rank, size_scale=2.6)
        args.ingest = True
    else:
        # C2: 5 % of the files CRLF.  The files as read (R) are CR-stripped while
        # packed into the arena (secret.go:121; the analyzer's packing step, before timing) and the
        # HBM-resident steps scan the stripped arena C; the value counts C's bytes.  The ingest leg
        # streams R itself and strips it on the GPU inside its timed region.
        R = corpus.generate(int(args.gb * 1e9), seed=corpus.SEED + rank, crlf_share=args.crlf)
        C = R.stripped() if args.crlf > 0 else R
        r_crlf, r_bytes = int(R.crlf.sum()), int(R.n_bytes)
        # R feeds only the ingest leg (single-process C2 runs): otherwise free it -- under torchrun
        # each rank would hold its corpus twice (2 x 20 GB of host memory per GPU)
        if args.crlf <= 0 or world > 1 or args.ingest or args.ingest_steps <= 0:
            R = None
    t_gen = time.time() - t_gen
    kinds_raw = np.ones(R.n_files, dtype=np.uint8) if R is not None else None  # every text file: CR strip

    h2d_peak = None
    host_leg = [False]  # the ingest leg of a resident run: submit() streams the host arena
    emissions = 1
    layer_unreg = []  # c4 --transform gather: the mapped layers' unregister calls
    if layer is None:
        dev = torch.device("cuda", local)
        if args.ingest:
            # host-resident corpus in a page-locked pool (the caller's pinned arena pool): every
            # step streams it through the engine's staging ring (RunHost)
            unregister = secret.HostRegister(C.arena)
            h2d_peak = measure_h2d(dev)
            d_arena = d_offs = d_paths = d_poffs = None
        else:
            d_arena = torch.from_numpy(C.arena).to(dev)
            d_offs = torch.from_numpy(C.offsets.view(np.int64)).to(dev)
            # the paths are input too: packed in HBM beside the contents (GPU allow-path prefilter)
            pp, poffs = C.packed_paths()
            d_paths = torch.from_numpy(pp).to(dev)
            d_poffs = torch.from_numpy(poffs.view(np.int64)).to(dev)
        torch.cuda.synchronize()
        t_c = time.time()
        calib = C.arena[:min(C.n_bytes, int(args.calib_mb * 1e6))] if args.calib_mb > 0 else None
        sc = secret.NewScanner(secret.ParseConfig(cfg_path) if cfg_path else None, device=local, calibration=calib)
        t_compile = time.time() - t_c

        def submit():
            if host_leg[0] and R is not None:  # the files as read; the GPU strips the CRs
                return sc.scan_arena_async(R.arena, R.offsets, R.path_ptrs, transform=kinds_raw)
            if args.ingest or host_leg[0]:
                return sc.scan_arena_async(C.arena, C.offsets, C.path_ptrs)
            return sc.scan_arena_async(C.arena, C.offsets, C.path_ptrs, dev_arena=d_arena.data_ptr(),
                                       dev_offsets=d_offs.data_ptr(), dev_paths=d_paths.data_ptr(),
                                       dev_path_offsets=d_poffs.data_ptr())

        emissions = max(1, int(round(args.gb * 1e9 / C.n_bytes))) if args.workload == "c5" else 1

        def run_steps(n, stats):
            # pipelined: step i+1's kernels run while step i's exact host pass finishes
            # (tsg_scan_submit; --depth 1 runs the steps back to back)
            inflight = []
            r = None
            for _ in range(n * emissions):  # c5: the pool once per emission (distinct ids: emission, file)
                inflight.append(submit())
                if len(inflight) >= args.depth:
                    r = inflight.pop(0).wait()
                    stats.append(r.stats())
            while inflight:
                r = inflight.pop(0).wait()
                stats.append(r.stats())
            last_res[0] = r
    else:
        from trivy_amd.analyzer import AnalyzerOptions, SecretAnalyzer
        from trivy_amd.analyzer.secret import Collector
        t_c = time.time()
        an = SecretAnalyzer(device=local)
        an.Init(AnalyzerOptions())
        t_compile = time.time() - t_c
        gx = args.transform in ("gpu", "gather")
        gth = args.transform == "gather" and args.workload == "c4"  # (tar layers only)
        colls = [Collector(an, args.arena_mb << 20, gx, gather=gth) for _ in range(args.collectors)]
        lworkers = an.LayerWorkers(args.layer_parallel, args.arena_mb << 20, args.collectors, gx, gth) \
            if layer_list is not None else None
        if gth and args.workload == "c4":  # the layer-buffer pool: registered once, outside the timed region
            t_r = time.time()
            layer_unreg = [secret.HostRegister(x, mapped=True) for x in (layer_list or [layer])]
            register_s = time.time() - t_r

        def run_steps(n, stats):
            for _ in range(n):
                st = {}
                if args.workload == "c1fs":
                    an.AnalyzeFS(layer, stats=st, materialize=False, colls=colls)
                elif layer_list is not None:  # the image's layers, --layer-parallel walks at once
                    per = []
                    t_l = time.time()
                    an.AnalyzeLayers(layer_list, materialize=False, stats=per, workers=lworkers, registered=gth)
                    for d in per:  # summed over the layers (walk_s / wait_s: summed over the workers)
                        for k2, v in d.items():
                            st[k2] = st.get(k2, 0) + v
                    st["layers_s"] = time.time() - t_l
                else:
                    an.AnalyzeLayer(layer, stats=st, materialize=False, colls=colls, registered=gth)
                stats.append(st)

    last_res = [None]  # the last step's ScanResult (findings checked against the oracle below)
    warm = []
    tw0 = time.time()
    run_steps(args.warmup, warm)
    while time.time() - tw0 < args.warmup_s:  # keep the GPU loaded until its clocks have settled
        run_steps(10, warm)
        args.warmup += 10
    warm_s = time.time() - tw0

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    cg0 = _cgroup_cpu()
    tc0 = _thread_cpu()
    t0 = time.time()
    stats = []
    run_steps(args.steps, stats)
    gathered = None
    if dist is not None and layer is None:
        # host-side findings gather (north_star): the job's result -- every rank's
        # findings of its shard -- merged on rank 0 in AnalysisResult.Sort order, inside the timed region
        tg = time.time()
        rec = last_res[0].records()
        pth = C.path_buf.reshape(-1, corpus.PATH_STRIDE)[rec["file"] % C.n_files].view("S%d" % corpus.PATH_STRIDE).ravel()
        merged = shard.gather_records(rec, pth, [r.ID for r in sc.Rules])
        if merged is not None:
            gathered = {"findings": int(len(merged["records"])), "ranks": world,
                        "files": int(len(np.unique(merged["paths"]))), "ms": round((time.time() - tg) * 1e3, 2),
                        "note": "once per job (the steps re-scan the same shards): tsg_result_records of every rank "
                                "gathered to rank 0 (gloo) and put in AnalysisResult.Sort order"}
    torch.cuda.synchronize()
    barrier()
    dt = time.time() - t0
    cg1 = _cgroup_cpu()
    tc1 = _thread_cpu()
    host_cpu = None
    if cg0 and cg1:  # the container's CPU use over the timed steps (quota throttling shows here)
        host_cpu = {"cpus_used": round((cg1["usage_usec"] - cg0["usage_usec"]) / (dt * 1e6), 2),
                    "throttled_ms": round((cg1.get("throttled_usec", 0) - cg0.get("throttled_usec", 0)) / 1e3, 1),
                    "quota_cpus": cg1.get("quota_cpus")}
    if tc0 and tc1:  # CPU-ms per step of this process, by thread name (the rest: threads that exited)
        host_cpu = host_cpu or {}
        per = {k: round((v - tc0[0].get(k, 0.0)) * 1e3 / args.steps, 2) for k, v in tc1[0].items()}
        per = {k: v for k, v in sorted(per.items(), key=lambda kv: -kv[1]) if v >= 0.05}
        total = round((tc1[1] - tc0[1]) * 1e3 / args.steps, 2)
        per["(exited threads)"] = round(total - sum(per.values()), 2)
        host_cpu["process_cpu_ms_per_step"] = total
        host_cpu["by_thread_ms_per_step"] = per
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    ms_step = dt / args.steps * 1e3
    last = stats[-1]

    # Ingest-inclusive leg of a resident c2 run (value stays the HBM-resident rate): the same corpus
    # page-locked on the host, every byte copied host->HBM inside the timed region through the
    # engine's staging ring and copy stream (tsg_scan_submit without a device arena).
    ingest = None
    unregister_leg = None
    res_timed = last_res[0]  # the timed steps' last result (parity below)
    # (single-process runs only: under torchrun every rank would page-lock its whole corpus)
    if layer is None and args.workload == "c2" and not args.ingest and args.ingest_steps > 0 and world == 1:
        del d_arena, d_offs
        torch.cuda.empty_cache()
        unregister_leg = secret.HostRegister(C.arena if R is None else R.arena)
        peak = measure_h2d(dev)
        peak_src = measure_h2d_from(C.arena if R is None else R.arena, local)
        host_leg[0] = True
        ist = []
        run_steps(1, ist)
        barrier()
        torch.cuda.synchronize()
        ti = time.time()
        ist = []
        run_steps(args.ingest_steps, ist)
        torch.cuda.synchronize()
        barrier()
        dti = time.time() - ti
        if dist is not None:
            t = torch.tensor([dti], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dti = float(t.item())
        leg_bytes = C.n_bytes if R is None else R.n_bytes
        h2d = leg_bytes * args.ingest_steps / dti / 1e9  # per GPU
        ingest = {"value": round(world * leg_bytes * args.ingest_steps / dti / 1e9, 3), "unit": "GB/s",
                  "steps": args.ingest_steps, "ms_per_step": round(dti / args.ingest_steps * 1e3, 3),
                  "achieved_h2d": round(h2d, 2), "h2d_peak_measured": peak, "frac_h2d": round(h2d / peak, 4),
                  "h2d_from_source_measured": peak_src,
                  "frac_h2d_source": round(h2d / peak_src, 4) if peak_src else None,
                  "h2d_chunks_per_scan": int(ist[-1].get("h2d_chunks", 0)),
                  "note": "same corpus and scanner, host-resident (page-locked) arena: H2D of every byte inside "
                          "the timed region, overlapped with the kernels (the engine's staging ring: one copier thread, "
                          "four staging buffers, copy stream)"
                          + ("; the files as read (%d CRLF), CR-stripped on the GPU (xform.hip) inside the timed "
                             "region" % int(R.crlf.sum()) if R is not None else "")}
    pre = "" if layer is None else "scan_"

    def avg(k):  # per-scan mean over the timed steps (c4 sums its batches per step)
        return sum(s[pre + k] for s in stats) / len(stats)
    kernels = {name: avg(k) for name, k in KERNELS}
    gpu_ms = avg("ms_gpu_total")
    scan_ms = kernels["filter_kernel (K1)"]
    breakdown = {k: round(avg(k), 3) for _, k in KERNELS}
    breakdown.update({k: round(avg(k), 3) for k in ("ms_fullscan_kernel", "ms_gpu_total", "ms_host_gpu_phase",
                                                     "ms_host_exact")})
    if layer is None:
        # per step: the arena bytes the timed steps scan.  (C2's files as read are 0.07 % larger --
        # the 5 % CRLF files' '\r' -- but the resident leg strips them while packing, before timing:
        # they are not counted; the ingest leg strips inside its timed region and counts them.)
        n_bytes, n_files = C.n_bytes * emissions, C.n_files * emissions
        arena_bytes = C.n_bytes  # per scan
        counts = {k: int(last[k]) for k in ("flagged_blocks", "anchor_hits", "follow_hits", "fullscan_pairs", "fold_sites",
                                            "candidates", "special_files", "findings")}
        # plain names: anchor_hits counts K2's exact anchor-item matches, follow_hits the hits
        # past the follow requirements that K2 emits to the verify kernel's NFA
        counts["anchor_item_matches"] = counts["anchor_hits"]
        counts["hits_to_verify"] = counts["follow_hits"]
        breakdown.update({k: round(avg(k), 3) for k in ("ms_host_allow_path", "ms_host_total")})
        # the pipeline's drain: the last scan's host work after its GPU phase (nothing overlaps it),
        # and the timed region beyond the steps' GPU time (fill, drain, gaps between scans)
        breakdown["ms_last_scan_after_gpu"] = round(last["ms_host_total"] - last["ms_host_gpu_phase"], 3)
        breakdown["ms_timed_minus_gpu"] = round(dt * 1e3 - args.steps * emissions * gpu_ms, 3)
        config_extra = {"bytes_per_gpu": n_bytes, "files_per_gpu": n_files, "pipeline_depth": args.depth,
                        "calibration_sample_bytes": int(calib.size) if calib is not None else 0,
                        "crlf_files": r_crlf,
                        "arena_bytes_after_cr_strip": C.n_bytes,
                        "input_bytes_as_read": r_bytes or C.n_bytes,
                        "value_numerator": "arena bytes (after the CR strip done while packing, before timing)",
                        "emissions_per_step": emissions, "pool_bytes": C.n_bytes,
                        "resident": "host (page-locked), H2D in the timed region" if args.ingest
                        else "HBM (copied once before timing)"}
    else:
        n_bytes = int(last["input_bytes"])  # bytes of the files analyzed, as read from the layer
        n_files = int(last["added"])
        arena_bytes = int(last["scan_bytes"])
        fs_wl = args.workload == "c1fs"
        keys = ("walked", "required", "added", "skipped_binary", "files", "dirs", "skipped_dirs", "nonregular") \
            if fs_wl else ("entries", "regular", "required", "added", "skipped_binary", "whiteouts")
        counts = {k: int(last[k]) for k in keys}
        counts.update({k: int(last["scan_" + k]) for k in ("candidates", "findings", "anchor_hits",
                                                            "follow_hits")})
        config_extra = {"walk_s_per_step": round(last["walk_s"], 3), "wait_s_per_step": round(last["wait_s"], 3),
                        "file_bytes_analyzed_per_gpu": n_bytes,
                        "arena_bytes_per_gpu": arena_bytes, "files_analyzed_per_gpu": n_files,
                        "arena_mb": args.arena_mb, "pipeline": "%d collectors (walk k+1 || scans k-%d..k)" % (args.collectors, args.collectors - 2),
                        "pre_transform": args.transform}
        if args.transform == "gather" and not fs_wl:
            config_extra["layer_register_s"] = round(register_s, 3)
            config_extra["gather_note"] = ("batches point into the layer (tsg_batch_ext v2 gather_base/gather_src); "
                                           "the GPU reads the files over PCIe from the mapped layer; the layer's "
                                           "one-time page-lock + map (layer_register_s) is outside the timed region")
        if fs_wl:
            config_extra["tree"] = "tmpfs (%s)" % os.path.dirname(layer)
        else:
            lsz = sum(int(x.size) for x in layer_list) if layer_list is not None else int(layer.size)
            config_extra["layer_bytes_per_gpu"] = lsz
            config_extra["layer_gbps"] = round(world * lsz * args.steps / dt / 1e9, 3)
            if layer_list is not None:
                config_extra["layers"] = [int(x.size) for x in layer_list]
                config_extra["layer_parallel"] = args.layer_parallel
                config_extra["pipeline"] = ("%d concurrent layer walks (AnalyzeLayers, image.go:202-235), each %s"
                                            % (args.layer_parallel, config_extra["pipeline"]))
                config_extra["walk_s_note"] = "walk_s / wait_s summed over the concurrent layer walks"
    value = world * n_bytes * args.steps / dt / 1e9
    alg_bytes = arena_bytes + 16 * (n_files // emissions)  # 1 B/arena byte + 16 B/file, per scan
    phase = alg_bytes / (gpu_ms * 1e-3) / 1e9  # §8(d): (arena + 16 n_files) / (t_prefilter + t_nfa)
    k1 = alg_bytes / (scan_ms * 1e-3) / 1e9
    dom = max(kernels, key=kernels.get)
    traffic = traffic_k1 = None
    if os.path.exists(args.traffic_file):
        try:
            tj = json.load(open(args.traffic_file))
            if tj.get("workload") == args.workload and abs(tj.get("gb", -1) - args.gb) < 1e-6:
                traffic = tj.get("phase_bytes_per_scan")
                traffic_k1 = tj.get("k1_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm",
                "kernel": "GPU phase per scan: %s (SURVEY.md §8(d) formula)" % " + ".join(kernels),
                "achieved": round(phase, 2), "peak": PEAK_HBM, "unit": "GB/s", "frac": round(phase / PEAK_HBM, 4),
                "traffic": traffic, "algorithmic_bytes": alg_bytes,
                "dominant_kernel": {"name": dom, "ms": round(kernels[dom], 3),
                                    "share": round(kernels[dom] / gpu_ms, 3) if gpu_ms else None},
                "k1": {"kernel": "filter_kernel (K1, streams every arena byte)", "achieved": round(k1, 2),
                       "frac": round(k1 / PEAK_HBM, 4), "traffic": traffic_k1},
                "traffic_source": os.path.relpath(args.traffic_file, ROOT) if traffic else None}
    if ingest is not None:
        roofline["achieved_h2d"] = ingest["achieved_h2d"]
        roofline["h2d_peak_measured"] = ingest["h2d_peak_measured"]
        roofline["frac_h2d"] = ingest["frac_h2d"]
        roofline["h2d_note"] = "per GPU, from the ingest leg (see \"ingest\")"
    if h2d_peak:
        h2d = n_bytes * args.steps / dt / 1e9  # per GPU: every byte of the step (all emissions) crossed PCIe
        roofline["achieved_h2d"] = round(h2d, 2)
        roofline["h2d_peak_measured"] = h2d_peak
        roofline["frac_h2d"] = round(h2d / h2d_peak, 4)
        roofline["h2d_note"] = ("per GPU: arena bytes / step time with every byte copied host->HBM in the timed region "
                                "(%d chunks per scan through the staging ring); peak = pinned hipMemcpyAsync on this box"
                                % int(last.get("h2d_chunks", 0)))

    if rank == 0:
        cpu = None
        parity = None
        if world == 1 and not args.no_cpu_baseline:
            cores = min(16, os.cpu_count() or 1)
            if layer is None:
                want, _ = oracle_sample(C, int(args.parity_mb * 1e6), cores, tmpdir, cfg_path)
                parity = parity_block(C, res_timed, want)
                if ingest is not None:
                    ingest["parity"] = parity_block(C, last_res[0], want)
                cpu = cpu_baseline(C, int(args.cpu_sample_mb * 1e6), [cores, 5], cfg_path, want,
                                   gpu_res=res_timed)
            elif args.workload == "c1fs":
                from trivy_amd.walker import Option
                res_fs = an.AnalyzeFS(layer, Option(), colls=colls)  # findings of the same walk, materialized
                cpu = cpu_baseline_fs(layer, cores, gpu_result=res_fs, parity_bytes=int(args.parity_mb * 1e6))
                parity = cpu.pop("parity", None)
            else:
                sample = corpus.generate_layer(int(args.cpu_sample_mb * 1e6), seed=corpus.SEED + rank)
                # (the same ingest mode as the timed steps: with --transform gather the sample's
                # batches are gathered from it, AnalyzeLayer page-locks and maps it for the call)
                res_l = an.AnalyzeLayer(sample, colls=[Collector(an, args.arena_mb << 20, gx, gather=gth)
                                                       for _ in range(args.collectors)])
                cpu = cpu_baseline_layer_cpp(sample, cores, gpu_result=res_l, parity_bytes=int(args.parity_mb * 1e6))
                parity = cpu.pop("parity", None)
        out = {
            "metric": "GB/s secret-scanned (whole node) at 1/2/4/8 MI355X; findings bit-exact vs CPU",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_s": round(warm_s, 2),
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic generator, seed 0x5EC2E7+rank; planted builtin-rule secrets%s)"
                    % (" and generated-rule samples" if args.workload in ("c3", "c3u", "c3f") else ""),
            "config": dict({"workload": wl_desc % args.gb, "workload_id": args.workload,
                            "parallelism": "files sharded, dp%d" % world,
                            "rules_compile_s": round(t_compile, 2),
                            "host_numa_node": numa_node}, **config_extra,
                           **({"devices_shared": "%d ranks on %d GPU(s), round-robin: a rehearsal of the "
                                                 "N-rank path, not a scaling number" % (world, n_dev)}
                              if shared_devices else {})),
            "roofline": roofline,
            "ingest": ingest,
            "cpu_baseline": cpu,
            "parity": parity,
            "gather": gathered,
            "legs": ("N=1: resident steps, ingest leg (c2), oracle parity sample, CPU baseline" if world == 1 else
                     "N>1: resident steps and the rank-0 findings gather only; the ingest leg, the parity sample "
                     "and the CPU baseline run at N=1 (every rank would page-lock its corpus / rerun the CPU "
                     "reference)"),
            "breakdown_ms": breakdown,
            "host_cpu": host_cpu,
            "counts": counts,
            "gen_s": round(t_gen, 2),
        }
        print(json.dumps(out), flush=True)
        if ingest is not None and "parity" in ingest and ingest["parity"]["mismatches"]:
            sys.exit("parity (ingest leg): %d of %d sample files differ from the oracle (first: %s)"
                     % (ingest["parity"]["mismatches"], ingest["parity"]["files"], ingest["parity"]["first_mismatch"]))
        full = (cpu or {}).get("gpu_vs_cpuref_all_files")
        if full and full["mismatches"]:
            sys.exit("parity: %d of %d files of the CPU-baseline sample differ from the restated reference "
                     "(first: %s)" % (full["mismatches"], full["files"], full.get("first_mismatch")))
        if parity is not None and parity["mismatches"]:
            sys.exit("parity: %d of %d sample files differ from the oracle (first: %s)"
                     % (parity["mismatches"], parity["files"], parity["first_mismatch"]))
    if args.workload == "c1fs":
        import shutil
        shutil.rmtree(layer, ignore_errors=True)
    if cfg_path:
        os.remove(cfg_path)
    if h2d_peak:
        unregister()
    if unregister_leg is not None:
        unregister_leg()
    for u in layer_unreg:
        u()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
