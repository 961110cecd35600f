"""GPU parity on the bench's own corpus generator (trivy_amd/csrc/corpus.cpp).

The bench (BASELINE configs[1]/[2]) scans corpora made by the C++ generator:
log-normal file sizes up to 10 MiB, 0.1 % minified lines over 10 KiB, 2 %
UTF-8 files with fold runes and invalid bytes, planted secrets.  These tests
scan a whole generated arena through the C-ABI (the same call the bench
times) and compare every selected file -- the multi-MiB ones, files holding a
> 10 KiB line, fold-rune files and a random sample -- field for field with
the oracle (pkg/fanal/secret/scanner.go:377-463 restated).  The oracle runs
in a process pool (it is pure Python).
"""
import multiprocessing as mp
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

POOL = min(16, os.cpu_count() or 1)


def _oracle_worker(args):
    items, cfg_path = args
    from oracle import secret_scanner as osc
    sc = osc.new_scanner(osc.parse_config(cfg_path) if cfg_path else None)
    return [(i, sc.scan(p, b)) for i, p, b in items]


def _oracle(items, cfg_path=None):
    """items: [(index, path, content)] -> {index: oracle result}, largest files spread first."""
    items = sorted(items, key=lambda t: -len(t[2]))
    shards = [items[k::POOL] for k in range(POOL)]
    ctx = mp.get_context("spawn")
    with ctx.Pool(POOL) as pool:
        out = {}
        for part in pool.map(_oracle_worker, [(s, cfg_path) for s in shards if s]):
            out.update(part)
    return out


def _select(C, rng, sample_bytes):
    sizes = np.diff(C.offsets.astype(np.int64))
    big = [int(i) for i in np.nonzero(sizes >= (1 << 20))[0]]
    chosen = set(big)
    long_line, fold = [], []
    for i in range(C.n_files):
        if len(long_line) >= 6 and len(fold) >= 12:
            break
        if sizes[i] > (1 << 20) or sizes[i] < 12 << 10:
            continue
        b = C.content(i)
        if len(long_line) < 6 and max(len(x) for x in b.split(b"\n")) > 10240:
            long_line.append(i)
        elif len(fold) < 12 and (b"\xe2\x84\xaa" in b or b"\xc5\xbf" in b or b"\xc4\xb0" in b):
            fold.append(i)
    chosen.update(long_line + fold)
    order = list(range(C.n_files))
    rng.shuffle(order)
    tot = 0
    for i in order:
        if tot >= sample_bytes:
            break
        if sizes[i] < (1 << 20):
            chosen.add(i)
            tot += int(sizes[i])
    return sorted(chosen), big, long_line, fold


def _check(C, res, chosen, want):
    from trivy_amd.secret.scanner import Secret  # noqa: F401
    n_find = 0
    for i in chosen:
        got = res.secrets([C.path(i)], lo=i)[0].to_dict()
        assert got == want[i], (i, C.path(i))
        n_find += len(want[i]["Findings"] or [])
    return n_find


def test_bench_corpus_c2_matches_oracle():
    """the Python oracle's own sample on the GPU side holds >= 500 findings
    (planted secrets 16x denser than the bench's corpus; 177 files, ~10 MB: the multi-MiB files,
    > 10 KiB lines, fold-rune files and a random 3 MB)."""
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    C = corpus.generate(int(160e6), seed=corpus.SEED + 7, secrets_per_byte=1.0 / 16384)
    chosen, big, long_line, fold = _select(C, random.Random(3), 3e6)
    assert len(big) >= 2 and long_line and fold, (len(big), len(long_line), len(fold))
    s = secret.NewScanner(None)
    res = s.scan_arena(C.arena, C.offsets, C.path_ptrs)
    want = _oracle([(i, C.path(i), C.content(i)) for i in chosen])
    n = _check(C, res, chosen, want)
    assert n >= 500, n


def test_bench_corpus_c3_matches_oracle(tmp_path):
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    y, samples = corpus.c3_rules()
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(y)
    C = corpus.generate_c3(int(24e6), samples, seed=corpus.SEED + 11, secrets_per_byte=1.0 / 16384)
    rng = random.Random(4)
    sizes = np.diff(C.offsets.astype(np.int64))
    small = [i for i in range(C.n_files) if sizes[i] < 200000]
    chosen = sorted(rng.sample(small, 160))
    s = secret.NewScanner(secret.ParseConfig(str(cfg)))
    res = s.scan_arena(C.arena, C.offsets, C.path_ptrs)
    want = _oracle([(i, C.path(i), C.content(i)) for i in chosen], str(cfg))
    n = _check(C, res, chosen, want)
    assert n > 20


def _cpuref(C, n_threads=16, cfg_path=None):
    """tsg_cpuref_scan (oracle/native/host_hooks.cpp, the restated reference CPU algorithm) over
    every file of C: the full-size completeness check (the Python oracle checks samples)."""
    import ctypes as c
    from oracle import hostlib
    import trivy_amd.secret as secret
    from trivy_amd.secret.scanner import ScanResult, _CBatch
    L = hostlib.lib()
    sc = secret.NewScanner(secret.ParseConfig(cfg_path) if cfg_path else None, lib=L, host_only=True)
    offs = np.ascontiguousarray(C.offsets)
    batch = _CBatch(C.n_files, C.arena.ctypes.data, offs.ctypes.data, None, None, C.path_ptrs.ctypes.data,
                    None, None)
    h = c.c_void_p()
    assert L.tsg_cpuref_scan(c.byref(sc._cg.g), c.byref(batch), n_threads, c.byref(h)) == 0
    return ScanResult(sc, h)


def test_c5_pool_streamed_twice_matches_oracle(monkeypatch):
    """BASELINE configs[4] (C5): a page-locked pool of mean-64-KiB files (size_scale 2.6) streamed
    host->HBM through the double-buffered ingest (RunHost, 16-MiB chunks) twice in flight, as the
    C5 bench re-emits it.  Both emissions: every file byte-identical to the restated reference
    CPU scan, and a sample field for field vs the oracle."""
    from bench import full_diff
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    monkeypatch.setenv("TSG_INGEST_CHUNK_MB", "16")
    C = corpus.generate(int(72e6), seed=corpus.SEED + 5, size_scale=2.6)
    assert C.n_bytes / C.n_files > 40e3
    unreg = secret.HostRegister(C.arena)
    try:
        s = secret.NewScanner(None)
        p1 = s.scan_arena_async(C.arena, C.offsets, C.path_ptrs)
        p2 = s.scan_arena_async(C.arena, C.offsets, C.path_ptrs)
        r1, r2 = p1.wait(), p2.wait()
    finally:
        unreg()
    assert r1.stats()["h2d_chunks"] >= 4
    ref = _cpuref(C)
    for r in (r1, r2):
        bad, first = full_diff(r, ref, C.n_files)
        assert bad == 0, (bad, C.path(first))
    chosen, big, _, _ = _select(C, random.Random(5), 2e6)
    want = _oracle([(i, C.path(i), C.content(i)) for i in chosen])
    assert _check(C, r2, chosen, want) > 5


def test_c2_corpus_every_file_matches_cpuref():
    """Candidate completeness at size: every file of a 256 MB C2 corpus (K1 -> K2 -> verify
    superset, exact host pass) byte-identical to the restated reference CPU scan."""
    from bench import full_diff
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    C = corpus.generate(int(256e6), seed=corpus.SEED + 13)
    res = secret.NewScanner(None).scan_arena(C.arena, C.offsets, C.path_ptrs)
    ref = _cpuref(C)
    bad, first = full_diff(res, ref, C.n_files)
    assert bad == 0, (bad, C.path(first) if first is not None else None)
    assert res.stats()["findings"] > 500


def test_c3f_fullscan_rules_every_file_matches_cpuref(tmp_path):
    """C3f: 2,000 generated rules of which ~5 % are bare, keyword-gated
    class runs ((?i)[a-z0-9/+]{32..48}) with neither a literal nor a rare class run, so every file
    holding a rule's keyword goes through fullscan_kernel.  Every file vs the restated reference
    CPU scan, a sample vs the oracle; the full-scan path must actually run."""
    from bench import full_diff
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    y, samples = corpus.c3_rules(fullscan_share=0.05)
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(y)
    C = corpus.generate_c3(int(48e6), samples, seed=corpus.SEED + 17, secrets_per_byte=1.0 / 16384)
    s = secret.NewScanner(secret.ParseConfig(str(cfg)))
    res = s.scan_arena(C.arena, C.offsets, C.path_ptrs)
    st = res.stats()
    assert st["fullscan_pairs"] > 0
    ref = _cpuref(C, cfg_path=str(cfg))
    bad, first = full_diff(res, ref, C.n_files)
    assert bad == 0, (bad, C.path(first) if first is not None else None)
    rng = random.Random(6)
    sizes = np.diff(C.offsets.astype(np.int64))
    withkw = [i for i in range(C.n_files) if sizes[i] < 400000 and b"kwf" in C.content(i)]
    small = [i for i in range(C.n_files) if sizes[i] < 200000]
    chosen = sorted(set(withkw[:40]) | set(rng.sample(small, 60)))
    want = _oracle([(i, C.path(i), C.content(i)) for i in chosen], str(cfg))
    assert _check(C, res, chosen, want) > 10


_VARIANT_CASE = {}


@pytest.mark.parametrize("env", [
    {},                                          # items + classes in LDS, 16-wave workgroups, first-byte test
    {"TSG_FOLD_WAVES": "4"},                      # the same staging in 4-wave workgroups
    {"TSG_FOLD_STAGE": "0"},                      # global tables, 4-wave workgroups
    {"TSG_FOLD_STAGE": "0", "TSG_FOLD_FIRST": "0"},  # ... without the first-byte test
    {"TSG_CONFIRM_STAGE_CLASSES": "0"},            # confirm kernel with its classes in global memory
], ids=["default", "waves4", "unstaged", "unstaged-nofirst", "confirm-global-classes"])
def test_c3_global_table_kernel_variants_match_cpuref(tmp_path, monkeypatch, env):
    """The global-table (2,087-rule) fold and confirm kernels in each selectable shape (engine.hip
    fold_kernel / confirm_kernel): every file of a C3 corpus holding fold
    runes byte-identical to the restated reference CPU scan, with the fold sites actually tried."""
    from bench import full_diff
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    for k in ("TSG_FOLD_WAVES", "TSG_FOLD_STAGE", "TSG_FOLD_FIRST", "TSG_CONFIRM_STAGE_CLASSES"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if "c3" not in _VARIANT_CASE:  # one corpus and one reference scan for every variant
        y, samples = corpus.c3_rules()
        cfg = tmp_path / "trivy-secret.yaml"
        cfg.write_text(y)
        C = corpus.generate_c3(int(32e6), samples, seed=corpus.SEED + 19, secrets_per_byte=1.0 / 16384)
        _VARIANT_CASE["c3"] = (C, str(cfg), _cpuref(C, cfg_path=str(cfg)))
    C, cfg, ref = _VARIANT_CASE["c3"]
    res = secret.NewScanner(secret.ParseConfig(cfg)).scan_arena(C.arena, C.offsets, C.path_ptrs)
    st = res.stats()
    assert st["fold_sites"] > 50, st["fold_sites"]
    bad, first = full_diff(res, ref, C.n_files)
    assert bad == 0, (bad, C.path(first) if first is not None else None)
    assert st["findings"] > 100


def _resident(s, C):
    """C's arena and offsets copied to HBM, scanned from there (the bench's resident path: the GPU
    finding materialisation, materialize.hip, needs the arena in HBM)."""
    import torch
    d_arena = torch.from_numpy(np.ascontiguousarray(C.arena)).to("cuda:0")
    d_offs = torch.from_numpy(np.ascontiguousarray(C.offsets).view(np.int64)).to("cuda:0")
    res = s.scan_arena(C.arena, C.offsets, C.path_ptrs, dev_arena=d_arena.data_ptr(), dev_offsets=d_offs.data_ptr())
    torch.cuda.synchronize()
    return res


def test_c2_corpus_resident_gpu_findings_calibrated_every_file():
    """The bench's exact configuration at 256 MB: a scanner compiled with a calibration sample (the
    corpus head; a rule compiler anchor choice: linear-client-secret on its class run), the arena in
    HBM, findings made on the GPU (materialize.hip) -- every file byte-identical to the restated
    reference CPU scan."""
    from bench import full_diff
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    C = corpus.generate(int(256e6), seed=corpus.SEED + 23)
    s = secret.NewScanner(None, calibration=C.arena[:16000000])
    assert any("(calibrated)" in s.rule_anchor(i) for i in range(len(s.Rules)))
    s.set_gpu_findings(True)
    res = _resident(s, C)
    ref = _cpuref(C)
    bad, first = full_diff(res, ref, C.n_files)
    assert bad == 0, (bad, C.path(first) if first is not None else None)
    assert res.stats()["findings"] > 500


def test_c3f_resident_gpu_findings_every_file(tmp_path):
    """C3f (finding-dense: the materialisation's target) resident in HBM with GPU findings: every
    file vs the restated reference CPU scan, a sample vs the oracle."""
    from bench import full_diff
    from trivy_amd import corpus
    import trivy_amd.secret as secret
    y, samples = corpus.c3_rules(fullscan_share=0.05)
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(y)
    C = corpus.generate_c3(int(48e6), samples, seed=corpus.SEED + 29, secrets_per_byte=1.0 / 16384)
    s = secret.NewScanner(secret.ParseConfig(str(cfg)), calibration=C.arena[:4000000])
    s.set_gpu_findings(True)
    res = _resident(s, C)
    ref = _cpuref(C, cfg_path=str(cfg))
    bad, first = full_diff(res, ref, C.n_files)
    assert bad == 0, (bad, C.path(first) if first is not None else None)
    assert res.stats()["findings"] > 10000
    rng = random.Random(8)
    sizes = np.diff(C.offsets.astype(np.int64))
    small = [i for i in range(C.n_files) if sizes[i] < 200000]
    chosen = sorted(rng.sample(small, 60))
    want = _oracle([(i, C.path(i), C.content(i)) for i in chosen], str(cfg))
    assert _check(C, res, chosen, want) > 10
