"""N>1 path: files shard across ranks, no data-path collective,
findings gathered to rank 0 in the reference's order.

CPU-only: world_size-2 gloo process group (127.0.0.1); each rank scans its LPT
shard through the native exact host tail (tsg_debug_host_tail, the same C++ tail
the GPU path feeds) and rank 0 compares the gathered, sorted result with the
oracle's single-process scan of the whole corpus.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import secret_scanner as osc
from tests.corpus import make_corpus
from trivy_amd.shard import shard_files, shard_loads


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _files(seed, n):
    # unique paths: secrets sort by FilePath only (analyzer.go:225-227), so equal paths would tie
    return [("d%04d/%s" % (i, p), b.replace(b"\r", b"")) for i, (p, b) in enumerate(make_corpus(seed, n))]


def _rank_main(rank, world, port, seed, n, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.test_host_tail import host_tail_scan
        from trivy_amd.shard import scan_sharded
        files = _files(seed, n)
        res = scan_sharded(files, lambda fs: host_tail_scan(None, fs), rank, world)
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump([s.to_dict() for s in res.Secrets], f)
        else:
            assert res is None
    finally:
        dist.destroy_process_group()


def _oracle_sorted(files):
    o = osc.new_scanner(None)
    secrets = [o.scan(p, b) for p, b in files]
    secrets = [s for s in secrets if s["Findings"]]
    secrets.sort(key=lambda s: s["FilePath"].encode("latin-1", "surrogateescape")
                 if isinstance(s["FilePath"], str) else s["FilePath"])
    for s in secrets:
        s["Findings"].sort(key=lambda f: (f["RuleID"], f["StartLine"]))
    return secrets


def test_shard_files_partition_and_balance():
    rng = np.random.default_rng(7)
    sizes = np.clip(rng.lognormal(np.log(8192), 1.5, 5000).astype(np.int64), 10, 10 << 20)
    for world in (1, 2, 3, 8):
        shards = shard_files(sizes, world)
        allidx = np.concatenate(shards)
        assert sorted(allidx.tolist()) == list(range(sizes.size))
        assert all(np.all(np.diff(s) > 0) for s in shards)
        loads = shard_loads(sizes, shards)
        # LPT: max load <= mean + largest item
        assert max(loads) <= sizes.sum() / world + sizes.max()
        assert shard_files(sizes, world)[0].tolist() == shards[0].tolist()  # deterministic


def test_shard_files_edge_cases():
    assert [s.tolist() for s in shard_files([], 2)] == [[], []]
    assert [s.tolist() for s in shard_files([5], 3)] == [[0], [], []]
    assert [s.tolist() for s in shard_files([1, 1, 1, 1], 2)] == [[0, 2], [1, 3]]
    with pytest.raises(ValueError):
        shard_files([1], 0)


@pytest.mark.timeout(300)
def test_two_rank_gloo_scan_matches_single_process(tmp_path):
    seed, n, world = 31, 160, 2
    out = tmp_path / "rank0.json"
    mp.start_processes(_rank_main, args=(world, _free_port(), seed, n, str(out)), nprocs=world,
                       join=True, start_method="spawn")
    got = json.loads(out.read_text())
    want = _oracle_sorted(_files(seed, n))
    assert len(want) > 5
    assert [s["FilePath"] for s in got] == [s["FilePath"] for s in want]
    assert got == want


def _rank_main_gpu(rank, world, port, seed, n, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import trivy_amd.secret as secret
        from trivy_amd.shard import scan_sharded
        dev = rank % torch.cuda.device_count()  # the 1-GPU box: both ranks share cuda:0
        sc = secret.NewScanner(None, device=dev)
        files = _files(seed, n)
        res = scan_sharded(files, lambda fs: sc.ScanBatch([secret.ScanArgs(p, b) for p, b in fs]), rank, world)
        if rank == 0:
            with open(out_path, "w") as f:
                json.dump([s.to_dict() for s in res.Secrets], f)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_rank_gpu_scan_matches_single_process(tmp_path):
    seed, n, world = 33, 160, 2
    out = tmp_path / "rank0.json"
    mp.start_processes(_rank_main_gpu, args=(world, _free_port(), seed, n, str(out)), nprocs=world,
                       join=True, start_method="spawn")
    got = json.loads(out.read_text())
    want = _oracle_sorted(_files(seed, n))
    assert len(want) > 5
    assert got == want


@pytest.mark.gpu
def test_two_scanners_one_process_concurrent():
    """One process, two Scanners (device ids 0 and 0 on the 1-GPU box; 0 and 1 on a node),
    shards scanned concurrently, merged and sorted as AnalysisResult.Sort vs the oracle."""
    import torch
    from oracle import secret_scanner as osc
    import trivy_amd.secret as secret
    from trivy_amd.analyzer.secret import AnalysisResult
    from trivy_amd.shard import scan_devices
    n_dev = torch.cuda.device_count()
    scanners = [secret.NewScanner(None, device=0), secret.NewScanner(None, device=1 if n_dev > 1 else 0)]
    # unique paths: AnalysisResult.Sort orders secrets by FilePath only (ties keep no defined order)
    files = [("d%04d/%s" % (i, p), b.replace(b"\r", b"")) for i, (p, b) in enumerate(make_corpus(61, 240))]
    got = scan_devices(files, scanners)
    o = osc.new_scanner(None)
    want = AnalysisResult()
    for p, b in files:
        r = o.scan(p, b)
        if r["Findings"]:
            want.Secrets.append(r)
    want.Secrets.sort(key=lambda s: s["FilePath"].encode("utf-8", "surrogateescape"))
    for s in want.Secrets:
        s["Findings"].sort(key=lambda f: (f["RuleID"].encode(), f["StartLine"]))
    assert [s.to_dict() for s in got.Secrets] == want.Secrets
    assert len(got.Secrets) > 5


def _rank_main_records(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from trivy_amd.secret.scanner import RECORD_DTYPE
        from trivy_amd.shard import gather_records
        rng = np.random.default_rng(100 + rank)
        n = 50
        rec = np.zeros(n, dtype=RECORD_DTYPE)
        rec["file"] = rng.integers(0, 20, n)
        rec["rule"] = rng.integers(0, 3, n)
        rec["start_line"] = rng.integers(1, 40, n)
        rec["end_line"] = rec["start_line"]
        rec["digest"] = rng.integers(0, 2 ** 62, n)
        paths = np.array([("r%d/f%02d" % (rank % 2, f)).encode() for f in rec["file"]], dtype="S16")
        merged = gather_records(rec, paths, ["zeta", "alpha", "mid"])
        if rank == 0:
            np.savez(out_path, rec=merged["records"], paths=merged["paths"], ranks=merged["ranks"])
        else:
            assert merged is None
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_records_gather_sorted(tmp_path):
    """shard.gather_records (bench.py's timed gather at N>1): every rank's records reach rank 0
    in FilePath, RuleID, StartLine order (analyzer.go:225-234)."""
    out = tmp_path / "merged.npz"
    mp.start_processes(_rank_main_records, args=(2, _free_port(), str(out)), nprocs=2, join=True,
                       start_method="spawn")
    d = np.load(out)
    rec, paths = d["rec"], d["paths"]
    assert len(rec) == 100
    ids = ["zeta", "alpha", "mid"]
    keys = [(p, ids[r], int(s)) for p, r, s in zip(paths, rec["rule"], rec["start_line"])]
    assert keys == sorted(keys)


def test_bench_gpus_flag_launches_the_ranks():
    """`bench.py --gpus 2` without a torchrun environment starts two rank processes itself
    (torch.distributed.run, one rank per GPU) before anything touches a GPU; --dry-run runs the
    rank / world plumbing, the max-over-ranks timing and the rank-0 findings gather on gloo.  The
    line reports the world that ran, and a --gpus / WORLD_SIZE disagreement fails loudly."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3
    assert d["gather"] == {"findings": 128, "ranks": 2}
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env2, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "--gpus 2 but WORLD_SIZE=1" in r.stderr
