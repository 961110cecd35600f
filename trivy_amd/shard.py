"""Multi-GPU sharding of a secret scan.

A scan shards naturally by file: every file is an independent unit
(`Scanner.Scan`, scanner.go:377-463, reads one file's content only), so ranks
partition the file list, scan their share on their own GPU and never exchange
file data.  There is no data-path collective.  The only cross-rank step is
the final gather of the (small, sparse) findings to one rank, which then
restores the reference's order: secrets by FilePath, findings by (RuleID,
StartLine) (`AnalysisResult.Sort`, pkg/fanal/analyzer/analyzer.go:225-234).

Partitioning is byte-balanced LPT (longest processing time first): files are
taken in decreasing size and each goes to the rank with the fewest bytes so
far, which bounds the largest shard by 4/3 of the optimum.  Within a shard
files keep their input order, so a rank's arena is a sub-sequence of the
caller's.
"""
import heapq
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from trivy_amd.analyzer.secret import AnalysisResult


def shard_files(sizes: Sequence[int], world: int) -> List[np.ndarray]:
    """LPT byte-balanced partition of file indices over `world` ranks.

    Returns one ascending index array per rank; every index appears in exactly
    one shard.  Ties (equal sizes, equal loads) break by index and rank, so the
    result is deterministic and identical on every rank."""
    if world < 1:
        raise ValueError("world must be >= 1")
    sizes = np.asarray(sizes, dtype=np.int64)
    order = np.lexsort((np.arange(sizes.size), -sizes))  # size desc, index asc
    heap = [(0, r) for r in range(world)]
    owner = np.empty(sizes.size, dtype=np.int64)
    for i in order:
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + int(sizes[i]), r))
    return [np.flatnonzero(owner == r) for r in range(world)]


def shard_loads(sizes: Sequence[int], shards: Sequence[np.ndarray]) -> List[int]:
    sizes = np.asarray(sizes, dtype=np.int64)
    return [int(sizes[s].sum()) for s in shards]


def gather_results(local: AnalysisResult, dst: int = 0, group=None) -> Optional[AnalysisResult]:
    """Gathers every rank's secrets to `dst` (torch.distributed, any backend that
    supports object collectives; gloo on the host).  On `dst` returns the merged
    and sorted AnalysisResult (analyzer.go:251-301 Merge, :225-234 Sort); None
    elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [None] * world if rank == dst else None
    dist.gather_object(local.Secrets, parts, dst=dst, group=group)
    if rank != dst:
        return None
    out = AnalysisResult()
    for p in parts:
        out.Merge(AnalysisResult(Secrets=list(p)))
    out.Sort()
    return out


def scan_sharded(files: Sequence[Tuple[str, bytes]], scan: Callable[[Sequence[Tuple[str, bytes]]], list],
                 rank: int, world: int, dst: int = 0, group=None) -> Optional[AnalysisResult]:
    """Scans this rank's LPT shard of `files` with `scan` (a batch scan returning
    one types.Secret per file, e.g. Scanner.ScanBatch over ScanArgs), keeps the
    secrets with findings (the analyzer drops the rest, secret.go:142-144) and
    gathers them to `dst`."""
    shard = shard_files([len(b) for _, b in files], world)[rank]
    mine = [files[i] for i in shard]
    res = AnalysisResult()
    if mine:
        for s in scan(mine):
            if s.Findings:
                res.Secrets.append(s)
    return gather_results(res, dst=dst, group=group)


def scan_devices(files: Sequence[Tuple[str, bytes]], scanners: Sequence) -> AnalysisResult:
    """One process, one Scanner per device (the shape of a Go drop-in: a scanner per
    GPU behind one analyzer): the LPT shards of `files` are
    submitted to the scanners concurrently (tsg_scan_submit; each device's GPU
    phase and host tail run on their own threads), then the secrets with
    findings are merged and sorted as AnalysisResult.Merge/Sort do
    (analyzer.go:251-301, :225-234)."""
    shards = shard_files([len(b) for _, b in files], len(scanners))
    pending = []
    for sc, shard in zip(scanners, shards):
        if len(shard) == 0:
            continue
        contents = [files[i][1] for i in shard]
        offs = np.zeros(len(contents) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(x) for x in contents], dtype=np.uint64)
        arena = np.frombuffer(b"".join(contents) + b"\0" * 64, dtype=np.uint8)
        paths = [files[i][0] for i in shard]
        pending.append((sc.scan_arena_async(arena, offs, paths), paths))
    out = AnalysisResult()
    for p, paths in pending:
        for s in p.wait().secrets(paths):
            if s.Findings:
                out.Merge(AnalysisResult(Secrets=[s]))
    out.Sort()
    return out


def gather_records(records: np.ndarray, paths: np.ndarray, rule_ids: Sequence[str], dst: int = 0,
                   group=None) -> Optional[dict]:
    """The compact form of the gather for large scans (bench.py under torchrun): every rank
    sends its finding records (tsg_result_records: file, rule index, start/end line, a digest of
    Match + Code lines) with each record's file path; `dst` concatenates them and restores the
    reference's order -- secrets by FilePath, findings by (RuleID, StartLine)
    (analyzer.go:225-234) -- with one lexsort.  Returns {"records", "paths", "ranks"} (sorted) on
    `dst`, None elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    parts = [None] * world if rank == dst else None
    dist.gather_object((records, paths), parts, dst=dst, group=group)
    if rank != dst:
        return None
    recs = np.concatenate([p[0] for p in parts]) if parts else records[:0]
    pths = np.concatenate([p[1] for p in parts]) if parts else paths[:0]
    ranks = np.concatenate([np.full(len(p[0]), r, dtype=np.int32) for r, p in enumerate(parts)])
    order_of_id = np.argsort(np.argsort(np.array(list(rule_ids), dtype=object)))  # RuleID rank per rule index
    key_rule = order_of_id[recs["rule"]] if len(recs) else np.zeros(0, dtype=np.int64)
    order = np.lexsort((recs["start_line"], key_rule, pths))
    return {"records": recs[order], "paths": pths[order], "ranks": ranks[order]}
