#!/usr/bin/env python3
"""Per-bucket K1 fire rates and per-item confirm counts on a C2 sample (CPU model).

Replays the streaming filter (tests/filter_model.py) and the confirm step's
exact item check over the first --mb MB of the bench corpus, and prints, per
bucket, its fire rate and items, and per item the exact occurrences (= anchor
hits K2 would emit, before file attribution) with the rule it anchors.
Diagnostic only: it sizes the post-filter work that VERDICT r01 flagged.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.filter_model import FilterModel, KIND_ANCHOR, KIND_KEYWORD, KIND_FOLD  # noqa: E402
from trivy_amd import corpus  # noqa: E402
from trivy_amd.secret.config import builtin_rules  # noqa: E402


def item_occ(fm, a, it):
    """bool array: item `it` matches starting at position p."""
    n = it["n"]
    cls = fm.item_cls[it["cls_off"]:it["cls_off"] + n]
    m = len(a) - n + 1
    if m <= 0:
        return np.zeros(0, dtype=bool)
    ok = np.ones(m, dtype=bool)
    for q in range(n):
        ok &= fm.classes[cls[q]][a[q:q + m]]
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=16)
    ap.add_argument("--calib-mb", type=float, default=0,
                    help="compile with a calibration sample of this size (tsg_compile_options), generated with "
                         "another seed than the evaluated sample")
    args = ap.parse_args()
    rules = builtin_rules()
    calib = None
    if args.calib_mb > 0:
        K = corpus.generate(int(args.calib_mb * 1e6), seed=corpus.SEED + 7777)
        calib = K.arena[:K.n_bytes].copy()
    fm = FilterModel(rules, calibration=calib)
    print("anchors moved by the calibration sample: %d" % fm.n_calibrated)
    C = corpus.generate(int(args.mb * 1e6))
    a = C.arena[:C.n_bytes]
    print("sample: %d files, %.1f MB" % (C.n_files, C.n_bytes / 1e6))
    fr = fm.fires(a)
    blocks = np.zeros(C.n_bytes // 16 + 1, dtype=bool)
    for j in range(fm.n_buckets - 1):
        nz = np.nonzero(fr[j])[0]
        blocks[nz >> 4] = True
        items = fm.bucket_items[fm.bucket_off[j]:fm.bucket_off[j + 1]]
        print("bucket %2d: fires %.2e /B  items %s" % (j, len(nz) / C.n_bytes, list(map(int, items))))
    print("flagged blocks: %.3f of blocks (%.2e per byte)" % (blocks.mean(), blocks.sum() / C.n_bytes))
    # per-item exact occurrences
    rows = []
    for k, it in enumerate(fm.items):
        occ = int(item_occ(fm, a, it).sum())
        ids = fm.item_ids[it["ids_off"]:it["ids_off"] + it["n_ids"]]
        kind = {KIND_ANCHOR: "anchor", KIND_KEYWORD: "kw", KIND_FOLD: "fold"}[it["kind"]]
        rows.append((occ, k, kind, it["n"], list(map(int, ids))))
    rows.sort(reverse=True)
    L = fm._cg  # noqa
    import ctypes as c
    from trivy_amd import _lib
    lib = _lib.lib()
    lib.tsg_debug_anchor.argtypes = [c.c_void_p, c.c_uint32] + [c.c_void_p] * 4
    lib.tsg_debug_rule_anchor.restype = c.c_char_p
    lib.tsg_debug_rule_anchor.argtypes = [c.c_void_p, c.c_uint32]
    tot = sum(r[0] for r in rows if r[2] == "anchor")
    print("anchor item occurrences: %d (%.2e per byte, x%.0f -> %.1f M at 20 GB)"
          % (tot, tot / C.n_bytes, 20e9 / C.n_bytes, tot * 20e9 / C.n_bytes / 1e6))
    for occ, k, kind, n, ids in rows[:40]:
        desc = ""
        if kind == "anchor":
            rr = c.c_uint32()
            ll = c.c_uint32()
            lo = c.c_int32()
            hi = c.c_int32()
            lib.tsg_debug_anchor(fm.h, ids[0], c.byref(rr), c.byref(ll), c.byref(lo), c.byref(hi))
            desc = "%s %s" % (rules[rr.value].ID, lib.tsg_debug_rule_anchor(fm.h, rr.value).decode())
        print("%9d  item %3d %-6s n=%2d ids=%s %s" % (occ, k, kind, n, ids[:4], desc))


if __name__ == "__main__":
    main()
