#!/usr/bin/env python3
"""CPU model of an 8-bucket K1 table over super-characters.

K1 (engine.hip filter_kernel) runs a bucketed shift-or over 15 item buckets + a newline bucket,
one 16-B table row per byte.  An 8-bucket table halves the LDS bytes and the v_lshl_or per byte
(k1x: 3.73 vs 4.98 ms on C2) but, with the same byte sets, flags 7x more 16-B blocks.  Here each
window slot's set is over super-characters (previous byte's bit f, byte) -- a 512-row table -- so
a bucket's union no longer allows every cross combination of its items' bytes.

The item windows are the product build's (least frequent <= 6 positions per item); the items are
re-clustered into 7 buckets by the same agglomerative rule as filter.cpp BuildFilter, with the fire
rate of a window estimated from super-character frequencies of a training sample (another seed),
and the flagged-block rate is measured on the first --mb MB of the C2 corpus.  Reported beside it:
the same simulator with plain byte sets at 16 and 8 buckets (the product's and the rejected shape).
Usage: python tools/superchar_model.py [--mb 30] [--bits 0,1,2,3,4,x,2:0+1]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.filter_model import FilterModel  # noqa: E402
from trivy_amd import corpus  # noqa: E402
from trivy_amd.secret.config import builtin_rules  # noqa: E402

W = 6  # window slots


def item_windows(fm):
    """Per item: (prev set, [W slot sets]) as bool[256] arrays (any = all True)."""
    anyb = np.ones(256, dtype=bool)
    out = []
    for it in fm.items:
        back, cls = it["back"], fm.item_cls[it["cls_off"]:it["cls_off"] + it["n"]]
        slots = []
        for s in range(W):
            q = back - W + s
            slots.append(fm.classes[cls[q]] if 0 <= q < it["n"] else anyb)
        q = back - W - 1
        prev = fm.classes[cls[q]] if 0 <= q < it["n"] else anyb
        out.append((prev, slots))
    return out


def super_sets(win, f):
    """Slot sets over super-characters f(prev) * 256 + byte: bool[W, 512]."""
    prev, slots = win
    out = np.zeros((W, 256 * (int(f.max()) + 1)), dtype=bool)
    for s in range(W):
        p = prev if s == 0 else slots[s - 1]
        bits = set(int(f[b]) for b in np.nonzero(p)[0])
        for bt in bits:
            out[s, bt * 256:(bt + 1) * 256] = slots[s]
    return out


def cluster(sets, prob, n_buckets):
    """Agglomerative merge (filter.cpp BuildFilter): always merge the pair whose union adds the
    least estimated fire rate Π_s P(slot set)."""
    cl = [s.copy() for s in sets]
    members = [[i] for i in range(len(sets))]
    cost = [float(np.prod([prob[s][x[s]].sum() for s in range(W)])) for x in cl]
    alive = list(range(len(cl)))
    while len(alive) > n_buckets:
        best = None
        for ai in range(len(alive)):
            i = alive[ai]
            for j in alive[ai + 1:]:
                u = cl[i] | cl[j]
                c = float(np.prod([prob[s][u[s]].sum() for s in range(W)]))
                d = c - cost[i] - cost[j]
                if best is None or d < best[0]:
                    best = (d, i, j, u, c)
        _, i, j, u, c = best
        cl[i], cost[i] = u, c
        members[i] += members[j]
        alive.remove(j)
    return [cl[i] for i in alive], [members[i] for i in alive]


def flagged_rate(a, buckets, idx):
    """Fraction of 16-B blocks with a window end of any bucket (zeros before the arena, as in K1)."""
    n = len(a)
    fire = np.zeros(n, dtype=bool)
    for B in buckets:
        ok = np.ones(n, dtype=bool)
        for s in range(W):
            sh = W - 1 - s
            col = B[s][idx]
            shifted = np.zeros(n, dtype=bool)
            shifted[sh:] = col[:n - sh] if sh else col
            ok &= shifted
        fire |= ok
    blocks = np.zeros(n // 16 + 1, dtype=bool)
    blocks[np.nonzero(fire)[0] >> 4] = True
    return blocks.mean(), fire.mean()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=30)
    ap.add_argument("--train-mb", type=float, default=8)
    ap.add_argument("--bits", default="0,1,2,3,4,6,x")
    args = ap.parse_args()
    fm = FilterModel(builtin_rules())
    wins = [w for w, it in zip(item_windows(fm), fm.items)]
    test = corpus.generate(int(args.mb * 1e6)).arena
    test = test[:int(args.mb * 1e6)]
    train = corpus.generate(int(args.train_mb * 1e6), seed=corpus.SEED + 100).arena[:int(args.train_mb * 1e6)]
    print("items %d, test %.0f MB, train %.0f MB" % (len(wins), len(test) / 1e6, len(train) / 1e6), flush=True)
    # plain byte sets (the product shape at 16 buckets, the rejected one at 8): same simulator
    bytefreq = np.bincount(train, minlength=256) / len(train)
    plain = [np.stack(w[1]) for w in wins]
    for nb in (15, 7):
        B, _ = cluster(plain, [bytefreq] * W, nb)
        blk, pos = flagged_rate(test, B, test)
        print("plain %2d item buckets: flagged blocks %.4f (fires %.2e / B)" % (nb, blk, pos), flush=True)
    for spec in args.bits.split(","):
        if spec == "x":
            f = np.array([((b >> 0) ^ (b >> 3)) & 1 for b in range(256)], dtype=np.uint16)
            name = "bit0^bit3"
        elif spec.startswith("2:"):  # two bits of the previous byte: a 1,024-row table
            k1, k2 = (int(x) for x in spec[2:].split("+"))
            f = np.array([((b >> k1) & 1) | (((b >> k2) & 1) << 1) for b in range(256)], dtype=np.uint16)
            name = "bits %d+%d" % (k1, k2)
        else:
            k = int(spec)
            f = np.array([(b >> k) & 1 for b in range(256)], dtype=np.uint16)
            name = "bit%d" % k

        def idx_of(a):
            prev = np.concatenate([[0], a[:-1]]).astype(np.uint16)
            return f[prev] * 256 + a.astype(np.uint16)
        itr = idx_of(train)
        freq = np.bincount(itr, minlength=256 * (int(f.max()) + 1)) / len(itr)
        S = [super_sets(w, f) for w in wins]
        B, mem = cluster(S, [freq] * W, 7)
        blk, pos = flagged_rate(test, B, idx_of(test))
        print("super-chars (%s) 7 item buckets: flagged blocks %.4f (fires %.2e / B); bucket sizes %s"
              % (name, blk, pos, sorted(len(m) for m in mem)), flush=True)


if __name__ == "__main__":
    main()
