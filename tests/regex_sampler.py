"""Random strings drawn from a Go regexp's language (test helper).

Walks the oracle's parsed AST (oracle.goregexp) and samples each node:
classes pick a member (biased to ASCII), repeats pick a count (capped),
alternations pick a branch; assertions emit nothing (the surrounding text may
then make the sample a non-match: those are useful decoys).
"""
import random

from oracle.goregexp import GoRegexp


def _pick(rng, ranges, ascii_bias=0.97):
    asc = [(lo, min(hi, 0x7E)) for lo, hi in ranges if lo <= 0x7E and min(hi, 0x7E) >= max(lo, 0x20)]
    asc = [(max(lo, 0x20), hi) for lo, hi in asc]
    if asc and rng.random() < ascii_bias:
        lo, hi = rng.choice(asc)
        return chr(rng.randint(lo, hi))
    lo, hi = rng.choice(ranges)
    hi = min(hi, 0x2FFFF)
    if lo > hi:
        lo = hi
    c = rng.randint(lo, hi)
    if 0xD800 <= c <= 0xDFFF:
        c = 0x41
    return chr(c)


def sample(node, rng, maxrep=6):
    k = node[0]
    if k == "class":
        return _pick(rng, node[1])
    if k in ("empty", "assert"):
        return ""
    if k in ("cat", "quote"):
        return "".join(sample(n, rng, maxrep) for n in node[1])
    if k == "alt":
        return sample(rng.choice(node[1]), rng, maxrep)
    if k == "cap":
        return sample(node[2], rng, maxrep)
    if k == "group":
        return sample(node[1], rng, maxrep)
    if k == "rep":
        _, lo, hi, _, sub = node
        top = lo + maxrep if hi == -1 else hi
        n = rng.randint(lo, max(lo, min(top, lo + 3 * maxrep)))
        return "".join(sample(sub, rng, maxrep) for _ in range(n))
    raise AssertionError(k)


def sample_regex(pattern, rng, maxrep=6):
    return sample(GoRegexp(pattern).ast, rng, maxrep).encode("utf-8")
