#!/usr/bin/env python3
"""Inclusive per-line profile inside one function (tools/sprof samples with
frame-pointer chains; build the library with -fno-omit-frame-pointer):
each sample is charged to the line of the innermost frame that lies in the
function whose name contains FUNC.
  python tools/sprof/incl.py /tmp/prof.txt libtsg_host ScanFile"""
import bisect
import collections
import subprocess
import sys


SRC = "scanner.cpp"


def main():
    global SRC
    path, want, func = sys.argv[1], sys.argv[2], sys.argv[3]
    if len(sys.argv) > 4:
        SRC = sys.argv[4]
    maps, libc = [], []
    for ln in open(path + ".maps"):
        parts = ln.split()
        if len(parts) >= 6 and "x" in parts[1] and "libc.so" in parts[5]:
            libc.append(tuple(int(x, 16) for x in parts[0].split("-")))
    for ln in open(path + ".maps"):
        parts = ln.split()
        if len(parts) >= 6 and "x" in parts[1] and want in parts[5]:
            a, b = (int(x, 16) for x in parts[0].split("-"))
            maps.append((a, b, int(parts[2], 16), parts[5]))
    import os
    lib = maps[0][3]
    if not os.path.exists(lib):  # a profile taken on another machine: the same library in this tree
        here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        for cand in ("trivy_amd", "oracle/build"):
            q = os.path.join(here, cand, os.path.basename(lib))
            if os.path.exists(q):
                lib = q
                break
    out = subprocess.run(["nm", "-C", "--defined-only", "-S", lib], capture_output=True, text=True).stdout
    ranges = []
    for ln in out.splitlines():
        p = ln.split(" ", 3)
        if len(p) == 4 and p[2] in "tTwW" and func in p[3]:
            ranges.append((int(p[0], 16), int(p[0], 16) + int(p[1], 16)))
    tot = 0
    hits = []
    for x in open(path):
        addrs = [int(v, 16) for v in x.split()]
        tot += 1
        in_libc = any(a <= addrs[0] < b for a, b in libc)
        # the stack-top word is a return address only for a libc leaf (memchr & co. keep no frame)
        cand = [addrs[0]] + ([addrs[1] - 1] if in_libc and len(addrs) > 1 else []) + [v - 1 for v in addrs[2:]]
        for v in cand:
            for a, b, off, _ in maps:
                if a <= v < b:
                    o = v - a + off
                    if any(lo <= o < hi for lo, hi in ranges):
                        hits.append(o)
                        break
            else:
                continue
            break
    uniq = sorted(set(hits))
    res = subprocess.run(["addr2line", "-i", "-a", "-C", "-e", lib] + ["%x" % o for o in uniq], capture_output=True,
                         text=True).stdout.splitlines()
    where, cur, chain = {}, None, []
    for ln in res + ["0xEND"]:
        if ln.startswith("0x"):
            if cur is not None:  # innermost line of the chain in a file named like the function's source
                own = [c for c in chain if SRC in c]
                where[cur] = (own[0] if own else chain[0] if chain else "?").split("/")[-1]
            cur = int(ln, 16) if ln != "0xEND" else None
            chain = []
        else:
            chain.append(ln)
    cnt = collections.Counter(where[o] for o in hits)
    print("samples %d, in %s: %d (%.1f%%)" % (tot, func, len(hits), 100.0 * len(hits) / max(1, tot)))
    for s, n in cnt.most_common(45):
        print("%6.1f%%  %s" % (100.0 * n / tot, s))


if __name__ == "__main__":
    main()
