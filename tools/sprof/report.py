#!/usr/bin/env python3
"""Symbolise tools/sprof samples: per function (nm) share of the samples in one library.
  python tools/sprof/report.py /tmp/prof.txt [libname-substring]"""
import bisect
import collections
import subprocess
import sys


def to_vaddr(lib):
    """File offset -> link-time address for a library's executable LOAD segments."""
    segs = []
    out = subprocess.run(["readelf", "-lW", lib], capture_output=True, text=True).stdout
    for ln in out.splitlines():
        p = ln.split()
        if p and p[0] == "LOAD" and "E" in "".join(p[6:-1]):
            segs.append((int(p[1], 16), int(p[2], 16), int(p[4], 16)))  # offset, vaddr, filesz
    def f(off):
        for o, v, n in segs:
            if o <= off < o + n:
                return off - o + v
        return off
    return f


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "libtsg"
    maps = []
    for ln in open(path + ".maps"):
        parts = ln.split()
        if len(parts) < 6 or "x" not in parts[1]:
            continue
        a, b = (int(x, 16) for x in parts[0].split("-"))
        maps.append((a, b, int(parts[2], 16), parts[5]))
    pcs = [int(x.split()[0], 16) for x in open(path)]
    libs = collections.Counter()
    per = collections.defaultdict(list)
    for pc in pcs:
        for a, b, off, name in maps:
            if a <= pc < b:
                libs[name] += 1
                per[name].append(pc - a + off)
                break
        else:
            libs["?"] += 1
    tot = len(pcs)
    print("samples %d" % tot)
    for name, n in libs.most_common(8):
        print("%6.1f%%  %s" % (100.0 * n / tot, name))
    for name in per:
        if want not in name:
            continue
        syms = []
        out = subprocess.run(["nm", "-C", "--defined-only", name], capture_output=True, text=True).stdout
        if not out.strip():
            out = subprocess.run(["nm", "-D", "-C", "--defined-only", name], capture_output=True, text=True).stdout
        for ln in out.splitlines():
            p = ln.split(" ", 2)
            if len(p) == 3 and p[1] in "tTwW":
                syms.append((int(p[0], 16), p[2]))
        syms.sort()
        addrs = [s[0] for s in syms]
        cnt = collections.Counter()
        va = to_vaddr(name)
        for off in per[name]:
            i = bisect.bisect_right(addrs, va(off)) - 1
            cnt[syms[i][1][:110] if i >= 0 else "?"] += 1
        print("--", name)
        for s, n in cnt.most_common(30):
            print("%6.1f%%  %s" % (100.0 * n / tot, s))


if __name__ == "__main__":
    main()


def lines(path, want):
    """Per source line (addr2line, innermost inline frame) of the library matching `want`."""
    maps = []
    for ln in open(path + ".maps"):
        parts = ln.split()
        if len(parts) >= 6 and "x" in parts[1]:
            a, b = (int(x, 16) for x in parts[0].split("-"))
            maps.append((a, b, int(parts[2], 16), parts[5]))
    offs, lib = [], None
    tot = 0
    tags = []
    for x in open(path):
        parts = x.split()
        pc = int(parts[0], 16)
        ra = int(parts[1], 16) if len(parts) > 1 else 0
        tot += 1
        tag = ""
        for a, b, off, name in maps:
            if a <= pc < b and "libc.so" in name:  # a leaf in libc: charge the line that called it
                pc, tag = ra, "libc<- "
                break
        for a, b, off, name in maps:
            if a <= pc < b and want in name:
                offs.append(pc - a + off)
                tags.append(tag)
                lib = name
    va = to_vaddr(lib)
    offs = [va(o) for o in offs]
    uniq = sorted(set(offs))
    out = subprocess.run(["addr2line", "-f", "-C", "-e", lib] + ["%x" % o for o in uniq], capture_output=True,
                         text=True).stdout.splitlines()
    where = {}
    for i, o in enumerate(uniq):
        fn, fl = out[2 * i], out[2 * i + 1]
        where[o] = "%s  %s" % (fl.split("/")[-1], fn[:70])
    cnt = collections.Counter(t + where[o] for o, t in zip(offs, tags))
    for s, n in cnt.most_common(40):
        print("%6.1f%%  %s" % (100.0 * n / tot, s))


if __name__ == "__main__" and len(sys.argv) > 3 and sys.argv[3] == "lines":
    lines(sys.argv[1], sys.argv[2])
