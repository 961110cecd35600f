"""Diagnose tsg_debug_xform mismatches: the identity-tile test's data, then the bytes
test's data three times in one process; per run xoff vs oracle and the first wrong byte."""
import ctypes as c
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import analyzer as oan  # noqa: E402
from trivy_amd import _lib  # noqa: E402

L = _lib.lib()
L.tsg_debug_xform.argtypes = [c.c_int, c.c_void_p, c.c_uint64, c.c_void_p, c.c_uint32, c.c_void_p, c.c_void_p,
                              c.c_uint64, c.c_void_p]


def identity_data():
    rng = random.Random(11)
    files, kinds = [], []
    for _ in range(3000):
        r = rng.random()
        n = rng.choice([0, 7, 100, 700, 1024, 1500, 2600, 5000, 12000])
        text = bytes(rng.choice(b"abcdefghij =:/\n") for _ in range(n))
        if r < 0.6:
            files.append(text)
            kinds.append(rng.choice([0, 1]))
        elif r < 0.8:
            b = bytearray(text)
            for _ in range(rng.randint(1, 15)):
                b.insert(rng.randint(0, len(b)), 13)
            files.append(bytes(b))
            kinds.append(1)
        elif r < 0.9:
            files.append(bytes(rng.choice(b"abcdef") for _ in range(n)))
            kinds.append(2)
        else:
            files.append(bytes(rng.choice(b"ab\x00\x01 z") for _ in range(n)))
            kinds.append(2)
    return files, kinds


def bytes_data():
    rng = random.Random(5)
    alpha = [b"a", b"Z", b" ", b"~", b"\x00", b"\x07", b"\r", b"\n", b"\xa0", b"\xa1", b"\xad", b"\xff", b"\x7f",
             b"\x1f"]
    files, kinds = [], []
    for _ in range(4000):
        n = rng.choice([0, 0, 1, 3, 4, 5, 6, 9, 15, 16, 17, 31, 63, 100, 1000, 1023, 1024, 1025, 3000, 9000])
        if rng.random() < 0.5:
            parts = []
            while sum(map(len, parts)) < n:
                parts.append(b"p" * rng.choice([1, 3, 4, 5, 6, 7, 20]) + rng.choice(alpha))
            b = b"".join(parts)[:n]
        else:
            b = b"".join(rng.choice(alpha) for _ in range(n))
        files.append(b)
        kinds.append(rng.choice([0, 1, 1, 2, 2]))
    return files, kinds


def check(name, files, kinds):
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in files])
    raw = np.frombuffer(b"".join(files) + b"\0" * 64, dtype=np.uint8)
    kd = np.array(kinds, dtype=np.uint8)
    out = np.zeros(int(offs[-1]) * 2 + 64, dtype=np.uint8)
    xoff = np.zeros(len(files) + 1, dtype=np.uint64)
    rc = L.tsg_debug_xform(0, raw.ctypes.data, int(offs[-1]), offs.ctypes.data, len(files), kd.ctypes.data,
                           out.ctypes.data, len(out), xoff.ctypes.data)
    want = [b if k == 0 else b.replace(b"\r", b"") if k == 1 else oan.extract_printable_bytes(b)
            for b, k in zip(files, kinds)]
    wo = np.zeros(len(files) + 1, dtype=np.uint64)
    wo[1:] = np.cumsum([len(x) for x in want])
    bad = np.nonzero(wo != xoff)[0]
    W = b"".join(want)
    G = out[:len(W)].tobytes()
    diff = np.nonzero(np.frombuffer(W, np.uint8) != np.frombuffer(G, np.uint8))[0]
    print(name, "rc", rc, "n_bytes", int(offs[-1]), "xoff mismatches", len(bad), bad[:5],
          "byte mismatches", len(diff))
    if len(bad):
        f = int(bad[0])
        print("  first bad xoff file", f, "got", int(xoff[f]), "want", int(wo[f]), "prev ok", int(xoff[f - 1]),
              int(wo[f - 1]), "raw off", int(offs[f]), "tile", int(offs[f]) // 1024)
    if len(diff):
        d0 = int(diff[0])
        f = int(np.searchsorted(wo, d0, side="right")) - 1
        print("  first wrong byte at", d0, "file", f, "kind", kinds[f], "raw off", int(offs[f]))
        print("  want", W[d0 - 8:d0 + 24])
        print("  got ", G[d0 - 8:d0 + 24])


check("identity", *identity_data())
bd = bytes_data()
for i in range(3):
    check("bytes%d" % i, *bd)
