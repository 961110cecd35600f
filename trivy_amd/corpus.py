"""Synthetic corpus (bench / large tests): wrapper of include/tsg_corpus.h."""
import ctypes as c
import json
import os
from pathlib import Path

import numpy as np

from . import _lib

POOL = Path(__file__).resolve().parent.parent / "tests/golden/secret_pool.json"
SEED = 0x5EC2E7
PATH_STRIDE = 64


def _declare(L):
    L.tsg_corpus_plan.restype = c.c_int64
    L.tsg_corpus_plan.argtypes = [c.c_uint64, c.c_uint64, c.c_void_p, c.c_uint64]
    L.tsg_corpus_fill.argtypes = [c.c_uint64, c.c_void_p, c.c_uint64, c.c_char_p, c.c_void_p, c.c_uint32,
                                  c.c_double, c.c_void_p, c.c_void_p, c.c_uint32, c.c_int]


class Corpus:
    """arena (uint8, +64 B zero pad), offsets (uint64, n+1), paths (char* array into a stride buffer)."""

    def __init__(self, arena, offsets, path_buf):
        self.arena = arena
        self.offsets = offsets
        self.path_buf = path_buf
        n = len(offsets) - 1
        self.path_ptrs = (path_buf.ctypes.data + np.arange(n, dtype=np.uint64) * PATH_STRIDE).astype(np.uint64)

    @property
    def n_files(self):
        return len(self.offsets) - 1

    @property
    def n_bytes(self):
        return int(self.offsets[-1])

    def path(self, i):
        raw = self.path_buf[i * PATH_STRIDE:(i + 1) * PATH_STRIDE].tobytes()
        return raw.split(b"\0", 1)[0].decode()

    def content(self, i):
        return self.arena[int(self.offsets[i]):int(self.offsets[i + 1])].tobytes()


def generate(target_bytes, seed=SEED, secrets_per_byte=1.0 / 262144, threads=None):
    L = _lib.lib()
    _declare(L)
    n = L.tsg_corpus_plan(seed, int(target_bytes), None, 0)
    offs = np.zeros(n + 1, dtype=np.uint64)
    L.tsg_corpus_plan(seed, int(target_bytes), offs.ctypes.data, n + 1)
    pool = json.loads(POOL.read_text())
    samples = [s.encode() for v in pool.values() for s in v]
    blob = b"".join(samples)
    poff = np.zeros(len(samples) + 1, dtype=np.uint64)
    poff[1:] = np.cumsum([len(s) for s in samples])
    total = int(offs[-1])
    arena = np.zeros(total + 64, dtype=np.uint8)
    paths = np.zeros(n * PATH_STRIDE, dtype=np.uint8)
    threads = threads or int(os.environ.get("TSG_HOST_THREADS", "16"))
    L.tsg_corpus_fill(seed, offs.ctypes.data, n, blob, poff.ctypes.data, len(samples), float(secrets_per_byte),
                      arena.ctypes.data, paths.ctypes.data, PATH_STRIDE, threads)
    return Corpus(arena, offs, paths)
