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
    L.tsg_corpus_crlf.restype = c.c_int64
    L.tsg_corpus_crlf.argtypes = [c.c_uint64, c.c_void_p, c.c_uint64, c.c_void_p, c.c_double, c.c_void_p, c.c_int]
    L.tsg_corpus_strip.argtypes = [c.c_void_p, c.c_uint64, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int]
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

    crlf = None  # per file: 1 = CRLF text (generate(crlf_share=...))

    def stripped(self, threads=None):
        """The analyzer's CR strip (secret.go:121) of every file: a Corpus over the
        stripped contents with the same paths (the arena the HBM-resident bench scans)."""
        L = _lib.lib()
        _declare(L)
        n = self.n_files
        offs = np.zeros(n + 1, dtype=np.uint64)
        out = np.zeros(self.n_bytes + 64, dtype=np.uint8)
        threads = threads or int(os.environ.get("TSG_HOST_THREADS", "16"))
        L.tsg_corpus_strip(self.offsets.ctypes.data, n, self.arena.ctypes.data, out.ctypes.data, offs.ctypes.data,
                           threads)
        S = Corpus(out[:int(offs[-1]) + 64], offs, self.path_buf)
        S.crlf = self.crlf
        return S

    def packed_paths(self):
        """The paths packed back to back (uint8, +16 B pad) and their n+1 offsets (uint64)."""
        rows = self.path_buf[:self.n_files * PATH_STRIDE].reshape(self.n_files, PATH_STRIDE)
        z = rows == 0
        lens = np.where(z.any(axis=1), z.argmax(axis=1), PATH_STRIDE).astype(np.uint64)
        offs = np.zeros(self.n_files + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(lens)
        keep = np.arange(PATH_STRIDE)[None, :] < lens[:, None].astype(np.int64)
        return np.concatenate([rows[keep], np.zeros(16, np.uint8)]), offs

    def content(self, i):
        return self.arena[int(self.offsets[i]):int(self.offsets[i + 1])].tobytes()


def generate(target_bytes, seed=SEED, secrets_per_byte=1.0 / 262144, threads=None, size_scale=1.0, crlf_share=0.0):
    """The C1/C2 generator; size_scale multiplies every planned file size (clipped at
    10 MiB, the total cut at target_bytes): C5's mean-64-KiB files use 2.6.
    crlf_share: that share of the files is CRLF text (5 % for C1/C2;
    Corpus.crlf marks them, Corpus.stripped() is the analyzer's CR strip)."""
    L = _lib.lib()
    _declare(L)
    n = L.tsg_corpus_plan(seed, int(target_bytes), None, 0)
    offs = np.zeros(n + 1, dtype=np.uint64)
    L.tsg_corpus_plan(seed, int(target_bytes), offs.ctypes.data, n + 1)
    if size_scale != 1.0:
        sizes = np.minimum(np.diff(offs).astype(np.float64) * size_scale, 10 << 20).astype(np.uint64)
        cum = np.cumsum(sizes)
        n = int(np.searchsorted(cum, int(target_bytes))) + 1
        n = min(n, len(sizes))
        offs = np.zeros(n + 1, dtype=np.uint64)
        offs[1:] = np.minimum(cum[:n], int(target_bytes))
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
    C = Corpus(arena, offs, paths)
    if crlf_share > 0:
        C.crlf = np.zeros(n, dtype=np.uint8)
        L.tsg_corpus_crlf(seed, offs.ctypes.data, n, arena.ctypes.data, float(crlf_share), C.crlf.ctypes.data, threads)
    return C


# ---- BASELINE configs[2] (C3): 2,000 generated custom rules ----
_C3_OPS = ["=", ">", ":=", "||:", "<=", "=>", ":"]


def c3_rules(n_rules=2000, seed=SEED, planted_share=0.10, unanchored_share=0.0, fullscan_share=0.0):
    """A trivy-secret.yaml text with n_rules custom rules and planted sample matches.

    60 %: generic assignment form (secret group), 40 %: literal-prefix token form;
    secret length L in [16, 64]; 1-3 keywords (4-12 chars, the first being the
    rule's literal); samples for `planted_share` of the rules.  With
    unanchored_share > 0 (the "C3u" variant) that share of
    the rules has no literal at a bounded offset -- a token of classes only,
    gated by its keyword -- so the engine full-scans the files where the gate is
    open.  With fullscan_share > 0 (the "C3f" variant) that
    share of the rules is a bare class run, (?i)[a-z0-9/+]{L} (L in [32, 48]),
    gated by its own keyword: neither a literal nor a rare class run anchors it
    (rules.cpp ExtractClassRun: a 6-window of that class is far above 1e-5),
    so every file holding the keyword goes through fullscan_kernel.  Returns
    (yaml_text, [sample bytes])."""
    import random
    rng = random.Random(seed ^ 0xC3)
    alnum = "abcdefghijklmnopqrstuvwxyz0123456789"
    lines = ["rules:"]
    samples = []
    urng = random.Random(seed ^ 0xC3A)
    frng = random.Random(seed ^ 0xC3F)
    for i in range(n_rules):
        L = rng.randint(16, 64)
        if fullscan_share and frng.random() < fullscan_share:
            kw = "kwf%04d" % i
            n = frng.randint(32, 48)
            lines += ["  - id: c3-fullscan-%04d" % i, "    category: Generated", "    title: Full-scan rule %d" % i,
                      "    severity: LOW", "    regex: '(?i)[a-z0-9/+]{%d}'" % n, "    keywords: [%s]" % kw]
            if frng.random() < 0.5:
                for _ in range(2):
                    tok = "".join(frng.choice(alnum + "/+") for _ in range(n))
                    samples.append(("%s: %s" % (kw, tok)).encode())
            continue
        if unanchored_share and urng.random() < unanchored_share:
            kw = "kwu%04d" % i
            rx = r"(?i)\b[g-z]{3}[0-9]{3}[._-][a-z0-9]{%d}\b" % (L // 2)
            lines += ["  - id: c3-unanchored-%04d" % i, "    category: Generated", "    title: Unanchored rule %d" % i,
                      "    severity: MEDIUM", "    regex: '%s'" % rx, "    keywords: [%s]" % kw]
            if urng.random() < planted_share * 3:
                for _ in range(3):
                    tok = "".join(urng.choice("ghijklmnopqrstuvwxyz") for _ in range(3)) + \
                          "".join(urng.choice("0123456789") for _ in range(3)) + urng.choice("._-") + \
                          "".join(urng.choice(alnum) for _ in range(L // 2))
                    samples.append(("%s = %s" % (kw, tok)).encode())
            continue
        generic = rng.random() < 0.6
        lit = ("kw%04d" % i) if generic else ("pfx%04d_" % i)
        kws = [lit] + ["".join(rng.choice(alnum) for _ in range(rng.randint(4, 12)))
                       for _ in range(rng.randint(0, 2))]
        if generic:
            rx = (r"(?i)(?P<key>%s[a-z0-9_ .\-,]{0,25})(=|>|:=|\|\|:|<=|=>|:).{0,5}['\"]"
                  r"(?P<secret>[a-z0-9]{%d})['\"]" % (lit, L))
        else:
            rx = r"%s[A-Za-z0-9]{%d}" % (lit, L)
        lines += ["  - id: c3-rule-%04d" % i, "    category: Generated", "    title: Generated rule %d" % i,
                  "    severity: %s" % rng.choice(["LOW", "MEDIUM", "HIGH", "CRITICAL"]),
                  "    regex: '%s'" % rx.replace("'", "''"),
                  "    keywords: [%s]" % ", ".join(kws)]
        if generic:
            lines.append("    secret-group-name: secret")
        if rng.random() < planted_share:
            for _ in range(3):
                if generic:
                    key = lit.upper() if rng.random() < 0.3 else lit
                    key += "".join(rng.choice("abcdefghijklmnopqrstuvwxyz0123456789_ .-,")
                                   for _ in range(rng.randint(0, 8)))
                    q = rng.choice("'\"")
                    s = "%s%s%s%s%s%s" % (key, rng.choice(_C3_OPS), " " * rng.randint(0, 3), q,
                                          "".join(rng.choice(alnum) for _ in range(L)), q)
                else:
                    s = lit + "".join(rng.choice(alnum + alnum.upper()[:26]) for _ in range(L))
                samples.append(s.encode())
    return "\n".join(lines) + "\n", samples


def generate_c3(target_bytes, rule_samples, seed=SEED, secrets_per_byte=1.0 / 262144, threads=None):
    """The C2 generator with the C3 rules' samples added to the planted pool."""
    L = _lib.lib()
    _declare(L)
    n = L.tsg_corpus_plan(seed, int(target_bytes), None, 0)
    offs = np.zeros(n + 1, dtype=np.uint64)
    L.tsg_corpus_plan(seed, int(target_bytes), offs.ctypes.data, n + 1)
    pool = json.loads(POOL.read_text())
    samples = [s.encode() for v in pool.values() for s in v] + list(rule_samples)
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


# ---- BASELINE configs[3] (C4): image layers of millions of small files ----
def generate_layer(target_file_bytes, seed=SEED, secrets_per_byte=1.0 / 262144, threads=None):
    """An uncompressed ustar layer (uint8 numpy array) holding ~target_file_bytes of file data."""
    L = _lib.lib()
    L.tsg_corpus_layer.restype = c.c_int64
    L.tsg_corpus_layer.argtypes = [c.c_uint64, c.c_uint64, c.c_char_p, c.c_void_p, c.c_uint32, c.c_double,
                                   c.c_void_p, c.c_uint64, c.c_int, c.POINTER(c.c_uint64)]
    pool = json.loads(POOL.read_text())
    samples = [s.encode() for v in pool.values() for s in v]
    blob = b"".join(samples)
    poff = np.zeros(len(samples) + 1, dtype=np.uint64)
    poff[1:] = np.cumsum([len(s) for s in samples])
    ne = c.c_uint64()
    total = L.tsg_corpus_layer(seed, int(target_file_bytes), blob, poff.ctypes.data, len(samples),
                               float(secrets_per_byte), None, 0, 1, c.byref(ne))
    out = np.empty(total, dtype=np.uint8)
    threads = threads or int(os.environ.get("TSG_HOST_THREADS", "16"))
    r = L.tsg_corpus_layer(seed, int(target_file_bytes), blob, poff.ctypes.data, len(samples),
                           float(secrets_per_byte), out.ctypes.data, total, threads, c.byref(ne))
    if r != total:
        raise RuntimeError("tsg_corpus_layer failed")
    return out
