"""Exact host tail (libtsg.so) vs the oracle on CPU.

Drives the C++ tail through the test hook ``tsg_debug_host_tail`` (whole-file
candidate windows, keyword gate from Go's bytes.ToLower) so that allow rules,
exclude blocks, group extraction, censoring, findLocation and the pdqsort
order are checked without a GPU.  The GPU candidate stage is covered by
tests/test_gpu_parity.py and tests/test_filter_model.py.
"""
import ctypes as c
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import hostlib
from oracle import secret_scanner as osc
from tests.corpus import make_corpus
from trivy_amd import _lib
from trivy_amd.secret import ParseConfig, builtin_allow_rules, builtin_rules
from trivy_amd.secret.scanner import CGlobal, ScanResult, _CBatch, _declare, _b

G = Path(__file__).resolve().parent / "golden"
CASES = json.loads((G / "scanner_cases.json").read_text())["cases"]


class _Owner:
    def __init__(self, L):
        self._L = L


def _assemble(cfg):
    b_rules, b_allow = builtin_rules(), builtin_allow_rules()
    if cfg is None:
        return b_rules, b_allow, []
    enabled = b_rules
    if cfg.EnableBuiltinRuleIDs:
        enabled = [r for r in b_rules if r.ID in cfg.EnableBuiltinRuleIDs]
    enabled = enabled + cfg.CustomRules
    rules = [r for r in enabled if r.ID not in cfg.DisableRuleIDs]
    allow = [a for a in b_allow + cfg.CustomAllowRules if a.ID not in cfg.DisableAllowRuleIDs]
    return rules, allow, cfg.ExcludeBlock.Regexes


def host_tail_scan(cfg, files, raw=False):
    L = hostlib.lib()
    _declare(L)
    rules, allow, exclude = _assemble(cfg)
    cg = CGlobal(rules, allow, exclude)
    contents = [b for _, b in files]
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in contents])
    arena = np.frombuffer(b"".join(contents) + b"\0" * 16, dtype=np.uint8)
    pb = [_b(p) for p, _ in files]
    parr = (c.c_char_p * max(1, len(pb)))(*pb)
    plen = np.array([len(p) for p in pb], dtype=np.uint64)
    batch = _CBatch(len(files), arena.ctypes.data, offs.ctypes.data, None, None,
                    c.cast(parr, c.c_void_p).value, plen.ctypes.data, None)
    h = c.c_void_p()
    if L.tsg_debug_host_tail(c.byref(cg.g), c.byref(batch), c.byref(h)) != 0:
        raise RuntimeError(hostlib.last_error())
    res = ScanResult(_Owner(L), h)
    return res if raw else res.secrets([p for p, _ in files])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] + "|" + c["config"] for c in CASES])
def test_host_tail_golden(case):
    cfg = ParseConfig(str(G / "scanner" / case["config"]))
    content = (G / "scanner" / case["input"]).read_bytes().replace(b"\r", b"")
    got = host_tail_scan(cfg, [(case["file_path"], content)])[0]
    assert got.to_dict() == case["want"]


@pytest.mark.parametrize("seed", [21, 22])
def test_host_tail_corpus_vs_oracle(seed):
    files = [(p, b.replace(b"\r", b"")) for p, b in make_corpus(seed, 150)]
    got = host_tail_scan(None, files)
    o = osc.new_scanner(None)
    n = 0
    for (p, b), g in zip(files, got):
        want = o.scan(p, b)
        assert g.to_dict() == want, p
        n += len(want["Findings"] or [])
    assert n > 5


def test_host_tail_many_findings_sort_order():
    # > 12 findings in one file exercises pdqsort beyond insertion sort
    body = b"\n".join(b"tok%02d ghp_%036d AKIA%016d " % (i, i * 7919 % 1000, i) for i in range(40))
    files = [("many.txt", body)]
    got = host_tail_scan(None, files)[0]
    want = osc.new_scanner(None).scan("many.txt", body)
    assert got.to_dict() == want
    assert len(want["Findings"]) > 12


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_host_tail_sort_keys_ties_and_prefixes(tmp_path, seed):
    """The findings sort compares packed keys (RuleID rank, the match's first 12 bytes, zero-padded)
    before whole matches: matches equal in those 12 bytes, matches that are prefixes of others,
    NUL bytes against the padding, exact duplicates on different lines, and two rules whose IDs
    order opposite to their definition -- the pdqsort permutation is the oracle's."""
    import random
    rng = random.Random(seed)
    cfg_path = tmp_path / "trivy-secret.yaml"
    cfg_path.write_text(
        "rules:\n"
        "  - id: zz-pfx\n    category: Custom\n    title: Z\n    severity: LOW\n"
        "    regex: 'PFX[a-c\\x00]{0,20}'\n"
        "  - id: aa-pfx\n    category: Custom\n    title: A\n    severity: LOW\n"
        "    regex: 'QFX[ab]{0,14}'\n")
    cfg = ParseConfig(str(cfg_path))
    alpha = [b"a", b"b", b"c", b"\x00"]
    lines, pool = [], []
    for i in range(600):
        if pool and rng.random() < 0.2:
            m = rng.choice(pool)  # an exact duplicate, elsewhere in the file
        elif rng.random() < 0.3:
            m = b"QFX" + b"".join(rng.choice(alpha[:2]) for _ in range(rng.randrange(0, 15)))
        else:
            head = b"aaaaaaaaa" if rng.random() < 0.5 else b""  # 12-byte ties
            m = b"PFX" + head + b"".join(rng.choice(alpha) for _ in range(rng.randrange(0, 21 - len(head))))
        pool.append(m)
        lines.append(b"v%d = %s ;" % (i, m))
    body = b"\n".join(lines)
    got = host_tail_scan(cfg, [("ties.txt", body)])[0]
    want = osc.new_scanner(osc.parse_config(str(cfg_path))).scan("ties.txt", body)
    assert got.to_dict() == want
    assert len(want["Findings"]) > 500


def test_host_tail_lazy_keyword_gate(tmp_path):
    """MatchKeywords is evaluated after the windowed search: keyword inside the match,
    elsewhere in the file (either case), only via U+0130 / U+212A folding, inside a
    longer word, or absent (scanner.go:174-186 semantics, checked against the oracle)."""
    cfg_path = tmp_path / "trivy-secret.yaml"
    cfg_path.write_text(
        "rules:\n"
        "  - id: gated\n    category: Custom\n    title: Gated\n    severity: HIGH\n"
        "    regex: 'tok_[a-z0-9]{8}'\n    keywords: [Kilo, 'mi.x']\n"
        "  - id: gated-in-match\n    category: Custom\n    title: In match\n    severity: LOW\n"
        "    regex: '(?i)zz[a-z]{4}[0-9]{3}'\n    keywords: [zzab]\n")
    cfg = ParseConfig(str(cfg_path))
    body = b"x = tok_abcdef12\n"
    files = [
        ("none.txt", body),
        ("lower.txt", body + b"kilo\n"),
        ("upper.txt", b"KILO " + body),
        ("mixed.txt", body + b"it is kIlO-ish\n"),
        ("dot.txt", body + b"MI.X\n"),
        ("dotmiss.txt", body + b"mixx mi_x\n"),
        ("kelvin.txt", body + "Kilo\n".encode()),
        ("dotless.txt", body + "Mİ.x\n".encode()),
        ("longs.txt", body + "ſilo kilo\n".encode()),
        ("partial.txt", body + b"kil\no\n"),
        ("inmatch.txt", b"ZZAB"[:4] + b"cd123 zzabcd999 zzxyzw000\n"),
        ("notinmatch.txt", b"zzxyzw000\n"),
        ("end.txt", body + b"kil"),
        ("start.txt", b"ilo" + body),
    ]
    got = host_tail_scan(cfg, files)
    o = osc.new_scanner(osc.parse_config(str(cfg_path)))
    for (p, b), g in zip(files, got):
        assert g.to_dict() == o.scan(p, b), p


def test_host_tail_c3_generated_rules(tmp_path):
    """The exact tail with 2,087 rules (BASELINE configs[2]) vs the oracle."""
    from trivy_amd.corpus import c3_rules
    from tests.test_gpu_parity import _c3_files
    y, samples = c3_rules()
    p = tmp_path / "trivy-secret.yaml"
    p.write_text(y)
    files = _c3_files(samples, 23, 40)
    got = host_tail_scan(ParseConfig(str(p)), files)
    o = osc.new_scanner(osc.parse_config(str(p)))
    n = 0
    for (path, b), g in zip(files, got):
        want = o.scan(path, b)
        assert g.to_dict() == want, path
        n += len(want["Findings"] or [])
    assert n > 10


def test_host_tail_c3u_unanchored_rules(tmp_path):
    """The exact tail with the C3u rules (10 % without a literal anchor) vs the oracle."""
    from trivy_amd.corpus import c3_rules
    from tests.test_gpu_parity import _c3_files
    y, samples = c3_rules(unanchored_share=0.1)
    p = tmp_path / "trivy-secret.yaml"
    p.write_text(y)
    files = _c3_files([s for s in samples if s.startswith(b"kwu")], 29, 30)
    got = host_tail_scan(ParseConfig(str(p)), files)
    o = osc.new_scanner(osc.parse_config(str(p)))
    n = 0
    for (path, b), g in zip(files, got):
        want = o.scan(path, b)
        assert g.to_dict() == want, path
        n += len(want["Findings"] or [])
    assert n > 5


CAND = np.dtype([("file", "<u4"), ("rule", "<u4"), ("wlo", "<i8"), ("whi", "<i8"), ("nl_before", "<i8"),
                 ("flags", "<u4"), ("nl_back", "<u4", (3,)), ("nl_fwd", "<u4", (3,)), ("pad", "<u4")])
assert CAND.itemsize == 64


def _windowed_candidates(files, n_rules, step, hints):
    """Every rule over every file in windows of `step` bytes, each carrying its
    '\\n' count and (hints) the last three '\\n' before it and the first three
    at or after it, as the GPU's finalize kernel writes them
    (Candidate::nl_back / nl_fwd)."""
    recs = []
    for f, (_, b) in enumerate(files):
        nl = np.flatnonzero(np.frombuffer(b, dtype=np.uint8) == 10)
        for lo in range(0, max(1, len(b)), step):
            before = nl[nl < lo]
            back = [0xFFFFFFFF] * 3
            fwd = [0xFFFFFFFF] * 3
            if hints:
                last = before[-3:][::-1]
                back = [lo - int(x) for x in last] + [0xFFFFFFFE] * (3 - len(last))
                nxt = nl[nl >= lo][:3]
                fwd = [int(x) - lo for x in nxt] + [0xFFFFFFFE] * (3 - len(nxt))
            for r in range(n_rules):
                recs.append((f, r, lo, min(len(b), lo + step - 1), len(before), 0, back, fwd, 0))
    return np.array(recs, dtype=CAND)


@pytest.mark.parametrize("hints", [False, True])
def test_host_tail_newline_hints(hints):
    """Code-context lines from the newline hints match the oracle: long lines
    before a match (farther than one 1-KiB GPU step), matches on the first
    lines, adjacent censored secrets and a multi-line key hiding newlines."""
    import random
    rng = random.Random(99)
    key, gh = b"AKIA" + b"Q" * 16, b"ghp_" + b"a1B2" * 9
    pk = (b"-----BEGIN RSA PRIVATE KEY-----\n" + b"MIIEow" * 12 + b"\n" + b"abcd" * 16 + b"\n"
          b"-----END RSA PRIVATE KEY-----")
    files = []
    for n, lens in enumerate([[0], [5], [3000], [9000, 3], [1500, 1500, 1500], [1, 2000, 1], [600, 0, 0]]):
        body = b"".join(bytes(rng.choice(b"xyz .,=") for _ in range(ln)) + b"\n" for ln in lens)
        files.append(("long%d.txt" % n, body + b"k = " + key + b"\n" + body + b"t=" + gh + b"\n"))
        files.append(("first%d.txt" % n, b"k = " + key + b" " + body))
        files.append(("pk%d.pem" % n, body + pk + b"\n" + b"x" * 2000 + b"\n" + key + b"\n"))
        files.append(("adj%d.txt" % n, body + key + b"\n" + gh + b"\n" + key + b"\n" + b"y" * 1100 + b"\n" + gh))
    L = hostlib.lib()
    _declare(L)
    rules, allow, exclude = _assemble(None)
    cg = CGlobal(rules, allow, exclude)
    contents = [b for _, b in files]
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in contents])
    arena = np.frombuffer(b"".join(contents) + b"\0" * 16, dtype=np.uint8)
    pb = [_b(p) for p, _ in files]
    parr = (c.c_char_p * len(pb))(*pb)
    plen = np.array([len(p) for p in pb], dtype=np.uint64)
    batch = _CBatch(len(files), arena.ctypes.data, offs.ctypes.data, None, None,
                    c.cast(parr, c.c_void_p).value, plen.ctypes.data, None)
    cands = _windowed_candidates(files, len(rules), 700, hints)
    h = c.c_void_p()
    if L.tsg_debug_host_tail_cands(c.byref(cg.g), c.byref(batch), cands.ctypes.data, len(cands), c.byref(h)) != 0:
        raise RuntimeError(hostlib.last_error())
    got = ScanResult(_Owner(L), h).secrets([p for p, _ in files])
    o = osc.new_scanner(None)
    n = 0
    for (p, b), g in zip(files, got):
        want = o.scan(p, b)
        assert g.to_dict() == want, p
        n += len(want["Findings"] or [])
    assert n > 40


def test_allow_path_literal_fast_path(tmp_path):
    """Allow-path regexes that are one literal (or one group of literal alternatives)
    with optional ^ / $ are matched by byte compares (Matcher::simple); the result must
    equal the regex's, including sources that only look literal (escaped anchors,
    trailing escaped '$', classes, an empty alternative, two groups)."""
    pats = [r"\.md$", r"^usr\/share\/", r"\/vendor\/", r"^exact\.txt$", r"a\$", r"b\\$", r"\d\.log$",
            r"^$x", r"c\.d", r"x.y", r"^opt\/(?:alpha|be|)\/", r"(?:gam|delt)a\.cfg$", r"^(?:one|two)$",
            r"q(?:r|s)(?:t|u)"]
    cfg_path = tmp_path / "trivy-secret.yaml"
    cfg_path.write_text("allow-rules:\n" + "".join(
        "  - id: p%d\n    path: '%s'\n" % (i, p.replace("'", "''")) for i, p in enumerate(pats)))
    cfg = ParseConfig(str(cfg_path))
    body = b"k = AKIA" + b"Q" * 16 + b"\n"
    paths = ["README.md", "README.mdx", "usr/share/x.txt", "x/usr/share/y", "src/vendor/z.go", "vendor/z.go",
             "exact.txt", "exact.txt2", "a$", "xa$y", "b\\", "b\\x", "3.log", "x.log", "c.d", "cxd", "xzy",
             "x.y", "plain.txt", "$x", "opt/alpha/k", "opt/be/k", "opt//k", "opt/beta/k", "x/opt/be/k",
             "gamma.cfg", "a/delta.cfg", "delt.cfg", "one", "two", "one2", "qrt", "qsu", "qrx", "x|y"]
    files = [(p, body) for p in paths]
    got = host_tail_scan(cfg, files)
    o = osc.new_scanner(osc.parse_config(str(cfg_path)))
    n_allowed = 0
    for (p, b), g in zip(files, got):
        want = o.scan(p, b)
        assert g.to_dict() == want, p
        n_allowed += not want["Findings"]
    assert n_allowed >= 8


def _fnv(h, b):
    for x in b:
        h = ((h ^ x) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def test_result_records_match_findings():
    """tsg_result_records (the multi-rank gather unit): one record per finding, in file order,
    with the rule index, lines and the documented FNV-1a digest of Match + Code lines."""
    import struct
    from trivy_amd.secret import builtin_rules
    files = [("d%03d/%s" % (i, p), b.replace(b"\r", b"")) for i, (p, b) in enumerate(make_corpus(23, 120))]
    res = host_tail_scan(None, files, raw=True)
    rec = res.records()
    got = res.secrets([p for p, _ in files])
    ids = [r.ID for r in builtin_rules()]
    want = []
    for i, s in enumerate(got):
        for f in s.Findings or []:
            h = _fnv(0xcbf29ce484222325, f.Match.encode("utf-8", "surrogateescape"))
            for ln in f.Code.Lines or []:
                h = _fnv(h, struct.pack("<q", ln.Number) + bytes([ln.IsCause, ln.FirstCause, ln.LastCause]))
                h = _fnv(h, ln.Content.encode("utf-8", "surrogateescape"))
            want.append((i, f.RuleID, f.StartLine, f.EndLine, h))
    assert len(want) > 5
    assert [(int(r["file"]), ids[r["rule"]], int(r["start_line"]), int(r["end_line"]), int(r["digest"]))
            for r in rec] == want


@pytest.mark.parametrize("seed", [77, 78, 79])
def test_host_tail_dense_findings_line_index(tmp_path, seed):
    """Files with many findings for their size take the per-file index of the newlines the
    censored content keeps (scanner.cpp ScanFile): line numbers, match lines over 100 B,
    code windows at the file's first and last lines, multi-line private keys whose newlines
    are censored, adjacent matches on one line and on consecutive lines -- vs the oracle.
    Several rules per file: their matches restart low, so the galloping searches for a
    finding's line and first span (FindingsHost) fall back to full ones between runs."""
    import random
    cfg_path = tmp_path / "trivy-secret.yaml"
    cfg_path.write_text(
        "rules:\n  - id: b64run\n    category: Custom\n    title: Base64 run\n    severity: LOW\n"
        "    regex: '(?i)[a-z0-9/+]{32,48}'\n    keywords: [blobkw]\n")
    cfg = ParseConfig(str(cfg_path))
    rng = random.Random(seed)
    alpha = b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
    pk = (b"-----BEGIN RSA PRIVATE KEY-----\n" + b"MIIEow" * 11 + b"\n" + b"abcd" * 16 + b"\n"
          b"-----END RSA PRIVATE KEY-----")
    files = []
    for i in range(60):
        parts = [b"blobkw"] if i % 5 else []
        for _ in range(rng.randint(6, 40)):
            r = rng.random()
            if r < 0.5:
                parts.append(bytes(rng.choice(alpha) for _ in range(rng.randint(20, 400))))
            elif r < 0.6:
                parts.append(pk)
            elif r < 0.75:
                parts.append(b"k = AKIA" + bytes(rng.choice(b"ABCDEFGHIJKLMNOPQRSTUVWXYZ234567") for _ in range(16)))
            elif r < 0.85:
                parts.append(b"x" * rng.randint(0, 300))
            else:
                parts.append(b"")
        sep = [b"\n", b" ", b"\n\n", b"="]
        body = b"".join(p + rng.choice(sep) for p in parts)
        files.append(("dense%02d.txt" % i, body))
    got = host_tail_scan(cfg, files)
    o = osc.new_scanner(osc.parse_config(str(cfg_path)))
    n = 0
    for (p, b), g in zip(files, got):
        want = o.scan(p, b)
        assert g.to_dict() == want, p
        n += len(want["Findings"] or [])
    assert n > 600


def test_host_tail_file_ids_past_2_pow_22():
    """Candidates of files whose ids need more than two 11-bit radix digits (>= 2^22, about 4.2 M
    files in one batch) are still grouped per file: the tail's LSD radix sort runs its passes over the
    file bits only.  Records shuffled so each file's candidates are interleaved with the others'."""
    import random
    key, gh = b"AKIA" + b"Q" * 16, b"ghp_" + b"a1B2" * 9
    real = [(b"a = 1\nk = " + key + b"\n" + b"t=" + gh + b"\n"),
            (b"t=" + gh + b"\nzz\nk = " + key + b"\n"),
            (b"nothing here\n"),
            (b"k = " + key + b" " + b"x" * 150 + b" t=" + gh + b"\n" + b"k = " + key + b"\n")]
    ids = [3, (1 << 21) + 5, (1 << 22) - 1, 1 << 22, (1 << 22) + 7, (1 << 23) + 11, (1 << 23) + 12]
    n_files = (1 << 23) + 64
    body = {f: real[k % len(real)] for k, f in enumerate(ids)}
    lens = np.zeros(n_files, dtype=np.uint64)
    for f, b in body.items():
        lens[f] = len(b)
    offs = np.zeros(n_files + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    arena = np.zeros(int(offs[-1]) + 16, dtype=np.uint8)
    for f, b in body.items():
        arena[int(offs[f]):int(offs[f]) + len(b)] = np.frombuffer(b, dtype=np.uint8)
    path = c.create_string_buffer(b"src/x.txt")
    own = {f: c.create_string_buffer(b"src/f%d.txt" % f) for f in ids}
    ptrs = np.full(n_files, c.addressof(path), dtype=np.uint64)
    plen = np.full(n_files, 9, dtype=np.uint64)
    for f, s in own.items():
        ptrs[f] = c.addressof(s)
        plen[f] = len(s.value)
    L = hostlib.lib()
    _declare(L)
    rules, allow, exclude = _assemble(None)
    cg = CGlobal(rules, allow, exclude)
    batch = _CBatch(n_files, arena.ctypes.data, offs.ctypes.data, None, None, ptrs.ctypes.data,
                    plen.ctypes.data, None)
    files = [(own[f].value.decode(), body[f]) for f in ids]
    cands = _windowed_candidates(files, len(rules), 40, True)
    cands["file"] = np.array(ids, dtype=np.uint32)[cands["file"]]
    cands = cands[np.random.default_rng(5).permutation(len(cands))]
    h = c.c_void_p()
    if L.tsg_debug_host_tail_cands(c.byref(cg.g), c.byref(batch), cands.ctypes.data, len(cands), c.byref(h)) != 0:
        raise RuntimeError(hostlib.last_error())
    res = ScanResult(_Owner(L), h)
    o = osc.new_scanner(None)
    n = 0
    for (p, b), f in zip(files, ids):
        want = o.scan(p, b)
        assert res.secrets([p], lo=f)[0].to_dict() == want, p
        for g in (f - 1, f + 1):  # the neighbours stay empty
            if g not in body and g < n_files:
                assert res.secrets(["src/x.txt"], lo=g)[0].to_dict() == osc.new_scanner(None).scan("src/x.txt", b"")
        n += len(want["Findings"] or [])
    rec = res.records()
    assert len(rec) == n > 10
    assert np.all(np.diff(rec["file"].astype(np.int64)) >= 0)
    assert set(rec["file"].tolist()) <= set(ids)


def _sort_case(rng, n, n_rules=4):
    """n findings: rule ids (two rules share an ID rank), matches from runs of '*' and a few letters
    (censored windows: long common prefixes, many exact ties)."""
    rank = np.array([2, 0, 2, 1][:n_rules], dtype=np.uint32)
    rule = rng.integers(0, n_rules, n).astype(np.uint32)
    pool = [b"*" * int(rng.integers(10, 60)) + bytes(rng.choice(list(b"ab *"), int(rng.integers(0, 5))))
            for _ in range(max(8, n // 6))]
    texts = [pool[int(rng.integers(0, len(pool)))] for _ in range(n)]
    off = np.zeros(n, dtype=np.uint32)
    off[1:] = np.cumsum([len(t) for t in texts])[:-1]
    return rule, rank, b"".join(texts), off, np.array([len(t) for t in texts], dtype=np.uint32), texts


def _native_sort(L, rule, rank, text, off, ln, threads):
    n = len(rule)
    out = np.zeros(n, dtype=np.uint32)
    L.tsg_debug_sort_findings.argtypes = [c.c_uint32, c.c_void_p, c.c_void_p, c.c_uint32, c.c_char_p, c.c_uint64,
                                          c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    assert L.tsg_debug_sort_findings(n, rule.ctypes.data, rank.ctypes.data, len(rank), text, len(text),
                                     off.ctypes.data, ln.ctypes.data, threads, out.ctypes.data) == 0
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_findings_sort_parallel_equals_sequential(seed):
    """SortFindingsParallel (the heaviest files' sort after GPU materialisation) spreads pdqsort's
    independent recursive calls over the pool; its permutation -- ties included -- is the sequential
    pdqsort's, and at a size the Python restatement finishes, Go's sort.Slice's (oracle/gosort.py)."""
    from oracle import gosort
    L = hostlib.lib()
    rng = np.random.default_rng(seed)
    rule, rank, text, off, ln, _ = _sort_case(rng, 120_000)
    seq = _native_sort(L, rule, rank, text, off, ln, 0)
    for threads in (2, 8, 16):
        assert np.array_equal(_native_sort(L, rule, rank, text, off, ln, threads), seq), threads
    rule, rank, text, off, ln, texts = _sort_case(rng, 6000)
    seq = _native_sort(L, rule, rank, text, off, ln, 0)
    assert np.array_equal(_native_sort(L, rule, rank, text, off, ln, 8), seq)
    items = list(range(len(rule)))
    gosort.sort_slice(items, lambda i, j: (rank[rule[i]], texts[i]) < (rank[rule[j]], texts[j]))
    assert np.array_equal(np.array(items, dtype=np.uint32), seq)
