"""Unanchored rules at scale (full-scan kernel): (file, rule) pairs with an open
keyword gate, files cut into chunks per lane, chunk entry states iterated to
the fixpoint.  Multi-MiB files with matches at and across chunk boundaries
(TSG_FULLSCAN_CHUNK forces small chunks), an unbounded repeat spanning many
chunks, gated-out files, and the C3u rule set -- all vs the oracle.
"""
import random

import pytest

from oracle import secret_scanner as osc

pytestmark = pytest.mark.gpu

RULES = (
    "rules:\n"
    "  - id: tok\n    category: Custom\n    title: Token\n    severity: HIGH\n"
    "    regex: '(?i)\\b[g-z]{3}[0-9]{3}[._-][a-z0-9]{12}\\b'\n    keywords: [gatekw]\n"
    "  - id: long\n    category: Custom\n    title: Long run\n    severity: LOW\n"
    "    regex: '[a-f]{2}[0-9]{2}_[a-z]+_end[0-9]'\n"
    "  - id: digits\n    category: Custom\n    title: Digits\n    severity: LOW\n"
    "    regex: '[0-9]{3}-[0-9]{4}-[0-9]{3}'\n    keywords: [call]\n")


def _files(rng):
    files = []
    filler = (b"lorem ipsum dolor sit amet 0123 consectetur " * 50 + b"\n")
    for i in range(6):
        body = bytearray(filler * (40 + 30 * i))  # ~90 KiB .. 0.5 MiB
        if i % 2 == 0:
            body[:0] = b"gatekw\n"
        for _ in range(20):  # tokens at random places, many across 4-KiB chunk edges
            at = rng.randrange(len(body) - 40)
            tok = (b" " + bytes(rng.choice(b"ghijkz") for _ in range(3)) + b"%03d" % rng.randrange(1000) +
                   b"_" + bytes(rng.choice(b"abc123xyz") for _ in range(12)) + b" ")
            body[at:at + len(tok)] = tok
        if i == 3:  # an unbounded repeat over ~40 KiB (10 chunks of 4 KiB)
            run = b" ab12_" + b"q" * 40000 + b"_end7 "
            body[5000:5000 + len(run)] = run
        if i == 4:
            body += b"\ncall 555-1234-999 now\n"
        files.append(("big%d.txt" % i, bytes(body)))
    # a multi-MiB file, gate open, token exactly at 4-KiB multiples
    big = bytearray(b"x" * (3 << 20))
    big[:7] = b"gatekw "
    for k in range(1, 200):
        at = k * 4096 * 3 - 5
        big[at:at + 21] = b" pqr777.abcdef123456 "
    files.append(("huge.txt", bytes(big)))
    return files


def _compare(secret, files, cfg):
    s = secret.NewScanner(secret.ParseConfig(cfg))
    o = osc.new_scanner(osc.parse_config(cfg))
    got = s.ScanBatch([secret.ScanArgs(FilePath=p, Content=b) for p, b in files])
    n = 0
    for (p, b), g in zip(files, got):
        want = o.scan(p, b)
        assert g.to_dict() == want, p
        n += len(want["Findings"] or [])
    return n


@pytest.mark.parametrize("chunk,class_runs,task", [("4096", "0", "4096"), ("65536", "0", "4096"),
                                                   ("4096", "0", "16"), ("4096", "1", "4096")])
def test_fullscan_chunks_vs_oracle(tmp_path, monkeypatch, chunk, class_runs, task):
    """class_runs 0: no literal anchors, the rules run in full-scan mode; 1: they are
    anchored on their runs of one-byte classes (rules.cpp ExtractClassRun).  Bounded rules
    run as lane tasks (task: TSG_FS_TASK_BYTES, 16 = the 8 x max_len minimum: many task
    edges inside tokens), the unbounded one wave-wide in chunks (TSG_FULLSCAN_CHUNK)."""
    import trivy_amd.secret as secret
    monkeypatch.setenv("TSG_FULLSCAN_CHUNK", chunk)
    monkeypatch.setenv("TSG_FS_TASK_BYTES", task)
    monkeypatch.setenv("TSG_CLASS_RUNS", class_runs)
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(RULES)
    n = _compare(secret, _files(random.Random(7)), str(cfg))
    assert n > 100


@pytest.mark.parametrize("class_runs", ["0", "1"])
def test_c3u_unanchored_rules_vs_oracle(tmp_path, monkeypatch, class_runs):
    """The C3u rule set (10 % of 2,000 generated rules without a literal anchor)."""
    import trivy_amd.secret as secret
    monkeypatch.setenv("TSG_CLASS_RUNS", class_runs)
    from trivy_amd.corpus import c3_rules
    from tests.test_gpu_parity import _c3_files
    y, samples = c3_rules(unanchored_share=0.1)
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(y)
    files = _c3_files([s for s in samples if s.startswith(b"kwu")] + samples[:50], 19, 120)
    assert _compare(secret, files, str(cfg)) > 20


FOLD_RULES = (
    "rules:\n"
    "  - id: tok-kw\n    category: Custom\n    title: Token gated by a k/i keyword\n    severity: HIGH\n"
    "    regex: '(?i)\\b[g-z]{3}[0-9]{3}[._-][a-z0-9]{12}\\b'\n    keywords: [kwink]\n"
    "  - id: anchored-kw\n    category: Custom\n    title: Anchored, gated\n    severity: LOW\n"
    "    regex: 'pfxtok_[a-z0-9]{10}'\n    keywords: [tikki]\n")


@pytest.mark.parametrize("class_runs", ["0", "1"])
def test_keyword_gate_through_fold_runes_vs_oracle(tmp_path, monkeypatch, class_runs):
    """bytes.ToLower maps U+212A to 'k' and U+0130 to 'i': keywords spelled with
    them open the gate (kwfold_kernel sets the bits); files holding the runes
    but not the keyword stay gated out of the full scan."""
    import trivy_amd.secret as secret
    monkeypatch.setenv("TSG_CLASS_RUNS", class_runs)
    K, I = "K".encode(), "İ".encode()
    tok = b" ghi123_abcdef123456 "
    atok = b" pfxtok_abcdefghij "
    pad = b"filler text 0123 " * 300 + b"\n"
    variants = [
        b"kwink",                       # ASCII
        K + b"w" + I + b"n" + K,        # every k / i through a fold rune
        b"KW" + I + b"NK",              # upper case + U+0130
        K + b"wink",                    # the rune at the start
        b"kwin" + K,                    # ... at the end
        b"kw" + K + b"nk",              # U+212A where 'i' belongs: no match
        b"kwi" + I + b"k",              # an extra rune: no match
    ]
    files = []
    for i, v in enumerate(variants):
        files.append(("v%d.txt" % i, pad + v + b"\n" + pad + tok + pad))
        files.append(("a%d.txt" % i, pad + b"t" + I + b"kk" + I + b" " + v + atok + pad))
    files.append(("runes-no-kw.txt", pad + K + I + b" x " + tok + pad))  # runes, keyword absent
    files.append(("deep.txt", pad * 40 + K + b"w" + I + b"nk" + pad * 40 + tok))
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(FOLD_RULES)
    n = _compare(secret, files, str(cfg))
    assert n >= 8


def test_fullscan_lists_overflow_and_grow(tmp_path, monkeypatch):
    """More open pairs (20,000 files, a keyword-less bounded rule) than the initial pair list
    (16,384) and more lane tasks (a 9 MB file cut into ~100-B tasks) than the initial task list
    (65,536): the scan sees the overflow, grows the lists to the counts and rescans.  Every file
    vs the restated reference CPU scan (tsg_cpuref_scan), a sample vs the oracle."""
    import numpy as np
    from bench import full_diff
    from tests.test_gpu_bench_corpus import _cpuref
    import trivy_amd.secret as secret
    monkeypatch.setenv("TSG_FS_TASK_BYTES", "16")
    monkeypatch.setenv("TSG_CLASS_RUNS", "0")
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text("rules:\n  - id: digits\n    category: Custom\n    title: Digits\n    severity: LOW\n"
                   "    regex: '[0-9]{3}-[0-9]{4}-[0-9]{3}'\n")
    rng = random.Random(3)
    contents = [b"x %03d-%04d-%03d y" % (i % 1000, i, i % 997) if i % 3 == 0 else b"nothing %d" % i
                for i in range(20000)]
    big = bytearray(b"ab 12-3456-789 " * (9_000_000 // 15))
    for k in range(300):
        at = rng.randrange(len(big) - 20)
        big[at:at + 14] = b" 123-4567-890 "
    contents.insert(7000, bytes(big))
    paths = ["f%05d.txt" % i for i in range(len(contents))]
    offs = np.zeros(len(contents) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in contents])
    arena = np.frombuffer(b"".join(contents) + b"\0" * 64, dtype=np.uint8)

    class C:  # the shape _cpuref / full_diff read
        pass
    C.arena, C.offsets, C.n_files = arena, offs, len(contents)
    keep = [np.frombuffer(p.encode() + b"\0", dtype=np.uint8) for p in paths]  # alive while C is
    C.path_ptrs = np.array([k.ctypes.data for k in keep], dtype=np.uint64)
    res = secret.NewScanner(secret.ParseConfig(str(cfg))).scan_arena(arena, offs, paths)
    st = res.stats()
    assert st["fullscan_pairs"] > 16384
    ref = _cpuref(C, cfg_path=str(cfg))
    bad, first = full_diff(res, ref, C.n_files)
    assert bad == 0, (bad, paths[first] if first is not None else None)
    assert st["findings"] > 3000
    o = osc.new_scanner(osc.parse_config(str(cfg)))
    got = res.secrets(paths)
    for i in list(range(0, 20001, 997)):
        if i != 7000:
            assert got[i].to_dict() == o.scan(paths[i], contents[i]), paths[i]
