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


@pytest.mark.parametrize("chunk", ["4096", "65536"])
def test_fullscan_chunks_vs_oracle(tmp_path, monkeypatch, chunk):
    import trivy_amd.secret as secret
    monkeypatch.setenv("TSG_FULLSCAN_CHUNK", chunk)
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(RULES)
    n = _compare(secret, _files(random.Random(7)), str(cfg))
    assert n > 100


def test_c3u_unanchored_rules_vs_oracle(tmp_path):
    """The C3u rule set (10 % of 2,000 generated rules without a literal anchor)."""
    import trivy_amd.secret as secret
    from trivy_amd.corpus import c3_rules
    from tests.test_gpu_parity import _c3_files
    y, samples = c3_rules(unanchored_share=0.1)
    cfg = tmp_path / "trivy-secret.yaml"
    cfg.write_text(y)
    files = _c3_files([s for s in samples if s.startswith(b"kwu")] + samples[:50], 19, 120)
    assert _compare(secret, files, str(cfg)) > 20
