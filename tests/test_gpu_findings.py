"""GPU finding materialisation (trivy_amd/csrc/materialize.hip) vs the
oracle and vs the host materialisation, on HBM-resident batches.

toFinding / findLocation (pkg/fanal/secret/scanner.go:475-558) and the censored
code lines (:431-446, :465-473) run on the GPU after the host's exact pass: the
cases below are the ones its line arithmetic can get wrong -- lines over 100 B
(the start-30 / end+20 cut) and over the 1-KiB search windows, matches that
span lines (the private-key rule: their '\\n' are censored), adjacent censored
matches on one line, findings on the first and on the last line (with and
without a final '\\n'), '\\n' hidden in censored spans between the code lines,
more than 12 findings in a file (pdqsort) and files at both ends of the arena.
"""
import random

import numpy as np
import pytest

from oracle import secret_scanner as osc

pytestmark = pytest.mark.gpu

AWS = b"AKIA" + b"Q" * 16
GH = b"ghp_" + b"a1B2" * 9
PK = (b"-----BEGIN RSA PRIVATE KEY-----\n" + b"MIIEow" * 12 + b"\n" + b"abcd" * 16 + b"\n"
      b"-----END RSA PRIVATE KEY-----")


def _edge_files(seed):
    rng = random.Random(seed)

    def noise(n):
        return bytes(rng.choice(b"xyz .,=;") for _ in range(n))

    files = [
        ("first_line.txt", b"k = " + AWS + b"\nnext\nmore\n"),
        ("only_line_no_nl.txt", b"t=" + GH),
        ("last_line_no_nl.txt", b"a\nb\nc\nk = " + AWS),
        ("last_line_nl.txt", b"a\nb\nc\nk = " + AWS + b"\n"),
        ("long_line.txt", b"head\n" + noise(300) + b" k = " + AWS + b" " + noise(500) + b"\ntail\n"),
        ("long_before.txt", noise(3000) + b"\n" + noise(2500) + b"\n" + noise(5000) + b" t=" + GH + b"\n" + noise(9000)),
        ("very_long_line.txt", noise(70000) + b" k = " + AWS + b" " + noise(70000)),
        ("adjacent.txt", b"x\n" + AWS + b" " + AWS + b";t=" + GH + b" " + AWS + b"\n" + b"y" * 150 + b"\n"),
        ("adjacent_long.txt", b"z" * 120 + AWS + AWS + b"," + GH + b"\n"),
        ("pk.pem", b"intro\n" + PK + b"\nafter\n" + b"k = " + AWS + b"\n"),
        ("pk_first.pem", PK + b"\n" + AWS),
        ("pk_twice.pem", b"a\n" + PK + b"\n" + PK + b"\nb\n"),
        ("blank_lines.txt", b"\n\n\n\nk = " + AWS + b"\n\n\n"),
        ("many.txt", b"\n".join(b"tok%02d ghp_%036d AKIA%016d " % (i, i * 7919 % 1000, i) for i in range(40))),
        ("cut_start.txt", AWS + b" " + noise(200) + b"\n"),
        ("cut_end.txt", noise(200) + b" " + AWS),
        ("nl_in_span_above.txt", PK + b"\nk = " + AWS + b"\n"),
        ("crlf_stripped.txt", (b"a\r\nk = " + AWS + b"\r\n").replace(b"\r", b"")),
        ("empty.txt", b""),
    ]
    for i in range(30):  # random mixes around 1-KiB window edges
        parts = []
        for _ in range(rng.randint(1, 6)):
            parts.append(noise(rng.choice([0, 1, 15, 16, 17, 63, 64, 99, 100, 101, 1000, 1023, 1024, 1025, 2100])))
            parts.append(rng.choice([b"\n", b"", b" "]))
            parts.append(rng.choice([b"k = " + AWS, b"t=" + GH, PK, b""]))
            parts.append(rng.choice([b"\n", b"", b"\n\n"]))
        files.append(("mix%02d.txt" % i, b"".join(parts)))
    return files


def _resident_scan(s, files):
    import torch
    contents = [b for _, b in files]
    paths = [p for p, _ in files]
    offs = np.zeros(len(files) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in contents])
    arena = np.frombuffer(b"".join(contents) + b"\0" * 64, dtype=np.uint8)
    d_arena = torch.from_numpy(arena.copy()).to("cuda:0")
    d_offs = torch.from_numpy(offs.view(np.int64)).to("cuda:0")
    r = s.scan_arena(arena, offs, paths, dev_arena=d_arena.data_ptr(), dev_offsets=d_offs.data_ptr())
    return r.secrets(paths), r


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_findings_edge_cases_vs_oracle_and_host(seed):
    import trivy_amd.secret as secret
    files = _edge_files(seed)
    s = secret.NewScanner(None)
    o = osc.new_scanner(None)
    assert s.set_gpu_findings(True) == 0  # (the default: on the host)
    gpu, r = _resident_scan(s, files)
    s.set_gpu_findings(False)
    host, _ = _resident_scan(s, files)
    s.set_gpu_findings(0)
    n = 0
    for (p, b), g, h in zip(files, gpu, host):
        want = o.scan(p, b)
        assert g.to_dict() == want, p
        assert h.to_dict() == want, p
        n += len(want["Findings"] or [])
    assert n > 80
    assert r.stats()["findings"] == n


def test_gpu_findings_dense_corpus_vs_oracle():
    """A corpus whose files hold many findings each (the C3f shape on builtin rules)."""
    import trivy_amd.secret as secret
    from tests.corpus import make_corpus
    rng = random.Random(5)
    files = []
    for p, b in make_corpus(77, 120):
        b = b.replace(b"\r", b"")
        cuts = sorted(rng.randrange(0, len(b) + 1) for _ in range(rng.randint(0, 25)))
        out, last = [], 0
        for c in cuts:
            out.append(b[last:c])
            out.append(rng.choice([b"k=" + AWS, b" t=" + GH + b" ", b"\n" + PK + b"\n", AWS]))
            last = c
        out.append(b[last:])
        files.append((p, b"".join(out)))
    s = secret.NewScanner(None)
    s.set_gpu_findings(True)
    o = osc.new_scanner(None)
    got, _ = _resident_scan(s, files)
    n = 0
    for (p, b), g in zip(files, got):
        want = o.scan(p, b)
        assert g.to_dict() == want, p
        n += len(want["Findings"] or [])
    assert n > 400
