"""Pin the CPU oracle against the reference's own golden tests.

Cases: pkg/fanal/secret/scanner_test.go:958-1330 (40 table entries) and
integration/testdata/secrets.json.golden, transcribed by tests/golden/make_fixtures.py.
"""
import json
from pathlib import Path

import pytest

from oracle import secret_scanner as osc

G = Path(__file__).resolve().parent / "golden"
CASES = json.loads((G / "scanner_cases.json").read_text())["cases"]


def _strip_cr(b):
    return b.replace(b"\r", b"")  # analyzer/secret/secret.go:121, scanner_test.go:1337


@pytest.mark.parametrize("case", CASES, ids=[c["name"] + "|" + c["config"] for c in CASES])
def test_oracle_matches_reference_golden(case):
    cfg = osc.parse_config(str(G / "scanner" / case["config"]))
    s = osc.new_scanner(cfg)
    content = _strip_cr((G / "scanner" / case["input"]).read_bytes())
    got = s.scan(case["file_path"], content)
    assert got == case["want"]


def test_oracle_integration_golden():
    d = json.loads((G / "integration" / "secrets.json").read_text())
    cfg = osc.parse_config(str(G / "integration" / "trivy-secret.yaml"))
    s = osc.new_scanner(cfg)
    for res in d["results"]:
        content = _strip_cr((G / "integration" / res["Target"]).read_bytes())
        got = s.scan(res["Target"], content)
        assert got["Findings"] == res["Secrets"]
