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


def test_config_scalars_decode_as_source_text(tmp_path):
    """ParseConfig decodes with gopkg.in/yaml.v3 into Go string fields (scanner.go:89-100) and
    Regexp.UnmarshalYAML compiles value.Value (:75-87): a scalar is its source text -- no YAML 1.1
    typing (0x1F -> 31, on -> True, 1_000 -> 1000) -- and only a plain null is the zero value.
    Checked for the mirror (trivy_amd.secret.config) and the oracle, then through the exact tail."""
    from oracle import secret_scanner as osc
    from trivy_amd.secret import ParseConfig
    p = tmp_path / "trivy-secret.yaml"
    p.write_text("rules:\n"
                 "  - id: 0\n    category: 1.50\n    title: true\n    severity: high\n"
                 "    regex: 0x1F\n    keywords: [1_000, on, 'null', ~, 007]\n"
                 "  - id: ~\n    title: null\n    category: 'null'\n    regex: '[a-z]+_0x1F'\n"
                 "    secret-group-name: ''\n"
                 "disable-rules: [no, 12]\n"
                 "allow-rules:\n  - id: yes\n    path: 0o17\n")
    m = ParseConfig(str(p))
    r0, r1 = m.CustomRules
    assert (r0.ID, r0.Category, r0.Title, r0.Severity, r0.Regex) == ("0", "1.50", "true", "HIGH", "0x1F")
    assert r0.Keywords == ["1_000", "on", "null", "", "007"]
    assert (r1.ID, r1.Title, r1.Category, r1.Regex, r1.SecretGroupName) == ("", "", "null", "[a-z]+_0x1F", "")
    assert m.DisableRuleIDs == ["no", "12"]
    assert (m.CustomAllowRules[0].ID, m.CustomAllowRules[0].Path) == ("yes", "0o17")
    o = osc.parse_config(str(p))
    q0, q1 = o.custom_rules
    assert (q0.id, q0.category, q0.title, q0.severity) == ("0", "1.50", "true", "HIGH")
    assert q0.keywords == ["1_000", "on", "null", "", "007"]
    assert (q1.id, q1.title, q1.category, q1.secret_group_name) == ("", "", "null", "")
    assert o.disable_rule_ids == ["no", "12"]
    assert o.custom_allow_rules[0].id == "yes"
    # the regex is the text 0x1F (matches "0x1F", not "31"); keyword "on" gates it
    from tests.test_host_tail import host_tail_scan
    files = [("a.txt", b"x = 0x1F on\n"), ("b.txt", b"x = 31 on\n"), ("c.txt", b"abc_0x1F\n")]
    got = host_tail_scan(m, files)
    oc = osc.new_scanner(o)
    for (path, b), g in zip(files, got):
        assert g.to_dict() == oc.scan(path, b), path
    assert got[0].Findings and got[0].Findings[0].RuleID == "0" and got[0].Findings[0].Title == "true"
    assert not got[1].Findings
    assert got[2].Findings and got[2].Findings[0].RuleID == ""
