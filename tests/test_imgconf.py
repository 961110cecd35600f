"""Image-config secret analyzer (pkg/fanal/analyzer/imgconf/secret/secret.go:39-62).

CPU: the MarshalIndent restatement scanned by the oracle reproduces the
reference's golden cases (tests/golden/imgconf_cases.json, transcribed from
secret_test.go:15-109).  GPU: the analyzer through the engine, field for field.
"""
import json
from pathlib import Path

import pytest

from oracle import secret_scanner as osc
from trivy_amd.analyzer.imgconf import ConfigAnalysisInput, MarshalIndentConfigFile

CASES = json.loads((Path(__file__).resolve().parent / "golden/imgconf_cases.json").read_text())["cases"]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_marshal_and_oracle_match_golden(case):
    if case["config"] is None:
        assert case["want"] is None
        return
    b = MarshalIndentConfigFile(case["config"], "  ", "")
    assert b.startswith(b"{\n  \"architecture\": \"\",\n  \"created\": \"0001-01-01T00:00:00Z\",")
    got = osc.new_scanner(None).scan("config.json", b)
    if case["want"] is None:
        assert not got["Findings"]
    else:
        assert got == case["want"]["Secret"]


def test_marshal_shapes():
    b = MarshalIndentConfigFile({"architecture": "amd64", "os": "linux",
                                 "rootfs": {"type": "layers", "diff_ids": ["sha256:ab"]},
                                 "config": {"Labels": {"b": "<x>", "a": "&"}, "Volumes": {"/data": {}},
                                            "Cmd": ["sh"], "Tty": True}}).decode()
    assert '"a": "\\u0026"' in b and '"b": "\\u003cx\\u003e"' in b  # HTML-safe, sorted map keys
    assert '"/data": {}' in b and '"Tty": true' in b
    assert b.index('"Cmd"') < b.index('"Labels"') < b.index('"Tty"') < b.index('"Volumes"')


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_imgconf_analyzer_golden(case):
    from trivy_amd.analyzer.imgconf import SecretAnalyzer
    a = SecretAnalyzer("")
    got = a.Analyze(ConfigAnalysisInput(Config=case["config"]))
    if case["want"] is None:
        assert got is None
    else:
        assert got.Secret.to_dict() == case["want"]["Secret"]


def test_marshal_history_and_healthcheck():
    """v1.History and v1.HealthConfig in struct declaration order (go-containerregistry v0.20.2 tags:
    History{author, created (a v1.Time struct: never omitted), created_by, comment, empty_layer};
    HealthConfig{Test, Interval, Timeout, StartPeriod, Retries} with Go field names).  Parity
    unpinned: the reference's tests cover Env only; the expected text follows the struct tags."""
    cfg = {"architecture": "amd64", "os": "linux",
           "history": [{"created_by": "RUN echo ghp_" + "a" * 36, "comment": "c", "empty_layer": True,
                        "author": "me"},
                       {"created": "2024-01-02T03:04:05Z", "created_by": "CMD sh", "empty_layer": False}],
           "config": {"Healthcheck": {"Retries": 3, "Test": ["CMD", "true"], "Interval": 1000000000}}}
    want = "\n".join([
        '{',
        '  "architecture": "amd64",',
        '  "created": "0001-01-01T00:00:00Z",',
        '  "history": [',
        '  {',
        '  "author": "me",',
        '  "created": "0001-01-01T00:00:00Z",',
        '  "created_by": "RUN echo ghp_' + "a" * 36 + '",',
        '  "comment": "c",',
        '  "empty_layer": true',
        '  },',
        '  {',
        '  "created": "2024-01-02T03:04:05Z",',
        '  "created_by": "CMD sh"',
        '  }',
        '  ],',
        '  "os": "linux",',
        '  "rootfs": {',
        '  "type": "",',
        '  "diff_ids": null',
        '  },',
        '  "config": {',
        '  "Healthcheck": {',
        '  "Test": [',
        '  "CMD",',
        '  "true"',
        '  ],',
        '  "Interval": 1000000000,',
        '  "Retries": 3',
        '  }',
        '  }',
        '  }'])
    got = MarshalIndentConfigFile(cfg, "  ", "").decode()
    assert got == want
    res = osc.new_scanner(None).scan("config.json", got.encode())
    assert [(f["RuleID"], f["StartLine"]) for f in res["Findings"]] == [("github-pat", 8)]
