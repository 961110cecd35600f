"""Builtin rule data and rule-compiler robustness (CPU).

* builtin_rules.json must be exactly what tools/extract_builtin_rules.py reads
  out of the reference (pkg/fanal/secret/builtin-rules.go:101-849,
  builtin-allow-rules.go:3-65) when the reference tree is present (build
  container only); this pins the 75 builtin rules no golden finding covers.
* Regression tests for rule shapes the compiler must survive.
"""
import ctypes as c
import json
import os
import sys
from pathlib import Path

import pytest

from trivy_amd import _lib
from trivy_amd.secret.config import AllowRule, Rule, builtin_allow_rules, builtin_rules
from trivy_amd.secret.scanner import CGlobal

ROOT = Path(__file__).resolve().parent.parent
REF = Path("/root/reference")


@pytest.mark.skipif(not (REF / "pkg/fanal/secret/builtin-rules.go").exists(), reason="reference tree absent")
def test_builtin_rules_json_reproduces_from_reference():
    sys.path.insert(0, str(ROOT / "tools"))
    try:
        import extract_builtin_rules as ex
    finally:
        sys.path.pop(0)
    want = ex.extract(str(REF))
    have = json.loads((ROOT / "trivy_amd/secret/builtin_rules.json").read_text())
    assert have == want


def test_builtin_rules_shape():
    rules, allow = builtin_rules(), builtin_allow_rules()
    assert len(rules) == 87 and len(allow) == 12
    assert len({r.ID for r in rules}) == 87
    for r in rules:
        assert r.Regex and r.ID and r.Title and r.Category
        _lib.regex_match(r.Regex, b"")  # compiles under the Go-syntax engine
    assert sum(1 for r in rules if r.SecretGroupName == "secret") == 50


def _compile(rules):
    L = _lib.lib()
    cg = CGlobal(rules, [], [])
    h = c.c_void_p()
    L.tsg_debug_compile.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    rc = L.tsg_debug_compile(c.byref(cg.g), c.byref(h))
    assert rc == 0, _lib.last_error()
    L.tsg_debug_compiled_free.argtypes = [c.c_void_p]
    L.tsg_debug_compiled_free(h)


def test_compile_long_literal_rule_terminates():
    # a 300-char literal: each char is a {1,1} element of the relaxed NFA; the
    # position budget must still be met (BuildNfa never ended)
    lit = "".join("abcdefghij"[i % 10] for i in range(300))
    _compile([Rule(ID="long", Regex=lit, Keywords=[lit[:8]])])
    _compile([Rule(ID="long2", Regex="(?i)x" + lit + "[0-9]{3}")])
    _compile([Rule(ID="alts", Regex="(" + lit + "|" + lit[::-1] + ")z")])


def test_empty_regex_is_a_regex():
    """regex: "" compiles in Go (Regexp.UnmarshalYAML) and matches everywhere."""
    _compile([Rule(ID="empty", Regex="")])


def test_empty_allow_path_allows_everything():
    from tests.test_host_tail import host_tail_scan
    from oracle import secret_scanner as osc
    from oracle.goregexp import GoRegexp
    from trivy_amd.secret.config import Config
    cfg = Config(CustomAllowRules=[AllowRule(ID="all", Path="")])
    files = [("a/b.txt", b"ghp_" + b"a" * 36), ("c.go", b"AKIA" + b"B" * 16)]
    got = host_tail_scan(cfg, files)
    o = osc.new_scanner(None)
    o.allow_rules.append(osc.AllowRule(id="all", path=GoRegexp("")))
    for (p, b), g in zip(files, got):
        assert g.to_dict() == o.scan(p, b)
        assert g.FilePath == p and g.Findings is None  # Secret{FilePath}: allowed path
