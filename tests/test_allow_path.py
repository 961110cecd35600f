"""Global AllowPath (scanner.go:57-59, 205-212) of the native scanner vs the oracle.

The native pass runs only the allow rules whose required literals can start at
some byte pair of the ASCII-lowered path (plus the rules without a usable
literal); this checks it stays exact: builtin allow paths, custom allow paths
with 1-byte / no literals, mixed case, non-ASCII and over-long paths.
"""
import random

from oracle import hostlib
from oracle import secret_scanner as osc
from trivy_amd.secret import NewScanner, ParseConfig

PIECES = ["usr", "share", "include", "lib", "local", "go", "python3.11", "gems", "src", "wordpress", "var", "log",
          "anaconda", "opt", "yarn-v1.22.0", "vendor", "locale", "locales", "test", "Test", "TESTS", "-test",
          "_test", ".test", "example", "EXAMPLE", "Examples", "a.md", "README.md", "x.mD", "node", "app", "é",
          "İ", "K", "ſ", "", "data", "docs"]


def _paths(seed, n):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        k = rng.randint(1, 6)
        p = "/".join(rng.choice(PIECES) for _ in range(k))
        if rng.random() < 0.3:
            p = "/" + p
        if rng.random() < 0.02:
            p = "d/" * 600 + p  # > 1024 bytes
        out.append(p)
    return out


def _check(cfg_path, paths):
    sc = NewScanner(ParseConfig(cfg_path) if cfg_path else None, lib=hostlib.lib(), host_only=True)
    o = osc.new_scanner(osc.parse_config(cfg_path) if cfg_path else None)
    for p in paths:
        assert sc.AllowPath(p) == o.allow_path(p), p


def test_allow_path_builtin_vs_oracle():
    _check(None, _paths(1, 4000) + ["usr/share/x", "Usr/share/x", "usr/local/lib/python3.9/a", "opt/yarn-v1./",
                                    "a.md", "a.MD", "b.md/c", "x/vendor/y", "testing", "ztest", "example"])


def test_allow_path_custom_rules_vs_oracle(tmp_path):
    cfg_path = tmp_path / "trivy-secret.yaml"
    cfg_path.write_text(
        "allow-rules:\n"
        "  - id: one-byte\n    description: d\n    path: 'q'\n"
        "  - id: no-literal\n    description: d\n    path: '^[a-c]+/[0-9]'\n"
        "  - id: alt\n    description: d\n    path: '(?i)(node|APP)/d'\n"
        "  - id: anchored\n    description: d\n    path: '^docs/.*\\.txt$'\n")
    _check(str(cfg_path), _paths(2, 3000) + ["abc/1", "q", "NODE/d", "app/D", "docs/x.txt", "Docs/x.txt", "ab/x"])
