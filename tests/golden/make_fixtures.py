#!/usr/bin/env python3
"""Dev-time converter: the reference's secret-scanner golden tests -> JSON fixtures.

Sources (read as text, in the build container only):
  * pkg/fanal/secret/scanner_test.go:22-1351   (40 table cases, expected types.Secret)
  * pkg/fanal/secret/testdata/*                (input files + YAML configs, copied verbatim)
  * integration/testdata/secrets.json.golden + fixtures/repo/secrets/*  (CLI golden)

Outputs (committed; the GPU box never reads /root/reference):
  tests/golden/scanner/<testdata files>
  tests/golden/scanner_cases.json
  tests/golden/integration/{deploy.sh,trivy-secret.yaml,secrets.json}

Only data leaves this script: expected findings are decoded from the Go struct
literals of the test file into plain JSON (field names as in pkg/fanal/types).
"""
import json
import re
import shutil
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent


class GoLit:
    """Tiny recursive-descent reader for the composite literals used in scanner_test.go."""

    TOK = re.compile(r'\s*(`[^`]*`|"(?:[^"\\]|\\.)*"|[A-Za-z_][\w.]*|\d+|\[\]|[{}(),:])', re.S)

    def __init__(self, text, env, cats):
        self.toks = []
        pos = 0
        while True:
            m = self.TOK.match(text, pos)
            if not m:
                rest = text[pos:].strip()
                assert rest == "", rest[:80]
                break
            self.toks.append(m.group(1))
            pos = m.end()
        self.i = 0
        self.env = env
        self.cats = cats

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else None

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def expect(self, t):
        got = self.next()
        assert got == t, (got, t, self.toks[self.i - 5:self.i + 5])

    def value(self):
        t = self.next()
        if t.startswith('"') or t.startswith("`"):
            return go_string(t)
        if t.isdigit():
            return int(t)
        if t in ("true", "false"):
            return t == "true"
        if t == "nil":
            return None
        if t == "[]":
            typ = self.next()  # element type
            return self.composite(list_of=typ)
        if t == "filepath.Join":
            self.expect("(")
            parts = []
            while self.peek() != ")":
                parts.append(self.value())
                if self.peek() == ",":
                    self.next()
            self.expect(")")
            return "/".join(parts)
        if t.startswith("secret.Category"):
            return self.cats[t.split(".", 1)[1]]
        if self.peek() == "{":
            return self.composite()
        if t in self.env:
            return self.env[t]
        raise ValueError("unknown token %r" % t)

    def composite(self, list_of=None):
        self.expect("{")
        if list_of is not None:
            out = []
            while self.peek() != "}":
                if self.peek() == "{":
                    out.append(self.composite())
                else:
                    out.append(self.value())
                if self.peek() == ",":
                    self.next()
            self.expect("}")
            return out
        out = {}
        while self.peek() != "}":
            key = self.next()
            self.expect(":")
            out[key] = self.value()
            if self.peek() == ",":
                self.next()
        self.expect("}")
        return out


def go_string(tok):
    if tok.startswith("`"):
        return tok[1:-1]
    return json.loads(tok)  # the test file uses only JSON-compatible escapes


def norm_line(line):
    return {
        "Number": line.get("Number", 0),
        "Content": line.get("Content", ""),
        "IsCause": line.get("IsCause", False),
        "Annotation": line.get("Annotation", ""),
        "Truncated": line.get("Truncated", False),
        "Highlighted": line.get("Highlighted", ""),
        "FirstCause": line.get("FirstCause", False),
        "LastCause": line.get("LastCause", False),
    }


def norm_finding(f):
    return {
        "RuleID": f.get("RuleID", ""),
        "Category": f.get("Category", ""),
        "Severity": f.get("Severity", ""),
        "Title": f.get("Title", ""),
        "StartLine": f.get("StartLine", 0),
        "EndLine": f.get("EndLine", 0),
        "Code": {"Lines": [norm_line(l) for l in (f.get("Code") or {}).get("Lines") or []]},
        "Match": f.get("Match", ""),
    }


def main(ref):
    ref = Path(ref)
    sdir = ref / "pkg/fanal/secret"
    src = (sdir / "scanner_test.go").read_text()
    rules_src = (sdir / "builtin-rules.go").read_text()
    cats = {m.group(1): json.loads(m.group(2)) for m in re.finditer(
        r'(Category\w+)\s*=\s*types\.SecretRuleCategory\(("[^"]*")\)', rules_src)}

    env = {}
    body = src[src.index("func TestSecretScanner"):]
    for m in re.finditer(r"\n\t(want\w+) := types\.SecretFinding(\{.*?\n\t\})(?=\n)", body, re.S):
        env[m.group(1)] = GoLit(m.group(2), env, cats).composite()

    tstart = body.index("tests := []struct {")
    tbody = body[tstart:]
    tbody = tbody[tbody.index("}{") + 1:]
    tbody = tbody[:tbody.index("\n\t}\n\n\tfor _, tt := range tests")] + "\n\t}"
    gl = GoLit(tbody, env, cats)
    raw_cases = gl.composite(list_of="case")

    out_dir = HERE / "scanner"
    out_dir.mkdir(exist_ok=True)
    for f in sorted((sdir / "testdata").iterdir()):
        shutil.copyfile(f, out_dir / f.name)

    cases = []
    for c in raw_cases:
        want = c.get("want") or {}
        findings = want.get("Findings")
        cases.append({
            "name": c["name"],
            "config": c["configPath"].replace("testdata/", "", 1),
            "input": c["inputFilePath"].replace("testdata/", "", 1),
            "file_path": c["inputFilePath"],
            "want": {
                "FilePath": want.get("FilePath", ""),
                "Findings": None if findings is None else [norm_finding(x) for x in findings],
            },
        })
    doc = {
        "source": "undistro/trivy@2024-12-20 pkg/fanal/secret/scanner_test.go:22-1351 "
                  "(TestSecretScanner table; inputs from pkg/fanal/secret/testdata)",
        "cases": cases,
    }
    (HERE / "scanner_cases.json").write_text(json.dumps(doc, indent=1, ensure_ascii=False) + "\n")

    idir = HERE / "integration"
    idir.mkdir(exist_ok=True)
    fx = ref / "integration/testdata/fixtures/repo/secrets"
    for name in ("deploy.sh", "trivy-secret.yaml"):
        shutil.copyfile(fx / name, idir / name)
    golden = json.loads((ref / "integration/testdata/secrets.json.golden").read_text())
    results = [{"Target": r["Target"], "Secrets": [norm_finding(s) for s in r["Secrets"]]}
               for r in golden["Results"] if r.get("Class") == "secret"]
    (idir / "secrets.json").write_text(json.dumps(
        {"source": "integration/testdata/secrets.json.golden (Results with Class=secret)",
         "results": results}, indent=1) + "\n")
    print("cases: %d, finding vars: %d" % (len(cases), len(env)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
