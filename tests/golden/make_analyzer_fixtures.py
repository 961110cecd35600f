#!/usr/bin/env python3
"""Dev-time converter: the reference's secret-analyzer golden tests -> fixtures.

Source (read as data, in the build container only):
  pkg/fanal/analyzer/secret/secret_test.go:16-258  (6 Analyze + 5 Required cases)
  pkg/fanal/analyzer/secret/testdata/*              (inputs and configs)

Outputs (committed; the GPU box never reads /root/reference):
  tests/golden/analyzer/testdata/...  text inputs and YAML configs, copied verbatim
  tests/golden/analyzer/testdata/secret.cpython-310.pyc.data (content of the case's .pyc path)
      NOT the reference's file: a synthetic binary made of the printable runs
      (> 4 bytes) that utils.ExtractPrintableBytes finds in it, separated by NUL
      bytes, so the extracted text -- all the analyzer scans -- is identical
  tests/golden/analyzer_cases.json  expected results, transcribed from the Go
      struct literals of secret_test.go:17-176 (wantFinding1/2, wantFindingGH_PAT)
"""
import json
import shutil
from pathlib import Path

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference/pkg/fanal/analyzer/secret/testdata")
OUT = HERE / "analyzer" / "testdata"


def _line(n, content, cause=False, first=False, last=False):
    return {"Number": n, "Content": content, "IsCause": cause, "Annotation": "", "Truncated": False,
            "Highlighted": content, "FirstCause": first, "LastCause": last}


def _finding(rule, cat, title, sev, s, e, match, lines):
    return {"RuleID": rule, "Category": cat, "Severity": sev, "Title": title, "StartLine": s,
            "EndLine": e, "Code": {"Lines": lines}, "Match": match}


L2 = 'generic secret line secret="*********"'
L5 = 'credentials: { user: "username" password: "123456789" }'
WANT1 = _finding("rule1", "general", "Generic Rule", "HIGH", 2, 2, L2, [   # secret_test.go:17-56
    _line(1, "--- ignore block start ---"), _line(2, L2, True, True, True),
    _line(3, "--- ignore block stop ---")])
WANT2 = _finding("rule1", "general", "Generic Rule", "HIGH", 4, 4, 'secret="**********"', [  # :57-94
    _line(2, L2), _line(3, "--- ignore block stop ---"),
    _line(4, 'secret="**********"', True, True, True), _line(5, L5)])
WANT_PAT = _finding("github-fine-grained-pat", "GitHub", "GitHub Fine-grained personal access tokens",  # :95-104
                    "CRITICAL", 1, 1,
                    'Binary file "/testdata/secret.cpython-310.pyc" matches a rule '
                    '"GitHub Fine-grained personal access tokens"', None)  # types.Code{}: Lines nil

ANALYZE = [  # secret_test.go:106-176
    {"name": "return results", "config": "testdata/config.yaml", "file": "testdata/secret.txt", "dir": ".",
     "want": {"Secrets": [{"FilePath": "testdata/secret.txt", "Findings": [WANT1, WANT2]}]}},
    {"name": "image scan return result", "config": "testdata/image-config.yaml", "file": "testdata/secret.txt",
     "dir": "", "want": {"Secrets": [{"FilePath": "/testdata/secret.txt", "Findings": [WANT1, WANT2]}]}},
    {"name": "image scan return nil", "config": "testdata/image-config.yaml", "file": "testdata/secret.doc",
     "dir": "", "want": None},
    {"name": "return nil when no results", "config": "", "file": "testdata/secret.txt", "dir": "", "want": None},
    {"name": "skip binary file", "config": "", "file": "testdata/binaryfile", "dir": "", "want": None},
    {"name": "python binary file", "config": "testdata/skip-tests-config.yaml",
     "file": "testdata/secret.cpython-310.pyc", "dir": "",
     "want": {"Secrets": [{"FilePath": "/testdata/secret.cpython-310.pyc", "Findings": [WANT_PAT]}]}},
]
REQUIRED = [  # secret_test.go:200-258 (config testdata/skip-tests-config.yaml)
    {"name": "pass regular file", "file": "testdata/secret.txt", "want": True},
    {"name": "skip small file", "file": "testdata/emptyfile", "want": False},
    {"name": "skip folder", "file": "testdata/node_modules/secret.txt", "want": False},
    {"name": "skip file", "file": "testdata/package-lock.json", "want": False},
    {"name": "skip extension", "file": "testdata/secret.doc", "want": False},
]


def printable_runs(data: bytes):
    runs, cur = [], bytearray()
    for b in data:
        if 0x20 <= b <= 0x7E or (b >= 0xA1 and b != 0xAD):
            cur.append(b)
            continue
        if len(cur) > 4:
            runs.append(bytes(cur))
        cur = bytearray()
    if len(cur) > 4:
        runs.append(bytes(cur))
    return runs


def main():
    (OUT / "node_modules").mkdir(parents=True, exist_ok=True)
    for name in ["config.yaml", "image-config.yaml", "skip-tests-config.yaml", "secret.txt", "secret.doc",
                 "binaryfile", "emptyfile", "package-lock.json", "node_modules/secret.txt"]:
        shutil.copyfile(REF / name, OUT / name)
    runs = printable_runs((REF / "secret.cpython-310.pyc").read_bytes())
    # stored under another name: *.pyc files are Python caches to git and gpurun
    (OUT / "secret.cpython-310.pyc.data").write_bytes(b"\x00\x00\x00\x00" + b"\x00".join(runs) + b"\x00")
    (HERE / "analyzer_cases.json").write_text(json.dumps({"analyze": ANALYZE, "required": REQUIRED}, indent=1))
    print("wrote", OUT, "and analyzer_cases.json")


if __name__ == "__main__":
    main()
