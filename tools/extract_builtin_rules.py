#!/usr/bin/env python3
"""Dev-time extractor: builtin secret rule DATA -> trivy_amd/secret/builtin_rules.json.

Reads the reference's rule table (pkg/fanal/secret/builtin-rules.go:77-849 and
builtin-allow-rules.go:3-65) as text and writes the rule data (ids, titles,
severities, categories, keyword lists and the *expanded* regex source strings)
as JSON.  Only data is emitted; the regex strings are what Go's
``regexp.MustCompile`` receives, i.e. ``fmt.Sprintf`` templates are expanded and
``MustCompileWithoutWordPrefix(s)`` becomes ``([^0-9a-zA-Z]|^)(s)``
(scanner.go:66-68).

Run once in the build container (``/root/reference`` is present there only):
    python tools/extract_builtin_rules.py /root/reference
"""
import json
import re
import sys
from pathlib import Path


def go_string(tok: str) -> str:
    """Decode a Go string literal (raw `...` or interpreted "...")."""
    if tok.startswith("`"):
        return tok[1:-1]
    assert tok.startswith('"') and tok.endswith('"'), tok
    body = tok[1:-1]
    out, i = [], 0
    simple = {"n": "\n", "t": "\t", "r": "\r", "\\": "\\", '"': '"', "'": "'",
              "a": "\a", "b": "\b", "f": "\f", "v": "\v"}
    while i < len(body):
        c = body[i]
        if c == "\\":
            n = body[i + 1]
            if n in simple:
                out.append(simple[n]); i += 2; continue
            if n == "x":
                out.append(chr(int(body[i + 2:i + 4], 16))); i += 4; continue
            if n == "u":
                out.append(chr(int(body[i + 2:i + 6], 16))); i += 6; continue
            raise ValueError("unsupported escape in %r" % tok)
        out.append(c); i += 1
    return "".join(out)


STR_TOK = r'(`[^`]*`|"(?:[^"\\]|\\.)*")'


def extract(ref_root: str) -> dict:
    """The builtin rule data of the reference tree at ref_root (what builtin_rules.json holds)."""
    src = Path(ref_root, "pkg/fanal/secret/builtin-rules.go").read_text()
    allow_src = Path(ref_root, "pkg/fanal/secret/builtin-allow-rules.go").read_text()

    cats = {m.group(1): go_string(m.group(2)) for m in re.finditer(
        r'(Category\w+)\s*=\s*types\.SecretRuleCategory\(' + STR_TOK + r'\)', src)}
    consts = {}
    cblock = re.search(r"// Reusable regex patterns\nconst \((.*?)\n\)", src, re.S).group(1)
    for m in re.finditer(r'(\w+)\s*=\s*' + STR_TOK, cblock):
        consts[m.group(1)] = go_string(m.group(2))
    start_word = consts["startWord"]

    body = src[src.index("var builtinRules = []Rule{"):]
    entries = re.split(r"\n\t\{\n", body)[1:]
    rules = []
    for e in entries:
        e = e.split("\n\t},")[0]
        rule = {}
        rule["id"] = go_string(re.search(r"ID:\s*" + STR_TOK, e).group(1))
        rule["category"] = cats[re.search(r"Category:\s*(\w+)", e).group(1)]
        rule["title"] = go_string(re.search(r"Title:\s*" + STR_TOK, e).group(1))
        sm = re.search(r"Severity:\s*" + STR_TOK, e)
        rule["severity"] = go_string(sm.group(1)) if sm else ""  # ionic-api-token has none
        m = re.search(r"Regex:\s*(MustCompileWithoutWordPrefix|MustCompile)\((.*)\),\n", e)
        fn, arg = m.group(1), m.group(2).strip()
        if arg.startswith("fmt.Sprintf("):
            inner = arg[len("fmt.Sprintf("):-1]
            tm = re.match(STR_TOK + r"\s*,\s*(.*)$", inner)
            tmpl = go_string(tm.group(1))
            args = [a.strip() for a in tm.group(2).split(",")]
            vals = [consts[a] for a in args]
            assert tmpl.count("%s") == len(vals)
            for v in vals:
                tmpl = tmpl.replace("%s", v, 1)
            pat = tmpl
        else:
            pat = go_string(arg)
        if fn == "MustCompileWithoutWordPrefix":
            pat = "%s(%s)" % (start_word, pat)
        rule["regex"] = pat
        g = re.search(r"SecretGroupName:\s*" + STR_TOK, e)
        rule["secret_group_name"] = go_string(g.group(1)) if g else ""
        km = re.search(r"Keywords:\s*\[\]string\{(.*)\}", e)
        rule["keywords"] = [go_string(t) for t in re.findall(STR_TOK, km.group(1))] if km else []
        rules.append(rule)

    allow = []
    abody = allow_src[allow_src.index("var builtinAllowRules"):]
    for e in re.split(r"\n\t\{\n", abody)[1:]:
        e = e.split("\n\t},")[0]
        r = {"id": go_string(re.search(r"ID:\s*" + STR_TOK, e).group(1)),
             "description": go_string(re.search(r"Description:\s*" + STR_TOK, e).group(1))}
        pm = re.search(r"Path:\s*MustCompile\(" + STR_TOK + r"\)", e)
        rm = re.search(r"Regex:\s*MustCompile\(" + STR_TOK + r"\)", e)
        r["path"] = go_string(pm.group(1)) if pm else None
        r["regex"] = go_string(rm.group(1)) if rm else None
        allow.append(r)

    return {
        "source": "undistro/trivy@2024-12-20 pkg/fanal/secret/builtin-rules.go:101-849, "
                  "builtin-allow-rules.go:3-65 (expanded regex source strings)",
        "rules": rules,
        "allow_rules": allow,
    }


DST = Path(__file__).resolve().parent.parent / "trivy_amd/secret/builtin_rules.json"


def main(ref_root: str) -> None:
    out = extract(ref_root)
    rules, allow, dst = out["rules"], out["allow_rules"], DST
    dst.write_text(json.dumps(out, indent=1, ensure_ascii=False) + "\n")
    print("wrote %d rules, %d allow rules -> %s" % (len(rules), len(allow), dst))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
