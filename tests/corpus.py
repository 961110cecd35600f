"""Small deterministic synthetic corpora for parity tests (test helper).

Mirrors the generator spec of SURVEY.md §8(d) at test scale: source-like
text with keyword collisions ("key", "task", "global", "live_", "-----",
"pk."), prose, base64/hex/JSON blobs, a share of UTF-8 (incl. U+0130,
U+212A, U+017F and invalid bytes), CRLF files (stripped before Scan, as the
analyzer does), long and minified lines, and planted secrets sampled from the
builtin rule regexes (some inside allow-listed paths).
"""
import base64
import json
import random
from pathlib import Path

from tests.regex_sampler import sample_regex

ROOT = Path(__file__).resolve().parent.parent
BUILTIN = json.loads((ROOT / "trivy_amd/secret/builtin_rules.json").read_text())

WORDS = ("key value task ask desk global blob live_ pk. config token secret password user name "
         "return function import from class def self data index buffer apikey access_key "
         "aws github slack stripe heroku twitter facebook discord linear lob mailgun hf_ sk "
         "SG. msg. eyJ dapi -----").split()
PATHS = ["src/main.py", "lib/util.go", "app/config.yaml", "deploy/run.sh", "web/index.js", "README.md",
         "test/fixtures.txt", "vendor/x/y.go", "docs/notes.txt", "pkg/service/handler.go", "examples/a.py",
         "etc/app.conf", "cmd/tool/main.go", "src/.env", "scripts/setup.sh"]


def _line(rng):
    n = max(1, int(rng.expovariate(1 / 6)))
    s = " ".join(rng.choice(WORDS) for _ in range(n))
    r = rng.random()
    if r < 0.1:
        s = "    " + s + " = '" + "".join(rng.choice("abcdef0123456789") for _ in range(rng.randint(4, 40))) + "'"
    elif r < 0.15:
        s = s + ": " + base64.b64encode(bytes(rng.getrandbits(8) for _ in range(rng.randint(8, 60)))).decode()
    return s


def make_file(rng, planted_rate=0.3, utf8_rate=0.1):
    lines = [_line(rng) for _ in range(rng.randint(0, 40))]
    if rng.random() < 0.02:
        lines.append("x" * rng.randint(100, 3000))  # long line
    if rng.random() < utf8_rate:
        specials = ["İ", "K", "ſ", "é", "日本語", "\udcff", "\udcc3", "naïve", "AKİA", "kEY", "ſk_live_"]
        for _ in range(rng.randint(1, 5)):
            i = rng.randint(0, len(lines))
            lines.insert(i, rng.choice(specials) + " " + _line(rng))
    text = "\n".join(lines)
    b = text.encode("utf-8", "surrogateescape")
    parts = [b]
    while rng.random() < planted_rate:
        rule = rng.choice(BUILTIN["rules"])
        sec = sample_regex(rule["regex"], rng, maxrep=4)
        pre = rng.choice([b" ", b"\n", b"=", b'"', b"export X=", b"", b"\t"])
        post = rng.choice([b" ", b"\n", b'"', b"", b".", b"\n\n"])
        pos = rng.randint(0, len(parts))
        parts.insert(pos, pre + sec + post)
    content = b"".join(parts)
    if rng.random() < 0.05:
        content = content.replace(b"\n", b"\r\n")
    return content


def make_corpus(seed, n_files, **kw):
    rng = random.Random(seed)
    files = []
    for i in range(n_files):
        path = rng.choice(PATHS)
        if rng.random() < 0.5:
            path = "d%d/%s" % (i, path)
        files.append((path, make_file(rng, **kw)))
    return files
