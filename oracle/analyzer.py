"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the secret analyzer's CPU path around Scanner.Scan
(undistro/trivy @ 2024-12-20):

* pkg/fanal/analyzer/secret/secret.go:28-62   skip lists
* pkg/fanal/analyzer/secret/secret.go:86-150  Init / Analyze
* pkg/fanal/analyzer/secret/secret.go:152-190 Required
* pkg/fanal/utils/utils.go:85-103, 128-160    IsBinary / ExtractPrintableBytes
* pkg/fanal/walker/tar.go:35-103              LayerTar.Walk (whiteouts, regular files)
* pkg/fanal/analyzer/analyzer.go:403-455      AnalyzeFile (Required gate, Dir "")

Tar headers are read with CPython's ``tarfile`` (an implementation independent
of the native walker), and Go's ``path.Clean`` / ``filepath.Ext`` / ``Base`` are
restated below.  Pinned by pkg/fanal/analyzer/secret/secret_test.go:16-258
(tests/golden/analyzer_cases.json, tests/test_oracle_golden.py).
"""
import io
import tarfile

from . import secret_scanner as osc

SKIP_FILES = ["go.mod", "go.sum", "package-lock.json", "yarn.lock", "pnpm-lock.yaml",
              "Pipfile.lock", "Gemfile.lock"]  # secret.go:29-37
SKIP_DIRS = [".git", "node_modules"]  # secret.go:38-41
SKIP_EXTS = [".jpg", ".png", ".gif", ".doc", ".pdf", ".bin", ".svg", ".socket", ".deb", ".rpm",
             ".zip", ".gz", ".gzip", ".tar"]  # secret.go:42-57
ALLOWED_BINARIES = [".pyc"]  # secret.go:59-61


def go_ext(p: str) -> str:  # path/filepath.Ext
    i = len(p) - 1
    while i >= 0 and p[i] != "/":
        if p[i] == ".":
            return p[i:]
        i -= 1
    return ""


def go_base(p: str) -> str:  # path/filepath.Base
    if p == "":
        return "."
    p = p.rstrip("/")
    if p == "":
        return "/"
    return p.rsplit("/", 1)[-1]


def go_path_clean(p: str) -> str:  # path.Clean: lexical processing, rooted ".." dropped
    if p == "":
        return "."
    rooted = p.startswith("/")
    parts = []
    for e in p.split("/"):
        if e in ("", "."):
            continue
        if e == "..":
            if parts and parts[-1] != "..":
                parts.pop()
            elif not rooted:
                parts.append("..")
            continue
        parts.append(e)
    out = ("/" if rooted else "") + "/".join(parts)
    return out if out else "."


def is_binary(content: bytes, size: int) -> bool:  # utils.go:85-103
    for b in content[:min(size, 300)]:
        if b < 7 or b == 11 or 13 < b < 27 or 27 < b < 0x20 or b == 0x7F:
            return True
    return False


def _is_print_byte(b: int) -> bool:  # unicode.IsPrint(rune(b)) for b < 256
    return 0x20 <= b <= 0x7E or (b >= 0xA1 and b != 0xAD)


def extract_printable_bytes(content: bytes) -> bytes:  # utils.go:128-160 (minLength = 4)
    out = bytearray()
    cur = bytearray()
    for b in content:
        if _is_print_byte(b):
            cur.append(b)
            continue
        if len(cur) > 4:
            out += cur + b"\n"
        cur = bytearray()
    if len(cur) > 4:
        out += cur + b"\n"
    return bytes(out)


class SecretAnalyzer:
    def __init__(self, config_path=""):  # Init, secret.go:86-101
        cfg = osc.parse_config(config_path)
        self.scanner = osc.new_scanner(cfg)
        self.config_path = config_path

    def required(self, file_path: str, size: int) -> bool:  # secret.go:152-190
        if size < 10:
            return False
        k = file_path.rfind("/")
        d, name = file_path[:k + 1], file_path[k + 1:]
        dirs = d.split("/")
        if any(s in dirs for s in SKIP_DIRS):
            return False
        if name in SKIP_FILES:
            return False
        if go_base(self.config_path) == file_path:
            return False
        if go_ext(name) in SKIP_EXTS:
            return False
        if self.scanner.allow_path(file_path):
            return False
        return True

    def prepare(self, file_path: str, dir_: str, content: bytes):
        """Analyze up to the Scan call (secret.go:103-136): None when skipped, else ScanArgs."""
        binary = is_binary(content, len(content))
        if binary and go_ext(file_path) not in ALLOWED_BINARIES:
            return None
        if not binary:
            data = content.replace(b"\r", b"")
        else:
            data = extract_printable_bytes(content)
        if dir_ == "":
            file_path = "/" + file_path
        return file_path, data, binary

    def analyze(self, file_path: str, dir_: str, content: bytes):  # secret.go:103-150
        args = self.prepare(file_path, dir_, content)
        if args is None:
            return None
        res = self.scanner.scan(args[0], args[1], args[2])
        if not res["Findings"]:
            return None
        return {"Secrets": [res]}


def walk_layer_tar(data: bytes):
    """LayerTar.Walk (walker/tar.go:35-103) with no skip paths: the regular files, as
    (filePath, size, content), plus the whiteout / opaque-dir counts."""
    files, wh, opq = [], 0, 0
    with tarfile.open(fileobj=io.BytesIO(data), mode="r:") as tf:
        for m in tf:
            name = m.name
            fp = go_path_clean(name).lstrip("/")
            fname = fp.rsplit("/", 1)[-1]
            if fname == ".wh..wh..opq":
                opq += 1
                continue
            if fname.startswith(".wh."):
                wh += 1
                continue
            if m.type not in (tarfile.REGTYPE, tarfile.AREGTYPE):  # Go: TypeReg (TypeRegA -> TypeReg)
                continue
            files.append((fp, m.size, tf.extractfile(m).read()))
    return files, wh, opq


def analyze_layer(analyzer: SecretAnalyzer, data: bytes):
    """The image-layer path: AnalyzeFile(dir="") for every walked regular file
    (analyzer.go:403-455).  Returns [(scan path, secret dict)] for files with findings."""
    out = []
    files, _, _ = walk_layer_tar(data)
    for fp, size, content in files:
        if not analyzer.required(fp, size):
            continue
        r = analyzer.analyze(fp, "", content)
        if r is not None:
            out.append(r["Secrets"][0])
    return out


# ---- FS.Walk (pkg/fanal/walker/fs.go:25-78), restated with os.scandir ----
DEFAULT_SKIP_DIRS = ["**/.git", "proc", "sys", "dev"]  # walker/walk.go:11-16


def doublestar_regex(pattern: str):
    """doublestar.Match (github.com/bmatcuk/doublestar/v4) as a Python regex over the whole
    path, by translation (an independent restatement of the native matcher): '**' as a whole
    component = zero or more directories ("a/**" also matches "a"), '*' / '?' / '[...]' never
    cross '/', '{a,b}' alternatives, '\\' escapes.  None for a malformed pattern."""
    import re
    out, i, n, depth = [], 0, len(pattern), 0
    while i < n:
        ch = pattern[i]
        comp = i == 0 or pattern[i - 1] == "/"
        if ch == "*" and comp and pattern[i:i + 2] == "**" and (i + 2 == n or pattern[i + 2] == "/"):
            if i + 2 == n:
                out.append(".*")
                i += 2
            else:
                out.append("(?:[^/]*/)*")  # zero or more whole components
                i += 3
            continue
        if ch == "/" and pattern[i:] == "/**":
            out.append("(?:/.*)?")
            i = n
            continue
        if ch == "*":
            out.append("[^/]*")
        elif ch == "?":
            out.append("[^/]")
        elif ch == "[":
            j = i + 1
            neg = j < n and pattern[j] in "!^"
            if neg:
                j += 1
            items, first = [], True
            while True:
                if j >= n:
                    return None
                if pattern[j] == "]" and not first:
                    break
                first = False
                if pattern[j] == "\\":
                    if j + 1 >= n:
                        return None
                    lo = pattern[j + 1]
                    j += 2
                else:
                    lo = pattern[j]
                    j += 1
                hi = lo
                if j + 1 < n and pattern[j] == "-" and pattern[j + 1] != "]":
                    if pattern[j + 1] == "\\":
                        if j + 2 >= n:
                            return None
                        hi = pattern[j + 2]
                        j += 3
                    else:
                        hi = pattern[j + 1]
                        j += 2
                items.append(re.escape(lo) + ("-" + re.escape(hi) if hi != lo else ""))
            cls = "".join(items)
            out.append("(?!/)[^%s]" % cls if neg else "(?=[^/])[%s]" % cls)
            i = j + 1
            continue
        elif ch == "{":
            out.append("(?:")
            depth += 1
        elif ch == "}" and depth:
            out.append(")")
            depth -= 1
        elif ch == "," and depth:
            out.append("|")
        elif ch == "\\":
            if i + 1 >= n:
                return None
            out.append(re.escape(pattern[i + 1]))
            i += 2
            continue
        else:
            out.append(re.escape(ch))
        i += 1
    if depth:
        return None
    return re.compile("(?s)" + "".join(out) + r"\Z")


def skip_path(path: str, patterns) -> bool:  # utils.SkipPath, utils.go:112-126
    path = path.lstrip("/")
    for p in patterns:
        rx = doublestar_regex(p)
        if rx is None:
            return False
        if rx.match(path):
            return True
    return False


def walk_fs(root: str, skip_dirs=(), skip_files=()):
    """FS.Walk + WalkDirFunc (fs.go:25-78): [(relPath, size)] of the regular files in
    filepath.WalkDir order (entries by name, directories not followed through symlinks),
    skip patterns already relative to root (BuildSkipPaths applied), defaultSkipDirs added,
    permission errors ignored."""
    import os
    import stat as st_
    skip_dirs = list(skip_dirs) + DEFAULT_SKIP_DIRS
    out = []
    rs = os.lstat(root)
    if not st_.S_ISDIR(rs.st_mode):
        if st_.S_ISREG(rs.st_mode) and not skip_path(".", skip_files):
            out.append((os.path.basename(root), rs.st_size))
        return out
    if skip_path(".", skip_dirs):  # WalkDir's first call is the root itself, relPath "." (fs.go:51-55)
        return out

    def walk(abs_dir, rel):
        try:
            names = sorted(os.listdir(abs_dir), key=lambda x: x.encode("utf-8", "surrogateescape"))
        except PermissionError:
            return
        for name in names:
            p = os.path.join(abs_dir, name)
            r = name if rel == "." else rel + "/" + name
            try:
                s = os.lstat(p)
            except FileNotFoundError:
                continue
            if st_.S_ISDIR(s.st_mode):
                if skip_path(r, skip_dirs):
                    continue
                walk(p, r)
            elif not st_.S_ISREG(s.st_mode):
                continue
            elif skip_path(r, skip_files):
                continue
            else:
                out.append((r, s.st_size))
    walk(root, ".")
    return out


def analyze_fs(analyzer: SecretAnalyzer, root: str, skip_dirs=(), skip_files=()):
    """`trivy fs` for the secret analyzer (artifact/local/fs.go:87-100 -> AnalyzeFile(dir=root)):
    [secret dict] of the files with findings, sorted as AnalysisResult.Sort."""
    import os
    out = []
    files = walk_fs(root, skip_dirs, skip_files)
    is_file = not os.path.isdir(root)
    # a file root: dir, filePath = path.Split(rootPath) (artifact/local/fs.go:90-93)
    dir_ = root[:root.rfind("/") + 1] if is_file else root
    for rel, size in files:
        if not analyzer.required(rel, size):
            continue
        with open(root if is_file else os.path.join(root, rel), "rb") as f:
            content = f.read()
        r = analyzer.analyze(rel, dir_, content)
        if r is not None:
            out.append(r["Secrets"][0])
    out.sort(key=lambda s: s["FilePath"].encode("utf-8", "surrogateescape")
             if isinstance(s["FilePath"], str) else s["FilePath"])
    for s in out:
        s["Findings"].sort(key=lambda f: (f["RuleID"], f["StartLine"]))
    return out
