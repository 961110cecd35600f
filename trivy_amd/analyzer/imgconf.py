"""Image-config secret analyzer: pkg/fanal/analyzer/imgconf/secret/secret.go over the engine.

The second caller of the secret Scanner ("must keep working"):
``Analyze`` marshals the image's v1.ConfigFile with ``json.MarshalIndent(cfg,
"  ", "")`` (secret.go:43-46) and scans it as ``config.json`` (:48-51); no
findings -> ``None`` (:53-56).

The v1.ConfigFile / v1.Config / v1.RootFS shapes and JSON tags follow
github.com/google/go-containerregistry v0.20.2 (go.mod:55, not vendored in the
reference): field order, ``omitempty`` and Time's RFC 3339 form decide every
line number of the scanned text.  The reference's three test cases
(imgconf/secret/secret_test.go:15-109) pin the Env-only shape
(tests/golden/imgconf_cases.json); other fields are restated from the
library's published struct tags (parity unpinned beyond the fixtures).
"""
import json
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from ..secret import NewScanner, ParseConfig, ScanArgs, Secret

TypeImageConfigSecret = "imgconf-secret"  # pkg/fanal/analyzer/const.go
analyzerVersion = 1                       # secret.go:15

# (json name, Go kind, omitempty) in declaration order
_CONFIG_FILE = [("architecture", "str", False), ("author", "str", True), ("container", "str", True),
                ("created", "time", True), ("docker_version", "str", True), ("history", "history", True),
                ("os", "str", False), ("rootfs", "rootfs", False), ("config", "config", False),
                ("os.version", "str", True), ("variant", "str", True), ("os.features", "list", True)]
_ROOTFS = [("type", "str", False), ("diff_ids", "list_null", False)]
_CONFIG = [("AttachStderr", "bool", True), ("AttachStdin", "bool", True), ("AttachStdout", "bool", True),
           ("Cmd", "list", True), ("Healthcheck", "health", True), ("Domainname", "str", True),
           ("Entrypoint", "list", True), ("Env", "list", True), ("Hostname", "str", True), ("Image", "str", True),
           ("Labels", "map", True), ("OnBuild", "list", True), ("OpenStdin", "bool", True),
           ("StdinOnce", "bool", True), ("Tty", "bool", True), ("User", "str", True), ("Volumes", "map", True),
           ("WorkingDir", "str", True), ("ExposedPorts", "map", True), ("ArgsEscaped", "bool", True),
           ("NetworkDisabled", "bool", True), ("MacAddress", "str", True), ("StopSignal", "str", True),
           ("Shell", "list", True)]
# v1.History (struct fields in declaration order; Created is a v1.Time struct, so
# omitempty never drops it: an unset time marshals as the zero time)
_HISTORY = [("author", "str", True), ("created", "time", True), ("created_by", "str", True),
            ("comment", "str", True), ("empty_layer", "bool", True)]
# v1.HealthConfig (no JSON names: the field names; time.Duration marshals as int64 nanoseconds)
_HEALTH = [("Test", "list", True), ("Interval", "int", True), ("Timeout", "int", True),
           ("StartPeriod", "int", True), ("Retries", "int", True)]
_ZERO_TIME = "0001-01-01T00:00:00Z"


def _go_string(s: str) -> str:
    """encoding/json string: HTML-safe escaping (<, >, & as \\u00XX; U+2028/9)."""
    out = json.dumps(s, ensure_ascii=False)
    return (out.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
            .replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))


def _value(v) -> Any:
    """A Go-marshalled value as a tree: ("obj", [(k, v)]), ("arr", [v]) or a JSON scalar text."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return json.dumps(v)
    if isinstance(v, str):
        return _go_string(v)
    if isinstance(v, dict):  # Go maps marshal with sorted keys
        return ("obj", [(k, _value(v[k])) for k in sorted(v)])
    if isinstance(v, (list, tuple)):
        return ("arr", [_value(x) for x in v])
    raise TypeError(type(v))


def _struct(fields, d: Dict[str, Any]):
    items = []
    for name, kind, omit in fields:
        v = d.get(name)
        if kind == "rootfs":
            items.append((name, _struct(_ROOTFS, v or {})))
            continue
        if kind == "config":
            items.append((name, _struct(_CONFIG, v or {})))
            continue
        if kind == "time":  # v1.Time wraps time.Time: a struct, never omitted
            items.append((name, _go_string(v or _ZERO_TIME)))
            continue
        if kind == "health":  # *HealthConfig: omitted when nil, else the struct (its own omitempty)
            if v is None:
                continue
            items.append((name, _struct(_HEALTH, v)))
            continue
        empty = v is None or v == "" or v is False or v == 0 or (isinstance(v, (list, dict)) and len(v) == 0)
        if omit and empty:
            continue
        if kind == "history":  # []History: each entry a struct
            items.append((name, ("arr", [_struct(_HISTORY, h or {}) for h in v])))
            continue
        if kind == "list_null" and v is None:
            items.append((name, "null"))
            continue
        if kind == "str":
            items.append((name, _go_string(v or "")))
        elif kind == "bool":
            items.append((name, "true" if v else "false"))
        elif kind == "int":
            items.append((name, str(int(v or 0))))
        else:
            items.append((name, _value(v)))
    return ("obj", items)


def _indent(tree, prefix: str, indent: str, depth: int, out: List[str]):
    if isinstance(tree, str):
        out.append(tree)
        return
    kind, items = tree
    open_, close = ("{", "}") if kind == "obj" else ("[", "]")
    if not items:
        out.append(open_ + close)
        return
    out.append(open_)
    for i, it in enumerate(items):
        out.append("\n" + prefix + indent * (depth + 1))
        if kind == "obj":
            k, v = it
            out.append(_go_string(k) + ": ")
            _indent(v, prefix, indent, depth + 1, out)
        else:
            _indent(it, prefix, indent, depth + 1, out)
        if i + 1 < len(items):
            out.append(",")
    out.append("\n" + prefix + indent * depth + close)


def MarshalIndentConfigFile(cfg: Dict[str, Any], prefix: str = "  ", indent: str = "") -> bytes:
    """json.MarshalIndent(v1.ConfigFile, prefix, indent) for a ConfigFile given as a dict with
    the JSON field names (secret.go:43)."""
    out: List[str] = []
    _indent(_struct(_CONFIG_FILE, cfg), prefix, indent, 0, out)
    return "".join(out).encode("utf-8")


@dataclass
class ConfigAnalysisInput:  # pkg/fanal/analyzer/config_analyzer.go:45-48
    OS: Any = None
    Config: Optional[Dict[str, Any]] = None  # v1.ConfigFile (JSON field names), None = nil


@dataclass
class ConfigAnalysisResult:  # config_analyzer.go:50-54 (the Secret part)
    Secret: Optional[Secret] = None


class SecretAnalyzer:
    """imgconf/secret.secretAnalyzer bound to the MI355X engine (secret.go:21-73)."""

    def __init__(self, configPath: str = "", device: int = 0):  # newSecretAnalyzer, secret.go:26-37
        try:
            c = ParseConfig(configPath)
        except Exception as e:
            raise RuntimeError("secret config error: %s" % e)
        self.scanner = NewScanner(c, device=device)

    def Analyze(self, input: ConfigAnalysisInput) -> Optional[ConfigAnalysisResult]:  # secret.go:39-62
        if input.Config is None:
            return None
        b = MarshalIndentConfigFile(input.Config, "  ", "")
        result = self.scanner.Scan(ScanArgs(FilePath="config.json", Content=b))
        if not result.Findings:
            return None
        return ConfigAnalysisResult(Secret=result)

    def Required(self, _os=None) -> bool:  # secret.go:64-66
        return True

    def Type(self) -> str:
        return TypeImageConfigSecret

    def Version(self) -> int:
        return analyzerVersion
