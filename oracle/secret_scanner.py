"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of the reference secret engine, pkg/fanal/secret/scanner.go
(undistro/trivy @ 2024-12-20).  Function names follow the Go ones; every
function cites the lines it restates.  Strings (paths, matches, code lines)
are kept as ``bytes`` internally and surfaced as ``str`` decoded with
``surrogateescape`` so that non-UTF-8 content round-trips losslessly.
"""
import json
from pathlib import Path

import yaml

from .goregexp import GoRegexp
from .gostd import bytes_to_lower, strings_to_lower, quote
from .gosort import sort_slice

_BUILTIN_JSON = Path(__file__).resolve().parent.parent / "trivy_amd/secret/builtin_rules.json"


def _s(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


def _b(s) -> bytes:
    if s is None:
        return b""
    if isinstance(s, bytes):
        return s
    return s.encode("utf-8", "surrogateescape")


class Rule:  # scanner.go:89-100
    def __init__(self, id, category="", title="", severity="", regex=None, keywords=(),
                 path=None, allow_rules=(), exclude_block=(), secret_group_name=""):
        self.id = id
        self.category = category
        self.title = title
        self.severity = severity
        self.regex = regex
        self.keywords = list(keywords or [])
        self.path = path
        self.allow_rules = list(allow_rules or [])
        self.exclude_block = list(exclude_block or [])
        self.secret_group_name = secret_group_name or ""

    def match_path(self, path: bytes) -> bool:  # scanner.go:170-172
        return self.path is None or self.path.match_string(path)

    def match_keywords(self, content: bytes) -> bool:  # scanner.go:174-186
        if len(self.keywords) == 0:
            return True
        lower = bytes_to_lower(content)
        for kw in self.keywords:
            if strings_to_lower(_b(kw)) in lower:
                return True
        return False

    def allow_path(self, path: bytes) -> bool:  # scanner.go:188-190
        return allow_rules_allow_path(self.allow_rules, path)

    def allow(self, match: bytes) -> bool:  # scanner.go:192-194
        return allow_rules_allow(self.allow_rules, match)

    def get_match_subgroups_locations(self, match_locs):  # scanner.go:155-168
        locs = []
        for i, name in enumerate(self.regex.subexp_names):
            if name == self.secret_group_name:
                locs.append((match_locs[2 * i], match_locs[2 * i + 1]))
        return locs


class AllowRule:  # scanner.go:196-201
    def __init__(self, id="", description="", regex=None, path=None):
        self.id, self.description, self.regex, self.path = id, description, regex, path


def allow_rules_allow_path(rules, path: bytes) -> bool:  # scanner.go:205-212
    for r in rules:
        if r.path is not None and r.path.match_string(path):
            return True
    return False


def allow_rules_allow(rules, match: bytes) -> bool:  # scanner.go:214-221
    for r in rules:
        if r.regex is not None and r.regex.match_string(match):
            return True
    return False


class _Blocks:  # scanner.go:237-275 (lazy, sync.Once)
    def __init__(self, content, regexes):
        self.content, self.regexes, self.locs = content, regexes, None

    def match(self, block):  # scanner.go:252-260
        if self.locs is None:
            self.locs = []
            for rx in self.regexes:
                for r in rx.find_all_index(self.content):
                    self.locs.append((r[0], r[1]))
        for s, e in self.locs:
            if s <= block[0] and block[1] <= e:  # Location.Match, scanner.go:233-235
                return True
        return False


def _compile(v):
    if v is None:
        return None
    if not isinstance(v, str):
        v = str(v)
    return GoRegexp(v)


def _yaml_value(node):
    """gopkg.in/yaml.v3 (go.mod:132) into the Config's Go types: a scalar decoded into a string
    field (and into Regexp.UnmarshalYAML, scanner.go:75-87, which compiles value.Value) is the
    node's text as written -- `0x1F` stays "0x1F", `true` stays "true" -- and a plain null
    scalar (~ / null / Null / NULL / empty) is the zero value (None here)."""
    if node is None:
        return None
    if isinstance(node, yaml.MappingNode):
        return {_yaml_value(k): _yaml_value(v) for k, v in node.value}
    if isinstance(node, yaml.SequenceNode):
        return [_yaml_value(v) for v in node.value]
    if node.style is None and node.value in ("~", "null", "Null", "NULL", ""):
        return None
    return node.value


def _go_string(v):  # a string field: its text, "" for null
    return "" if v is None else v


def _allow_rules_from_yaml(items):
    out = []
    for a in items or []:
        out.append(AllowRule(id=_go_string(a.get("id")), description=_go_string(a.get("description")),
                             regex=_compile(a.get("regex")), path=_compile(a.get("path"))))
    return out


def _exclude_from_yaml(block):
    return [_compile(_go_string(r)) for r in ((block or {}).get("regexes") or [])]


def convert_severity(sev) -> str:  # scanner.go:310-318
    sev = "" if sev is None else str(sev)
    if sev.lower() in ("low", "medium", "high", "critical", "unknown"):
        return sev.upper()
    return "UNKNOWN"


class Config:  # scanner.go:29-43
    def __init__(self):
        self.enable_builtin_rule_ids = []
        self.disable_rule_ids = []
        self.disable_allow_rule_ids = []
        self.custom_rules = []
        self.custom_allow_rules = []
        self.exclude_block = []


def parse_config(config_path):  # scanner.go:277-307
    if not config_path:
        return None
    p = Path(config_path)
    if not p.exists():
        return None
    doc = _yaml_value(yaml.compose(p.read_text(), Loader=yaml.SafeLoader)) or {}
    c = Config()
    c.enable_builtin_rule_ids = [_go_string(x) for x in doc.get("enable-builtin-rules") or []]
    c.disable_rule_ids = [_go_string(x) for x in doc.get("disable-rules") or []]
    c.disable_allow_rule_ids = [_go_string(x) for x in doc.get("disable-allow-rules") or []]
    for r in doc.get("rules") or []:
        c.custom_rules.append(Rule(
            id=_go_string(r.get("id")), category=_go_string(r.get("category")),
            title=_go_string(r.get("title")),
            severity=convert_severity(r.get("severity")),
            regex=_compile(r.get("regex")),
            keywords=[_go_string(k) for k in (r.get("keywords") or [])],
            path=_compile(r.get("path")),
            allow_rules=_allow_rules_from_yaml(r.get("allow-rules")),
            exclude_block=_exclude_from_yaml(r.get("exclude-block")),
            secret_group_name=_go_string(r.get("secret-group-name"))))
    c.custom_allow_rules = _allow_rules_from_yaml(doc.get("allow-rules"))
    c.exclude_block = _exclude_from_yaml(doc.get("exclude-block"))
    return c


_BUILTIN = None


def builtin_rules():
    """builtin-rules.go:101-849 / builtin-allow-rules.go:3-65 (data via builtin_rules.json)."""
    global _BUILTIN
    if _BUILTIN is None:
        d = json.loads(_BUILTIN_JSON.read_text())
        rules = [Rule(id=r["id"], category=r["category"], title=r["title"], severity=r["severity"],
                      regex=GoRegexp(r["regex"]), keywords=r["keywords"],
                      secret_group_name=r["secret_group_name"]) for r in d["rules"]]
        allow = [AllowRule(id=a["id"], description=a["description"], regex=_compile(a["regex"]),
                           path=_compile(a["path"])) for a in d["allow_rules"]]
        _BUILTIN = (rules, allow)
    return _BUILTIN


class Scanner:
    def __init__(self, rules, allow_rules, exclude_block):
        self.rules, self.allow_rules, self.exclude_block = rules, allow_rules, exclude_block

    # scanner.go:57-59
    def allow_path(self, path) -> bool:
        return allow_rules_allow_path(self.allow_rules, _b(path))

    def allow(self, match: bytes) -> bool:  # scanner.go:52-54
        return allow_rules_allow(self.allow_rules, match)

    def allow_location(self, rule, content, loc):  # scanner.go:150-153
        m = content[loc[0]:loc[1]]
        return self.allow(m) or rule.allow(m)

    def find_locations(self, rule, content):  # scanner.go:102-126
        if rule.regex is None:
            return []
        if rule.secret_group_name != "":
            return self.find_submatch_locations(rule, content)
        locs = []
        for idx in rule.regex.find_all_index(content):
            loc = (idx[0], idx[1])
            if self.allow_location(rule, content, loc):
                continue
            locs.append(loc)
        return locs

    def find_submatch_locations(self, rule, content):  # scanner.go:128-148
        out = []
        for m in rule.regex.find_all_submatch_index(content):
            loc = (m[0], m[1])
            if self.allow_location(rule, content, loc):
                continue
            out.extend(rule.get_match_subgroups_locations(m))
        return out

    def scan(self, file_path, content: bytes, binary=False):  # scanner.go:377-463
        path = _b(file_path)
        if self.allow_path(path):
            return {"FilePath": _s(path), "Findings": None}
        censored = None
        matched = []
        global_blocks = _Blocks(content, self.exclude_block)
        for rule in self.rules:
            if not rule.match_path(path):
                continue
            if rule.allow_path(path):
                continue
            if not rule.match_keywords(content):
                continue
            locs = self.find_locations(rule, content)
            if not locs:
                continue
            local_blocks = _Blocks(content, rule.exclude_block)
            for loc in locs:
                if global_blocks.match(loc) or local_blocks.match(loc):
                    continue
                if loc[0] < 0:
                    # Go would panic slicing with a non-participating group (-1)
                    raise RuntimeError("non-participating secret group (reference panics)")
                matched.append((rule, loc))
                if censored is None:
                    censored = bytearray(content)
                censored[loc[0]:loc[1]] = b"*" * (loc[1] - loc[0])  # censorLocation :465-473
        findings = []
        for rule, loc in matched:  # scanner.go:438-446
            f = to_finding(rule, loc, bytes(censored))
            if binary:
                f["Match"] = "Binary file %s matches a rule %s" % (quote(path), quote(_b(rule.title)))
                f["Code"] = {"Lines": None}  # types.Code{}: Lines is nil -> JSON null
            findings.append(f)
        if not findings:
            return {"FilePath": "", "Findings": None}

        def less(x, y):  # scanner.go:452-457 (Go string compare == bytewise)
            if x["RuleID"] != y["RuleID"]:
                return _b(x["RuleID"]) < _b(y["RuleID"])
            return _b(x["Match"]) < _b(y["Match"])

        sort_slice(findings, less)
        return {"FilePath": _s(path), "Findings": findings}


def new_scanner(config):  # scanner.go:320-364
    b_rules, b_allow = builtin_rules()
    if config is None:
        return Scanner(list(b_rules), list(b_allow), [])
    enabled = list(b_rules)
    if config.enable_builtin_rule_ids:
        enabled = [r for r in b_rules if r.id in config.enable_builtin_rule_ids]
    enabled = enabled + config.custom_rules
    rules = [r for r in enabled if r.id not in config.disable_rule_ids]
    allow = list(b_allow) + config.custom_allow_rules
    allow = [a for a in allow if a.id not in config.disable_allow_rule_ids]
    return Scanner(rules, allow, config.exclude_block)


def to_finding(rule, loc, content):  # scanner.go:475-488
    start_line, end_line, code, match_line = find_location(loc[0], loc[1], content)
    return {
        "RuleID": rule.id,
        "Category": rule.category,
        "Severity": "UNKNOWN" if rule.severity == "" else rule.severity,
        "Title": rule.title,
        "StartLine": start_line,
        "EndLine": end_line,
        "Code": code,
        "Match": _s(match_line),
    }


def find_location(start, end, content):  # scanner.go:495-558
    start_line_num = content.count(b"\n", 0, start)
    line_start = content.rfind(b"\n", 0, start)
    line_start = 0 if line_start == -1 else line_start + 1
    line_end = content.find(b"\n", start)
    if line_end == -1:
        line_end = len(content)
    if line_end - line_start > 100:
        line_start = line_start if start - line_start - 30 < 0 else start - 30
        line_end = line_end if end + 20 > line_end else end + 20
    match_line = content[line_start:line_end]
    end_line_num = start_line_num + content.count(b"\n", start, end)

    lines = content.split(b"\n")
    code_start = max(start_line_num - 2, 0)
    code_end = min(end_line_num + 2, len(lines))
    out = []
    found_first = False
    for i, raw in enumerate(lines[code_start:code_end]):
        real = code_start + i
        in_cause = start_line_num <= real <= end_line_num
        if len(raw) > 100:
            s = match_line if in_cause else raw[:100]
        else:
            s = raw
        out.append({
            "Number": code_start + i + 1, "Content": _s(s), "IsCause": in_cause,
            "Annotation": "", "Truncated": False, "Highlighted": _s(s),
            "FirstCause": (not found_first) and in_cause, "LastCause": False,
        })
        found_first = found_first or in_cause
    for ln in reversed(out):
        if ln["IsCause"]:
            ln["LastCause"] = True
            break
    return start_line_num + 1, end_line_num + 1, {"Lines": out}, match_line
