"""Secret rule configuration: pkg/fanal/secret/scanner.go:29-100,196-226,277-318.

Regexes are validated by compiling them with the native Go-semantics engine
(the reference fails ParseConfig on a bad regex, scanner.go:75-87).
"""
import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Optional

import yaml

from .. import _lib

_BUILTIN = Path(__file__).resolve().parent / "builtin_rules.json"


class ConfigError(Exception):
    pass


def _check_regex(src, where):
    if src is None:
        return None
    src = str(src)
    try:
        _lib.regex_match(src, b"")
    except ValueError as e:
        raise ConfigError("regexp compile error (%s): %s" % (where, e))
    return src


@dataclass
class AllowRule:  # scanner.go:196-201
    ID: str = ""
    Description: str = ""
    Regex: Optional[str] = None
    Path: Optional[str] = None


@dataclass
class ExcludeBlock:  # scanner.go:223-226
    Description: str = ""
    Regexes: List[str] = field(default_factory=list)


@dataclass
class Rule:  # scanner.go:89-100
    ID: str = ""
    Category: str = ""
    Title: str = ""
    Severity: str = ""
    Regex: Optional[str] = None
    Keywords: List[str] = field(default_factory=list)
    Path: Optional[str] = None
    AllowRules: List[AllowRule] = field(default_factory=list)
    ExcludeBlock: ExcludeBlock = field(default_factory=ExcludeBlock)
    SecretGroupName: str = ""


@dataclass
class Config:  # scanner.go:29-43
    EnableBuiltinRuleIDs: List[str] = field(default_factory=list)
    DisableRuleIDs: List[str] = field(default_factory=list)
    DisableAllowRuleIDs: List[str] = field(default_factory=list)
    CustomRules: List[Rule] = field(default_factory=list)
    CustomAllowRules: List[AllowRule] = field(default_factory=list)
    ExcludeBlock: ExcludeBlock = field(default_factory=ExcludeBlock)


# yaml.v3 (gopkg.in/yaml.v3 v3.0.1, go.mod:132) decodes a scalar into a Go `string` field -- and
# Regexp.UnmarshalYAML compiles value.Value (scanner.go:75-87) -- as the node's source text: `id: 0`
# is "0", `regex: 0x1F` is "0x1F", `title: true` is "true"; only a plain null (~, null, Null, NULL or
# nothing) is the zero value ("" / a nil *Regexp).  So the document is composed into nodes and read
# by their text, not constructed with PyYAML's YAML 1.1 typing (0x1F -> 31, on -> True).
_PLAIN_NULL = ("~", "null", "Null", "NULL", "")


def _node(n, where="config"):
    if n is None:
        return None
    if isinstance(n, yaml.MappingNode):
        out = {}
        for k, v in n.value:
            out[_text(_node(k, where), where)] = _node(v, where)
        return out
    if isinstance(n, yaml.SequenceNode):
        return [_node(v, where) for v in n.value]
    if n.style is None and n.value in _PLAIN_NULL:
        return None
    return n.value


def _text(v, where) -> str:  # a Go string field
    if v is None:
        return ""
    if not isinstance(v, str):
        raise ConfigError("secrets config decode error: %s: cannot unmarshal a %s into a string"
                          % (where, "sequence" if isinstance(v, list) else "mapping"))
    return v


def _texts(v, where):  # a Go []string field
    if v is None:
        return []
    if not isinstance(v, list):
        raise ConfigError("secrets config decode error: %s: cannot unmarshal a scalar into a list" % where)
    return [_text(x, where) for x in v]


def _load_yaml(text):
    try:
        return _node(yaml.compose(text, Loader=yaml.SafeLoader)) or {}
    except yaml.YAMLError as e:
        raise ConfigError("secrets config decode error: %s" % e)


def convert_severity(sev) -> str:  # scanner.go:310-318
    sev = "" if sev is None else str(sev)
    if sev.lower() in ("low", "medium", "high", "critical", "unknown"):
        return sev.upper()
    return "UNKNOWN"


def _allow_rules(items, where):
    out = []
    for a in items or []:
        out.append(AllowRule(ID=_text(a.get("id"), where), Description=_text(a.get("description"), where),
                             Regex=_check_regex(a.get("regex"), where),
                             Path=_check_regex(a.get("path"), where)))
    return out


def _exclude(block, where):
    block = block or {}
    return ExcludeBlock(Description=_text(block.get("description"), where),
                        Regexes=[_check_regex(_text(r, where), where) for r in (block.get("regexes") or [])])


def ParseConfig(config_path) -> Optional[Config]:  # scanner.go:277-307
    if not config_path:
        return None
    p = Path(config_path)
    if not p.exists():
        return None
    doc = _load_yaml(p.read_text())
    c = Config()
    c.EnableBuiltinRuleIDs = _texts(doc.get("enable-builtin-rules"), "enable-builtin-rules")
    c.DisableRuleIDs = _texts(doc.get("disable-rules"), "disable-rules")
    c.DisableAllowRuleIDs = _texts(doc.get("disable-allow-rules"), "disable-allow-rules")
    for r in doc.get("rules") or []:
        rid = _text(r.get("id"), "rules")
        c.CustomRules.append(Rule(
            ID=rid, Category=_text(r.get("category"), rid), Title=_text(r.get("title"), rid),
            Severity=convert_severity(_text(r.get("severity"), rid)),
            Regex=_check_regex(r.get("regex"), rid),
            Keywords=_texts(r.get("keywords"), rid),
            Path=_check_regex(r.get("path"), rid),
            AllowRules=_allow_rules(r.get("allow-rules"), rid),
            ExcludeBlock=_exclude(r.get("exclude-block"), rid),
            SecretGroupName=_text(r.get("secret-group-name"), rid)))
    c.CustomAllowRules = _allow_rules(doc.get("allow-rules"), "allow-rules")
    c.ExcludeBlock = _exclude(doc.get("exclude-block"), "exclude-block")
    return c


_CACHE = None


def _load_builtin():
    global _CACHE
    if _CACHE is None:
        d = json.loads(_BUILTIN.read_text())
        rules = [Rule(ID=r["id"], Category=r["category"], Title=r["title"], Severity=r["severity"],
                      Regex=r["regex"], Keywords=list(r["keywords"]), SecretGroupName=r["secret_group_name"])
                 for r in d["rules"]]
        allow = [AllowRule(ID=a["id"], Description=a["description"], Regex=a["regex"], Path=a["path"])
                 for a in d["allow_rules"]]
        _CACHE = (rules, allow)
    return _CACHE


def builtin_rules() -> List[Rule]:  # builtin-rules.go:87-90 GetBuiltinRules
    return list(_load_builtin()[0])


def builtin_allow_rules() -> List[AllowRule]:
    return list(_load_builtin()[1])
