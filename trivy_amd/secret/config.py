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


def convert_severity(sev) -> str:  # scanner.go:310-318
    sev = "" if sev is None else str(sev)
    if sev.lower() in ("low", "medium", "high", "critical", "unknown"):
        return sev.upper()
    return "UNKNOWN"


def _allow_rules(items, where):
    out = []
    for a in items or []:
        out.append(AllowRule(ID=str(a.get("id", "") or ""), Description=str(a.get("description", "") or ""),
                             Regex=_check_regex(a.get("regex"), where),
                             Path=_check_regex(a.get("path"), where)))
    return out


def _exclude(block, where):
    block = block or {}
    return ExcludeBlock(Description=str(block.get("description", "") or ""),
                        Regexes=[_check_regex(r, where) for r in (block.get("regexes") or [])])


def ParseConfig(config_path) -> Optional[Config]:  # scanner.go:277-307
    if not config_path:
        return None
    p = Path(config_path)
    if not p.exists():
        return None
    try:
        doc = yaml.safe_load(p.read_text()) or {}
    except yaml.YAMLError as e:
        raise ConfigError("secrets config decode error: %s" % e)
    c = Config()
    c.EnableBuiltinRuleIDs = [str(x) for x in doc.get("enable-builtin-rules") or []]
    c.DisableRuleIDs = [str(x) for x in doc.get("disable-rules") or []]
    c.DisableAllowRuleIDs = [str(x) for x in doc.get("disable-allow-rules") or []]
    for r in doc.get("rules") or []:
        rid = str(r.get("id", "") or "")
        c.CustomRules.append(Rule(
            ID=rid, Category=str(r.get("category", "") or ""), Title=str(r.get("title", "") or ""),
            Severity=convert_severity(r.get("severity")),
            Regex=_check_regex(r.get("regex"), rid),
            Keywords=[str(k) for k in (r.get("keywords") or [])],
            Path=_check_regex(r.get("path"), rid),
            AllowRules=_allow_rules(r.get("allow-rules"), rid),
            ExcludeBlock=_exclude(r.get("exclude-block"), rid),
            SecretGroupName=str(r.get("secret-group-name", "") or "")))
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
