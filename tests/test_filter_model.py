"""Streaming prefilter (K1) semantics on CPU: every true match is covered.

The CPU model (tests/filter_model.py) replays the compiled bucketed shift-or
tables and the exact confirm step.  For files without fold runes (U+0130,
U+212A, U+017F: those go through the careful pass) every match of every rule
regex -- found by the native Go-regexp engine over the whole file -- must start
inside the window of some anchor hit of that rule, and files
holding a fold rune must be flagged.  Rule sets: the builtin rules and the
golden configs' custom rules.
"""
import ctypes as c
import json
import random
from pathlib import Path

import numpy as np
import pytest
import yaml

from tests.corpus import make_corpus
from tests.filter_model import FilterModel, RuleInfo
from tests.regex_sampler import sample_regex
from trivy_amd import _lib
from trivy_amd.secret import ParseConfig, builtin_rules

ROOT = Path(__file__).resolve().parent.parent
FOLDS = (b"\xc4\xb0", b"\xe2\x84\xaa", b"\xc5\xbf")
NOISE = ["the quick brown fox ", "key=", "secret: ", "\n", "  ", "'", '"', "AKIA", "ghp_", "sk_live_",
         "é", "日本", "\udcff", "-----BEGIN ", "=>", "xoxb-", "eyJ", ".", "hooks.slack.com", "\t", ",", "_",
         "0123456789abcdef", "aws_", "live_", "test_", "SG.", "pk.", "linear ", "token: "]


def _anchors(model):
    L = _lib.lib()
    L.tsg_debug_anchor.argtypes = [c.c_void_p, c.c_uint32] + [c.c_void_p] * 4
    out = []
    j = 0
    while True:
        r, ln, lo, hi = c.c_uint32(), c.c_uint32(), c.c_int32(), c.c_int32()
        if L.tsg_debug_anchor(model.h, j, c.byref(r), c.byref(ln), c.byref(lo), c.byref(hi)) != 0:
            return out
        out.append((r.value, ln.value, lo.value, hi.value))
        j += 1


def _rule_kw(model, i):
    L = _lib.lib()
    L.tsg_debug_rule.argtypes = [c.c_void_p, c.c_uint32, c.c_void_p]
    ri = RuleInfo()
    L.tsg_debug_rule(model.h, i, c.byref(ri))
    if ri.gate != 1 or not ri.n_kw:
        return []
    return list(np.ctypeslib.as_array((c.c_uint32 * ri.n_kw).from_address(ri.kw_ids)))


def _pack(contents):
    offs = np.zeros(len(contents) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(x) for x in contents])
    arena = np.frombuffer(b"".join(contents), dtype=np.uint8)
    return arena, offs


def _check(rules, contents, calibration=None):
    model = FilterModel(rules, calibration=calibration)
    if calibration is not None:
        assert model.n_calibrated >= 1  # (the samples below make the compiler move an anchor)
    anchors = _anchors(model)
    arena, offs = _pack(contents)
    hits, folds = model.run(arena, offs)
    special = {f for f, _ in folds}
    reqs = model.anchor_reqs()
    windows = {}
    for f, end, aid in hits:
        # the confirm kernel drops hits failing the anchor's follow requirements
        if not model.follow_possible(reqs[aid], contents[f], end):
            continue
        r, lit_len, lo, hi = anchors[aid]
        lit = end - lit_len
        windows.setdefault((f, r), []).append((max(0, lit - hi), lit - lo))
    n_matches = 0
    for f, content in enumerate(contents):
        has_fold = any(s in content for s in FOLDS)
        assert has_fold == (f in special), (f, content)
        if has_fold:
            continue
        for r, rule in enumerate(rules):
            if not rule.Regex:
                continue
            for m in _lib.regex_find_all(rule.Regex, content):
                if m[0] == m[1]:
                    continue  # empty matches come from unanchored rules (full-scan path)
                if not any(lo <= m[0] <= hi for lo, hi in windows.get((f, r), [])):
                    raise AssertionError("rule %s match %r at %d not covered" % (rule.ID, content[m[0]:m[1]], m[0]))
                n_matches += 1
    return n_matches, len(hits)


def _planted_texts(rng, rules, n):
    out = []
    for _ in range(n):
        parts = []
        for _ in range(rng.randint(1, 30)):
            if rng.random() < 0.35:
                rule = rng.choice(rules)
                if rule.Regex:
                    parts.append(sample_regex(rule.Regex, rng, maxrep=4))
            else:
                parts.append(rng.choice(NOISE).encode("utf-8", "surrogateescape"))
        out.append(b"".join(parts))
    return out


@pytest.mark.parametrize("seed", range(4))
def test_builtin_planted_matches_covered(seed):
    rules = builtin_rules()
    rng = random.Random(300 + seed)
    n, _ = _check(rules, _planted_texts(rng, rules, 120))
    assert n > 50


@pytest.mark.parametrize("seed", [11, 12])
def test_builtin_corpus_matches_covered(seed):
    files = make_corpus(seed, 80)
    contents = [b.replace(b"\r", b"") for _, b in files]
    n, hits = _check(builtin_rules(), contents)
    assert n > 0


def test_fold_runes_flag_files():
    rules = builtin_rules()
    contents = [b"plain ascii\n", b"x\xc4\xb0y", b"\xe2\x84\xaa", b"ab\xc5\xbf", b"\xc4\xc4", b"\xe2\x84",
                b"\xc5\xbf\xc5\xbf", b""]
    model = FilterModel(rules)
    arena, offs = _pack(contents)
    _, folds = model.run(arena, offs)
    assert folds == {(1, 5), (2, 5), (3, 3), (6, 3)}


def test_golden_custom_rules_covered():
    rng = random.Random(9)
    for f in sorted((ROOT / "tests/golden/scanner").glob("*.yaml")):
        d = yaml.safe_load(f.read_text()) or {}
        if not d.get("rules"):
            continue
        try:
            cfg = ParseConfig(str(f))
        except ValueError:
            continue
        rules = builtin_rules() + list(cfg.CustomRules or [])
        custom = [r for r in rules if r.Regex]
        _check(rules, _planted_texts(rng, custom, 25))


def test_newline_bucket_shape():
    m = FilterModel(builtin_rules())
    nlb = m.n_buckets - 1
    assert m.bucket_off[nlb + 1] == m.bucket_off[nlb]  # no items
    assert list(np.nonzero(m.allowed(nlb, 0))[0]) == [10]
    for s in (1, 2, 3):
        assert m.allowed(nlb, s).all()
    for s in (4, 5, 6, 7):
        assert not m.allowed(nlb, s).any()
    for j in range(nlb):  # item buckets carry fires through slots 6, 7
        assert m.allowed(j, 6).all() and m.allowed(j, 7).all()


def test_keyword_bits_exact_ascii():
    """GPU keyword bits = ASCII case-insensitive keyword presence (files without U+0130/U+212A)."""
    rules = builtin_rules()
    m = FilterModel(rules)
    L = _lib.lib()
    L.tsg_debug_keyword.restype = c.c_char_p
    L.tsg_debug_keyword.argtypes = [c.c_void_p, c.c_uint32]
    kws = []
    while True:
        k = L.tsg_debug_keyword(m.h, len(kws))
        if k is None:
            break
        kws.append(k)
    rng = random.Random(5)
    contents = _planted_texts(rng, rules, 60)
    contents += [k.upper() + b" x" for k in kws] + [b"a" + k + b"b" for k in kws] + [kws[0][:-1]]
    arena, offs = _pack(contents)
    got = set()
    m.run(arena, offs, got)
    want = set()
    for f, content in enumerate(contents):
        low = content.lower()
        for i, k in enumerate(kws):
            if k in low:
                want.add((f, i))
    with_items = {int(m.item_ids[it["ids_off"]]) for it in m.items if it["kind"] == 0}
    gated = {int(x) for r in range(len(rules)) for x in _rule_kw(m, r)}
    assert with_items and with_items <= gated
    assert {(f, i) for f, i in want if i in with_items} == got


def test_class_run_anchors_cover_matches():
    """Rules without a required literal anchored on a run of one-byte classes
    (rules.cpp ExtractClassRun): every match holds the run at its bounded offset,
    so K1/K2 + the follow requirements still cover every match."""
    from trivy_amd.secret.config import Rule
    import re as _re
    srcs = [r"(?i)\b[g-z]{3}[0-9]{3}[._-][a-z0-9]{12}\b",
            r"[a-f]{2}[0-9]{2}_[a-z]+_end[0-9]",
            r"[0-9]{3}-[0-9]{4}-[0-9]{3}",
            r"(?i)(?:^|\s)[k-s]{2}[0-9]{4}[:=][A-Z0-9]{8}",
            r"x?[0-9]{2}\.[0-9]{2}\.[0-9]{4}-[a-z]{2}"]
    rules = builtin_rules() + [Rule(ID="cr%d" % i, Category="C", Title="t", Severity="LOW",
                                    Regex=s)
                               for i, s in enumerate(srcs)]
    m = FilterModel(rules)
    L = _lib.lib()
    L.tsg_debug_rule_anchor.restype = c.c_char_p
    L.tsg_debug_rule_anchor.argtypes = [c.c_void_p, c.c_uint32]
    descs = [L.tsg_debug_rule_anchor(m.h, len(rules) - len(srcs) + i).decode() for i in range(len(srcs))]
    assert all("classes" in d for d in descs), descs
    rng = random.Random(11)
    n, _ = _check(rules, _planted_texts(rng, rules[-len(srcs):], 60))
    assert n > 40


def _calibration_sample(seed):
    """Bytes in which some builtin literal anchors are common words (linear, heroku, intercom,
    mailgun ...) and hex / base64 runs are rare: the compiler then anchors those rules on their
    class runs (tsg_compile_options)."""
    rng = random.Random(seed)
    words = [b"linear ", b"linear-gradient(", b"heroku ", b"intercom ", b"mailgun ", b"asana ", b"discord ",
             b"the ", b"value = ", b"x", b"\n", b"if (a) ", b"return b; "]
    return b"".join(rng.choice(words) for _ in range(200000))


@pytest.mark.parametrize("seed", range(3))
def test_calibrated_anchors_cover_matches(seed):
    """With a calibration sample the rule compiler may anchor a rule on a class run instead of its
    literal (rules.cpp CompileRules): every match must still be covered (the class run is a fixed run
    every match holds, at a bounded offset)."""
    rules = builtin_rules()
    rng = random.Random(500 + seed)
    texts = _planted_texts(rng, rules, 120)
    texts += [b"color: linear-gradient(" + t for t in texts[:20]]
    n, _ = _check(rules, texts, calibration=_calibration_sample(seed))
    assert n > 50
