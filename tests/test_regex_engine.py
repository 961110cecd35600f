"""Native Go-regexp engine (exact host pass) vs the oracle -- CPU only.

Covers every builtin rule regex (pkg/fanal/secret/builtin-rules.go), the golden
configs' custom regexes, and the builtin allow-rule regexes, on texts mixing
noise, planted samples of each regex's language, non-ASCII runes, invalid UTF-8
and the fold-special runes U+212A / U+017F / U+0130.  Also checks that a
search restricted to start windows that contain every true match start equals
the unrestricted search (the GPU-candidate contract).
"""
import json
import random
from pathlib import Path

import pytest
import yaml

from oracle.goregexp import GoRegexp
from oracle.gostd import bytes_to_lower
from tests.regex_sampler import sample_regex
from trivy_amd import _lib

ROOT = Path(__file__).resolve().parent.parent
BUILTIN = json.loads((ROOT / "trivy_amd/secret/builtin_rules.json").read_text())


def _golden_custom_regexes():
    out = []
    for f in sorted((ROOT / "tests/golden/scanner").glob("*.yaml")):
        d = yaml.safe_load(f.read_text()) or {}
        for r in d.get("rules") or []:
            if r.get("regex"):
                out.append(str(r["regex"]))
            for a in r.get("allow-rules") or []:
                for k in ("regex", "path"):
                    if a.get(k):
                        out.append(str(a[k]))
        for a in d.get("allow-rules") or []:
            for k in ("regex", "path"):
                if a.get(k):
                    out.append(str(a[k]))
    return sorted(set(out))


# Nullable loop bodies such as (a|)+ are excluded: CPython's backtracker and
# Go's Pike VM (which the native engine follows) record different captures for
# the final empty iteration; no rule uses that construct.
PATTERNS = ([r["regex"] for r in BUILTIN["rules"]]
            + [a[k] for a in BUILTIN["allow_rules"] for k in ("regex", "path") if a[k]]
            + _golden_custom_regexes()
            + [r"a*", r"x{2,5}?y", r"(?m)^ab$", r"\bfoo\b", r"(?i)straße", r"(?s).{0,3}z",
               r"[^\x00-\x7f]+", r"\x{FFFD}", r"(?U)a+b", r"(?i)k+s", r"^", r"$", r"(?i)[^k]",
               # one greedy class repeat (FindAll's class-run path, goregex.cpp FindAllRun)
               r"(?i)[a-z0-9/+]{32,48}", r"[0-9]{3}", r"(?P<secret>[a-f0-9]{8,})", r"(?i)[ks]{2,4}",
               r"[^\s]{3,5}", r"((?:[a-c]){2,3})", r"(?i)(?P<x>[k-s]+)", r"\S{4}", r"[^a]{1,2}", r"[\x{FFFD}a]{2}",
               # literals (Regex::Match's byte search, goregex.cpp MatchLiteral) and near-literals that are not
               r"(?i)example", r"abc", r"(?i)(ex)(?:am)ple", r"a\.b", r"(?i)akia", r"[xX]y", r"(?i)ke", r"(?i)s",
               r"(?i)ſ", r"é", r"(?i)^ex"])

NOISE = ["the quick brown fox ", "key=", "secret: ", "\n", "  ", "'", '"', "AKIA", "ghp_",
         "sk_live_", "K", "ſ", "İ", "é", "日本", "\udcff", "-----BEGIN ", "=>",
         "xoxb-", "eyJ", ".", "hooks.slack.com", "\t", ",", "_", "0123456789abcdef"]


def _text(rng, pats, n_parts=40):
    parts = []
    for _ in range(n_parts):
        if rng.random() < 0.35:
            parts.append(sample_regex(rng.choice(pats), rng))
        else:
            parts.append(rng.choice(NOISE).encode("utf-8", "surrogateescape"))
    return b"".join(parts)


@pytest.mark.parametrize("idx", range(len(PATTERNS)))
def test_native_regex_matches_oracle(idx):
    pat = PATTERNS[idx]
    ref = GoRegexp(pat)
    rng = random.Random(1000 + idx)
    for trial in range(25):
        text = _text(rng, [pat], n_parts=rng.randint(1, 30))
        want = ref.find_all_submatch_index(text)
        got = _lib.regex_find_all(pat, text, submatch=True)
        assert got == want, (pat, text)
        assert _lib.regex_match(pat, text) == ref.match_string(text)


@pytest.mark.parametrize("idx", range(len(PATTERNS)))
def test_windowed_search_equals_full(idx):
    pat = PATTERNS[idx]
    rng = random.Random(7 + idx)
    for trial in range(15):
        text = _text(rng, [pat], n_parts=rng.randint(1, 30))
        full = _lib.regex_find_all(pat, text, submatch=True)
        if any(m[0] == m[1] for m in full):
            continue  # nullable patterns are never anchored (whole-file path)
        # any superset of the true starts must give the same answer
        ws = []
        for m in full:
            lo = max(0, m[0] - rng.randint(0, 4))
            ws.append((lo, m[0] + rng.randint(0, 4)))
        for _ in range(rng.randint(0, 4)):
            a = rng.randint(0, max(0, len(text)))
            ws.append((a, a + rng.randint(0, 8)))
        ws.sort()
        merged = []
        for lo, hi in ws:
            if merged and lo <= merged[-1][1] + 1:
                merged[-1] = (merged[-1][0], max(hi, merged[-1][1]))
            else:
                merged.append((lo, hi))
        got = _lib.regex_find_all(pat, text, submatch=True, windows=merged)
        assert got == full, (pat, text, merged)


def test_bytes_to_lower_matches_oracle():
    rng = random.Random(5)
    for _ in range(200):
        b = _text(rng, [r"(?i)[a-z]{3}"], n_parts=rng.randint(0, 12))
        assert _lib.go_bytes_to_lower(b) == bytes_to_lower(b)


def test_compile_errors_agree():
    bad = ["a**", "(", "[a", "x{2}{3}", "\\1", "(?P<>a)", "a{1001}", "*a", "(?i", "[z-a]", "\\pL"]
    for p in bad:
        with pytest.raises(ValueError):
            GoRegexp(p)
        with pytest.raises(ValueError):
            _lib.regex_find_all(p, b"abc")


@pytest.mark.parametrize("idx", range(4))
def test_backtracker_equals_pike_vm(idx):
    """The bit-state backtracker, the Pike VM and the backtracker falling back to
    the Pike VM mid-search (8-position budget) give the same FindAll result,
    whole-text and windowed, for every builtin and golden custom regex."""
    rng = random.Random(7000 + idx)
    L = _lib.lib()
    try:
        for pat in PATTERNS + [r"(a|)+", r"(a*)+$", r"(?:(a)|b)*c"]:
            text = _text(rng, [pat], n_parts=12)
            wins = None
            if rng.random() < 0.5 and text:
                pts = sorted(rng.randrange(len(text)) for _ in range(6))
                wins = [(pts[k], pts[k + 1]) for k in range(0, 6, 2)]
            res = []
            for mode in (0, 1, 2):
                L.tsg_debug_regex_engine(mode)
                res.append(_lib.regex_find_all(pat, text, submatch=True, windows=wins))
            assert res[0] == res[1] == res[2], (pat, text, wins)
    finally:
        L.tsg_debug_regex_engine(0)


LITERALS = [r"(?i)example", r"abc", r"(?i)(ex)(?:am)ple", r"a\.b", r"(?i)akia", r"[xX]y", r"x", r"(?i)ghp_",
            # not literals (fold orbits past ASCII, non-ASCII runes, anchors): the engines decide
            r"(?i)ke", r"(?i)s", r"(?i)ſ", r"é", r"(?i)^ex", r"ex$", r"\bex"]


def test_literal_match_equals_engine():
    """Regex::Match's byte search for literal regexes (goregex.cpp MatchLiteral, auto
    mode only) against the Pike VM (mode 1) and the oracle, on texts with mixed case,
    the fold-special runes K (U+212A) / ſ (U+017F) / İ (U+0130) and invalid UTF-8."""
    rng = random.Random(4242)
    L = _lib.lib()
    alphabet = ["e", "E", "x", "X", "a", "A", "m", "p", "l", "L", "k", "K", "s", "ſ", "K", "İ", "é", "\udcff",
                "b", "c", ".", "y", "Y", "i", "g", "h", "_", "\n"]
    try:
        for pat in LITERALS:
            ref = GoRegexp(pat)
            for _ in range(150):
                parts = [rng.choice(alphabet) for _ in range(rng.randint(0, 14))]
                if rng.random() < 0.3:
                    parts.insert(rng.randint(0, len(parts)), sample_regex(pat, rng).decode("utf-8", "surrogateescape"))
                text = "".join(parts).encode("utf-8", "surrogateescape")
                L.tsg_debug_regex_engine(0)
                auto = _lib.regex_match(pat, text)
                L.tsg_debug_regex_engine(1)
                vm = _lib.regex_match(pat, text)
                assert auto == vm == ref.match_string(text), (pat, text)
    finally:
        L.tsg_debug_regex_engine(0)
