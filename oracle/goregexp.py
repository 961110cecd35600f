"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement of Go 1.22 ``regexp`` (syntax ``regexp/syntax`` with the Perl flag
set that ``regexp.Compile`` uses: ClassNL | OneLine | PerlX | UnicodeGroups) for
the secret scanner's calls (pkg/fanal/secret/scanner.go:112, 130, 171, 207, 216,
264).

Design: parse the Go pattern into a small AST with Go's rules (scoped
``(?imsU)`` flags, ``(?P<n>)``/``(?<n>)``, ``\\Q..\\E``, octal/hex escapes,
ASCII Perl classes, POSIX classes, repeat limits, "a**" rejection, ``(?i)``
closing literals and classes under simple case folding), then emit an
*explicit* CPython ``re`` pattern: every literal/class becomes a bracket
expression of code points, ``$`` -> ``\\Z``, ``\\b`` -> ASCII look-arounds,
named groups -> positional groups (Go allows duplicate names).  CPython's
backtracking engine returns the leftmost-first (Perl-order) match and
submatches, which is exactly Go's ``regexp`` (non-POSIX) contract.

Input text is matched as ``bytes.decode('utf-8', 'surrogateescape')`` so that
each invalid byte is one code point standing for U+FFFD of width 1, as in
``utf8.DecodeRune``; classes containing U+FFFD therefore also contain the
escape range U+DC80..U+DCFF, and results are mapped back to byte offsets.
FindAll iteration restates ``(*Regexp).allMatches`` (empty-match rules).
"""
import re

from .gostd import decode, byte_offsets, fold_orbit

MAX_RUNE = 0x10FFFF
MAX_REPEAT = 1000


class GoRegexpError(ValueError):
    pass


# ----------------------------------------------------------------------------
# character classes as sorted, merged range lists
# ----------------------------------------------------------------------------

def clean(ranges):
    rs = sorted(ranges)
    out = []
    for lo, hi in rs:
        if out and lo <= out[-1][1] + 1:
            if hi > out[-1][1]:
                out[-1] = (out[-1][0], hi)
        else:
            out.append((lo, hi))
    return out


def negate(ranges):
    out, nxt = [], 0
    for lo, hi in clean(ranges):
        if lo > nxt:
            out.append((nxt, lo - 1))
        nxt = hi + 1
    if nxt <= MAX_RUNE:
        out.append((nxt, MAX_RUNE))
    return out


def fold_ranges(ranges):
    """appendFoldedRange: close each range under simple case folding."""
    out = list(ranges)
    for lo, hi in ranges:
        if hi - lo > 0x3000 and lo <= 0x80:
            # huge ranges: fold only the cased part we know about cheaply
            span_hi = min(hi, 0x1FFFF)
        else:
            span_hi = hi
        for cp in range(lo, span_hi + 1):
            for o in fold_orbit(cp):
                if not (lo <= o <= hi):
                    out.append((o, o))
    return clean(out)


PERL = {
    "d": [(0x30, 0x39)],
    "s": [(0x09, 0x0A), (0x0C, 0x0D), (0x20, 0x20)],
    "w": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
}

POSIX = {
    "alnum": [(0x30, 0x39), (0x41, 0x5A), (0x61, 0x7A)],
    "alpha": [(0x41, 0x5A), (0x61, 0x7A)],
    "ascii": [(0x00, 0x7F)],
    "blank": [(0x09, 0x09), (0x20, 0x20)],
    "cntrl": [(0x00, 0x1F), (0x7F, 0x7F)],
    "digit": [(0x30, 0x39)],
    "graph": [(0x21, 0x7E)],
    "lower": [(0x61, 0x7A)],
    "print": [(0x20, 0x7E)],
    "punct": [(0x21, 0x2F), (0x3A, 0x40), (0x5B, 0x60), (0x7B, 0x7E)],
    "space": [(0x09, 0x0D), (0x20, 0x20)],
    "upper": [(0x41, 0x5A)],
    "word": [(0x30, 0x39), (0x41, 0x5A), (0x5F, 0x5F), (0x61, 0x7A)],
    "xdigit": [(0x30, 0x39), (0x41, 0x46), (0x61, 0x66)],
}

# ----------------------------------------------------------------------------
# AST: ('class', ranges) ('empty',) ('assert', kind) ('cat', [..]) ('alt', [..])
#      ('cap', idx, sub) ('rep', min, max(-1 = inf), greedy, sub)
# ----------------------------------------------------------------------------


class _Parser:
    def __init__(self, pat: str):
        self.s = pat
        self.i = 0
        self.fi = False  # (?i)
        self.fm = False  # (?m)  (clears OneLine)
        self.fs = False  # (?s)
        self.fU = False  # (?U)
        self.ncap = 0
        self.names = [""]

    def err(self, msg):
        raise GoRegexpError("error parsing regexp: %s: `%s`" % (msg, self.s))

    def peek(self, k=0):
        j = self.i + k
        return self.s[j] if j < len(self.s) else None

    def parse(self):
        node = self.alt()
        if self.i < len(self.s):
            if self.s[self.i] == ")":
                self.err("unexpected )")
            self.err("trailing input")
        return node

    def alt(self):
        branches = [self.concat()]
        while self.peek() == "|":
            self.i += 1
            branches.append(self.concat())
        return branches[0] if len(branches) == 1 else ("alt", branches)

    def concat(self):
        items = []
        while True:
            c = self.peek()
            if c is None or c in "|)":
                break
            if c in "*+?":
                self.err("missing argument to repetition operator")
            if c == "{" and self._repeat_spec(self.i) is not None:
                self.err("missing argument to repetition operator")
            atom = self.atom()
            if atom is None:  # flag group (?i)
                continue
            atom = self.repeats(atom)
            if atom[0] == "quote":
                items.extend(atom[1])
            else:
                items.append(atom)
        if not items:
            return ("empty",)
        return items[0] if len(items) == 1 else ("cat", items)

    def _repeat_spec(self, j):
        m = re.match(r"\{(\d+)(,(\d*))?\}", self.s[j:])
        if not m:
            return None
        lo = int(m.group(1))
        if m.group(2) is None:
            hi = lo
        elif m.group(3) == "":
            hi = -1
        else:
            hi = int(m.group(3))
        return lo, hi, m.end()

    def repeats(self, atom):
        last = None
        while True:
            c = self.peek()
            if c in ("*", "+", "?"):
                lo, hi = {"*": (0, -1), "+": (1, -1), "?": (0, 1)}[c]
                ln = 1
            elif c == "{":
                spec = self._repeat_spec(self.i)
                if spec is None:
                    return atom
                lo, hi, ln = spec
                if lo > MAX_REPEAT or hi > MAX_REPEAT or (hi >= 0 and lo > hi):
                    self.err("invalid repeat count")
            else:
                return atom
            if last is not None:
                self.err("invalid nested repetition operator")
            self.i += ln
            greedy = True
            if self.peek() == "?":
                self.i += 1
                greedy = False
            if self.fU:
                greedy = not greedy
            if atom[0] == "quote":
                # \Q..\E: repetition applies to the last literal only
                lits = atom[1]
                atom = ("quote", lits[:-1] + [("rep", lo, hi, greedy, lits[-1])])
            else:
                atom = ("rep", lo, hi, greedy, atom)
            last = c

    def literal(self, cp):
        if self.fi:
            orb = fold_orbit(cp)
            return ("class", clean([(o, o) for o in orb]))
        return ("class", [(cp, cp)])

    def atom(self):
        c = self.s[self.i]
        if c == "(":
            return self.group()
        if c == "[":
            return self.cls()
        if c == ".":
            self.i += 1
            if self.fs:
                return ("class", [(0, MAX_RUNE)])
            return ("class", [(0, 9), (11, MAX_RUNE)])
        if c == "^":
            self.i += 1
            return ("assert", "bol" if self.fm else "bot")
        if c == "$":
            self.i += 1
            return ("assert", "eol" if self.fm else "eot")
        if c == "\\":
            return self.escape_atom()
        self.i += 1
        return self.literal(ord(c))

    def group(self):
        s = self.s
        if s.startswith("(?P<", self.i) or (s.startswith("(?<", self.i) and not s.startswith("(?<=", self.i) and not s.startswith("(?<!", self.i)):
            start = self.i + (4 if s.startswith("(?P<", self.i) else 3)
            end = s.find(">", start)
            if end < 0:
                self.err("invalid named capture")
            name = s[start:end]
            if not name or not re.fullmatch(r"[A-Za-z0-9_]+", name):
                self.err("invalid named capture")
            self.i = end + 1
            return self.capture(name)
        if s.startswith("(?", self.i):
            j = self.i + 2
            neg = False
            fl = {"i": self.fi, "m": self.fm, "s": self.fs, "U": self.fU}
            seen = False
            while j < len(s):
                ch = s[j]
                if ch in "imsU":
                    fl[ch] = not neg
                    seen = True
                elif ch == "-":
                    if neg:
                        self.err("invalid or unsupported Perl syntax")
                    neg = True
                    seen = False
                elif ch == ":" or ch == ")":
                    if neg and not seen:
                        self.err("invalid or unsupported Perl syntax")
                    if ch == ")" and not seen and not neg:
                        self.err("missing argument to repetition operator" if False else "invalid or unsupported Perl syntax")
                    break
                else:
                    self.err("invalid or unsupported Perl syntax")
                j += 1
            else:
                self.err("missing closing )")
            if s[j] == ")":
                # (?flags): affects the rest of the current group
                self.fi, self.fm, self.fs, self.fU = fl["i"], fl["m"], fl["s"], fl["U"]
                self.i = j + 1
                return None
            # (?flags:re) scoped, non-capturing
            saved = (self.fi, self.fm, self.fs, self.fU)
            self.fi, self.fm, self.fs, self.fU = fl["i"], fl["m"], fl["s"], fl["U"]
            self.i = j + 1
            sub = self.alt()
            if self.peek() != ")":
                self.err("missing closing )")
            self.i += 1
            self.fi, self.fm, self.fs, self.fU = saved
            return ("group", sub)
        self.i += 1
        return self.capture("", opened=True)

    def capture(self, name, opened=False):
        self.ncap += 1
        idx = self.ncap
        self.names.append(name)
        saved = (self.fi, self.fm, self.fs, self.fU)
        sub = self.alt()
        if self.peek() != ")":
            self.err("missing closing )")
        self.i += 1
        self.fi, self.fm, self.fs, self.fU = saved
        return ("cap", idx, sub)

    def hexval(self, txt):
        try:
            v = int(txt, 16)
        except ValueError:
            self.err("invalid escape sequence")
        if v > MAX_RUNE:
            self.err("invalid escape sequence")
        return v

    def escape_rune(self):
        """parseEscape: returns a code point; self.i points after the backslash."""
        s = self.s
        if self.i >= len(s):
            self.err("trailing backslash at end of expression")
        c = s[self.i]
        self.i += 1
        if c in "1234567":
            nxt = self.peek()
            if nxt is None or not ("0" <= nxt <= "7"):
                self.err("invalid escape sequence")
            c = "0"
            self.i -= 1
        if c == "0":
            v = 0
            for _ in range(2):
                nxt = self.peek()
                if nxt is not None and "0" <= nxt <= "7":
                    v = v * 8 + int(nxt)
                    self.i += 1
                else:
                    break
            return v
        if c == "x":
            if self.peek() == "{":
                end = s.find("}", self.i)
                if end < 0 or end == self.i + 1:
                    self.err("invalid escape sequence")
                v = self.hexval(s[self.i + 1:end])
                self.i = end + 1
                return v
            txt = s[self.i:self.i + 2]
            if len(txt) < 2 or not re.fullmatch(r"[0-9A-Fa-f]{2}", txt):
                self.err("invalid escape sequence")
            self.i += 2
            return int(txt, 16)
        simple = {"a": 7, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11}
        if c in simple:
            return simple[c]
        if ord(c) < 0x80 and not c.isalnum():
            return ord(c)
        self.err("invalid escape sequence")

    def escape_atom(self):
        s = self.s
        self.i += 1
        if self.i >= len(s):
            self.err("trailing backslash at end of expression")
        c = s[self.i]
        if c in "AzbB":
            self.i += 1
            return ("assert", {"A": "bot", "z": "eot", "b": "wordb", "B": "nwordb"}[c])
        if c in "dDsSwW":
            self.i += 1
            rng = PERL[c.lower()]
            return ("class", negate(rng) if c.isupper() else list(rng))
        if c in "pP":
            self.err("unicode classes unsupported in oracle")
        if c == "Q":
            end = s.find("\\E", self.i + 1)
            lit = s[self.i + 1:] if end < 0 else s[self.i + 1:end]
            self.i = len(s) if end < 0 else end + 2
            lits = [self.literal(ord(ch)) for ch in lit]
            if not lits:
                return ("empty",)
            return ("quote", lits)
        return self.literal(self.escape_rune())

    def cls(self):
        s = self.s
        self.i += 1
        negated = False
        if self.peek() == "^":
            negated = True
            self.i += 1
        ranges = []
        first = True
        while True:
            c = self.peek()
            if c is None:
                self.err("missing closing ]")
            if c == "]" and not first:
                self.i += 1
                break
            first = False
            if c == "[" and self.peek(1) == ":":
                m = re.match(r"\[:(\^?)([a-z]+):\]", s[self.i:])
                if m and m.group(2) in POSIX:
                    rng = POSIX[m.group(2)]
                    if m.group(1):
                        rng = negate(rng)
                    ranges += fold_ranges(rng) if self.fi else rng
                    self.i += m.end()
                    continue
            if c == "\\" and self.peek(1) in tuple("dDsSwW"):
                k = self.peek(1)
                rng = PERL[k.lower()]
                ranges += negate(rng) if k.isupper() else rng
                self.i += 2
                continue
            if c == "\\" and self.peek(1) in ("p", "P"):
                self.err("unicode classes unsupported in oracle")
            lo = self.class_char()
            hi = lo
            if self.peek() == "-" and self.peek(1) is not None and self.peek(1) != "]":
                self.i += 1
                hi = self.class_char()
                if hi < lo:
                    self.err("invalid character class range")
            if self.fi:
                ranges += fold_ranges([(lo, hi)])
            else:
                ranges.append((lo, hi))
        ranges = clean(ranges)
        if negated:
            ranges = negate(ranges)
        return ("class", ranges)

    def class_char(self):
        c = self.s[self.i]
        if c == "\\":
            self.i += 1
            return self.escape_rune()
        self.i += 1
        return ord(c)


# ----------------------------------------------------------------------------
# emission to CPython re
# ----------------------------------------------------------------------------

_WORD = "[0-9A-Za-z_]"
_ASSERT = {
    "bot": r"\A",
    "eot": r"\Z",
    "bol": r"(?:\A|(?<=\n))",
    "eol": r"(?=\n|\Z)",
    "wordb": r"(?:(?<!%s)(?=%s)|(?<=%s)(?!%s))" % ((_WORD,) * 4),
    "nwordb": r"(?:(?<=%s)(?=%s)|(?<!%s)(?!%s))" % ((_WORD,) * 4),
}


def _cp(c):
    return "\\U%08x" % c if c > 0xFFFF else "\\u%04x" % c


def _emit_class(ranges):
    has_fffd = any(lo <= 0xFFFD <= hi for lo, hi in ranges)
    rs = []
    for lo, hi in ranges:  # Go never produces surrogate runes from input
        if hi < 0xD800 or lo > 0xDFFF:
            rs.append((lo, hi))
        else:
            if lo < 0xD800:
                rs.append((lo, 0xD7FF))
            if hi > 0xDFFF:
                rs.append((0xE000, hi))
    if has_fffd:
        rs.append((0xDC80, 0xDCFF))
    rs = clean(rs)
    if not rs:
        return "(?!)"
    body = "".join(_cp(lo) if lo == hi else _cp(lo) + "-" + _cp(hi) for lo, hi in rs)
    return "[" + body + "]"


def _emit(node):
    kind = node[0]
    if kind == "class":
        return _emit_class(node[1])
    if kind == "empty":
        return ""
    if kind == "assert":
        return _ASSERT[node[1]]
    if kind == "cat":
        return "".join(_emit(n) for n in node[1])
    if kind == "alt":
        return "(?:" + "|".join(_emit(n) for n in node[1]) + ")"
    if kind == "cap":
        return "(" + _emit(node[2]) + ")"
    if kind == "group":
        return "(?:" + _emit(node[1]) + ")"
    if kind == "rep":
        _, lo, hi, greedy, sub = node
        if hi == -1:
            q = "*" if lo == 0 else ("+" if lo == 1 else "{%d,}" % lo)
        elif lo == hi:
            q = "{%d}" % lo
        elif lo == 0 and hi == 1:
            q = "?"
        else:
            q = "{%d,%d}" % (lo, hi)
        return "(?:" + _emit(sub) + ")" + q + ("" if greedy else "?")
    if kind == "quote":
        return "".join(_emit(n) for n in node[1])
    raise AssertionError(kind)


class GoRegexp:
    """regexp.Regexp restatement (only the methods scanner.go calls)."""

    def __init__(self, pattern: str):
        if isinstance(pattern, bytes):
            pattern = pattern.decode("utf-8", "surrogateescape")
        self.pattern = pattern
        p = _Parser(pattern)
        ast = p.parse()
        self.ast = ast
        self.subexp_names = p.names  # index 0 is the whole match (""), as SubexpNames()
        self.num_subexp = p.ncap
        self.py = _emit(ast)
        self._re = re.compile(self.py)

    def __repr__(self):
        return "GoRegexp(%r)" % self.pattern

    def _prep(self, b: bytes):
        s = decode(b)
        return s, byte_offsets(s, b)

    def find_all_submatch_index(self, b: bytes):
        """FindAllSubmatchIndex(b, -1) with byte offsets; -1 for unset groups."""
        s, offs = self._prep(b)
        out = []
        end = len(s)
        pos, prev_end = 0, -1
        while pos <= end:
            m = self._re.search(s, pos)
            if m is None:
                break
            accept = True
            if m.end() == pos:  # empty match
                if m.start() == prev_end:
                    accept = False
                pos += 1
            else:
                pos = m.end()
            prev_end = m.end()
            if accept:
                idx = []
                for g in range(self.num_subexp + 1):
                    a, z = m.span(g)
                    if a < 0:
                        idx += [-1, -1]
                    elif offs is None:
                        idx += [a, z]
                    else:
                        idx += [offs[a], offs[z]]
                out.append(idx)
        return out

    def find_all_index(self, b: bytes):
        return [m[:2] for m in self.find_all_submatch_index(b)]

    def match_string(self, b: bytes) -> bool:
        if isinstance(b, str):
            b = b.encode("utf-8", "surrogateescape")
        return self._re.search(decode(b)) is not None


def compile(pattern):
    return GoRegexp(pattern)
