"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatements of the Go 1.22 standard-library behaviour the secret scanner
depends on (Go source is not in the image; semantics restated from the
published package documentation):

* ``decode_runes``      -- utf8.DecodeRune: invalid byte -> U+FFFD width 1
* ``bytes_to_lower``    -- bytes.ToLower (pkg/fanal/secret/scanner.go:178)
* ``strings_to_lower``  -- strings.ToLower (scanner.go:180)
* ``quote``             -- strconv.Quote, i.e. fmt's %q (scanner.go:442)
* ``fold_orbit``        -- unicode.SimpleFold orbit (regexp (?i) semantics)

Non-ASCII case mappings come from CPython's ``unicodedata`` (Unicode 13.0)
while Go 1.22 ships Unicode 15.0: parity for non-ASCII letters is UNPINNED
(no reference test exercises it).
"""
import unicodedata

RUNE_ERROR = 0xFFFD


def surrogate_to_rune(cp: int) -> int:
    """A ``surrogateescape`` code point stands for one invalid byte == U+FFFD."""
    return RUNE_ERROR if 0xDC80 <= cp <= 0xDCFF else cp


def decode(b: bytes) -> str:
    """UTF-8 decode with Go's rune model: every invalid byte becomes one
    surrogate code point (width 1), exactly as utf8.DecodeRune yields
    (RuneError, 1) for it.  Valid sequences decode to one code point."""
    return b.decode("utf-8", "surrogateescape")


def byte_offsets(s: str, b: bytes):
    """Prefix table: char index -> byte offset (identity when ``b`` is ASCII)."""
    if len(s) == len(b):
        return None
    offs = [0] * (len(s) + 1)
    o = 0
    for i, ch in enumerate(s):
        offs[i] = o
        cp = ord(ch)
        if cp < 0x80 or 0xDC80 <= cp <= 0xDCFF:
            o += 1
        elif cp < 0x800:
            o += 2
        elif cp < 0x10000:
            o += 3
        else:
            o += 4
    offs[len(s)] = o
    return offs


def go_lower_rune(cp: int) -> int:
    """unicode.ToLower (simple mapping)."""
    if cp < 0x80:
        return cp + 32 if 65 <= cp <= 90 else cp
    if 0xD800 <= cp <= 0xDFFF:
        return cp
    if cp == 0x130:  # UnicodeData simple lowercase of U+0130 is U+0069
        return 0x69
    low = chr(cp).lower()
    return ord(low) if len(low) == 1 else cp


def _map_lower(b: bytes) -> bytes:
    out = []
    for ch in decode(b):
        cp = surrogate_to_rune(ord(ch))
        out.append(chr(go_lower_rune(cp)))
    return "".join(out).encode("utf-8", "surrogatepass")


def bytes_to_lower(b: bytes) -> bytes:
    """bytes.ToLower: ASCII fast path, else bytes.Map(unicode.ToLower, s)
    with invalid bytes re-encoded as U+FFFD (EF BF BD)."""
    if b.isascii():
        return b.lower()
    return _map_lower(b)


def strings_to_lower(b: bytes) -> bytes:
    """strings.ToLower -- same mapping for our purposes."""
    return bytes_to_lower(b)


def _is_print(cp: int) -> bool:
    """unicode.IsPrint: L, M, N, P, S and the ASCII space."""
    if cp == 0x20:
        return True
    if 0xD800 <= cp <= 0xDFFF:
        return False
    cat = unicodedata.category(chr(cp))
    return cat[0] in "LMNPS"


def quote(b: bytes) -> str:
    """strconv.Quote of a Go string held as bytes."""
    out = ['"']
    for ch in decode(b):
        cp = ord(ch)
        if 0xDC80 <= cp <= 0xDCFF:  # invalid byte
            out.append("\\x%02x" % (cp - 0xDC00))
            continue
        if ch == '"' or ch == "\\":
            out.append("\\" + ch)
            continue
        if _is_print(cp):
            out.append(ch)
            continue
        esc = {7: "\\a", 8: "\\b", 12: "\\f", 10: "\\n", 13: "\\r", 9: "\\t", 11: "\\v"}
        if cp in esc:
            out.append(esc[cp])
        elif cp < 0x20 or cp == 0x7F:
            out.append("\\x%02x" % cp)
        elif cp < 0x10000:
            out.append("\\u%04x" % cp)
        else:
            out.append("\\U%08x" % cp)
    out.append('"')
    return "".join(out)


# --- unicode.SimpleFold orbits -------------------------------------------------

_ORBITS = None


def _fold_key(cp: int) -> int:
    if cp in (0x130, 0x131):  # no simple case folding for dotted/dotless i
        return cp
    if 0xD800 <= cp <= 0xDFFF:
        return cp
    c = chr(cp)
    up = c.upper()
    if len(up) == 1:
        low = up.lower()
        if len(low) == 1:
            return ord(low)
    low = c.lower()
    if len(low) == 1:
        return ord(low)
    return cp


def _build_orbits():
    groups = {}
    for cp in range(0x110000):
        k = _fold_key(cp)
        if k != cp:
            groups.setdefault(k, {k}).add(cp)
    orbits = {}
    for k, members in groups.items():
        # a key must itself map to itself to be a proper orbit representative
        fs = frozenset(members)
        for m in members:
            orbits[m] = fs
    return orbits


def fold_orbit(cp: int):
    """All runes equivalent to ``cp`` under simple case folding (incl. cp)."""
    global _ORBITS
    if cp < 0x80:
        c = chr(cp)
        if c in "kK":
            return frozenset((0x4B, 0x6B, 0x212A))
        if c in "sS":
            return frozenset((0x53, 0x73, 0x17F))
        if c.isalpha():
            return frozenset((ord(c.lower()), ord(c.upper())))
        return frozenset((cp,))
    if _ORBITS is None:
        _ORBITS = _build_orbits()
    return _ORBITS.get(cp, frozenset((cp,)))
