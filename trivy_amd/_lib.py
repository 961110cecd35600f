"""ctypes binding of trivy_amd/libtsg.so (the C-ABI declared in include/*.h).

The library is built in-tree by trivy_amd/_build.py (``__graft_entry__.build()``).
There is no fallback: if the shared object is missing, importing the product
fails loudly.
"""
import ctypes
import os
from pathlib import Path

# TSG_LIB: an alternative build of the same library (tools/build_variant.py, tuning runs)
_PATH = Path(os.environ.get("TSG_LIB") or Path(__file__).resolve().parent / "libtsg.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not _PATH.exists():
            raise ImportError("trivy_amd native library %s is missing: run __graft_entry__.build()" % _PATH)
        _lib = ctypes.CDLL(str(_PATH), mode=os.RTLD_NOW | ctypes.RTLD_GLOBAL)
        _declare(_lib)
    return _lib


def _declare(L):
    c = ctypes
    L.tsg_last_error.restype = c.c_char_p
    L.tsg_regex_find_all.restype = c.c_int
    L.tsg_regex_find_all.argtypes = [c.c_char_p, c.c_char_p, c.c_uint64, c.c_int,
                                     c.POINTER(c.c_int64), c.c_uint32, c.POINTER(c.c_int64),
                                     c.c_uint64, c.POINTER(c.c_uint64), c.POINTER(c.c_int32)]
    L.tsg_regex_match.restype = c.c_int
    L.tsg_regex_match.argtypes = [c.c_char_p, c.c_char_p, c.c_uint64]
    L.tsg_go_bytes_to_lower.restype = c.c_int64
    L.tsg_go_bytes_to_lower.argtypes = [c.c_char_p, c.c_uint64, c.c_char_p, c.c_uint64]


def last_error(L=None):
    """Thread-local error text of library L (default libtsg.so)."""
    L = L if L is not None else lib()
    L.tsg_last_error.restype = ctypes.c_char_p
    e = L.tsg_last_error()
    return e.decode("utf-8", "replace") if e else ""


def regex_find_all(pattern: str, text: bytes, submatch=True, windows=None):
    """Go FindAll[Submatch]Index through the native engine -> list of index lists."""
    L = lib()
    pat = pattern.encode("utf-8", "surrogateescape")
    wbuf, nw = None, 0
    if windows is not None:
        flat = [x for w in windows for x in w]
        wbuf = (ctypes.c_int64 * max(1, len(flat)))(*flat)
        nw = len(windows)
    cap = 1 << 12
    while True:
        out = (ctypes.c_int64 * cap)()
        n = ctypes.c_uint64()
        ncap = ctypes.c_int32()
        rc = L.tsg_regex_find_all(pat, text, len(text), 1 if submatch else 0, wbuf, nw, out, cap,
                                  ctypes.byref(n), ctypes.byref(ncap))
        if rc != 0:
            raise ValueError(last_error())
        if n.value <= cap:
            break
        cap = n.value
    k = 2 * (ncap.value + 1) if submatch else 2
    flat = list(out[:n.value])
    return [flat[i:i + k] for i in range(0, len(flat), k)]


def regex_match(pattern: str, text: bytes) -> bool:
    rc = lib().tsg_regex_match(pattern.encode("utf-8", "surrogateescape"), text, len(text))
    if rc < 0:
        raise ValueError(last_error())
    return rc == 1


def go_bytes_to_lower(b: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(b) * 3 + 4)
    n = lib().tsg_go_bytes_to_lower(b, len(b), out, len(out))
    return out.raw[:n]
