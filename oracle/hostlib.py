"""ctypes loader of oracle/build/libtsg_host.so (TEST INFRASTRUCTURE).

Loaded RTLD_LOCAL: it carries its own copy of the libtsg.so C-ABI, and handles
it creates (scanners, results) must go back to it -- pass ``hostlib.lib()`` as
the ``_lib`` of trivy_amd's Scanner / SecretAnalyzer.  Only tests/, smoke() and
bench.py's cpu_baseline use it.
"""
import ctypes as c
import os
from pathlib import Path

# TSG_HOSTLIB: an alternative build of the same library (tools/sanitize.sh: ASan/UBSan, TSan)
_PATH = Path(os.environ.get("TSG_HOSTLIB") or Path(__file__).resolve().parent / "build" / "libtsg_host.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not _PATH.exists():
            raise ImportError("%s is missing: run __graft_entry__.build()" % _PATH)
        L = c.CDLL(str(_PATH), mode=os.RTLD_NOW | os.RTLD_LOCAL)
        L.tsg_last_error.restype = c.c_char_p
        for name in ("tsg_debug_host_tail", "tsg_debug_scanner_host_only"):
            getattr(L, name).restype = c.c_int
        L.tsg_debug_host_tail.argtypes = [c.c_void_p, c.c_void_p, c.POINTER(c.c_void_p)]
        L.tsg_debug_host_tail_cands.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_uint64,
                                                c.POINTER(c.c_void_p)]
        L.tsg_debug_scanner_host_only.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
        L.tsg_cpuref_scan.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.POINTER(c.c_void_p)]
        _lib = L
    return _lib


def last_error():
    e = lib().tsg_last_error()
    return e.decode("utf-8", "replace") if e else ""
