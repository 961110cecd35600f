#!/usr/bin/env python3
"""Print the compiled GPU tables' facts for a rule set (no GPU needed)."""
import ctypes as c
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trivy_amd import _lib  # noqa: E402
from trivy_amd.secret import ParseConfig, builtin_rules, builtin_allow_rules  # noqa: E402
from trivy_amd.secret.scanner import CGlobal, _CTableInfo  # noqa: E402


def compiled(rules, allow=(), exclude=()):
    L = _lib.lib()
    cg = CGlobal(rules, allow, exclude)
    h = c.c_void_p()
    L.tsg_debug_compile.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    if L.tsg_debug_compile(c.byref(cg.g), c.byref(h)) != 0:
        raise ValueError(_lib.last_error())
    return L, h, cg


def main():
    rules = builtin_rules()
    if len(sys.argv) > 1:
        cfg = ParseConfig(sys.argv[1])
        rules = rules + cfg.CustomRules
    L, h, cg = compiled(rules, builtin_allow_rules())
    t = _CTableInfo()
    L.tsg_debug_compiled_info.argtypes = [c.c_void_p, c.c_void_p]
    L.tsg_debug_compiled_info(h, c.byref(t))
    print({k: getattr(t, k) for k, _ in t._fields_})


if __name__ == "__main__":
    main()


def anchors(rules):
    L, h, cg = compiled(rules)
    L.tsg_debug_anchor.argtypes = [c.c_void_p, c.c_uint32] + [c.c_void_p] * 4
    L.tsg_debug_keyword.argtypes = [c.c_void_p, c.c_uint32]
    L.tsg_debug_keyword.restype = c.c_char_p
    out = {}
    j = 0
    while True:
        r, ln, lo, hi = c.c_uint32(), c.c_uint32(), c.c_int32(), c.c_int32()
        if L.tsg_debug_anchor(h, j, c.byref(r), c.byref(ln), c.byref(lo), c.byref(hi)) != 0:
            break
        out.setdefault(rules[r.value].ID, []).append((ln.value, lo.value, hi.value))
        j += 1
    return out
