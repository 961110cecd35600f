"""CPU model of the scan kernel's automaton (test helper, not product code).

Reads the compiled tables through include/tsg_debug.h and replays the K1
semantics in Python: the bytes.ToLower symbol stream (C4 B0 -> 'i',
E2 84 AA -> 'k'; C5 BF -> 's' for anchors only), keyword bits per file and
anchor hits with the lookahead filter.  Used to check the gate's exactness
and the anchors' superset property against the oracle without a GPU.
"""
import ctypes as c

import numpy as np

from trivy_amd import _lib
from trivy_amd.secret.scanner import CGlobal, _CTableInfo


class _RuleInfo(c.Structure):
    _fields_ = [("nfa_words", c.c_uint32), ("gate", c.c_uint32), ("anchored", c.c_uint32),
                ("has_regex", c.c_uint32), ("nfa", c.c_void_p), ("kw_ids", c.c_void_p), ("n_kw", c.c_uint32)]


class Tables:
    def __init__(self, rules):
        L = _lib.lib()
        self._cg = CGlobal(rules, [], [])
        h = c.c_void_p()
        L.tsg_debug_compile.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
        if L.tsg_debug_compile(c.byref(self._cg.g), c.byref(h)) != 0:
            raise ValueError(_lib.last_error())
        self.h = h
        L.tsg_debug_compiled_info.argtypes = [c.c_void_p, c.c_void_p]
        info = _CTableInfo()
        L.tsg_debug_compiled_info(h, c.byref(info))
        self.info = {k: getattr(info, k) for k, _ in info._fields_}
        cm, tr, oo, oi = c.c_void_p(), c.c_void_p(), c.c_void_p(), c.c_void_p()
        no = c.c_uint32()
        L.tsg_debug_ac.argtypes = [c.c_void_p] + [c.c_void_p] * 5
        L.tsg_debug_ac(h, c.byref(cm), c.byref(tr), c.byref(oo), c.byref(oi), c.byref(no))
        ns, nc = self.info["ac_states"], self.info["ac_classes"]
        self.cmap = np.ctypeslib.as_array((c.c_uint8 * 256).from_address(cm.value)).copy()
        self.trans = np.ctypeslib.as_array((c.c_uint16 * (ns * nc)).from_address(tr.value)).copy()
        self.out_off = np.ctypeslib.as_array((c.c_uint32 * (ns + 1)).from_address(oo.value)).copy()
        self.out_items = np.ctypeslib.as_array((c.c_uint32 * max(1, no.value)).from_address(oi.value)).copy()
        self.nc = nc
        L.tsg_debug_rule.argtypes = [c.c_void_p, c.c_uint32, c.c_void_p]
        self.rules = []
        for i in range(len(rules)):
            ri = _RuleInfo()
            L.tsg_debug_rule(h, i, c.byref(ri))
            kws = list(np.ctypeslib.as_array((c.c_uint32 * max(1, ri.n_kw)).from_address(ri.kw_ids))[:ri.n_kw]) \
                if ri.n_kw else []
            self.rules.append({"gate": ri.gate, "anchored": ri.anchored, "kw": kws})
        L.tsg_debug_anchor.argtypes = [c.c_void_p, c.c_uint32] + [c.c_void_p] * 4
        self.anchors = []
        j = 0
        while True:
            r, ln, lo, hi = c.c_uint32(), c.c_uint32(), c.c_int32(), c.c_int32()
            if L.tsg_debug_anchor(h, j, c.byref(r), c.byref(ln), c.byref(lo), c.byref(hi)) != 0:
                break
            self.anchors.append((r.value, ln.value, lo.value, hi.value))
            j += 1

    def symbols(self, b: bytes):
        """(class, byte-end) per symbol of the lowered stream (fold sequences collapse)."""
        out = []
        i, n = 0, len(b)
        cm = self.cmap
        ci, ck, cs = cm[ord("i")], cm[ord("k")], cm[ord("s")]
        while i < n:
            x = b[i]
            m = cm[x]
            if m >= 0xFD:
                if x == 0xC4 and i + 1 < n and b[i + 1] == 0xB0:
                    out.append((ci, i + 2)); i += 2; continue
                if x == 0xE2 and i + 2 < n and b[i + 1] == 0x84 and b[i + 2] == 0xAA:
                    out.append((ck, i + 3)); i += 3; continue
                if x == 0xC5 and i + 1 < n and b[i + 1] == 0xBF:
                    out.append((cs, i + 2)); i += 2; continue
                m = 0
            out.append((m, i + 1))
            i += 1
        return out

    def run(self, b: bytes):
        """Returns (keyword id set, [(anchor id, literal end)], n flagged positions)."""
        st = 0
        kws, hits, flagged = set(), [], 0
        for cls, end in self.symbols(b):
            e = int(self.trans[st * self.nc + int(cls)])
            st = e & 0x7FFF
            if e & 0x8000:
                flagged += 1
                for item in self.out_items[self.out_off[st]:self.out_off[st + 1]]:
                    item = int(item)
                    if item >> 28 == 0:
                        kws.add(item & 0x0FFFFFFF)
                    else:
                        hits.append((item & 0x0FFFFFFF, end))
        return kws, hits, flagged
