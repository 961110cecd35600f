"""Scanner: pkg/fanal/secret/scanner.go:320-463 over the MI355X engine.

``NewScanner`` assembles the rule set exactly as the reference does
(scanner.go:320-364) and hands the resulting Global to ``tsg_scanner_new``;
``Scan``/``ScanBatch`` submit contents through ``tsg_scan`` and decode the
findings into ``types.Secret``-shaped objects (pkg/fanal/types/secret.go).
"""
import ctypes
import json
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from .. import _lib
from .config import AllowRule, Config, Rule, builtin_allow_rules, builtin_rules

c = ctypes


class _CAllowRule(c.Structure):
    _fields_ = [("id", c.c_char_p), ("regex", c.c_char_p), ("path", c.c_char_p)]


class _CRule(c.Structure):
    _fields_ = [("id", c.c_char_p), ("category", c.c_char_p), ("title", c.c_char_p),
                ("severity", c.c_char_p), ("regex", c.c_char_p), ("path", c.c_char_p),
                ("secret_group_name", c.c_char_p), ("keywords", c.POINTER(c.c_char_p)),
                ("n_keywords", c.c_uint32), ("allow_rules", c.POINTER(_CAllowRule)),
                ("n_allow_rules", c.c_uint32), ("exclude_regexes", c.POINTER(c.c_char_p)),
                ("n_exclude_regexes", c.c_uint32)]


class _CGlobal(c.Structure):
    _fields_ = [("rules", c.POINTER(_CRule)), ("n_rules", c.c_uint32),
                ("allow_rules", c.POINTER(_CAllowRule)), ("n_allow_rules", c.c_uint32),
                ("exclude_regexes", c.POINTER(c.c_char_p)), ("n_exclude_regexes", c.c_uint32)]


class _CBatch(c.Structure):
    _fields_ = [("n_files", c.c_uint32), ("host_arena", c.c_void_p), ("host_offsets", c.c_void_p),
                ("dev_arena", c.c_void_p), ("dev_offsets", c.c_void_p), ("paths", c.c_void_p),
                ("path_lens", c.c_void_p), ("binary", c.c_void_p), ("transform", c.c_void_p),
                ("dev_paths", c.c_void_p), ("dev_path_offsets", c.c_void_p)]  # frozen (round-4 layout)


class _CBatchExt(c.Structure):  # tsg_batch_ext: struct_size first, then the fields past tsg_batch
    _fields_ = [("struct_size", c.c_uint32), ("base", _CBatch),
                ("host_paths", c.c_void_p), ("host_path_offsets", c.c_void_p),
                ("gather_base", c.c_void_p), ("gather_src", c.c_void_p)]


BATCH_EXT_SIZE_V1 = _CBatchExt.gather_base.offset  # TSG_BATCH_EXT_SIZE_V1 (round 5: host paths)
BATCH_EXT_SIZE_V2 = c.sizeof(_CBatchExt)  # TSG_BATCH_EXT_SIZE_V2 (round 6: + gather_base / gather_src)


class _CCompileOptions(c.Structure):  # tsg_compile_options (versioned: struct_size first)
    _fields_ = [("struct_size", c.c_uint32), ("reserved", c.c_uint32), ("calib", c.c_void_p),
                ("calib_bytes", c.c_uint64)]


COMPILE_OPTIONS_SIZE_V1 = c.sizeof(_CCompileOptions)


def compile_options(calibration):
    """(buffer kept alive, tsg_compile_options) for a calibration sample."""
    buf = np.frombuffer(calibration, dtype=np.uint8) if isinstance(calibration, (bytes, bytearray)) \
        else np.ascontiguousarray(calibration, dtype=np.uint8)
    return buf, _CCompileOptions(COMPILE_OPTIONS_SIZE_V1, 0, buf.ctypes.data if len(buf) else None, len(buf))


class _CStats(c.Structure):
    _fields_ = [(n, c.c_uint64) for n in ("bytes", "files", "anchor_hits", "candidates", "special_files",
                                          "findings")] + \
               [(n, c.c_double) for n in ("ms_scan_kernel", "ms_verify_kernel", "ms_fullscan_kernel",
                                          "ms_gpu_total", "ms_host_gpu_phase", "ms_host_allow_path",
                                          "ms_host_exact", "ms_host_total")] + \
               [("flagged_blocks", c.c_uint64), ("ms_careful_kernel", c.c_double),
                ("follow_hits", c.c_uint64)] + \
               [(n, c.c_double) for n in ("ms_chunkmap_kernel", "ms_confirm_kernel", "ms_nfa_kernel",
                                          "ms_finalize_kernel", "ms_h2d_span")] + \
               [("h2d_chunks", c.c_uint64), ("fullscan_pairs", c.c_uint64), ("fold_sites", c.c_uint64),
                ("ms_xform_kernel", c.c_double)]


class _CTableInfo(c.Structure):
    _fields_ = [(n, c.c_uint32) for n in ("n_rules", "n_keywords", "n_anchors", "n_filter_items",
                                          "n_filter_buckets", "filter_window", "n_fullscan_rules",
                                          "nfa_words_total")] + \
               [("filter_table_bytes", c.c_uint64), ("filter_est_fp", c.c_double)]


def _declare(L):
    if getattr(L, "_tsg_scanner_declared", False):
        return
    L.tsg_scanner_new.argtypes = [c.POINTER(_CGlobal), c.c_int, c.POINTER(c.c_void_p)]
    L.tsg_scanner_new_ex.argtypes = [c.POINTER(_CGlobal), c.c_int, c.c_void_p, c.POINTER(c.c_void_p)]
    L.tsg_scanner_free.argtypes = [c.c_void_p]
    L.tsg_scanner_allow_path.argtypes = [c.c_void_p, c.c_char_p, c.c_uint64]
    L.tsg_scan.argtypes = [c.c_void_p, c.POINTER(_CBatch), c.POINTER(c.c_void_p)]
    L.tsg_scan_submit.argtypes = [c.c_void_p, c.POINTER(_CBatch), c.POINTER(c.c_void_p)]
    L.tsg_scan_ext.argtypes = [c.c_void_p, c.POINTER(_CBatchExt), c.POINTER(c.c_void_p)]
    L.tsg_scan_submit_ext.argtypes = [c.c_void_p, c.POINTER(_CBatchExt), c.POINTER(c.c_void_p)]
    L.tsg_scan_wait.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    L.tsg_result_free.argtypes = [c.c_void_p]
    L.tsg_result_json.argtypes = [c.c_void_p, c.POINTER(c.c_void_p), c.POINTER(c.c_uint64)]
    L.tsg_result_json_range.argtypes = [c.c_void_p, c.c_uint32, c.c_uint32, c.POINTER(c.c_void_p),
                                        c.POINTER(c.c_uint64)]
    L.tsg_result_stats.argtypes = [c.c_void_p, c.POINTER(_CStats)]
    if hasattr(L, "tsg_result_records"):
        L.tsg_result_records.argtypes = [c.c_void_p, c.c_void_p, c.c_uint64]
        L.tsg_result_records.restype = c.c_uint64
    L.tsg_scanner_table_info.argtypes = [c.c_void_p, c.POINTER(_CTableInfo)]
    L.tsg_scanner_rule_anchor.argtypes = [c.c_void_p, c.c_uint32]
    L.tsg_scanner_rule_anchor.restype = c.c_char_p
    L.tsg_host_register.argtypes = [c.c_void_p, c.c_uint64]
    L.tsg_host_register_mapped.argtypes = [c.c_void_p, c.c_uint64]
    L.tsg_host_unregister.argtypes = [c.c_void_p]
    L._tsg_scanner_declared = True


def _b(s) -> Optional[bytes]:
    if s is None:
        return None
    if isinstance(s, bytes):
        return s
    return str(s).encode("utf-8", "surrogateescape")


def _s(latin: str) -> str:
    """JSON strings from the library carry raw bytes as latin-1 code points."""
    return latin.encode("latin-1").decode("utf-8", "surrogateescape")


@dataclass
class Line:  # pkg/fanal/types/misconf.go:52-61
    Number: int = 0
    Content: str = ""
    IsCause: bool = False
    Annotation: str = ""
    Truncated: bool = False
    Highlighted: str = ""
    FirstCause: bool = False
    LastCause: bool = False


@dataclass
class Code:  # misconf.go:48-50 (Lines is None for binary files: types.Code{})
    Lines: Optional[List[Line]] = field(default_factory=list)


@dataclass
class SecretFinding:  # pkg/fanal/types/secret.go:10-20
    RuleID: str = ""
    Category: str = ""
    Severity: str = ""
    Title: str = ""
    StartLine: int = 0
    EndLine: int = 0
    Code: Code = field(default_factory=Code)
    Match: str = ""

    def to_dict(self):
        return {"RuleID": self.RuleID, "Category": self.Category, "Severity": self.Severity,
                "Title": self.Title, "StartLine": self.StartLine, "EndLine": self.EndLine,
                "Code": {"Lines": None if self.Code.Lines is None else [dict(l.__dict__) for l in self.Code.Lines]},
                "Match": self.Match}


@dataclass
class Secret:  # pkg/fanal/types/secret.go:5-8
    FilePath: str = ""
    Findings: Optional[List[SecretFinding]] = None

    def to_dict(self):
        return {"FilePath": self.FilePath,
                "Findings": None if self.Findings is None else [f.to_dict() for f in self.Findings]}


@dataclass
class ScanArgs:  # scanner.go:366-370
    FilePath: str
    Content: bytes
    Binary: bool = False


class CGlobal:
    """tsg_global built from an assembled rule set (keeps the C strings alive)."""

    def __init__(self, rules: Sequence[Rule], allow_rules: Sequence[AllowRule], exclude_regexes: Sequence[str]):
        self.Rules = list(rules)
        self.AllowRules = list(allow_rules)
        self.ExcludeRegexes = list(exclude_regexes)
        self._keep = []
        self.g = self._build_global()

    def _cstrs(self, items):
        arr = (c.c_char_p * max(1, len(items)))(*[_b(x) for x in items])
        self._keep.append(arr)
        return arr

    def _callow(self, items):
        arr = (_CAllowRule * max(1, len(items)))()
        for i, a in enumerate(items):
            arr[i].id = _b(a.ID)
            arr[i].regex = _b(a.Regex)  # None = no regex; "" is a regex (matches everything)
            arr[i].path = _b(a.Path)
        self._keep.append(arr)
        return arr

    def _build_global(self):
        rs = (_CRule * max(1, len(self.Rules)))()
        for i, r in enumerate(self.Rules):
            x = rs[i]
            x.id, x.category, x.title, x.severity = _b(r.ID), _b(r.Category), _b(r.Title), _b(r.Severity)
            x.regex = _b(r.Regex)
            x.path = _b(r.Path)
            x.secret_group_name = _b(r.SecretGroupName or "")
            x.keywords = self._cstrs(r.Keywords)
            x.n_keywords = len(r.Keywords)
            x.allow_rules = self._callow(r.AllowRules)
            x.n_allow_rules = len(r.AllowRules)
            x.exclude_regexes = self._cstrs(r.ExcludeBlock.Regexes)
            x.n_exclude_regexes = len(r.ExcludeBlock.Regexes)
        self._keep.append(rs)
        return _CGlobal(rs, len(self.Rules), self._callow(self.AllowRules), len(self.AllowRules),
                        self._cstrs(self.ExcludeRegexes), len(self.ExcludeRegexes))


class Scanner:
    """secret.Scanner: an assembled Global bound to one HIP device."""

    def __init__(self, rules: Sequence[Rule], allow_rules: Sequence[AllowRule], exclude_regexes: Sequence[str],
                 device: int = 0, lib=None, host_only: bool = False, calibration=None):
        """lib: the C-ABI library (default libtsg.so).  host_only (tests): a scanner without a
        GPU engine from the oracle's library (oracle/hostlib.py), whose tsg_scan fails."""
        self.Rules = list(rules)
        self.AllowRules = list(allow_rules)
        self.ExcludeRegexes = list(exclude_regexes)
        L = lib if lib is not None else _lib.lib()
        _declare(L)
        self._L = L
        self._cg = CGlobal(rules, allow_rules, exclude_regexes)
        g = self._cg.g
        h = c.c_void_p()
        if host_only:
            rc = L.tsg_debug_scanner_host_only(c.byref(g), c.byref(h))
        elif calibration is not None:
            keep, opt = compile_options(calibration)
            rc = L.tsg_scanner_new_ex(c.byref(g), int(device), c.byref(opt), c.byref(h))
        else:
            rc = L.tsg_scanner_new(c.byref(g), int(device), c.byref(h))
        if rc != 0:
            raise RuntimeError("tsg_scanner_new failed: %s" % _lib.last_error(L))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.tsg_scanner_free(h)
            self._h = None

    # --- reference API -----------------------------------------------------
    def AllowPath(self, path) -> bool:  # scanner.go:57-59
        p = _b(path)
        return self._L.tsg_scanner_allow_path(self._h, p, len(p)) == 1

    def Scan(self, args: ScanArgs) -> Secret:  # scanner.go:377-463
        return self.ScanBatch([args])[0]

    def ScanBatch(self, args: Sequence[ScanArgs]) -> List[Secret]:
        contents = [a.Content for a in args]
        offs = np.zeros(len(contents) + 1, dtype=np.uint64)
        if contents:
            offs[1:] = np.cumsum([len(x) for x in contents], dtype=np.uint64)
        arena = b"".join(contents) + b"\0" * 16
        res = self.scan_arena(arena, offs, [a.FilePath for a in args],
                              binary=[bool(a.Binary) for a in args])
        return res.secrets([a.FilePath for a in args])

    # --- batched arena API (analyzer / bench) -------------------------------
    def scan_arena_async(self, arena, offsets, paths, binary=None, dev_arena=None, dev_offsets=None,
                         dev_paths=None, dev_path_offsets=None, transform=None):
        """Pipelined scan (tsg_scan_submit): returns a PendingScan; .wait() gives the ScanResult.
        The arrays passed must stay alive until then (the PendingScan keeps references)."""
        keep, batch = self._batch(arena, offsets, paths, binary, dev_arena, dev_offsets, dev_paths,
                                  dev_path_offsets, transform)
        h = c.c_void_p()
        rc = self._L.tsg_scan_submit(self._h, c.byref(batch), c.byref(h))
        if rc != 0:
            raise RuntimeError("tsg_scan_submit failed: %s" % _lib.last_error(self._L))
        return PendingScan(self, h, (keep, batch))

    def _batch(self, arena, offsets, paths, binary, dev_arena, dev_offsets, dev_paths=None, dev_path_offsets=None,
               transform=None):
        """transform: per-file pre-transform kinds (uint8; 1 = CR strip, 2 = printable runs) run on the
        GPU over the host arena (the bytes as read)."""
        n = len(offsets) - 1
        arena_buf = np.frombuffer(arena, dtype=np.uint8) if isinstance(arena, (bytes, bytearray)) else arena
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        plen = None
        if isinstance(paths, np.ndarray) and paths.dtype == np.uint64:
            parr, plen_ptr = paths, None  # char* table (caller keeps the strings alive)
            paths_addr = paths.ctypes.data
        else:
            pb = [_b(p) for p in paths]
            parr = (c.c_char_p * max(1, n))(*pb)
            plen = np.array([len(p) for p in pb], dtype=np.uint64) if n else np.zeros(1, np.uint64)
            paths_addr = c.cast(parr, c.c_void_p).value
            plen_ptr = plen.ctypes.data
        bin_arr = np.array(binary, dtype=np.uint8) if binary is not None else None
        batch = _CBatch(n, arena_buf.ctypes.data, offs.ctypes.data,
                        dev_arena, dev_offsets, paths_addr, plen_ptr,
                        bin_arr.ctypes.data if bin_arr is not None else None,
                        transform.ctypes.data if transform is not None else None,
                        dev_paths, dev_path_offsets)
        return (arena_buf, offs, parr, plen, bin_arr, transform), batch

    def scan_arena(self, arena, offsets, paths, binary=None, dev_arena=None, dev_offsets=None, dev_paths=None,
                   dev_path_offsets=None, host_paths=None, host_path_offsets=None, gather_base=None,
                   gather_src=None, transform=None):
        """One batch (tsg_scan).  dev_arena / dev_offsets: the contents already in HBM;
        dev_paths / dev_path_offsets: the paths packed in HBM (GPU allow-path prefilter);
        host_paths / host_path_offsets (numpy u8 / u64): the paths packed in host memory, passed
        through the versioned tsg_batch_ext (tsg_scan_ext).  gather_base (a uint8 array registered
        with HostRegister(mapped=True)) / gather_src (u64): file f's bytes as read are
        gather_base[gather_src[f]:][:offsets[f+1]-offsets[f]] -- arena None, transform (u8 per file:
        1 text, 2 binary) required (tsg_batch_ext v2)."""
        n = len(offsets) - 1
        if gather_base is not None:
            if arena is not None or transform is None or gather_src is None:
                raise ValueError("scan_arena(gather): arena None, gather_src and transform required")
            arena = np.zeros(1, np.uint8)  # (not passed: host_arena is NULL in a gathered batch)
        arena_buf = np.frombuffer(arena, dtype=np.uint8) if isinstance(arena, (bytes, bytearray)) else arena
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        if isinstance(paths, np.ndarray) and paths.dtype == np.uint64:
            parr, plen_ptr = paths, None  # char* table (caller keeps the strings alive)
            paths_addr = paths.ctypes.data
        else:
            pb = [_b(p) for p in paths]
            parr = (c.c_char_p * max(1, n))(*pb)
            plen = np.array([len(p) for p in pb], dtype=np.uint64) if n else np.zeros(1, np.uint64)
            paths_addr = c.cast(parr, c.c_void_p).value
            plen_ptr = plen.ctypes.data
        bin_arr = np.array(binary, dtype=np.uint8) if binary is not None else None
        kinds = np.ascontiguousarray(transform, dtype=np.uint8) if transform is not None else None
        batch = _CBatch(n, None if gather_base is not None else arena_buf.ctypes.data, offs.ctypes.data,
                        dev_arena, dev_offsets, paths_addr, plen_ptr,
                        bin_arr.ctypes.data if bin_arr is not None else None,
                        kinds.ctypes.data if kinds is not None else None,
                        dev_paths, dev_path_offsets)
        h = c.c_void_p()
        if gather_base is not None:
            gsrc = np.ascontiguousarray(gather_src, dtype=np.uint64)
            ext = _CBatchExt(BATCH_EXT_SIZE_V2, batch,
                             host_paths.ctypes.data if host_paths is not None else None,
                             host_path_offsets.ctypes.data if host_path_offsets is not None else None,
                             gather_base.ctypes.data, gsrc.ctypes.data)
            rc = self._L.tsg_scan_ext(self._h, c.byref(ext), c.byref(h))
        elif host_paths is not None:
            ext = _CBatchExt(BATCH_EXT_SIZE_V1, batch, host_paths.ctypes.data, host_path_offsets.ctypes.data)
            rc = self._L.tsg_scan_ext(self._h, c.byref(ext), c.byref(h))
        else:
            rc = self._L.tsg_scan(self._h, c.byref(batch), c.byref(h))
        if rc != 0:
            raise RuntimeError("tsg_scan failed: %s" % _lib.last_error(self._L))
        return ScanResult(self, h)

    def set_gpu_findings(self, mode) -> int:
        """Findings of HBM-resident batches on the GPU (materialize.h; True / 1), on the host
        (False / 0, the default) or on the GPU while the exact pass is the bound (2)
        (tsg_debug_scanner_gpu_findings); returns the previous mode."""
        self._L.tsg_debug_scanner_gpu_findings.argtypes = [c.c_void_p, c.c_int]
        return self._L.tsg_debug_scanner_gpu_findings(self._h, int(mode))

    def table_info(self):
        t = _CTableInfo()
        self._L.tsg_scanner_table_info(self._h, c.byref(t))
        return {k: getattr(t, k) for k, _ in t._fields_}

    def rule_anchor(self, i):
        return self._L.tsg_scanner_rule_anchor(self._h, i).decode()


class PendingScan:
    def __init__(self, scanner, h, keep):
        self._sc = scanner
        self._h = h
        self._keep = keep

    def __del__(self):
        # dropped without wait(): the native scan thread still borrows the
        # arena / offsets / paths kept here, so join it before they are freed
        h = getattr(self, "_h", None)
        if h:
            r = c.c_void_p()
            self._sc._L.tsg_scan_wait(h, c.byref(r))
            self._h = None
            if r:
                self._sc._L.tsg_result_free(r)

    def wait(self):
        r = c.c_void_p()
        rc = self._sc._L.tsg_scan_wait(self._h, c.byref(r))
        self._h = None
        self._keep = None
        if rc != 0:
            raise RuntimeError("tsg_scan failed: %s" % _lib.last_error(self._sc._L))
        return ScanResult(self._sc, r)


RECORD_DTYPE = np.dtype([("file", "<u4"), ("rule", "<u4"), ("start_line", "<i8"), ("end_line", "<i8"),
                         ("digest", "<u8")])  # tsg_record


class ScanResult:
    def __init__(self, scanner, h):
        self._sc = scanner
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._sc._L.tsg_result_free(self._h)
            self._h = None

    def stats(self):
        s = _CStats()
        self._sc._L.tsg_result_stats(self._h, c.byref(s))
        return {k: getattr(s, k) for k, _ in s._fields_}

    def raw(self, lo=None, hi=None):
        p = c.c_void_p()
        n = c.c_uint64()
        if lo is None:
            self._sc._L.tsg_result_json(self._h, c.byref(p), c.byref(n))
        elif self._sc._L.tsg_result_json_range(self._h, lo, hi, c.byref(p), c.byref(n)) != 0:
            raise IndexError((lo, hi))
        return json.loads(c.string_at(p, n.value).decode("ascii"))

    def raw_text(self, lo, hi) -> bytes:
        """The JSON text of files [lo, hi) (tsg_result_json_range), unparsed: byte-for-byte
        comparisons of two results."""
        p = c.c_void_p()
        n = c.c_uint64()
        if self._sc._L.tsg_result_json_range(self._h, lo, hi, c.byref(p), c.byref(n)) != 0:
            raise IndexError((lo, hi))
        return c.string_at(p, n.value)

    def records(self) -> np.ndarray:
        """One compact record per finding (tsg_result_records): file, rule index, lines, digest."""
        L = self._sc._L
        n = L.tsg_result_records(self._h, None, 0)
        out = np.empty(n, dtype=RECORD_DTYPE)
        if n:
            L.tsg_result_records(self._h, out.ctypes.data, n)
        return out

    def secrets(self, paths, lo=None) -> List[Secret]:
        """types.Secret per file (files [lo, lo + len(paths)) when lo is given)."""
        out = []
        raw = self.raw() if lo is None else self.raw(lo, lo + len(paths))
        for path, fr in zip(paths, raw):
            kind = fr["kind"]
            if kind == 0:
                out.append(Secret())
            elif kind == 1:
                out.append(Secret(FilePath=path))
            else:
                fs = []
                for f in fr["findings"]:
                    raw = f["Code"]["Lines"]
                    lines = None if raw is None else [
                        Line(Number=l["Number"], Content=_s(l["Content"]), IsCause=l["IsCause"],
                             Highlighted=_s(l["Highlighted"]), FirstCause=l["FirstCause"],
                             LastCause=l["LastCause"]) for l in raw]
                    fs.append(SecretFinding(RuleID=_s(f["RuleID"]), Category=_s(f["Category"]),
                                            Severity=_s(f["Severity"]), Title=_s(f["Title"]),
                                            StartLine=f["StartLine"], EndLine=f["EndLine"],
                                            Code=Code(Lines=lines), Match=_s(f["Match"])))
                out.append(Secret(FilePath=path, Findings=fs))
        return out


def HostRegister(buf, lib=None, mapped: bool = False):
    """Page-lock a numpy buffer (tsg_host_register) so host-resident batches in it stream
    asynchronously to the GPU; returns an unregister callable.  mapped: also map it into the
    device's address space (tsg_host_register_mapped) -- a tar layer a gathering collector's
    batches are read from (Collector(gather=True))."""
    L = lib if lib is not None else _lib.lib()
    _declare(L)
    reg = L.tsg_host_register_mapped if mapped else L.tsg_host_register
    if reg(buf.ctypes.data, buf.nbytes) != 0:
        raise RuntimeError("tsg_host_register failed: %s" % _lib.last_error(L))
    return lambda: L.tsg_host_unregister(buf.ctypes.data)


def NewScanner(config: Optional[Config], device: int = 0, lib=None, host_only: bool = False,
               calibration=None) -> Scanner:
    """scanner.go:320-364.  calibration (optional, bytes / uint8 array): a sample of the bytes the
    scanner will see, e.g. its first batch -- the rule compiler then picks between a rule's literal
    and class-run anchors by their fire rates on it (tsg_compile_options); findings never change."""
    b_rules, b_allow = builtin_rules(), builtin_allow_rules()
    if config is None:
        return Scanner(b_rules, b_allow, [], device, lib, host_only, calibration)
    enabled = b_rules
    if config.EnableBuiltinRuleIDs:
        enabled = [r for r in b_rules if r.ID in config.EnableBuiltinRuleIDs]
    enabled = enabled + list(config.CustomRules)
    rules = [r for r in enabled if r.ID not in config.DisableRuleIDs]
    allow = b_allow + list(config.CustomAllowRules)
    allow = [a for a in allow if a.ID not in config.DisableAllowRuleIDs]
    return Scanner(rules, allow, list(config.ExcludeBlock.Regexes), device, lib, host_only, calibration)
