"""pkg/fanal/walker over the native batch walk (include/tsg_analyzer.h tsg_fs_walk_*).

* ``Option``                       -- walk.go:18-21 (SkipFiles, SkipDirs)
* ``FS().BuildSkipPaths(base, p)`` -- fs.go:102-155: CLI skip paths -> paths relative to the root
* ``CleanSkipPaths`` / ``SkipPath`` -- pkg/fanal/utils/utils.go:105-126 (doublestar.Match natively)
* ``FS().Walk(root, opt)``         -- fs.go:25-39 + WalkDirFunc :41-78 as a native handle that
  feeds batch collectors (SecretAnalyzer.AnalyzeFS); ``FS().Files(root, opt)`` lists the
  (FilePath, size) pairs the walk yields, in WalkDir order.
"""
import ctypes as c
import os
import posixpath
from dataclasses import dataclass, field
from typing import List

from .. import _lib

defaultSizeThreshold = 100 << 20             # walk.go:9 (cachedFile temp-file spill, tar walker only)
defaultSkipDirs = ["**/.git", "proc", "sys", "dev"]  # walk.go:11-16 (added by the native walk)


class _CFsStats(c.Structure):
    _fields_ = [(n, c.c_uint64) for n in ("files", "dirs", "skipped_dirs", "skipped_files", "nonregular",
                                          "perm_errors")]


class _CFsAddStats(c.Structure):
    _fields_ = [(n, c.c_uint64) for n in ("walked", "required", "skipped_binary", "added", "input_bytes")]


def _declare(L):
    if getattr(L, "_tsg_walker_declared", False):
        return
    L.tsg_fs_walk_new.argtypes = [c.c_char_p, c.POINTER(c.c_char_p), c.c_uint32, c.POINTER(c.c_char_p),
                                  c.c_uint32, c.POINTER(c.c_void_p)]
    L.tsg_fs_walk_free.argtypes = [c.c_void_p]
    L.tsg_fs_walk_stats.argtypes = [c.c_void_p, c.POINTER(_CFsStats)]
    L.tsg_collector_add_fs.argtypes = [c.c_void_p, c.c_void_p, c.POINTER(_CFsAddStats)]
    L.tsg_doublestar_match.argtypes = [c.c_char_p, c.c_char_p]
    L._tsg_walker_declared = True


def _b(s) -> bytes:
    return s if isinstance(s, bytes) else str(s).encode("utf-8", "surrogateescape")


@dataclass
class Option:  # walk.go:18-21
    SkipFiles: List[str] = field(default_factory=list)
    SkipDirs: List[str] = field(default_factory=list)


def CleanSkipPaths(skipPaths: List[str]) -> List[str]:  # utils.go:105-110
    return [posixpath.normpath(p.replace(os.sep, "/")).lstrip("/") if p else "." for p in skipPaths]


def Match(pattern: str, path: str, lib=None) -> int:
    """doublestar.Match: 1 / 0, -1 for a malformed pattern."""
    L = lib or _lib.lib()
    _declare(L)
    return L.tsg_doublestar_match(_b(pattern), _b(path))


def SkipPath(path: str, skipPaths: List[str], lib=None) -> bool:  # utils.go:112-126
    path = path.lstrip("/")
    for p in skipPaths:
        m = Match(p, path, lib)
        if m < 0:
            return False
        if m:
            return True
    return False


class FSWalk:
    """A native walk over one root (the handle tsg_collector_add_fs consumes)."""

    def __init__(self, root: str, opt: Option, lib=None):
        self._L = lib or _lib.lib()
        _declare(self._L)
        sd = [_b(p) for p in opt.SkipDirs]
        sf = [_b(p) for p in opt.SkipFiles]
        ad = (c.c_char_p * max(1, len(sd)))(*sd)
        af = (c.c_char_p * max(1, len(sf)))(*sf)
        h = c.c_void_p()
        if self._L.tsg_fs_walk_new(_b(root), ad, len(sd), af, len(sf), c.byref(h)) != 0:
            raise RuntimeError("tsg_fs_walk_new failed: %s" % _lib.last_error(self._L))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.tsg_fs_walk_free(self._h)
            self._h = None

    def stats(self) -> dict:
        s = _CFsStats()
        self._L.tsg_fs_walk_stats(self._h, c.byref(s))
        return {k: getattr(s, k) for k, _ in s._fields_}


class FS:  # fs.go:19-23
    def BuildSkipPaths(self, base: str, paths: List[str]) -> List[str]:  # fs.go:102-155
        absBase = os.path.abspath(base)
        rel_paths = []
        for path in paths:
            absSkip = os.path.abspath(path)
            rel = os.path.relpath(absSkip, absBase)
            if not os.path.isabs(path) and rel.startswith(".."):
                relPath = path  # #1: relative to the root as given
            else:
                relPath = rel   # #2 / #3: relative to the root
            rel_paths.append(relPath.replace(os.sep, "/"))
        return CleanSkipPaths(rel_paths)

    def Walk(self, root: str, opt: Option, lib=None) -> FSWalk:  # fs.go:25-39
        o = Option(SkipFiles=self.BuildSkipPaths(root, opt.SkipFiles),
                   SkipDirs=self.BuildSkipPaths(root, opt.SkipDirs))
        return FSWalk(root, o, lib)
