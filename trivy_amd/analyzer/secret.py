"""SecretAnalyzer: pkg/fanal/analyzer/secret/secret.go over the MI355X engine.

Same names and behaviour as the Go analyzer (undistro/trivy @ 2024-12-20):

* ``SecretAnalyzer.Init(opt)``      -- secret.go:86-101 (ParseConfig + NewScanner)
* ``SecretAnalyzer.Required(p, fi)`` -- secret.go:152-190 (tsg_analyzer_required)
* ``SecretAnalyzer.Analyze(input)`` -- secret.go:103-150: binary gate, CR strip or
  printable extraction, "/" prefix for image files, Scan, nil without findings
* ``Type()`` = "secret" (analyzer/const.go:140), ``Version()`` = 1 (secret.go:26)

and the batched forms the engine is built for (the analyzer group's goroutine
per file, analyzer.go:403-455, becomes a batch collector feeding one arena):

* ``AnalyzeBatch(inputs)``  -- Analyze for many files, one GPU submission per arena
* ``AnalyzeLayer(tar)``     -- LayerTar.Walk (walker/tar.go:35-103) + AnalyzeFile's
  Required gate + Analyze for every regular file of an uncompressed layer,
  parsed natively into double-buffered pinned arenas (tsg_collector_add_tar)
* ``AnalyzeLayers(tars, base)`` -- the image artifact's layer pipeline
  (artifact/image/image.go:202-235): `parallel` layer walks at once into one
  engine, base layers with the secret analyzer disabled

Every transform runs in libtsg.so (include/tsg_analyzer.h); there is no CPU
fallback for the scan itself.
"""
import ctypes
import collections
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

from .. import _lib
from ..secret import NewScanner, ParseConfig, Secret
from ..secret.scanner import ScanResult

c = ctypes
TypeSecret = "secret"  # pkg/fanal/analyzer/const.go:140
version = 1            # secret.go:26
TSG_SKIPPED, TSG_FULL = -1, -2


class _CTarStats(c.Structure):
    _fields_ = [(n, c.c_uint64) for n in ("entries", "regular", "required", "added", "skipped_binary",
                                          "whiteouts", "opaque_dirs", "input_bytes")]


def _declare(L):
    if getattr(L, "_tsg_analyzer_declared", False):
        return
    L.tsg_is_binary.argtypes = [c.c_char_p, c.c_uint64]
    L.tsg_extract_printable.argtypes = [c.c_char_p, c.c_uint64, c.c_char_p]
    L.tsg_extract_printable.restype = c.c_uint64
    L.tsg_strip_cr.argtypes = [c.c_char_p, c.c_uint64, c.c_char_p]
    L.tsg_strip_cr.restype = c.c_uint64
    L.tsg_analyzer_new.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_void_p)]
    L.tsg_analyzer_free.argtypes = [c.c_void_p]
    L.tsg_analyzer_walk_end.argtypes = [c.c_void_p]
    L.tsg_analyzer_set_walk_ahead.argtypes = [c.c_void_p, c.c_int]
    L.tsg_analyzer_required.argtypes = [c.c_void_p, c.c_char_p, c.c_uint64, c.c_int64]
    L.tsg_collector_new.argtypes = [c.c_void_p, c.c_uint64, c.POINTER(c.c_void_p)]
    L.tsg_collector_free.argtypes = [c.c_void_p]
    L.tsg_collector_add.argtypes = [c.c_void_p, c.c_char_p, c.c_uint64, c.c_char_p, c.c_char_p, c.c_uint64]
    L.tsg_collector_add.restype = c.c_int64
    L.tsg_collector_add_tar.argtypes = [c.c_void_p, c.c_void_p, c.c_uint64, c.POINTER(c.c_uint64),
                                        c.POINTER(_CTarStats)]
    L.tsg_collector_files.argtypes = [c.c_void_p]
    L.tsg_collector_files.restype = c.c_uint32
    L.tsg_collector_bytes.argtypes = [c.c_void_p]
    L.tsg_collector_bytes.restype = c.c_uint64
    L.tsg_collector_input_bytes.argtypes = [c.c_void_p]
    L.tsg_collector_input_bytes.restype = c.c_uint64
    L.tsg_collector_file.argtypes = [c.c_void_p, c.c_uint32, c.POINTER(c.c_void_p), c.POINTER(c.c_uint64),
                                     c.POINTER(c.c_void_p), c.POINTER(c.c_uint64), c.POINTER(c.c_int)]
    L.tsg_collector_submit.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    L.tsg_collector_reset.argtypes = [c.c_void_p]
    L.tsg_collector_set_gpu_transform.argtypes = [c.c_void_p, c.c_int]
    L.tsg_collector_set_gather.argtypes = [c.c_void_p, c.c_int]
    L.tsg_scan_wait.argtypes = [c.c_void_p, c.POINTER(c.c_void_p)]
    L._tsg_analyzer_declared = True


def _b(s) -> bytes:
    return s if isinstance(s, bytes) else str(s).encode("utf-8", "surrogateescape")


# ---- utils (pkg/fanal/utils/utils.go) -------------------------------------
def IsBinary(content: bytes, fileSize: int) -> bool:  # utils.go:85-103
    L = _lib.lib()
    _declare(L)
    return L.tsg_is_binary(content, min(int(fileSize), len(content))) == 1


def ExtractPrintableBytes(content: bytes) -> bytes:  # utils.go:128-160
    L = _lib.lib()
    _declare(L)
    out = c.create_string_buffer(len(content) + len(content) // 5 + 2)
    n = L.tsg_extract_printable(content, len(content), out)
    return out.raw[:n]


def StripCR(content: bytes) -> bytes:  # bytes.ReplaceAll(content, "\r", ""), secret.go:121
    L = _lib.lib()
    _declare(L)
    out = c.create_string_buffer(max(1, len(content)))
    n = L.tsg_strip_cr(content, len(content), out)
    return out.raw[:n]


# ---- analyzer types (pkg/fanal/analyzer/analyzer.go) -----------------------
@dataclass
class SecretScannerOption:  # analyzer.go:56-58
    ConfigPath: str = ""


@dataclass
class AnalyzerOptions:  # analyzer.go:44-54 (the secret analyzer's part)
    SecretScannerOption: SecretScannerOption = field(default_factory=SecretScannerOption)


@dataclass
class FileInfo:  # the os.FileInfo facts the analyzer reads
    size: int

    def Size(self) -> int:
        return self.size


@dataclass
class AnalysisInput:  # analyzer.go:81-88
    Dir: str
    FilePath: str
    Info: FileInfo
    Content: bytes  # or a readable binary file object


@dataclass
class AnalysisResult:  # analyzer.go:99-136 (the Secrets part)
    Secrets: List[Secret] = field(default_factory=list)

    def Merge(self, other: Optional["AnalysisResult"]):  # analyzer.go:251-301
        if other is not None:
            self.Secrets.extend(other.Secrets)

    def Sort(self):  # analyzer.go:225-234
        self.Secrets.sort(key=lambda s: _b(s.FilePath))
        for sec in self.Secrets:
            if sec.Findings:
                sec.Findings.sort(key=lambda f: (_b(f.RuleID), f.StartLine))


def _read(content) -> bytes:
    if isinstance(content, (bytes, bytearray, memoryview)):
        return bytes(content)
    data = content.read()
    if hasattr(content, "seek"):
        content.seek(0)
    return data


class Collector:
    """A batch arena (tsg_collector): Analyze's pre-scan half for many files."""

    def __init__(self, analyzer: "SecretAnalyzer", arena_bytes: int = 256 << 20, gpu_transform: bool = False,
                 gather: bool = False):
        """gpu_transform: files enter the arena as read and the CR strip / printable
        extraction runs on the GPU at scan time (tsg_collector_set_gpu_transform).
        gather (needs gpu_transform; tar walks): the walk copies nothing -- the GPU gathers
        the batch's files from the layer buffer, which the caller registers with
        HostRegister(buf, mapped=True) and keeps until the batch is waited on; one batch
        holds one layer's files (tsg_collector_set_gather)."""
        self._L = analyzer._L
        self._an = analyzer  # the C collector borrows the analyzer (and its walk state)
        if not analyzer._h:
            raise RuntimeError("Collector: the analyzer has no scanner (Init first)")
        h = c.c_void_p()
        if self._L.tsg_collector_new(analyzer._h, int(arena_bytes), c.byref(h)) != 0:
            raise RuntimeError("tsg_collector_new failed: %s" % _lib.last_error(self._L))
        self._h = h
        if gpu_transform and self._L.tsg_collector_set_gpu_transform(h, 1) != 0:
            raise RuntimeError("tsg_collector_set_gpu_transform failed: %s" % _lib.last_error(self._L))
        if gather and self._L.tsg_collector_set_gather(h, 1) != 0:
            raise RuntimeError("tsg_collector_set_gather failed: %s" % _lib.last_error(self._L))
        self.gather = bool(gather)
        self._keep = []

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.tsg_collector_free(self._h)
            self._h = None

    def add(self, path: str, dir_: str, content: bytes) -> int:
        p = _b(path)
        return self._L.tsg_collector_add(self._h, p, len(p), _b(dir_), content, len(content))

    def add_tar(self, buf, cursor: int, stats: _CTarStats):
        """Walk the layer from ``cursor``: (1 when full / 0 at the end, next cursor).
        With the analyzer's walk-ahead on, the next window of the layer is indexed on a
        background thread after a return of 1, so the analyzer keeps ``buf`` alive until
        the walk ends (0, an error, or SecretAnalyzer.WalkEnd) -- tsg_analyzer.h."""
        cur = c.c_uint64(cursor)
        addr = buf.ctypes.data if hasattr(buf, "ctypes") else c.cast(c.c_char_p(buf), c.c_void_p).value
        self._an._walk_buf = buf
        rc = self._L.tsg_collector_add_tar(self._h, addr, len(buf), c.byref(cur), c.byref(stats))
        if rc != 1:  # the walk ended (the C side joined any background index)
            self._an._walk_buf = None
        if rc < 0:
            raise ValueError("tar layer: %s" % _lib.last_error(self._L))
        return rc, cur.value

    def files(self) -> int:
        return self._L.tsg_collector_files(self._h)

    def nbytes(self) -> int:
        return self._L.tsg_collector_bytes(self._h)

    def input_bytes(self) -> int:
        return self._L.tsg_collector_input_bytes(self._h)

    def file(self, i: int):
        """(scan path, transformed content, binary) of batch file i."""
        pp, pl, cp, cl, bn = c.c_void_p(), c.c_uint64(), c.c_void_p(), c.c_uint64(), c.c_int()
        if self._L.tsg_collector_file(self._h, i, c.byref(pp), c.byref(pl), c.byref(cp), c.byref(cl),
                                      c.byref(bn)) != 0:
            raise IndexError(i)
        path = c.string_at(pp, pl.value).decode("utf-8", "surrogateescape")
        data = c.string_at(cp, cl.value) if cl.value else b""
        return path, data, bool(bn.value)

    def paths(self) -> List[str]:
        return [self.file(i)[0] for i in range(self.files())]

    def submit(self) -> "PendingBatch":
        h = c.c_void_p()
        if self._L.tsg_collector_submit(self._h, c.byref(h)) != 0:
            raise RuntimeError("tsg_collector_submit failed: %s" % _lib.last_error(self._L))
        return PendingBatch(self, h)

    def reset(self):
        self._L.tsg_collector_reset(self._h)


class PendingBatch:
    def __init__(self, coll: Collector, h):
        self.coll, self._h = coll, h

    def __del__(self):
        # dropped without wait() (e.g. an exception in the caller's loop): the
        # scan thread still reads the collector's arena, so join it first
        h = getattr(self, "_h", None)
        if h:
            r = c.c_void_p()
            self.coll._L.tsg_scan_wait(h, c.byref(r))
            self._h = None
            if r:
                self.coll._L.tsg_result_free(r)
            self.coll.reset()

    def wait(self, materialize: bool = True):
        """Per batch file: the Secret when it has findings (Analyze's result), else None.
        materialize=False: only the batch's tsg_stats (dict), no per-file objects."""
        r = c.c_void_p()
        rc = self.coll._L.tsg_scan_wait(self._h, c.byref(r))
        self._h = None
        if rc != 0:
            raise RuntimeError("tsg_scan failed: %s" % _lib.last_error(self.coll._L))
        res = ScanResult(_ScannerRef(self.coll._L), r)
        out = ([s if s.Findings else None for s in res.secrets(self.coll.paths())] if materialize
               else res.stats())
        del res
        self.coll.reset()
        return out


class _ScannerRef:  # what ScanResult needs of its scanner
    def __init__(self, L):
        self._L = L


def _pipeline(colls, fill, take):
    """Fill the collectors in turn (fill(coll) -> True at the end of the input) and submit
    each batch; with n collectors, n - 1 scans stay in flight while the next batch is
    filled (a collector is refilled only after its scan was taken).  Returns the seconds
    spent filling and waiting."""
    inflight = collections.deque()
    k, done = 0, False
    t_walk = t_wait = 0.0
    try:
        while not done:
            coll = colls[k]
            t0 = time.perf_counter()
            done = fill(coll)
            t_walk += time.perf_counter() - t0
            if coll.files():
                inflight.append(coll.submit())
            t0 = time.perf_counter()
            while len(inflight) > len(colls) - 1:
                take(inflight.popleft())
            t_wait += time.perf_counter() - t0
            k = (k + 1) % len(colls)
        t0 = time.perf_counter()
        while inflight:
            take(inflight.popleft())
        t_wait += time.perf_counter() - t0
    finally:
        while inflight:  # an error left batches in flight: join them before the arenas go
            inflight.popleft().__del__()
    return t_walk, t_wait


class SecretAnalyzer:
    """analyzer/secret.SecretAnalyzer bound to the MI355X engine."""

    def __init__(self, scanner=None, configPath: str = "", device: int = 0, lib=None, host_only: bool = False):
        """lib / host_only: as trivy_amd.secret.Scanner (tests drive the host logic on CPU)."""
        self._L = lib if lib is not None else _lib.lib()
        _declare(self._L)
        self.device = device
        self._host_only = host_only
        self._h = None
        self._walk_buf = None  # the layer buffer of a walk in progress (Collector.add_tar)
        self.scanner = None
        self.configPath = configPath
        if scanner is not None:
            self._bind(scanner, configPath)

    def _bind(self, scanner, configPath):
        if self._h:
            self._L.tsg_analyzer_free(self._h)
            self._h = None
            self._walk_buf = None
        self.scanner = scanner
        self.configPath = configPath
        h = c.c_void_p()
        if self._L.tsg_analyzer_new(scanner._h, _b(configPath), c.byref(h)) != 0:
            raise RuntimeError("tsg_analyzer_new failed: %s" % _lib.last_error(self._L))
        self._h = h
        # walk-ahead: this object keeps the layer buffer alive until the walk ends
        self._L.tsg_analyzer_set_walk_ahead(h, 1)

    def WalkEnd(self):
        """Ends a tar walk (joins its background index): the layer buffer may go after this."""
        if self._h:
            self._L.tsg_analyzer_walk_end(self._h)
        self._walk_buf = None

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.tsg_analyzer_free(self._h)  # joins a walk's background index
            self._h = None
        self._walk_buf = None

    # --- reference API ------------------------------------------------------
    def Init(self, opt: AnalyzerOptions):  # secret.go:86-101
        path = opt.SecretScannerOption.ConfigPath
        if self.scanner is not None and path == self.configPath:
            return None
        try:
            cfg = ParseConfig(path)
        except Exception as e:  # xerrors.Errorf("secret config error: %w", err)
            raise RuntimeError("secret config error: %s" % e)
        self._bind(NewScanner(cfg, device=self.device, lib=self._L, host_only=self._host_only), path)
        return None

    def Type(self) -> str:
        return TypeSecret

    def Version(self) -> int:
        return version

    def Required(self, filePath: str, fi) -> bool:  # secret.go:152-190
        p = _b(filePath)
        size = fi.Size() if hasattr(fi, "Size") else int(fi)
        return self._L.tsg_analyzer_required(self._h, p, len(p), int(size)) == 1

    def Analyze(self, input: AnalysisInput) -> Optional[AnalysisResult]:  # secret.go:103-150
        return self.AnalyzeBatch([input])[0]

    # --- batched forms ------------------------------------------------------
    def AnalyzeBatch(self, inputs: Sequence[AnalysisInput], arena_bytes: int = 256 << 20,
                     gpu_transform: bool = False) -> List[Optional[AnalysisResult]]:
        out: List[Optional[AnalysisResult]] = [None] * len(inputs)
        coll = Collector(self, arena_bytes, gpu_transform)
        idx: List[int] = []

        def flush():
            if not idx:
                return
            for k, sec in zip(idx, coll.submit().wait()):
                if sec is not None:
                    out[k] = AnalysisResult(Secrets=[sec])
            idx.clear()

        for k, inp in enumerate(inputs):
            data = _read(inp.Content)
            for _ in range(2):
                r = coll.add(inp.FilePath, inp.Dir, data)
                if r == TSG_FULL:
                    flush()
                    continue
                if r >= 0:
                    idx.append(k)
                elif r != TSG_SKIPPED:
                    raise RuntimeError("tsg_collector_add failed: %s" % _lib.last_error(self._L))
                break
        flush()
        return out

    def AnalyzeFS(self, root: str, opt=None, arena_bytes: int = 256 << 20, stats: Optional[dict] = None,
                  materialize: bool = True, colls: Optional[List["Collector"]] = None,
                  gpu_transform: bool = False) -> AnalysisResult:
        """`trivy fs` for this analyzer: FS.Walk (walker/fs.go:25-78) + AnalyzeFile's Required +
        Analyze for every regular file under root, read natively into double-buffered pinned
        arenas (tsg_collector_add_fs); one collector fills while the others' batches scan.
        FilePath is the path relative to root (Dir = root, no '/' prefix: secret.go:130-135)."""
        from ..walker import FS, Option, _CFsAddStats
        w = FS().Walk(root, opt or Option(), lib=self._L)
        result = AnalysisResult()
        scan_tot: dict = {}
        st = _CFsAddStats()

        def take(p):
            out = p.wait(materialize)
            if materialize:
                result.Secrets.extend(sec for sec in out if sec is not None)
            else:
                for k2, v in out.items():
                    scan_tot[k2] = scan_tot.get(k2, 0) + v
        colls = colls or [Collector(self, arena_bytes, gpu_transform), Collector(self, arena_bytes, gpu_transform)]
        def fill(coll):
            rc = self._L.tsg_collector_add_fs(coll._h, w._h, c.byref(st))
            if rc < 0:
                raise RuntimeError("fs walk: %s" % _lib.last_error(self._L))
            return rc == 0
        t_walk, t_wait = _pipeline(colls, fill, take)
        if stats is not None:
            stats.update({n: getattr(st, n) for n, _ in st._fields_})
            stats.update(w.stats())
            stats.update({"scan_" + k2: v for k2, v in scan_tot.items()})
            stats.update({"walk_s": t_walk, "wait_s": t_wait})
        result.Sort()
        return result

    def AnalyzeLayer(self, layer, arena_bytes: int = 256 << 20, stats: Optional[dict] = None,
                     materialize: bool = True, colls: Optional[List[Collector]] = None,
                     gpu_transform: bool = False, gather: bool = False,
                     registered: bool = False) -> AnalysisResult:
        """Every regular file of an uncompressed tar layer (bytes or a uint8 numpy array),
        as the image artifact's AnalyzeFile(dir="") would run it.  The collectors (two by
        default) are filled in turn while the others' batches are on the GPU.  materialize=False
        (bench): findings stay in the engine; stats gets the summed scan counters.
        gather (with gpu_transform; or collectors made with gather=True): the GPU reads the files
        in the layer itself (no arena copy); the layer, a uint8 numpy array, is registered
        page-locked and mapped for the call unless `registered` says the caller holds it so
        (HostRegister(layer, mapped=True): a pinned layer-buffer pool registers once)."""
        result = AnalysisResult()
        scan_tot: dict = {}

        def take(p):
            out = p.wait(materialize)
            if materialize:
                result.Secrets.extend(sec for sec in out if sec is not None)
            else:
                for k2, v in out.items():
                    scan_tot[k2] = scan_tot.get(k2, 0) + v
        st = _CTarStats()
        colls = colls or [Collector(self, arena_bytes, gpu_transform or gather, gather) for _ in range(2)]
        cursor = 0
        unregister = None
        if any(cl.gather for cl in colls) and not registered:
            from ..secret.scanner import HostRegister
            if not hasattr(layer, "ctypes"):
                raise TypeError("AnalyzeLayer(gather): the layer must be a numpy uint8 array")
            unregister = HostRegister(layer, self._L, mapped=True)

        def fill(coll):
            nonlocal cursor
            rc, cursor = coll.add_tar(layer, cursor, st)
            if rc == 1 and coll.files() == 0:
                raise RuntimeError("tar layer: an entry does not fit an empty collector")
            return rc == 0
        try:
            t_walk, t_wait = _pipeline(colls, fill, take)
        finally:  # the layer buffer may go away after this call (tsg_analyzer.h buffer lifetime)
            self.WalkEnd()
            if unregister is not None:  # every batch read from it was waited on (_pipeline)
                unregister()
        if stats is not None:
            stats.update({n: getattr(st, n) for n, _ in st._fields_})
            stats.update({"scan_" + k2: v for k2, v in scan_tot.items()})
            stats.update({"walk_s": t_walk, "wait_s": t_wait})
        return result


    def LayerWorkers(self, parallel: int = 2, arena_bytes: int = 256 << 20, collectors: int = 2,
                     gpu_transform: bool = False, gather: bool = False) -> list:
        """AnalyzeLayers' workers, for reuse across calls: per worker an analyzer bound to this scanner
        (its own tar-walk state) and its collectors (pinned arenas: allocating them per call would
        cost a hipHostMalloc each, and freeing them waits for the device)."""
        out = []
        for _ in range(max(1, parallel)):
            sub = SecretAnalyzer(self.scanner, self.configPath, device=self.device, lib=self._L,
                                 host_only=self._host_only)
            out.append((sub, [Collector(sub, arena_bytes, gpu_transform or gather, gather)
                              for _ in range(max(1, collectors))]))
        return out

    def AnalyzeLayers(self, layers: Sequence, base: Optional[Sequence[bool]] = None, parallel: int = 2,
                      arena_bytes: int = 256 << 20, collectors: int = 2, gpu_transform: bool = False,
                      materialize: bool = True, stats: Optional[list] = None,
                      workers: Optional[list] = None, gather: bool = False,
                      registered: bool = False) -> List[AnalysisResult]:
        """The image artifact's layer inspection for this analyzer (pkg/fanal/artifact/image/image.go:
        202-235): a pipeline of `parallel` workers over the layers, each running inspectLayer's walk
        (AnalyzeLayer) of one layer at a time; a base layer (base[i] true, the image's base diff IDs)
        has the secret analyzer disabled (image.go:208-211) and yields an empty result without a walk.
        Each worker owns an analyzer (its own tar-walk state) and collectors bound to this scanner, so
        the walks of several layers feed the one engine -- its staging ring interleaves their batches'
        copies and kernels.  Returns one AnalysisResult per layer, in the order given, each sorted as
        inspectLayer sorts its result (analyzer.go:225-234).  stats (a list): per layer, the
        AnalyzeLayer stats dict (None for base layers).  workers: from LayerWorkers (then `parallel`,
        `arena_bytes`, `collectors`, `gpu_transform` and `gather` are theirs).  gather / registered:
        as AnalyzeLayer (the layers are then uint8 numpy arrays)."""
        import threading
        if self.scanner is None:
            raise RuntimeError("AnalyzeLayers: the analyzer has no scanner (Init first)")
        n = len(layers)
        base = list(base) if base is not None else [False] * n
        if len(base) != n:
            raise ValueError("AnalyzeLayers: base flags must match the layers")
        results: List[Optional[AnalysisResult]] = [None] * n
        per: List[Optional[dict]] = [None] * n
        todo = collections.deque(i for i in range(n) if not base[i])
        for i in range(n):
            if base[i]:
                results[i] = AnalysisResult()
        lock = threading.Lock()
        errors: List[BaseException] = []

        if workers is None:
            workers = self.LayerWorkers(min(parallel, max(1, len(todo))), arena_bytes, collectors, gpu_transform,
                                        gather)

        def worker(sub, colls):
            while True:
                with lock:
                    if errors or not todo:
                        return
                    i = todo.popleft()
                st: dict = {}
                try:
                    r = sub.AnalyzeLayer(layers[i], stats=st, materialize=materialize, colls=colls,
                                         registered=registered)
                except BaseException as e:  # the pipeline stops at the first error (parallel.Pipeline)
                    with lock:
                        errors.append(e)
                    return
                r.Sort()
                results[i], per[i] = r, st

        threads = [threading.Thread(target=worker, args=w, name="tsg-layer-%d" % k)
                   for k, w in enumerate(workers[:max(1, len(todo))])]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        if stats is not None:
            stats[:] = per
        return results  # type: ignore[return-value]


def NewSecretAnalyzer(s=None, configPath: str = "") -> SecretAnalyzer:  # secret.go:79-84
    return SecretAnalyzer(s, configPath)
