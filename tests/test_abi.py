"""The drop-in C-ABI (include/*.h) is what libtsg.so exports, and nothing CPU-scan-shaped.

* every function include/*.h declares is exported by trivy_amd/libtsg.so;
* the CPU-only test hooks and the CPU reference scan (oracle/native/tsg_oracle.h)
  are exported by the oracle's library only, never by the product library.
No compute calls: loading and symbol lookup work without a GPU.
"""
import ctypes
import re
from pathlib import Path

from oracle import hostlib
from trivy_amd import _lib

ROOT = Path(__file__).resolve().parent.parent
DECL = re.compile(r"^\s*(?:const\s+)?[\w\s\*]+?\b(tsg_\w+)\s*\(", re.M)


def _declared(path):
    text = re.sub(r"/\*.*?\*/", "", Path(path).read_text(), flags=re.S)
    return sorted(set(DECL.findall(text)))


def test_product_exports_every_declared_symbol():
    L = _lib.lib()
    names = [n for h in sorted((ROOT / "include").glob("*.h")) for n in _declared(h)]
    assert len(names) > 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_cpu_scan_hooks_are_not_in_the_product():
    L = _lib.lib()
    hooks = _declared(ROOT / "oracle/native/tsg_oracle.h")
    assert set(hooks) >= {"tsg_debug_host_tail", "tsg_debug_host_tail_cands", "tsg_debug_scanner_host_only",
                          "tsg_cpuref_scan"}
    for n in hooks:
        try:
            getattr(L, n)
            present = True
        except AttributeError:
            present = False
        assert not present, n
    H = hostlib.lib()
    for n in hooks:
        assert hasattr(H, n), n


def test_scanner_new_fails_loudly_without_gpu():
    """No HIP device here: tsg_scanner_new must fail (no CPU fallback in the product)."""
    import torch
    if torch.cuda.is_available():
        return
    from trivy_amd.secret import NewScanner
    try:
        NewScanner(None)
    except RuntimeError as e:
        assert "tsg_scanner_new failed" in str(e)
    else:
        raise AssertionError("a scanner was created without a GPU")


def _c_layout(tmp_path):
    """sizeof / offsetof of the batch structs as a C compiler lays them out from include/tsg_scanner.h."""
    import subprocess
    src = tmp_path / "probe.c"
    src.write_text('#include <stdio.h>\n#include "tsg_scanner.h"\nint main(void){printf("%zu %zu %zu %zu %u %zu %u\\n",'
                   ' sizeof(tsg_batch), sizeof(tsg_batch_ext), offsetof(tsg_batch_ext, base),'
                   ' offsetof(tsg_batch_ext, host_paths), (unsigned)TSG_BATCH_EXT_SIZE_V1,'
                   ' offsetof(tsg_batch_ext, gather_base), (unsigned)TSG_BATCH_EXT_SIZE_V2); return 0;}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    return [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]


def test_batch_struct_layouts(tmp_path):
    """The frozen tsg_batch is the round-4 layout (11 fields, no host paths); tsg_batch_ext carries
    struct_size first; the ctypes mirror agrees with the C compiler."""
    from trivy_amd.secret.scanner import _CBatch, _CBatchExt, BATCH_EXT_SIZE_V1, BATCH_EXT_SIZE_V2
    size_b, size_e, off_base, off_hp, v1, off_gb, v2 = _c_layout(tmp_path)
    assert size_b == 8 + 10 * 8 == ctypes.sizeof(_CBatch)  # n_files (+pad) and ten pointers
    assert off_base == _CBatchExt.base.offset == 8
    assert off_hp == _CBatchExt.host_paths.offset
    # v1 (round 5) ends after the host paths; v2 (round 6) adds the gather fields after them
    assert v1 == off_gb == _CBatchExt.gather_base.offset == BATCH_EXT_SIZE_V1 == 112
    assert v2 == size_e == ctypes.sizeof(_CBatchExt) == BATCH_EXT_SIZE_V2 == 128


def test_scan_ext_refuses_unknown_struct_size():
    """A tsg_batch_ext whose struct_size the library does not know is refused before anything is read
    (no scanner or GPU needed: the check comes first)."""
    from trivy_amd.secret.scanner import _CBatchExt, _declare, BATCH_EXT_SIZE_V1
    L = _lib.lib()
    _declare(L)
    for bogus in (0, 7, BATCH_EXT_SIZE_V1 - 8, BATCH_EXT_SIZE_V1 + 8, BATCH_EXT_SIZE_V1 + 24, 0xFFFFFFFF):
        b = _CBatchExt()
        b.struct_size = bogus
        h = ctypes.c_void_p()
        assert L.tsg_scan_ext(None, ctypes.byref(b), ctypes.byref(h)) < 0
        assert "struct_size %d" % bogus in _lib.last_error(L)
        assert not h.value
        assert L.tsg_scan_submit_ext(None, ctypes.byref(b), ctypes.byref(h)) < 0
        assert not h.value
