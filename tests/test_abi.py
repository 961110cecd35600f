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
