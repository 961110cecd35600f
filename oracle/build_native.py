"""Builds oracle/build/libtsg_host.so (TEST INFRASTRUCTURE, see oracle/native/tsg_oracle.h).

The product's host objects (trivy_amd/_obj, made by trivy_amd/_build.py) plus
oracle/native/*.cpp: the CPU-only test hooks and the C++ restatement of the
reference CPU algorithm used as bench.py's CPU baseline.  libtsg.so itself
exports none of these.
"""
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
OUT = HERE / "build" / "libtsg_host.so"


def build(verbose=False):
    sys.path.insert(0, str(ROOT))
    from trivy_amd import _build
    _build.build(verbose)
    objdir = HERE / "build" / "obj"
    objdir.mkdir(parents=True, exist_ok=True)
    hdrs = list((HERE / "native").glob("*.h")) + list(_build.CSRC.glob("*.h")) + list((ROOT / "include").glob("*.h"))
    objs = []
    for src in sorted((HERE / "native").glob("*.cpp")):
        obj = objdir / (src.stem + ".o")
        objs.append(obj)
        if _build._stale(obj, [src] + hdrs):
            cmd = ["g++"] + _build.CXXFLAGS + ["-I", str(HERE / "native"), "-c", str(src), "-o", str(obj)]
            if verbose:
                print(" ".join(cmd))
            _build._run(cmd)
    prod = sorted(_build.BUILD.glob("*.o"))
    if not OUT.exists() or _build._stale(OUT, objs + prod):
        _build._run([_build.HIPCC, "--offload-arch=gfx950", "-shared", "-o", str(OUT)] + [str(o) for o in objs + prod]
                    + ["-lpthread"])
    return OUT


if __name__ == "__main__":
    print(build(verbose=True))
