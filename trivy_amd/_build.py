"""In-tree build of the native library trivy_amd/libtsg.so (gfx950 only).

Host C++ (*.cpp) is compiled with g++, device code (*.hip) with
``hipcc --offload-arch=gfx950``, and everything is linked with hipcc into one
shared object that ships with the repo snapshot to the GPU box.
"""
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OUT = PKG / "libtsg.so"
BUILD = PKG / "_obj"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

CXXFLAGS = ["-O3", "-g1", "-fno-omit-frame-pointer", "-march=x86-64-v3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-I", str(CSRC),
            "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROCM, "include"),
            "-I", str(PKG.parent / "include")]
HIPFLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-I", str(CSRC),
            "-I", str(PKG.parent / "include"), "-munsafe-fp-atomics"]


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("build failed: " + " ".join(cmd))
    return r.stdout


def _stale(obj, deps):
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(verbose=False):
    BUILD.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.h")) + list(CSRC.glob("*.inc")) + list((PKG.parent / "include").glob("*.h"))
    objs = []
    jobs = []
    for src in sorted(CSRC.glob("*.cpp")):
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if _stale(obj, [src] + headers):
            jobs.append(["g++"] + CXXFLAGS + ["-c", str(src), "-o", str(obj)])
    for src in sorted(CSRC.glob("*.hip")):
        obj = BUILD / (src.stem + ".hip.o")
        objs.append(obj)
        if _stale(obj, [src] + headers):
            jobs.append([HIPCC] + HIPFLAGS + ["-c", str(src), "-o", str(obj)])
    procs = []
    for cmd in jobs:
        if verbose:
            print(" ".join(cmd))
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = False
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out)
            failed = True
    if failed:
        raise RuntimeError("native build failed")
    if jobs or not OUT.exists() or _stale(OUT, objs):
        _run([HIPCC, "--offload-arch=gfx950", "-shared", "-o", str(OUT)] + [str(o) for o in objs]
             + ["-lpthread"])
    return OUT


if __name__ == "__main__":
    print(build(verbose=True))
