#!/usr/bin/env python3
"""Build libtsg.so variants with compile-time tuning macros (engine.hip TSG_C_*).

  python tools/build_variant.py NAME -DTSG_C_THREADS=256 -DTSG_C_WIN=112
writes trivy_amd/_variants/NAME/libtsg.so; run with TSG_LIB=<that path>.
Tuning aid only: the product is the default build (__graft_entry__.build()).
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from trivy_amd import _build  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
d = _build.PKG / "_variants" / name
d.mkdir(parents=True, exist_ok=True)
_build.BUILD = d / "obj"
_build.OUT = d / "libtsg.so"
_build.HIPFLAGS = _build.HIPFLAGS + defs
print(_build.build())
