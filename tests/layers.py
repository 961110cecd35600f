"""Synthetic uncompressed container-image layers (test helper).

Builds tar archives with CPython's tarfile in the three header formats Go's
archive/tar reads (USTAR, GNU, PAX) holding what LayerTar.Walk must handle
(pkg/fanal/walker/tar.go:35-103): regular files (text, CRLF, binary, .pyc-like
binaries, tiny files), names longer than 100 bytes (GNU 'L' / PAX path
records / USTAR prefix), directories, symlinks, hard links, whiteouts and
opaque-dir markers, files under skipped dirs / names / extensions and under
builtin allow paths, with planted builtin-rule secrets.
"""
import io
import random
import tarfile

from tests.corpus import make_file

DIRS = ["usr/lib/python3/site-packages/pkg", "etc/app", "opt/service/conf", "home/user/.config",
        "usr/share/doc/tool", "app/node_modules/dep", "srv/www/.git/objects", "var/lib/data",
        "root/deploy/scripts", "usr/local/lib/very/deeply/nested/directory/structure/for/testing/long/names"]
NAMES = ["config.yaml", "settings.py", "README.md", "run.sh", "index.js", "server.go", "secrets.env",
         "package-lock.json", "image.png", "data.bin", "notes.txt", "main.c", "app.conf", "tool.pyc"]


def make_layer(seed: int, n_files: int, fmt=tarfile.GNU_FORMAT) -> bytes:
    rng = random.Random(seed)
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w", format=fmt) as tf:
        made_dirs = set()
        for i in range(n_files):
            d = rng.choice(DIRS)
            if d not in made_dirs and rng.random() < 0.5:
                ti = tarfile.TarInfo(d + "/")
                ti.type = tarfile.DIRTYPE
                tf.addfile(ti)
                made_dirs.add(d)
            name = rng.choice(NAMES)
            if rng.random() < 0.1:
                name = "x" * rng.randint(60, 140) + "_" + name  # long names
            path = "%s/%d_%s" % (d, i, name)
            if rng.random() < 0.05:
                path = "./" + path
            if rng.random() < 0.03:
                path = "/" + path
            if rng.random() < 0.02:  # names path.Clean rewrites: "//", "/./", "/../"
                path = path.replace("/", rng.choice(["//", "/./", "/x/../"]), 1)
            r = rng.random()
            if r < 0.04:
                ti = tarfile.TarInfo(d + "/.wh." + name)  # whiteout
                tf.addfile(ti)
                continue
            if r < 0.06:
                ti = tarfile.TarInfo(d + "/.wh..wh..opq")
                tf.addfile(ti)
                continue
            if r < 0.10:
                ti = tarfile.TarInfo(path + ".lnk")
                ti.type = tarfile.SYMTYPE
                ti.linkname = "../target"
                tf.addfile(ti)
                continue
            if r < 0.12:
                ti = tarfile.TarInfo(path + ".hard")
                ti.type = tarfile.LNKTYPE
                ti.linkname = d + "/other"
                tf.addfile(ti)
                continue
            if r < 0.16:
                data = bytes(rng.getrandbits(8) for _ in range(rng.randint(0, 400)))  # binary
            elif r < 0.19:
                data = b"\x00" * 16 + make_file(rng, planted_rate=0.8) + b"\x01" * 8  # binary w/ text runs
                if rng.random() < 0.6:
                    path += ".pyc"
            elif r < 0.22:
                data = b"tiny"[:rng.randint(0, 4)]
            else:
                data = make_file(rng, planted_rate=0.35)
                if rng.random() < 0.15:
                    data = data.replace(b"\n", b"\r\n")
            ti = tarfile.TarInfo(path)
            ti.size = len(data)
            ti.mode = 0o644
            tf.addfile(ti, io.BytesIO(data))
    return buf.getvalue()
