"""C4 ingest probe: native tar walk alone (host-only scanner) at several thread counts."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trivy_amd import corpus  # noqa: E402
from trivy_amd.analyzer import AnalyzerOptions, SecretAnalyzer  # noqa: E402
from trivy_amd.analyzer.secret import Collector, _CTarStats  # noqa: E402

layer = corpus.generate_layer(int(float(os.environ.get("GB", "4")) * 1e9))
from oracle import hostlib  # noqa: E402
a = SecretAnalyzer(lib=hostlib.lib(), host_only=True)
a.Init(AnalyzerOptions())
coll = Collector(a, 256 << 20)
st = _CTarStats()
cur, t = 0, time.time()
while True:
    rc, cur = coll.add_tar(layer, cur, st)
    coll.reset()
    if rc == 0:
        break
dt = time.time() - t
print("threads=%s walk %.3f s  %.2f GB/s layer  %.2f GB/s analyzed  files %d" % (
    os.environ.get("TSG_HOST_THREADS", "16"), dt, layer.size / dt / 1e9, st.input_bytes / dt / 1e9, st.added))
