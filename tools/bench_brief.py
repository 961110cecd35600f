"""One-line summary of a bench.py JSON result: value, GPU phase, per-kernel ms, counts."""
import json
import sys

for p in sys.argv[1:]:
    d = json.loads(open(p).read().strip().splitlines()[-1])
    b, c = d.get("breakdown_ms", {}), d.get("counts", {})
    ks = " ".join("%s=%.3f" % (k[3:].replace("_kernel", ""), v) for k, v in b.items() if k.endswith("_kernel"))
    print("value=%.1f gpu=%.3f %s | %s" % (d["value"], b.get("ms_gpu_total", 0), ks,
                                          " ".join("%s=%s" % kv for kv in c.items())))
