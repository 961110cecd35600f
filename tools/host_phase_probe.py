#!/usr/bin/env python3
"""Where a bench step's wall time goes on the GPU box (profiling aid, not a test):
tsg_scan (GPU phase + host tail, with TSG_TAIL_DEBUG phase totals on stderr), stats(), result free."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trivy_amd import corpus  # noqa: E402
import trivy_amd.secret as secret  # noqa: E402

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
C = corpus.generate(int(gb * 1e9))
d_arena = torch.from_numpy(C.arena).cuda()
d_offs = torch.from_numpy(C.offsets.view(np.int64)).cuda()
torch.cuda.synchronize()
sc = secret.NewScanner(None, device=0)
for i in range(3):
    t0 = time.time()
    r = sc.scan_arena(C.arena, C.offsets, C.path_ptrs, dev_arena=d_arena.data_ptr(), dev_offsets=d_offs.data_ptr())
    t1 = time.time()
    s = r.stats()
    t2 = time.time()
    del r
    t3 = time.time()
    print("step %d: scan %.1f ms (gpu phase %.1f, exact %.1f, host total %.1f) stats %.2f ms free %.1f ms" %
          (i, (t1 - t0) * 1e3, s["ms_host_gpu_phase"], s["ms_host_exact"], s["ms_host_total"], (t2 - t1) * 1e3,
           (t3 - t2) * 1e3), flush=True)
