"""Host issue cost of a render call vs its GPU time: R renders of part (0, N) rotated over F
replicas / streams, timing the issuing loop (no synchronisation) and the whole run.
One JSON line per (N, F).

    python tools/diag_launch.py [renders]
"""
import json
import os
import sys
import tempfile
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402

import rtgpu  # noqa: E402
import scenes  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 160
d = tempfile.mkdtemp()
xml = scenes.synthetic_heightfield(d)
os.chdir(d)
hs = rtgpu.HostScene(xml)
F = 8
reps = [rtgpu.DeviceScene(hs, 0) for _ in range(F)]
c = hs.camera(0)
H, W = c["height"], c["width"]
bufs = [(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"),
         torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")) for _ in range(F)]
streams = [torch.cuda.Stream() for _ in range(F)]
ptrs = [(b[0].data_ptr(), b[1].data_ptr(), s.cuda_stream) for b, s in zip(bufs, streams)]
for n in (1, 8):
    for f in (1, 8):
        for k in range(2 * F):
            reps[k % f].render_device(*ptrs[k % f], part=(0, n))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(R):
            reps[k % f].render_device(*ptrs[k % f], part=(0, n))
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"N": n, "F": f, "renders": R, "issue_us_per_render": round((t1 - t0) / R * 1e6, 1),
                          "total_us_per_render": round((t2 - t0) / R * 1e6, 1)}), flush=True)
