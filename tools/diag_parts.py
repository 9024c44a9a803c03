"""Diagnostics for the N-GPU partition on one GPU: part (r, N) of the headline frame timed
alone (the latency floor of a small grid), per kernel, and F parts of F independent frames in
flight at once (F scene replicas, each on its own stream: what a GPU of an N-GPU node does
when a step carries F frames).  Prints one JSON line per (N, F).

    python tools/diag_parts.py [steps]
"""
import json
import os
import sys
import tempfile
import time

# RTG_DIAG_QUEUES: hardware queues per process (HIP's default is 4): more streams than queues
# share them and serialise
if os.environ.get("RTG_DIAG_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ["RTG_DIAG_QUEUES"]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402

import rtgpu  # noqa: E402
import scenes  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
d = tempfile.mkdtemp()
xml = scenes.synthetic_heightfield(d)
os.chdir(d)
hs = rtgpu.HostScene(xml)
FS = [int(x) for x in os.environ.get("RTG_DIAG_F", "1,2,4,8").split(",")]
FMAX = max(FS)
reps = [rtgpu.DeviceScene(hs, 0) for _ in range(FMAX)]
c = hs.camera(0)
H, W = c["height"], c["width"]
bufs = [(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"),
         torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")) for _ in range(FMAX)]
streams = [torch.cuda.Stream() for _ in range(FMAX)]


def run(n, part, f, nsteps):
    for _ in range(2):
        for k in range(f):
            reps[k].render_device(bufs[k][0].data_ptr(), bufs[k][1].data_ptr(), streams[k].cuda_stream, part=(part, n))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(nsteps):
        for k in range(f):
            reps[k].render_device(bufs[k][0].data_ptr(), bufs[k][1].data_ptr(), streams[k].cuda_stream, part=(part, n))
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / nsteps * 1e3


base = run(1, 0, 1, steps)
for n in (1, 2, 4, 8):
    # the slowest part of N (bands are dealt b % N; part 0 has the most bands)
    kt = {}
    for _ in range(5):
        reps[0].render_device(bufs[0][0].data_ptr(), bufs[0][1].data_ptr(), streams[0].cuda_stream,
                              flags=rtgpu.RTG_RENDER_TIMING, part=(0, n))
        for k, v in reps[0].timings().items():
            kt[k] = kt.get(k, 0.0) + v / 5
    for f in FS:
        ms = run(n, 0, f, steps)
        # f frames' part 0 per ms; an N-GPU node renders f whole frames in this time
        eff = base * f / (n * ms)
        print(json.dumps({"N": n, "frames_in_flight": f, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default"), "ms_per_step": round(ms, 4),
                          "kernels_ms_one_part": {k: round(v, 4) for k, v in kt.items()},
                          "predicted_efficiency": round(eff, 4),
                          "predicted_mrays_s": round(4147193 * f * n / (n * ms * 1e-3) / 1e6, 1)}), flush=True)
