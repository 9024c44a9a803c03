"""Part (r, N) of the headline frame with F frames in flight (F scene replicas, each on its own
stream), per part: the time per part-frame and the host's issue time -- what one GPU of an
N-GPU node does per step (bench.py part_scaling, alone, for A/B of run-time settings).

    RTG_DIAG_F=8 RTG_DIAG_N=8 python tools/diag_parts8.py [steps]

RTG_DIAG_PARTS=0,3 renders only those parts (e.g. under rocprofv3 --kernel-trace, whose
trace tools/trace_parts.py reads).
"""
import json
import os
import sys
import tempfile
import time

F = int(os.environ.get("RTG_DIAG_F", "8"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", str(F + 1))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402

import rtgpu  # noqa: E402
import scenes  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 320
    N = int(os.environ.get("RTG_DIAG_N", "8"))
    d = tempfile.mkdtemp()
    xml = scenes.synthetic_heightfield(d)
    os.chdir(d)
    hs = rtgpu.HostScene(xml)
    reps = [rtgpu.DeviceScene(hs, 0) for _ in range(F)]
    bufs = [(torch.empty((1080, 1920, 3), dtype=torch.float32, device="cuda"),
             torch.empty((1080, 1920, 3), dtype=torch.uint8, device="cuda")) for _ in range(F)]
    streams = [torch.cuda.Stream() for _ in range(F)]
    full = []
    only = os.environ.get("RTG_DIAG_PARTS")
    sel = [int(x) for x in only.split(",")] if only else list(range(N))
    for parts in ((0, 1),) + tuple((r, N) for r in sel):
        def step(k):
            h, l = bufs[k % F]
            reps[k % F].render_device(h.data_ptr(), l.data_ptr(), streams[k % F].cuda_stream, seed=7, part=parts)
        for k in range(2 * F):
            step(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            step(k)
        issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        full.append({"part": list(parts), "ms": round(el / steps * 1e3, 4), "issue_ms": round(issue / steps * 1e3, 4)})
    frame = full[0]["ms"]
    worst = max(p["ms"] for p in full[1:])
    print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith(("RTG_", "HIP_", "GPU_MAX"))},
                      "F": F, "N": N, "frame_ms": frame, "max_part_ms": worst,
                      "predicted_efficiency": round(frame / (N * worst), 4), "parts": full}), flush=True)


if __name__ == "__main__":
    main()
