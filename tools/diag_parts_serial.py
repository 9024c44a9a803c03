"""One configuration's frame and its parts of N rendered one at a time (one stream, synchronised
after each render): the GPU time a part costs alone against 1/N of the frame, with no other
frame in flight to fill its tails.  Under rocprofv3 --kernel-trace, tools/trace_groups.py
then splits the kernels by grid size (frame / part).

    python tools/diag_parts_serial.py [c3|c3ton|c4|headline] [N] [reps]"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402

import rtgpu  # noqa: E402
import scenes  # noqa: E402


def scene(cfg, d):
    if cfg == "c3":
        return scenes.config_c3(d)
    if cfg == "c3ton":
        return scenes.config_c3_ton(d, os.path.join(ROOT, "tests", "golden", "scenes", "ton_Roosendaal_smooth_ply"))
    if cfg == "c4":
        return scenes.config_c4(d)
    return scenes.synthetic_heightfield(d)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    d = tempfile.mkdtemp()
    xml = scene(cfg, d)
    os.chdir(d)
    hs = rtgpu.HostScene(xml)
    ds = rtgpu.DeviceScene(hs, 0)
    c = hs.camera(0)
    H, W = c["height"], c["width"]
    hdr = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    ldr = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def timed(part):
        for _ in range(2):
            ds.render_device(hdr.data_ptr(), ldr.data_ptr(), st, seed=3, part=part)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ds.render_device(hdr.data_ptr(), ldr.data_ptr(), st, seed=3, part=part)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2] * 1e3

    full = timed((0, 1))
    parts = [timed((r, N)) for r in range(N)]
    out = {"config": cfg, "N": N, "full_ms": round(full, 4), "part_ms": [round(x, 4) for x in parts],
           "sum_parts_ms": round(sum(parts), 4), "serial_efficiency": round(full / (N * max(parts)), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
