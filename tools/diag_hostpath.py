"""rtg_render's host-buffer path (the CLI's, main.cpp:164-195) on the headline frame: one frame at
a time into page-locked frames: the kernels writing into the frame directly (the default for
page-locked frames), render + copy (RTG_HOST_DIRECT=0), and the chunked path (RTG_HOST_CHUNKS, rtg_api.cpp render_chunked) --
beside the device-resident frame (rtg_render_device + synchronize) it is compared with.
Usage: python tools/diag_hostpath.py [frames]"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))

import torch  # noqa: E402,F401  (one HIP runtime: torch first, rtgpu.lib())

import rtgpu  # noqa: E402
import scenes  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    d = tempfile.mkdtemp()
    xml = scenes.synthetic_heightfield(d, K=100352)
    os.chdir(d)
    hs = rtgpu.HostScene(xml)
    ds = rtgpu.DeviceScene(hs, 0)
    H, W = 1080, 1920
    pl = rtgpu.PinnedArray((H, W, 3), "uint8")
    hdr = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
    ldr = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()

    def dev():
        ds.render_device(hdr.data_ptr(), ldr.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()

    def host():
        ds.render(0, out=(None, pl.array))

    cases = [("device", {}, dev), ("host_copy", {"RTG_HOST_DIRECT": "0"}, host), ("host_direct", {}, host)]
    for c in (2, 4):
        cases.append((f"host_chunks{c}", {"RTG_HOST_CHUNKS": str(c)}, host))
    ref = None
    for rep in range(2):
        for name, env, fn in cases:
            for k in ("RTG_HOST_CHUNKS", "RTG_HOST_CHUNK_COPY", "RTG_HOST_DIRECT"):
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(3):
                fn()
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            ms = (time.perf_counter() - t0) / n * 1e3
            if fn is host:
                if ref is None:
                    ref = pl.array.copy()
                same = bool((pl.array == ref).all())
            else:
                same = None
            print(json.dumps({"case": name, "rep": rep, "ms_per_frame": round(ms, 4), "same_ldr": same}), flush=True)


if __name__ == "__main__":
    main()
