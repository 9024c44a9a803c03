"""Diagnostics: per-frame time of the headline on the default stream vs a dedicated stream,
with and without per-frame event records in the timed loop.  python tools/diag_streams.py [steps]"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402

import rtgpu  # noqa: E402
import scenes  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
d = tempfile.mkdtemp()
xml = scenes.synthetic_heightfield(d)
os.chdir(d)
hs = rtgpu.HostScene(xml)
a = rtgpu.DeviceScene(hs, 0)
c = hs.camera(0)
H, W = c["height"], c["width"]
hdr = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
ldr = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
own = torch.cuda.Stream()


def run(stream, events):
    sp = stream.cuda_stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for _ in range(3):
        a.render_device(hdr.data_ptr(), ldr.data_ptr(), sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        if events:
            ev[k][0].record(stream)
        a.render_device(hdr.data_ptr(), ldr.data_ptr(), sp)
        if events:
            ev[k][1].record(stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for rep in range(2):
    for stream, sname in ((torch.cuda.default_stream(), "default"), (own, "own")):
        for events in (True, False):
            print(f"{sname:8s} stream, events={events}: {run(stream, events):.4f} ms/frame", flush=True)
