"""Diagnostics: does overlapping two halves of the headline frame on two streams hide the
kernel-boundary drain?  Two replicas of the scene on GPU 0 (separate work buffers) render
the two interleaved 16-row-band halves (part 0/1 of 2) on two streams, against one replica
rendering the whole frame on one stream.  python tools/diag_split.py [steps]"""
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
b = rtgpu.DeviceScene(hs, 0)
c = hs.camera(0)
H, W = c["height"], c["width"]
hdr = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
ldr = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()


def one():
    a.render_device(hdr.data_ptr(), ldr.data_ptr(), s1.cuda_stream)


def split():
    a.render_device(hdr.data_ptr(), ldr.data_ptr(), s1.cuda_stream, part=(0, 2))
    b.render_device(hdr.data_ptr(), ldr.data_ptr(), s2.cuda_stream, part=(1, 2))


def timeit(f):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


for f, name in ((one, "one stream, whole frame"), (split, "two streams, two halves"),
                (one, "one stream, whole frame"), (split, "two streams, two halves")):
    print(f"{name}: {timeit(f):.4f} ms/frame", flush=True)
ref = hdr.clone()
one()
torch.cuda.synchronize()
ref = hdr.clone()
split()
torch.cuda.synchronize()
print("identical:", bool(torch.equal(ref.view(torch.int32), hdr.view(torch.int32))), flush=True)
