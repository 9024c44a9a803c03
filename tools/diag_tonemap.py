"""Tonemapper parity and cost on the GPU: differing bytes against the reference's own
goldens (tests/golden/tonemap.npz) and the CPU restatement on full-HD inputs, and the
device time of one 1080p / 4K tonemap.  Run on the GPU box: python tools/diag_tonemap.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "advanced-cpu-raytracing_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle_bind as ob  # noqa: E402
import rtgpu  # noqa: E402


def diff(a, b):
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    return int((d != 0).sum()), int(d.max())


for i, (name, (key, burn, sat, gamma), ref) in enumerate(ob.tonemap_goldens()):
    got = rtgpu.tonemap(ob.load_golden(name), key, burn, sat, gamma)
    print("golden", i, name, (key, burn, sat, gamma), "differing bytes / max", diff(got, ref), "of", ref.size,
          flush=True)

rng = np.random.default_rng(4)
hdr = rng.lognormal(3.0, 1.5, size=(1080, 1920, 3)).astype(np.float32)
hdr[::97, ::89] = 0.0
for params in [(0.18, 1.0, 1.0, 2.2), (0.05, 10.0, 0.7, 2.4), (0.5, 0.0, 1.0, 1.0)]:
    got = rtgpu.tonemap(hdr, *params)
    ref = ob.tonemap(hdr, *params)
    print("fullhd", params, "differing bytes / max", diff(got, ref), "of", ref.size, flush=True)

print("log-sum mode (RTG_TM_SEQSUM):", os.environ.get("RTG_TM_SEQSUM", "library default"))
for (h, w, kind) in [(1080, 1920, "lognormal"), (2160, 3840, "lognormal"), (1080, 1920, "hover")]:
    a = rng.lognormal(1.0, 1.0, size=(h, w, 3)) if kind == "lognormal" else rng.uniform(0.0, 1.98, size=(h, w, 3))
    x = torch.from_numpy(a.astype(np.float32)).cuda()
    y = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
    p = rtgpu.TonemapParams(0.18, 1.0, 1.0, 2.2)
    st = torch.cuda.current_stream().cuda_stream
    f = rtgpu.lib().rtg_tonemap_device
    for _ in range(2):
        f(ctypes.c_void_p(x.data_ptr()), w, h, ctypes.byref(p), ctypes.c_void_p(y.data_ptr()), 0, ctypes.c_void_p(st))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        f(ctypes.c_void_p(x.data_ptr()), w, h, ctypes.byref(p), ctypes.c_void_p(y.data_ptr()), 0, ctypes.c_void_p(st))
    torch.cuda.synchronize()
    print("tonemap", kind, w, "x", h, "ms", round((time.perf_counter() - t) / 5 * 1e3, 3), flush=True)
