"""k_primary time for row bands of C3 (is the per-wave cost or the tail the problem?)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402,F401

import rtgpu  # noqa: E402
import scenes  # noqa: E402

d = tempfile.mkdtemp()
os.chdir(d)
xml = scenes.config_c3(d, spp=1)
hs = rtgpu.HostScene(xml)
ds = rtgpu.DeviceScene(hs, 0)
for rows in ((0, 1080), (112, 176), (112, 128), (128, 144), (400, 464), (0, 112), (176, 1080)):
    for _ in range(2):
        ds.render(0, rows=rows, flags=rtgpu.RTG_RENDER_TIMING)
        t = ds.timings()
    ds.reset_stats()
    ds.render(0, rows=rows, flags=rtgpu.RTG_RENDER_COUNT_STATS)
    st = ds.stats()
    print(rows, {k: round(v, 3) for k, v in t.items()}, st["node_visits"], st["tri_tests"], flush=True)
