"""Diagnostics: per-kernel timings of one configuration on the wavefront pipeline and the
fused kernel, with traversal statistics.  python tools/diag_config.py c3 [spp]"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402,F401

import rtgpu  # noqa: E402
import scenes  # noqa: E402

cfg = sys.argv[1]
d = tempfile.mkdtemp()
kw = {}
if len(sys.argv) > 2:
    kw["spp"] = int(sys.argv[2])
if cfg == "c2":
    xml = scenes.config_c2(d, os.path.join(ROOT, "tests", "golden", "scenes", "cornell_conductors.xml"))
elif cfg == "headline":
    xml = scenes.synthetic_heightfield(d)
else:
    xml = getattr(scenes, "config_" + cfg)(d, **kw)
os.chdir(d)
hs = rtgpu.HostScene(xml)
ds = rtgpu.DeviceScene(hs, 0)
print(cfg, hs.counts(), hs.camera(0), flush=True)
for flags, name in ((0, "default"), (rtgpu.RTG_RENDER_FUSED, "fused"), (rtgpu.RTG_RENDER_TREE, "tree")):
    ds.reset_stats()
    ds.render(0, flags=flags | rtgpu.RTG_RENDER_COUNT_STATS)
    st = ds.stats()
    for _ in range(2):
        ds.render(0, flags=flags | rtgpu.RTG_RENDER_TIMING)
        t = ds.timings()
    print(name, {k: round(v, 3) for k, v in t.items()}, st, flush=True)
