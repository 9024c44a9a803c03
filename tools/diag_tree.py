"""Tree-pipeline run of one configuration (rocprofv3 target).  python tools/diag_tree.py c5 [spp]"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402,F401

import rtgpu  # noqa: E402
import scenes  # noqa: E402

cfg = sys.argv[1]
kw = {"spp": int(sys.argv[2])} if len(sys.argv) > 2 else {}
d = tempfile.mkdtemp()
xml = scenes.config_c2(d, os.path.join(ROOT, "tests", "golden", "scenes", "cornell_conductors.xml")) if cfg == "c2" \
    else getattr(scenes, "config_" + cfg)(d, **kw)
os.chdir(d)
hs = rtgpu.HostScene(xml)
ds = rtgpu.DeviceScene(hs, 0)
for _ in range(2):
    ds.render(0, flags=rtgpu.RTG_RENDER_TREE | rtgpu.RTG_RENDER_TIMING)
print(ds.timings(), flush=True)
