"""Path-tracing throughput (fused kernel): python tools/diag_pt.py [scene] [size] [spp]"""
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401

import oracle_bind as ob  # noqa: E402
import rtgpu  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "pt_cornell"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 512
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
src = open(os.path.join(ROOT, "tests", "golden", "scenes", name + ".xml")).read()
src = re.sub(r"<ImageResolution>[^<]*</ImageResolution>", f"<ImageResolution>{size} {size}</ImageResolution>", src)
src = ob.with_samples(src, spp)
d = tempfile.mkdtemp()
xml = os.path.join(d, "s.xml")
open(xml, "w").write(src)
hs = rtgpu.HostScene(xml)
ds = rtgpu.DeviceScene(hs, 0)
ds.reset_stats()
ds.render(0, flags=rtgpu.RTG_RENDER_COUNT_STATS)
st = ds.stats()
rays = st["camera_rays"] + st["secondary_rays"] + st["shadow_rays"]
for _ in range(2):
    t0 = time.perf_counter()
    ds.render(0, flags=rtgpu.RTG_RENDER_TIMING)
    t = ds.timings()
    el = time.perf_counter() - t0
k = sum(t.values())
print(f"{name} {size}^2 x {spp} spp: rays {rays} ({rays / (size * size * spp):.2f}/sample), kernels {t} ms,"
      f" {rays / (k * 1e-3) / 1e6:.0f} Mrays/s (kernel), wall {el * 1e3:.1f} ms", flush=True)
