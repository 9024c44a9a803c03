"""Path tracing: device-resident frame time of the fused kernel vs the wavefront path tracer
(rtg_path.hip, RTG_RENDER_TREE; with path regeneration and with a pass per sample), per scene at size^2 x spp.  Rays per frame from a counted
fused render.  One JSON line per (scene, path).

    python tools/diag_ptwave.py [size] [spp] [scene ...]
"""
import json
import os
import re
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import oracle_bind as ob  # noqa: E402
import rtgpu  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
names = sys.argv[3:] or ["pt_cornell", "pt_nee", "pt_rr"]
for name in names:
    src = open(os.path.join(ROOT, "tests", "golden", "scenes", name + ".xml")).read()
    src = re.sub(r"<ImageResolution>[^<]*</ImageResolution>", f"<ImageResolution>{size} {size}</ImageResolution>", src)
    src = ob.with_samples(src, spp)
    d = tempfile.mkdtemp()
    xml = os.path.join(d, "s.xml")
    open(xml, "w").write(src)
    hs = rtgpu.HostScene(xml)
    ds = rtgpu.DeviceScene(hs, 0)
    hdr = torch.empty((size, size, 3), dtype=torch.float32, device="cuda")
    ldr = torch.empty((size, size, 3), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ds.reset_stats()
    ds.render_device(hdr.data_ptr(), ldr.data_ptr(), st, flags=rtgpu.RTG_RENDER_FUSED | rtgpu.RTG_RENDER_COUNT_STATS)
    torch.cuda.synchronize()
    s = ds.stats()
    rays = s["camera_rays"] + s["secondary_rays"] + s["shadow_rays"]
    ref = None
    for path, flags, regen in (("fused", rtgpu.RTG_RENDER_FUSED, "1"), ("wavefront_regen", rtgpu.RTG_RENDER_TREE, "1"),
                               ("wavefront_noregen", rtgpu.RTG_RENDER_TREE, "0")):
        os.environ["RTG_PATH_REGEN"] = regen    # read per render (rtg_path.hip path_pass_samples)
        for _ in range(2):
            ds.render_device(hdr.data_ptr(), ldr.data_ptr(), st, flags=flags)
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            ds.render_device(hdr.data_ptr(), ldr.data_ptr(), st, flags=flags)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        img = hdr.cpu().numpy()
        same = None if ref is None else bool((img.view("uint32") == ref.view("uint32")).all())
        ref = img if ref is None else ref
        print(json.dumps({"scene": name, "size": size, "spp": spp, "path": path, "ms_per_frame": round(ms, 3),
                          "rays": rays, "rays_per_sample": round(rays / (size * size * spp), 3),
                          "mrays_s": round(rays / ms / 1e3, 1), "bit_identical_to_fused": same}), flush=True)
    ds.close()
    hs.close()
