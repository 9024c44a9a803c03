"""Deferred large leaves (k_bigleaf / k_hitfix) on a large-leaf configuration: pending pixels and
the ones whose winner failed the leaf-box check (counters of a production render: with
RTG_DEFER_DIAG=1, set here, k_hitfix counts them in extend_wide_visits / extend_fallbacks).

    python tools/diag_defer.py [c3|c3ton|c4]"""
import json
import os
import sys
import tempfile

os.environ["RTG_DEFER_DIAG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "advanced-cpu-raytracing_amd"))
import torch  # noqa: E402,F401

import rtgpu  # noqa: E402
import scenes  # noqa: E402


def main():
    for cfg in sys.argv[1:] or ["c3", "c3ton", "c4"]:
        d = tempfile.mkdtemp()
        if cfg == "c3":
            xml = scenes.config_c3(d)
        elif cfg == "c3ton":
            xml = scenes.config_c3_ton(d, os.path.join(ROOT, "tests", "golden", "scenes", "ton_Roosendaal_smooth_ply"))
        else:
            xml = scenes.config_c4(d)
        os.chdir(d)
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, 0)
        ds.render(0, seed=1)
        ds.reset_stats()
        ds.render(0, seed=1)
        st = ds.stats()
        c = hs.camera(0)
        print(json.dumps({"config": cfg, "camera_rays": c["width"] * c["height"] * c["spp"],
                          "pending": st["extend_wide_visits"], "checked_out": st["extend_fallbacks"]}), flush=True)


if __name__ == "__main__":
    main()
