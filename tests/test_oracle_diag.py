"""The oracle's per-pixel diagnostics (oracle_render_pixel) on the CPU: without flips it is the
full render's pixel bit for bit; flipping an environment lookup that lies near a texel boundary
changes the pixel (test_gpu_configs.py uses it to explain C4's pixels outside the bound)."""
import os

import numpy as np

import oracle_bind as ob
import rtgpu

SCENES = os.path.join(ob.GOLDEN, "scenes")


def test_render_pixel_equals_render():
    old = os.getcwd()
    os.chdir(SCENES)
    try:
        hs = rtgpu.HostScene("env_light.xml")
        hdr, _, _ = ob.render(hs, seed=9)
        h, w, _ = hdr.shape
        rng = np.random.default_rng(0)
        flipped = 0
        for y, x in zip(rng.integers(0, h, 40), rng.integers(0, w, 40)):
            v, n = ob.render_pixel(hs, int(x), int(y), seed=9, env_eps=0.05)
            assert np.array_equal(v.view(np.uint32), hdr[y, x].view(np.uint32)), (y, x)
            if n:
                f, _ = ob.render_pixel(hs, int(x), int(y), seed=9, env_eps=0.05, env_flip=(1 << n) - 1)
                flipped += int(not np.array_equal(f, v))
        assert flipped > 0
    finally:
        os.chdir(old)
