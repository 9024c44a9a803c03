"""GPU photographic tonemapper (rtg_tonemap, rtg_render on <Tonemap> cameras) against the
reference's Tonemapper::Tonemap outputs (tests/golden/tonemap.npz) and the CPU restatement.

Exact: the log-average luminance is the reference's sequential double sum in pixel order
(k_tm_seqsum), so every byte equals the reference's -- measured 0 differing bytes on the 12
goldens and the three full-HD cases (tools/diag_tonemap.py).  The device library's double
log / exp / pow could in principle round differently from glibc's on some input; none of
these inputs shows it."""
import os

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu

pytestmark = pytest.mark.gpu

SCENES = os.path.join(ob.GOLDEN, "scenes")


def _close(got, ref):
    d = np.abs(got.astype(np.int32) - ref.astype(np.int32))
    return float(np.mean(d == 0)), int(d.max())


@pytest.mark.parametrize("case", range(12))
def test_tonemap_matches_reference(case):
    name, (key, burn, sat, gamma), ref = ob.tonemap_goldens()[case]
    got = rtgpu.tonemap(ob.load_golden(name), key, burn, sat, gamma)
    exact, mx = _close(got, ref)
    assert exact == 1.0, (name, exact, mx)


@pytest.mark.parametrize("params", [(0.18, 1.0, 1.0, 2.2), (0.05, 10.0, 0.7, 2.4), (0.5, 0.0, 1.0, 1.0)])
def test_tonemap_full_hd_vs_oracle(params):
    rng = np.random.default_rng(4)
    hdr = rng.lognormal(3.0, 1.5, size=(1080, 1920, 3)).astype(np.float32)
    hdr[::97, ::89] = 0.0                     # black pixels: R / y_i = NaN -> clipped to 0
    got = rtgpu.tonemap(hdr, *params)
    ref = ob.tonemap(hdr, *params)
    exact, mx = _close(got, ref)
    assert exact == 1.0, (exact, mx)


def test_render_tonemapped_camera(tmp_path):
    s = open(os.path.join(SCENES, "env_light.xml")).read().replace(
        "<ImageName>env_light.png</ImageName>",
        "<ImageName>env_light.hdr</ImageName>\n            <Tonemap><TMO>Photographic</TMO>"
        "<TMOOptions>0.18 1</TMOOptions><Saturation>1.0</Saturation><Gamma>2.2</Gamma></Tonemap>")
    xml = tmp_path / "tm.xml"
    xml.write_text(s)
    old = os.getcwd()
    os.chdir(SCENES)
    try:
        hs = rtgpu.HostScene(str(xml))
        assert hs.camera(0)["tonemapped"]
        ds = rtgpu.DeviceScene(hs, 0)
        hdr, ldr = ds.render(0)
        # the LDR output is the tonemapped image of the float output (main.cpp:187-192)
        assert np.array_equal(ldr, rtgpu.tonemap(hdr, 0.18, 1.0, 1.0, 2.2))
        exact, mx = _close(ldr, ob.tonemap(hdr, 0.18, 1.0, 1.0, 2.2))
        assert exact == 1.0, (exact, mx)
        # a row band keeps the clamp (the tonemapper needs the whole image)
        _, band = ds.render(0, rows=(0, 8))
        assert np.array_equal(band[:8], ob.clamp_ldr(hdr[:8]))
    finally:
        os.chdir(old)
