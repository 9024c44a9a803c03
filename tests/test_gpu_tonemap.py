"""GPU photographic tonemapper (rtg_tonemap, rtg_render on <Tonemap> cameras) against the
reference's Tonemapper::Tonemap outputs (tests/golden/tonemap.npz) and the CPU restatement.

Exact: the log-average luminance is the reference's sequential double sum in pixel order
(k_tm_seqsum), so every byte equals the reference's -- measured 0 differing bytes on the 12
goldens and the three full-HD cases (tools/diag_tonemap.py).  The device library's double
log / exp / pow could in principle round differently from glibc's on some input; none of
these inputs shows it."""
import math
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


def _seq_log_average(hdr):
    """tonemapper.h:35-48 in Python floats (doubles, math.log = glibc's log, the sum in order)."""
    x = hdr.reshape(-1, 3).astype(np.float64)
    lum = 0.2126 * x[:, 0] + 0.7152 * x[:, 1] + 0.0722 * x[:, 2]
    delta = float(np.float32(0.01))
    s = 0.0
    for v in (lum + delta).tolist():
        s += math.log(v)
    return math.exp(s / len(lum))


def _log_inputs():
    rng = np.random.default_rng(11)
    yield "lognormal_1080p", rng.lognormal(0.0, 1.5, size=(1080, 1920, 3)).astype(np.float32)
    yield "bright", rng.lognormal(3.0, 1.0, size=(480, 640, 3)).astype(np.float32)
    # luminance around 0.99: log terms around zero, the running sum hovers near 0
    yield "hover", rng.uniform(0.0, 1.98, size=(480, 640, 3)).astype(np.float32)
    yield "flat_zero_logs", np.full((300, 500, 3), 0.99, np.float32)
    yield "black", np.zeros((200, 333, 3), np.float32)
    yield "ragged_1x1", np.full((1, 1, 3), 2.0, np.float32)
    yield "ragged_7x150", rng.lognormal(0.0, 2.0, size=(7, 150, 3)).astype(np.float32)
    # 4K, a sum that crosses zero and many binades: the mode-3 summaries fail and succeed
    yield "mixed_4k", np.concatenate([rng.lognormal(1.0, 1.0, size=(1080, 3840, 3)),
                                      rng.lognormal(-2.0, 1.0, size=(1080, 3840, 3))]).astype(np.float32)


@pytest.mark.parametrize("name,hdr", list(_log_inputs()), ids=[n for n, _ in _log_inputs()])
def test_log_average_sequential(name, hdr):
    """The windowed sums -- with the windows summarised in parallel first (mode 3, the default)
    and without (mode 2) -- equal the plain sequential chain (mode 1) bit for bit, and all equal
    the reference's host sum (glibc log) to the last bit where the device log agrees with
    glibc's (asserted within 1e-15 relative; exact equality is reported)."""
    win = rtgpu.tonemap_log_average(hdr, 2)
    summ = rtgpu.tonemap_log_average(hdr, 3)
    chain = rtgpu.tonemap_log_average(hdr, 1)
    assert win == chain or (math.isnan(win) and math.isnan(chain)), (name, win.hex(), chain.hex())
    assert summ == chain or (math.isnan(summ) and math.isnan(chain)), (name, summ.hex(), chain.hex())
    dflt = rtgpu.tonemap_log_average(hdr, -1)
    assert dflt == summ or (math.isnan(dflt) and math.isnan(summ))
    ref = _seq_log_average(hdr)
    print(name, "window == chain;", "== host reference" if win == ref else f"host {ref!r} vs {win!r}")
    assert abs(win - ref) <= 1e-15 * abs(ref), (name, win, ref)
