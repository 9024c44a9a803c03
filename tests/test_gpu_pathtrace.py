"""Path tracing (ComputeGlobalIllumination, raytracer.cpp:135-191) and mesh lights
(MeshLight::getSample, meshLight.h:27-47; SampleDirectLighting :780-803) on the GPU.

* Per pixel, GPU == CPU oracle on the same counter-RNG keys (tolerance 1e-4 relative,
  north_star's bound), every pixel, with the same camera / secondary / shadow ray counts (a
  GI direction computed with a last-ulp different sinf/acosf could flip a grazing hit; on the
  six scenes at 4 spp none does).
* Against the reference itself: statistical goldens (tests/golden/pt_*.npz, and
  <name>_avg.npz for the area-light, environment-light, DOF + motion-blur and C3 fixtures: the
  per-pixel mean of 1024 reference samples and its variance) vs the GPU at 4096 spp, 8x8-block
  z-scores.
* Mesh-light sampling has no reference golden (the reference's face draw is out of range
  in 1 of faceCount+1 draws): GPU == oracle only, on every render path.
"""
import os

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu

pytestmark = pytest.mark.gpu

REL = 1e-4
SCENES = os.path.join(ob.GOLDEN, "scenes")
AVG = sorted(k for k, v in ob.manifest().items() if v["kind"] == "stochastic_avg")
PARITY = AVG + ["pt_meshlight", "mesh_light"]


def _scene(tmp_path, name, spp):
    xml = tmp_path / (name + ".xml")
    xml.write_text(ob.with_samples(open(os.path.join(SCENES, name + ".xml")).read(), spp))
    old = os.getcwd()
    os.chdir(SCENES)                  # PLY files resolve from the current directory (parser.cpp:1404)
    try:
        return rtgpu.HostScene(str(xml))
    finally:
        os.chdir(old)


@pytest.mark.parametrize("name", PARITY)
def test_gpu_equals_oracle(name, tmp_path):
    hs = _scene(tmp_path, name, 4)
    ds = rtgpu.DeviceScene(hs, 0)
    ds.reset_stats()
    hdr, ldr = ds.render(0, seed=99, flags=rtgpu.RTG_RENDER_COUNT_STATS)
    st = ds.stats()
    ohdr, _, ost = ob.render(hs, seed=99)
    r = ob.compare(hdr, ohdr, REL)
    print(name, r, st, ost)
    # round 4: every pixel within the bound and the same rays on all six scenes (a last-ulp
    # different sinf / acosf in a GI direction moved one triangle test of pt_cornell, no ray)
    assert r["n_fail"] == 0, r
    assert np.array_equal(ldr, ob.clamp_ldr(hdr))
    for k in ("camera_rays", "secondary_rays", "shadow_rays"):
        assert st[k] == ost[k], (k, st[k], ost[k])


STOCH = sorted(k for k, v in ob.manifest().items() if v["kind"] == "stochastic" and "avg_samples" in v)


@pytest.mark.parametrize("name", AVG + STOCH)
def test_gpu_statistical_vs_reference(name, tmp_path):
    hs = _scene(tmp_path, name, 4096)
    ds = rtgpu.DeviceScene(hs, 0)
    hdr, _ = ds.render(0, seed=5)
    ok, info = ob.zscore_ok(ob.block_zscores(hdr, name, 4096))
    print(name, info)
    assert ok, info


def test_mesh_light_every_path(tmp_path):
    """A LightMesh sampled by direct lighting (no path tracing): the wavefront pipeline, the
    fused kernel and the oracle agree."""
    xml = tmp_path / "ml0.xml"
    xml.write_text(open(os.path.join(SCENES, "mesh_light.xml")).read().replace(
        "<MaxRecursionDepth>1</MaxRecursionDepth>", "<MaxRecursionDepth>0</MaxRecursionDepth>"))
    hs = rtgpu.HostScene(str(xml))
    ds = rtgpu.DeviceScene(hs, 0)
    a, _ = ds.render(0, seed=3)
    b, _ = ds.render(0, seed=3, flags=rtgpu.RTG_RENDER_FUSED)
    ds.render(0, flags=rtgpu.RTG_RENDER_TIMING)
    t = ds.timings()
    assert "k_primary" in t or "k_frame" in t            # the wavefront pipeline ran
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), ob.compare(a, b)
    o, _, _ = ob.render(hs, seed=3)
    r = ob.compare(a, o, REL)
    assert r["rel_pass"] == 1.0, r


def test_mesh_light_tree_pipeline(tmp_path):
    """Mesh lights in the wavefront ray-tree pipeline (a mirror sphere spawns children)."""
    s = open(os.path.join(SCENES, "mesh_light.xml")).read().replace('<Sphere id="1">\n            <Material>4</Material>', '<Sphere id="1">\n            <Material>5</Material>')
    xml = tmp_path / "ml_tree.xml"
    xml.write_text(s)
    hs = rtgpu.HostScene(str(xml))
    ds = rtgpu.DeviceScene(hs, 0)
    a, _ = ds.render(0, seed=3, flags=rtgpu.RTG_RENDER_TREE)
    b, _ = ds.render(0, seed=3, flags=rtgpu.RTG_RENDER_FUSED)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), ob.compare(a, b)
    o, _, _ = ob.render(hs, seed=3)
    assert ob.compare(a, o, REL)["rel_pass"] == 1.0


def test_path_tracing_deterministic_across_row_bands(tmp_path):
    """Counter-based RNG: rendering the reference's 8 row bands separately gives the same
    image as one launch (GPU-count independence of the sample-parallel / band split)."""
    hs = _scene(tmp_path, "pt_cornell", 2)
    ds = rtgpu.DeviceScene(hs, 0)
    full, _ = ds.render(0, seed=17)
    out = np.zeros_like(full)
    for t in range(8):
        band, _ = ds.render(0, rows=(t * 8, t * 8 + 8), seed=17)
        out[t * 8:t * 8 + 8] = band[t * 8:t * 8 + 8]
    assert np.array_equal(out.view(np.uint32), full.view(np.uint32))


PT_ONLY = ["pt_cornell", "pt_nee", "pt_rr", "pt_meshlight"]


def _bits(a):
    return a.view(np.uint32)


# step kernel modes: as chosen by the camera (regeneration with Russian roulette), with path
# regeneration forced, and with a pass per sample
MODES = {"default": {}, "regen": {"RTG_PATH_REGEN": "1"}, "noregen": {"RTG_PATH_REGEN": "0"}}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", PT_ONLY)
@pytest.mark.parametrize("spp", [1, 4])
def test_path_wavefront_equals_fused(name, spp, mode, tmp_path, monkeypatch):
    """The wavefront path tracer (rtg_path.hip, forced with RTG_RENDER_TREE) gives the fused
    kernel's image bit for bit: the same node steps (rtg_node.hpp) on the same RNG keys -- with
    the step as one kernel (the default), with or without path regeneration (a finished sample's
    slot starting the pixel's next sample inside the pass; by default with Russian roulette).
    The first render plans its
    later passes from its first; the second runs planned throughout."""
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    hs = _scene(tmp_path, name, spp)
    ds = rtgpu.DeviceScene(hs, 0)
    b, lb = ds.render(0, seed=11, flags=rtgpu.RTG_RENDER_FUSED)
    for _ in range(2):
        a, la = ds.render(0, seed=11, flags=rtgpu.RTG_RENDER_TREE)
        assert np.array_equal(_bits(a), _bits(b)), ob.compare(a, b)
        assert np.array_equal(la, lb)
    ds.render(0, seed=11, flags=rtgpu.RTG_RENDER_TREE | rtgpu.RTG_RENDER_TIMING)
    assert "path_iterations" in ds.timings()


@pytest.mark.parametrize("env", ["RTG_PATH_SYNC", "RTG_PATH_PLAN_TIGHT"])
def test_path_wavefront_host_driven_and_overflow(env, tmp_path, monkeypatch):
    """Every pass host-driven (RTG_PATH_SYNC), and plans one iteration short
    (RTG_PATH_PLAN_TIGHT: every planned pass leaves paths, the render is redone host-driven):
    the same image as the fused kernel."""
    monkeypatch.setenv(env, "1")
    hs = _scene(tmp_path, "pt_nee", 4)
    ds = rtgpu.DeviceScene(hs, 0)
    b, _ = ds.render(0, seed=5, flags=rtgpu.RTG_RENDER_FUSED)
    for _ in range(2):
        a, _ = ds.render(0, seed=5, flags=rtgpu.RTG_RENDER_TREE)
        assert np.array_equal(_bits(a), _bits(b)), ob.compare(a, b)


@pytest.mark.parametrize("name", ["pt_cornell", "pt_nee"])
def test_path_wavefront_stats_and_bands(name, tmp_path, monkeypatch):
    """Ray counts of the wavefront path tracer equal the fused kernel's; row bands rendered
    separately give the whole frame (part_pixel mapping of the path queues)."""
    hs = _scene(tmp_path, name, 2)
    ds = rtgpu.DeviceScene(hs, 0)
    ds.reset_stats()
    ds.render(0, seed=17, flags=rtgpu.RTG_RENDER_FUSED | rtgpu.RTG_RENDER_COUNT_STATS)
    sf = ds.stats()
    ds.reset_stats()
    full, _ = ds.render(0, seed=17, flags=rtgpu.RTG_RENDER_TREE | rtgpu.RTG_RENDER_COUNT_STATS)
    sw = ds.stats()
    for k in ("camera_rays", "secondary_rays", "shadow_rays"):
        assert sw[k] == sf[k], (k, sw[k], sf[k])
    out = np.zeros_like(full)
    for t in range(4):
        band, _ = ds.render(0, rows=(t * 16, t * 16 + 16), seed=17, flags=rtgpu.RTG_RENDER_TREE)
        out[t * 16:t * 16 + 16] = band[t * 16:t * 16 + 16]
    assert np.array_equal(_bits(out), _bits(full))


@pytest.mark.parametrize("regen", ["1", "0"])
def test_path_regeneration_passes_and_sample_ranges(regen, tmp_path, monkeypatch):
    """Regeneration across pass boundaries (70 spp: passes of 64 and 6 samples per slot) and
    with sample ranges accumulated separately (RTG_RENDER_ACCUM_ONLY, samples [0, 3) and
    [3, 7)): the fused kernel's bits, so each pixel's samples are still summed in sample order."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("RTG_PATH_REGEN", regen)
    hs = _scene(tmp_path, "pt_rr", 70)
    ds = rtgpu.DeviceScene(hs, 0)
    b, lb = ds.render(0, seed=23, flags=rtgpu.RTG_RENDER_FUSED)
    for _ in range(2):
        a, la = ds.render(0, seed=23, flags=rtgpu.RTG_RENDER_TREE)
        assert np.array_equal(_bits(a), _bits(b)), ob.compare(a, b)
        assert np.array_equal(la, lb)
    h, w = a.shape[:2]
    for s0, n in ((0, 3), (3, 4)):
        accs = []
        for flags in (rtgpu.RTG_RENDER_FUSED, rtgpu.RTG_RENDER_TREE):
            acc = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda:0")
            ds.render_device(0, 0, 0, accum_ptr=acc.data_ptr(), flags=flags | rtgpu.RTG_RENDER_ACCUM_ONLY,
                             sample_begin=s0, sample_count=n, seed=23)
            torch.cuda.synchronize()
            accs.append(acc.cpu().numpy())
        assert np.array_equal(_bits(accs[0]), _bits(accs[1]))


@pytest.mark.parametrize("cap", ["8", "48", "4096"])
def test_path_regeneration_iteration_bound(cap, tmp_path, monkeypatch):
    """Passes with path regeneration run many iterations (up to 64 samples per slot, Russian
    roulette chains); a plan grown from a long first pass (its iterations + a quarter) must stay
    within the per-pass bound the iteration counters are sized for (kPathMaxIter, lowered here
    with RTG_PATH_ITER_CAP): capped, a pass that needs more leaves paths, the render is redone
    host-driven and a pass past the bound falls back to the fused kernel -- the fused kernel's
    bits whichever happens (rtg_path.hip path_run)."""
    monkeypatch.setenv("RTG_PATH_REGEN", "1")
    monkeypatch.setenv("RTG_PATH_ITER_CAP", cap)
    hs = _scene(tmp_path, "pt_rr", 64)
    ds = rtgpu.DeviceScene(hs, 0)
    b, lb = ds.render(0, seed=29, flags=rtgpu.RTG_RENDER_FUSED)
    for _ in range(3):
        a, la = ds.render(0, seed=29, flags=rtgpu.RTG_RENDER_TREE)
        assert np.array_equal(_bits(a), _bits(b)), ob.compare(a, b)
        assert np.array_equal(la, lb)
