"""k_shadow's walk against the per-lane reference-order walk (RTG_RENDER_EXACT_SHADOW).
The shipped wavefront walk (RTG_SHADOW_MODE 3, rtg_common.hpp trace_any_wide) decides
CastShadowRay (raytracer.cpp:585-623, a boolean) on the any-hit tree (rtg_ahb.cpp: binned
SAH over the reference's leaves), by exact sufficient / necessary conditions on each face's
reference leaf box with a reference-walk fallback; the A/B trees (RTG_AHB=split: large leaves
split into faces with padded boxes, RTG_AHB=ref: the reference's BVH collapsed) and the A/B
builds' walks (1: wave packets of the per-lane walk, 2: climbing
from the ray's origin leaf) pass the same tests.  Every image must be bit-identical -- on
every golden scene, through the wavefront, ray-tree and fused pipelines, at the headline's
full size and on C2-C5 at full size."""
import os

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu

pytestmark = pytest.mark.gpu

SCENES = os.path.join(ob.GOLDEN, "scenes")
NAMES = sorted(ob.manifest())


@pytest.fixture(scope="module", autouse=True)
def _cwd():
    old = os.getcwd()
    os.chdir(SCENES)
    yield
    os.chdir(old)


def _same(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


@pytest.mark.parametrize("flags", [0, rtgpu.RTG_RENDER_TREE])
@pytest.mark.parametrize("name", NAMES)
def test_wide_shadow_equals_reference_walk(name, flags):
    hs = rtgpu.HostScene(name + ".xml")
    ds = rtgpu.DeviceScene(hs, 0)
    hdr, ldr = ds.render(0, flags=flags)
    ehdr, eldr = ds.render(0, flags=flags | rtgpu.RTG_RENDER_EXACT_SHADOW)
    assert _same(hdr, ehdr) and _same(ldr, eldr)


@pytest.mark.parametrize("mode", ["split", "ref"])
@pytest.mark.parametrize("name", NAMES)
def test_anyhit_tree_modes(name, mode, monkeypatch):
    monkeypatch.setenv("RTG_AHB", mode)
    hs = rtgpu.HostScene(name + ".xml")
    ds = rtgpu.DeviceScene(hs, 0)
    hdr, ldr = ds.render(0)
    ehdr, eldr = ds.render(0, flags=rtgpu.RTG_RENDER_EXACT_SHADOW)
    assert _same(hdr, ehdr) and _same(ldr, eldr)


def _stats(ds, flags):
    ds.reset_stats()
    ds.render(0, flags=flags | rtgpu.RTG_RENDER_COUNT_STATS)
    return ds.stats()


def test_wide_shadow_headline_full_size(tmp_path):
    import scenes
    xml = scenes.synthetic_heightfield(str(tmp_path), K=100352)
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, 0)
        hdr, ldr = ds.render(0)
        ehdr, eldr = ds.render(0, flags=rtgpu.RTG_RENDER_EXACT_SHADOW)
        assert _same(hdr, ehdr) and _same(ldr, eldr)
        # the production render (what bench.py times) against the CPU restatement itself
        ohdr, oldr, _ = ob.render(hs)
        r = ob.compare(hdr, ohdr)
        assert r["n_fail"] == 0 and _same(ldr, oldr), r
        w = _stats(ds, 0)
        e = _stats(ds, rtgpu.RTG_RENDER_EXACT_SHADOW)
        print("wide", w, "\nexact", e)
        assert w["shadow_rays"] == e["shadow_rays"] > 0
        # extend rays untouched; the shipped any-hit walk (RTG_SHADOW_MODE 3: the 4-wide BVH)
        # fetches well under half the nodes of the reference's top-down walk, with almost no
        # rays left to the reference walk
        shadow_keys = ("shadow_node_visits", "shadow_tri_tests", "shadow_wide_visits", "shadow_fallbacks")
        assert {k: v for k, v in w.items() if k not in shadow_keys} == {k: v for k, v in e.items() if k not in shadow_keys}
        assert e["shadow_fallbacks"] == 0 and e["shadow_wide_visits"] == 0
        assert 0 < w["shadow_wide_visits"] < 0.5 * e["shadow_node_visits"]
        assert w["shadow_fallbacks"] < 1e-3 * w["shadow_rays"]
    finally:
        os.chdir(old)


@pytest.mark.parametrize("cfg", ["c5", "c2"])
def test_wide_shadow_configs(tmp_path, cfg):
    """C5 (ray trees, spheres, Perlin) reduced to 480x270 x 1 spp; C2 (conductors) at 200x200."""
    import scenes
    root = os.path.dirname(SCENES)
    if cfg == "c5":
        xml = scenes.config_c5(str(tmp_path), K=200000, width=480, height=270, spp=1)
    else:
        xml = scenes.config_c2(str(tmp_path), os.path.join(SCENES, "cornell_conductors.xml"), width=200, height=200)
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, 0)
        for flags in (0, rtgpu.RTG_RENDER_TREE, rtgpu.RTG_RENDER_FUSED):
            hdr, _ = ds.render(0, flags=flags)
            ehdr, _ = ds.render(0, flags=flags | rtgpu.RTG_RENDER_EXACT_SHADOW)
            assert _same(hdr, ehdr), flags
    finally:
        os.chdir(old)
    assert root


@pytest.mark.parametrize("cfg", ["c3", "c3ton", "c4", "c5"])
@pytest.mark.parametrize("mode", ["exact", "split"])
def test_wide_shadow_configs_full_size(tmp_path, cfg, mode, monkeypatch):
    """C3 (70k blob, area light, 4 spp), C3 on ton_Roosendaal, C4 (instances, 16 spp) and C5
    (870k, 4K, 64 spp) at their BASELINE sizes: the shipped render against the reference
    walk, every pixel, with the default tree and with large leaves split (RTG_AHB=split,
    which large-leaf scenes C3, C3-ton and C4 then take)."""
    import scenes
    monkeypatch.setenv("RTG_AHB", mode)
    if cfg == "c3":
        xml = scenes.config_c3(str(tmp_path))
    elif cfg == "c3ton":
        xml = scenes.config_c3_ton(str(tmp_path), os.path.join(SCENES, "ton_Roosendaal_smooth_ply"))
    elif cfg == "c4":
        xml = scenes.config_c4(str(tmp_path))
    else:
        xml = scenes.config_c5(str(tmp_path))
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, 0)
        hdr, ldr = ds.render(0)
        ehdr, eldr = ds.render(0, flags=rtgpu.RTG_RENDER_EXACT_SHADOW)
        diff = int((hdr.view(np.uint32) != ehdr.view(np.uint32)).any(axis=2).sum())
        print(cfg, "differing pixels", diff)
        assert diff == 0 and _same(ldr, eldr)
        st = _stats(ds, 0)
        print(cfg, {k: st[k] for k in ("shadow_rays", "shadow_wide_visits", "shadow_tri_tests", "shadow_fallbacks")})
    finally:
        os.chdir(old)

