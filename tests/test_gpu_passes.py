"""Multi-sample passes (RenderParams::slabs, rtg_api.cpp pass_slabs): the wavefront and ray-tree
pipelines carry several consecutive samples of the rendered pixels in one pass (~16 Mi camera
rays), so a GPU holding 1/N of a frame still launches full grids, and a frame pays the tail of
its slowest waves once per pass.  Each pixel's colours of a pass are added to its accumulation
in sample order (accum_samples: renderThreadMain's spp loop, main.cpp:80-121), so the image must
be the one of one-sample passes (RTG_RENDER_SAMPLE_PASSES) bit for bit -- in every layout of the
wavefront pipeline (fused, one light, general, deferred large leaves, instances), on the ray
trees (host-driven first pass, planned passes, a short last pass), for frame parts and for
accumulate-only sample ranges.  The full-size C3 / C4 / C5 renders of test_gpu_configs.py run
the multi-sample passes against the CPU restatement."""
import os

import numpy as np
import pytest

import multigpu
import oracle_bind as ob
import rtgpu
import scenes

pytestmark = pytest.mark.gpu

SCENES = os.path.join(ob.GOLDEN, "scenes")
ONE = rtgpu.RTG_RENDER_SAMPLE_PASSES


@pytest.fixture()
def in_tmp(tmp_path):
    old = os.getcwd()
    os.chdir(tmp_path)
    yield str(tmp_path)
    os.chdir(old)


def _same(a, b):
    return np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)) and np.array_equal(a[1], b[1])


def _fixture(name, in_tmp, spp, width=None, height=None):
    src = os.path.join(SCENES, name + ".xml")
    os.chdir(SCENES)                       # the fixtures' relative PLY / texture paths
    hs0 = rtgpu.HostScene(src)
    c = hs0.camera(0)
    hs0.close()
    return scenes.with_resolution(src, os.path.join(in_tmp, name + "_spp.xml"), width or c["width"],
                                  height or c["height"], spp)


def _case(name, in_tmp):
    if name == "c3_small":
        return scenes.config_c3(in_tmp, K=20000, width=320, height=180, spp=4), 0
    if name == "c4_small":
        return scenes.config_c4(in_tmp, n_side=3, K_tree=4000, width=320, height=180, spp=6), 0
    if name == "synth_fused":
        return scenes.synthetic_heightfield(in_tmp, K=10000, width=320, height=180, spp=3), 0
    if name in ("c5_dragon", "cornell_dielectric", "spheres_mirror"):
        return _fixture(name, in_tmp, 5, 320, 240), rtgpu.RTG_RENDER_TREE
    return scenes.with_depth(_fixture(name, in_tmp, 4), os.path.join(in_tmp, name + "_d0.xml"), 0), 0


@pytest.mark.parametrize("name", ["synth_fused", "area_light", "env_light", "brdf_lights", "transforms_textures",
                                  "c3_small", "c4_small", "c5_dragon", "cornell_dielectric", "spheres_mirror"])
def test_sample_passes_equal_one_sample_passes(name, in_tmp, monkeypatch):
    xml, flags = _case(name, in_tmp)
    hs = rtgpu.HostScene(xml)
    ds = rtgpu.DeviceScene(hs, 0)
    c = hs.camera(0)
    spp = c["spp"]
    assert spp > 1
    one = ds.render(0, seed=21, flags=flags | ONE)
    multi = ds.render(0, seed=21, flags=flags)            # every sample in one pass at this size
    again = ds.render(0, seed=21, flags=flags)            # (ray trees: the planned passes)
    # passes of two samples and a short last one (spp odd) or of three
    monkeypatch.setenv("RTG_PASS_RAYS", str(c["width"] * c["height"] * 2))
    two = ds.render(0, seed=21, flags=flags)
    print(name, spp, "differing pixels", int((one[0].view(np.uint32) != multi[0].view(np.uint32)).any(axis=2).sum()))
    assert _same(one, multi) and _same(one, again) and _same(one, two)
    # a frame part: the same rows as the whole frame
    part = ds.render(0, seed=21, flags=flags, part=(1, 3))
    runs = multigpu.part_runs(0, c["height"], 1, 3)
    for a, b in runs:
        assert np.array_equal(part[0][a:b].view(np.uint32), one[0][a:b].view(np.uint32)), (a, b)


@pytest.mark.parametrize("name,flags", [("c3_small", 0), ("c5_dragon", rtgpu.RTG_RENDER_TREE)])
def test_sample_passes_accumulate_ranges(name, flags, in_tmp):
    """RTG_RENDER_ACCUM_ONLY over a sample range (how samples split across devices: each device
    writes its range's weighted sum, rtg_resolve_accum adds them): ranges [0, 2) and [2, spp) in
    multi-sample passes equal the same ranges in one-sample passes."""
    torch = pytest.importorskip("torch")
    xml, f0 = _case(name, in_tmp)
    flags |= f0
    hs = rtgpu.HostScene(xml)
    ds = rtgpu.DeviceScene(hs, 0)
    c = hs.camera(0)
    H, W, spp = c["height"], c["width"], c["spp"]

    def acc(b, n, extra):
        a = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0")
        ds.render_device(0, 0, 0, accum_ptr=a.data_ptr(), flags=flags | extra | rtgpu.RTG_RENDER_ACCUM_ONLY,
                         seed=8, sample_begin=b, sample_count=n)
        torch.cuda.synchronize()
        return a.cpu().numpy()

    for b, n in ((0, 2), (2, spp - 2)):
        one, multi = acc(b, n, ONE), acc(b, n, 0)
        assert np.array_equal(one.view(np.uint32), multi.view(np.uint32)), (b, n)


def test_timed_samples_reports_the_last_pass(in_tmp, monkeypatch):
    """rtg_scene_timed_samples: the samples the timed stages covered (bench.py prices the timed
    pass's algorithmic bytes with it)."""
    xml, _ = _case("c3_small", in_tmp)
    hs = rtgpu.HostScene(xml)
    ds = rtgpu.DeviceScene(hs, 0)
    ds.render(0, flags=rtgpu.RTG_RENDER_TIMING)
    ds.timings()
    assert ds.timed_samples() == 4
    ds.render(0, flags=rtgpu.RTG_RENDER_TIMING | ONE)
    assert ds.timed_samples() == 1
    c = hs.camera(0)
    monkeypatch.setenv("RTG_PASS_RAYS", str(c["width"] * c["height"] * 3))   # passes of 2 + 2
    ds.render(0, flags=rtgpu.RTG_RENDER_TIMING)
    assert ds.timed_samples() == 2


@pytest.mark.parametrize("name", ["c5_dragon", "cornell_dielectric", "spheres_mirror"])
def test_tree_passes_on_two_streams(name, in_tmp, monkeypatch):
    """The ray trees' planned passes rotate over several streams with their own level buffers
    (rtg_tree.hip tree_streams), the resolves kept in sample order by events: with two or three
    streams the image of one stream bit for bit -- with multi-sample passes, one-sample passes
    (many planned passes, every stream in use) and a frame part."""
    xml, flags = _case(name, in_tmp)
    hs = rtgpu.HostScene(xml)
    ds = rtgpu.DeviceScene(hs, 0)
    out = {}
    for streams in ("1", "2", "3"):
        monkeypatch.setenv("RTG_TREE_STREAMS", streams)
        for extra in (0, ONE):
            ds.render(0, seed=5, flags=flags | extra)                  # makes the plan
            out[streams, extra] = ds.render(0, seed=5, flags=flags | extra)
        out[streams, "part"] = ds.render(0, seed=5, flags=flags | ONE, part=(1, 2))
    for k in (0, ONE, "part"):
        assert _same(out["1", k], out["2", k]) and _same(out["1", k], out["3", k]), k
