"""BASELINE.json configurations C2-C5 at their full sizes on the GPU.

The reduced versions of C2, C3 and C5 are reference goldens (tests/golden, checked by
test_gpu_parity.py).  Here each configuration is rendered at full size on the GPU and
checked against the CPU restatement on the same seeded RNG keys -- whole image where the
oracle finishes in seconds, a band of rows otherwise -- plus the size-independent
property the configuration offers (C5: deterministic, so 64 spp == 1 spp to rounding).
C4 (MeshInstance forest) has no reference golden: the reference crashes on it (see
tests/golden/make_goldens.py), so it is pinned only through the restatement.
"""
import os

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu
import scenes

pytestmark = pytest.mark.gpu

REL = 1e-4
SCENES = os.path.join(ob.GOLDEN, "scenes")


@pytest.fixture()
def in_tmp(tmp_path):
    old = os.getcwd()
    os.chdir(tmp_path)
    yield str(tmp_path)
    os.chdir(old)


def _scene(xml):
    hs = rtgpu.HostScene(xml)
    return hs, rtgpu.DeviceScene(hs, 0)


def test_c2_cornell_800(in_tmp):
    xml = scenes.config_c2(in_tmp, os.path.join(SCENES, "cornell_conductors.xml"))
    hs, ds = _scene(xml)
    assert hs.camera(0)["width"] == 800
    hdr, ldr = ds.render(0)
    ohdr, _, _ = ob.render(hs)
    r = ob.compare(hdr, ohdr, REL)
    print(r)
    assert r["rel_pass"] == 1.0, r
    assert np.array_equal(ldr, ob.clamp_ldr(hdr))


def test_c3_blob_1080p_4spp(in_tmp):
    """Whole image (8.3 M camera rays + area-light shadow rays) against the restatement."""
    xml = scenes.config_c3(in_tmp)
    hs, ds = _scene(xml)
    c = hs.camera(0)
    assert (c["width"], c["height"], c["spp"]) == (1920, 1080, 4) and hs.counts()["faces"] > 69000
    hdr, _ = ds.render(0, seed=11)
    ohdr, _, _ = ob.render(hs, seed=11)
    r = ob.compare(hdr, ohdr, REL)
    print(r)
    assert r["n_fail"] == 0, r


def test_c3_ton_roosendaal_1080p_4spp(in_tmp):
    """C3 on the reference's own 62k-triangle ton_Roosendaal mesh, whole image."""
    xml = scenes.config_c3_ton(in_tmp, os.path.join(SCENES, "ton_Roosendaal_smooth_ply"))
    hs, ds = _scene(xml)
    c = hs.camera(0)
    assert (c["width"], c["height"], c["spp"]) == (1920, 1080, 4) and hs.counts()["faces"] > 62000
    hdr, _ = ds.render(0, seed=13)
    ohdr, _, _ = ob.render(hs, seed=13)
    r = ob.compare(hdr, ohdr, REL)
    print(r)
    assert r["n_fail"] == 0, r


# C4's pixels outside the bound, all eight bands (round 4, seed 5): 5 pixels (10 values)
C4_FAIL_CAP = 5


def test_c4_forest_1080p_16spp(in_tmp):
    """Eight 16-row bands against the oracle.  The only pixels outside the 1e-4 bound are
    explained one by one: the spherical environment light's lookup (sphericalEnvironmentLight.h:
    22-34) truncates width * u and height * v to a texel, u and v coming from atan2f / acosf, so
    a last-ulp different device result at a coordinate within ulps of a texel boundary picks the
    neighbouring texel.  Each failing pixel must be reproduced by the oracle with some of its
    lookups that lie within 2e-3 texel of a boundary flipped (ob.explain_env_flips), and their
    number may not exceed this round's count."""
    xml = scenes.config_c4(in_tmp)
    hs, ds = _scene(xml)
    c = hs.camera(0)
    assert (c["width"], c["height"], c["spp"]) == (1920, 1080, 16) and hs.counts()["objects"] == 102
    hdr, _ = ds.render(0, seed=5)
    # eight 16-row bands spread over the frame (128 rows x 1920 x 16 spp = 3.9 M camera rays)
    total = 0
    for r0 in (48, 176, 304, 432, 560, 688, 816, 944):
        rows = (r0, r0 + 16)
        ohdr, _, _ = ob.render(hs, rows=rows, seed=5)
        r = ob.compare(hdr[rows[0]:rows[1]], ohdr[rows[0]:rows[1]], REL)
        nbad, unexplained = ob.explain_env_flips(hs, hdr[rows[0]:rows[1]], ohdr[rows[0]:rows[1]], rows, seed=5)
        print(rows, r, "failing pixels", nbad, "unexplained", unexplained)
        assert not unexplained, (rows, unexplained)
        total += nbad
    assert total <= C4_FAIL_CAP, total


def test_c5_dragon_4k_64spp(in_tmp):
    torch = pytest.importorskip("torch")
    xml = scenes.config_c5(in_tmp)
    hs, ds = _scene(xml)
    c = hs.camera(0)
    W, H = c["width"], c["height"]
    assert (W, H, c["spp"]) == (3840, 2160, 64) and hs.counts()["faces"] > 860000
    hdr64, _ = ds.render(0)
    # one sample pass, device accumulation buffer
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0")
    ds.render_device(0, 0, 0, accum_ptr=acc.data_ptr(), flags=rtgpu.RTG_RENDER_ACCUM_ONLY, sample_begin=0,
                     sample_count=1)
    torch.cuda.synchronize()
    a = acc.cpu().numpy()
    hdr1 = a[..., :3] / a[..., 3:4]
    # deterministic scene, jitter discarded (main.cpp:83): every sample traces the pixel centre
    r = ob.compare(hdr64, hdr1, 1e-5)
    print("64 vs 1 spp", r)
    assert r["rel_pass"] == 1.0, r
    # eight 16-row bands spread over the frame (sky, Perlin ground, mirror sphere and the
    # dielectric mesh's reflect / refract trees), 491 k pixel trees against the restatement
    for r0 in (160, 400, 640, 880, 1120, 1360, 1600, 1840):
        rows = (r0, r0 + 16)
        oacc, _ = ob.render(hs, rows=rows, sample_begin=0, sample_count=1, accum=True)
        r = ob.compare(a[rows[0]:rows[1]], oacc[rows[0]:rows[1]], REL)
        print("vs oracle", rows, r)
        assert r["rel_pass"] == 1.0, (rows, r)


@pytest.mark.parametrize("cfg", ["c3", "c4"])
def test_large_leaf_cooperative_walk_small(cfg, in_tmp):
    """Meshes whose midpoint BVH keeps leaves of hundreds of faces take the wave-cooperative
    leaf test; with instances the walk runs under partial exec masks.  Whole image vs the
    oracle, and the wavefront pipeline == the fused kernel bit for bit."""
    if cfg == "c3":
        xml = scenes.config_c3(in_tmp, K=20000, width=320, height=180, spp=1)
    else:
        xml = scenes.config_c4(in_tmp, n_side=3, K_tree=4000, width=320, height=180, spp=1)
    hs, ds = _scene(xml)
    hdr, _ = ds.render(0, seed=3)
    ohdr, _, _ = ob.render(hs, seed=3)
    r = ob.compare(hdr, ohdr, REL)
    print(r)
    assert r["n_fail"] == 0, r
    xml0 = scenes.with_depth(xml, os.path.join(in_tmp, "d0.xml"), 0)
    hs0, ds0 = _scene(xml0)
    a, _ = ds0.render(0, seed=3)
    b, _ = ds0.render(0, seed=3, flags=rtgpu.RTG_RENDER_FUSED)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("name", ["c3_small", "c4_small", "c3_blob", "berserker", "windmill", "tower", "car_smooth"])
def test_deferred_large_leaves(name, in_tmp, monkeypatch):
    """Large-leaf scenes: the camera walk defers its large leaves to k_bigleaf and settles each
    pixel in k_hitfix (the winner's leaf box checked at next_up(t), rtg_common.hpp DeferCtx), the
    shadow walk queues its large leaves to k_bigleaf_any (AnyDefer) -- bit for bit the image of the cooperative
    reference walk (RTG_DEFER=0), of camera deferral alone (RTG_DEFER_ANY=0) and of the counting
    render (which never defers)."""
    if name == "c3_small":
        xml = scenes.config_c3(in_tmp, K=20000, width=320, height=180, spp=1)
    elif name == "c4_small":
        xml = scenes.config_c4(in_tmp, n_side=3, K_tree=4000, width=320, height=180, spp=2)
    else:
        xml = os.path.join(SCENES, name + ".xml")
        os.chdir(SCENES)
    hs, ds = _scene(xml)
    xml0 = scenes.with_depth(xml, os.path.join(in_tmp, "d0.xml"), 0)   # wavefront pipeline (no ray trees)
    hs0, ds0 = _scene(xml0)
    a, la = ds0.render(0, seed=9)
    c, lc = ds0.render(0, seed=9, flags=rtgpu.RTG_RENDER_COUNT_STATS)
    monkeypatch.setenv("RTG_DEFER_ANY", "0")   # shadow rays: the cooperative walk
    d, ld = ds0.render(0, seed=9)
    monkeypatch.setenv("RTG_DEFER", "0")
    b, lb = ds0.render(0, seed=9)
    n = int((a.view(np.uint32) != b.view(np.uint32)).any(axis=2).sum())
    m = int((a.view(np.uint32) != d.view(np.uint32)).any(axis=2).sum())
    print(name, "differing pixels", n, "(shadow deferral alone:", m, ")")
    assert n == 0 and m == 0 and np.array_equal(la, lb) and np.array_equal(la, ld)
    assert np.array_equal(a.view(np.uint32), c.view(np.uint32))


@pytest.mark.parametrize("case,pad_objects,pad_faces,deferred", [
    ("objects_under", 4093, 0, True),          # 4 095 objects, the blob is object 4 094
    ("objects_over", 4095, 0, False),          # 4 097 objects, the blob is object 4 096 (13 bits)
    ("faces_under", 0, 2 ** 20 - 19802 - 1000, True),
    ("faces_over", 0, 2 ** 20, False),         # the blob's face records start past 2^20
])
def test_deferral_gate(case, pad_objects, pad_faces, deferred, in_tmp, monkeypatch):
    """The deferred-leaf key packs (t, object, face) into 32 + 12 + 20 bits (rtg_common.hpp
    obj_key), so the camera walk defers only scenes of fewer than 4 096 objects and 2^20 faces
    (rtg_wave.hpp launch_wave_t).  Padding meshes before the large-leaf blob put its object index
    and face records on either side of those limits: below them the deferring walk runs (pending
    pixels counted with RTG_DEFER_DIAG=1), above them it must not (a key would alias), and either
    way the image is bit for bit the cooperative walk's (RTG_DEFER=0) and the oracle's."""
    xml = scenes.config_defer_gate(in_tmp, pad_objects=pad_objects, pad_faces=pad_faces)
    hs, ds = _scene(xml)
    n = hs.counts()
    assert (n["objects"] > 4096) == (pad_objects > 4094) and (n["faces"] >= 2 ** 20) == (pad_faces >= 2 ** 20)
    monkeypatch.setenv("RTG_DEFER_DIAG", "1")
    ds.reset_stats()
    a, la = ds.render(0, seed=4)
    pending = ds.stats()["extend_wide_visits"]
    monkeypatch.delenv("RTG_DEFER_DIAG")
    print(case, n, "pending pixels", pending)
    assert (pending > 0) == deferred, pending
    monkeypatch.setenv("RTG_DEFER", "0")
    b, lb = ds.render(0, seed=4)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(la, lb)
    ohdr, _, _ = ob.render(hs, seed=4)
    r = ob.compare(a, ohdr, REL)
    print(r)
    assert r["n_fail"] == 0, r


def test_defer_buffer_grows_with_the_part(in_tmp):
    """The deferred-leaf buffer's layout (keys, entries, states) depends on the pixel count it
    was sized for: after a counted full frame (large wave buffers) and a one-row render (a small
    queue), a larger row range under the 1 024-entry floor must not reuse it (rtg_api.cpp
    ensure_defer).  Each row range equals the same rows of a whole-frame render."""
    xml = scenes.config_defer_gate(in_tmp, width=160, height=90)
    hs, ds = _scene(xml)
    full, _ = ds.render(0, seed=6)
    ds.render(0, seed=6, flags=rtgpu.RTG_RENDER_COUNT_STATS)
    for rows in ((40, 41), (40, 43), (38, 44)):       # 160, 480, 960 pixels
        h, _ = ds.render(0, seed=6, rows=rows)
        assert np.array_equal(h[rows[0]:rows[1]].view(np.uint32), full[rows[0]:rows[1]].view(np.uint32)), rows
