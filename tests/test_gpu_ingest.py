"""Device scene ingest: the reference's midpoint BVH (mesh.cpp:23-156)
and face order built on the GPU (rtg_bvh.hip) from a description loaded with
RTG_LOAD_DEVICE_BVH must equal the host build bit for bit -- the walk's node records, the
face records in BVH order, and therefore every rendered pixel and traversal counter."""
import os
import time

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu

pytestmark = pytest.mark.gpu

SCENES = os.path.join(ob.GOLDEN, "scenes")
NAMES = ["simple", "spheres_mirror", "cornell_dielectric", "scienceTree", "scienceTree_diamond", "berserker",
         "transforms_textures", "ply_quads", "synth_10k", "c2_cornell", "c3_blob", "c5_dragon", "bump_normal",
         "mesh_light", "pt_cornell"]


@pytest.fixture(autouse=True)
def _cwd():
    old = os.getcwd()
    os.chdir(SCENES)
    yield
    os.chdir(old)


def _pair(xml):
    host = rtgpu.HostScene(xml)
    dev = rtgpu.HostScene(xml, device_bvh=True)
    assert dev.counts()["nodes"] == 0 and dev.counts()["faces"] == host.counts()["faces"]
    return host, dev, rtgpu.DeviceScene(host, 0), rtgpu.DeviceScene(dev, 0)


def _same_bvh(a, b):
    na, ta = a.export_bvh()
    nb, tb = b.export_bvh()
    assert na.shape == nb.shape and ta.shape == tb.shape, (na.shape, nb.shape, ta.shape, tb.shape)
    assert np.array_equal(na.view(np.uint32), nb.view(np.uint32))
    assert np.array_equal(ta.view(np.uint32), tb.view(np.uint32))
    return na.shape[0], ta.shape[0]


@pytest.mark.parametrize("name", NAMES)
def test_device_bvh_equals_host_bvh(name):
    hs, hd, ds_h, ds_d = _pair(name + ".xml")
    nn, nf = _same_bvh(ds_h, ds_d)
    ds_h.reset_stats()
    ds_d.reset_stats()
    a, _ = ds_h.render(0, flags=rtgpu.RTG_RENDER_COUNT_STATS, seed=7)
    b, _ = ds_d.render(0, flags=rtgpu.RTG_RENDER_COUNT_STATS, seed=7)
    print(name, nn, "nodes", nf, "faces")
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert ds_h.stats() == ds_d.stats()


@pytest.mark.parametrize("K", [100352, 869558])
def test_device_bvh_full_size(tmp_path, K):
    """The headline height field and a C5-size (870k-triangle) mesh."""
    import scenes
    if K == 100352:
        xml = scenes.synthetic_heightfield(str(tmp_path), K=K, width=1920, height=1080)
    else:
        xml = scenes.config_c5(str(tmp_path), width=384, height=216, spp=1)
    os.chdir(tmp_path)
    t0 = time.perf_counter()
    host = rtgpu.HostScene(xml)
    t1 = time.perf_counter()
    dev = rtgpu.HostScene(xml, device_bvh=True)
    t2 = time.perf_counter()
    ds_h = rtgpu.DeviceScene(host, 0)
    t3 = time.perf_counter()
    ds_d = rtgpu.DeviceScene(dev, 0)
    t4 = time.perf_counter()
    print(f"K={K}: host load+bvh {t1 - t0:.3f}s + create {t3 - t2:.3f}s | load {t2 - t1:.3f}s + device bvh/create "
          f"{t4 - t3:.3f}s")
    nn, nf = _same_bvh(ds_h, ds_d)
    assert nf >= K * 0.99


@pytest.mark.parametrize("extra", [[], ["--host-bvh"]])
def test_cli_drop_in(tmp_path, extra):
    """The drop-in CLI (`rtgpu scene.xml`, main.cpp:132-202): same PNG as the library render,
    with the BVH built on the GPU (default) or on the host."""
    import re
    import shutil
    import subprocess
    from PIL import Image
    exe = os.path.join(os.path.dirname(rtgpu.LIB_PATH), "rtgpu")
    src = open(os.path.join(SCENES, "cornell_dielectric.xml")).read()
    m = re.search(r"<ImageName>([^<]*)</ImageName>", src)
    (tmp_path / "s.xml").write_text(src)
    r = subprocess.run([exe, "s.xml"] + extra, cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Rendering took" in r.stdout
    png = tmp_path / (os.path.splitext(m.group(1))[0] + ".png")
    got = np.asarray(Image.open(png).convert("RGB"))
    hs = rtgpu.HostScene(str(tmp_path / "s.xml"))
    _, ldr = rtgpu.DeviceScene(hs, 0).render(0)
    assert np.array_equal(got, ldr)
    shutil.rmtree(tmp_path, ignore_errors=True)
