"""Host scene ingest (the reference's parser semantics, parser.cpp) observed through the
flattened description and through renders of the CPU oracle."""
import os

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu
import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")


def render(xml, **kw):
    hs = rtgpu.HostScene(xml)
    hdr, ldr, st = ob.render(hs, **kw)
    return hs, hdr, st


def _scene(tmp_path, text, name="s.xml"):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


BASE = """<Scene>
    <BackgroundColor>1 2 3</BackgroundColor>
    <Cameras>
        <Camera id="1">
            <Position>0 0 0</Position>
            <Gaze>0 0 -1</Gaze>
            <Up>0 1 0</Up>
            <NearPlane>-1 1 -1 1</NearPlane>
            <NearDistance>1</NearDistance>
            <ImageResolution>8 8</ImageResolution>
            <ImageName>a.png</ImageName>
        </Camera>
        CAM2
    </Cameras>
    <Lights>
        <AmbientLight>10 10 10</AmbientLight>
        <PointLight id="1"><Position>0 0 0</Position><Intensity>100 100 100</Intensity></PointLight>
    </Lights>
    <Materials>
        MATS
    </Materials>
    <VertexData>
        -1 -1 -2
        1 -1 -2
        0 1 -2
    </VertexData>
    <Objects>
        <Triangle id="1"><Material>MAT</Material><Indices>1 2 3</Indices></Triangle>
    </Objects>
</Scene>
"""


def make(tmp_path, mats, mat=1, cam2=""):
    return _scene(tmp_path, BASE.replace("MATS", mats).replace("MAT<", f"{mat}<").replace(
        "<Material>MAT</Material>", f"<Material>{mat}</Material>").replace("CAM2", cam2))


def test_background_and_miss(tmp_path):
    m = '<Material id="1"><AmbientReflectance>1 1 1</AmbientReflectance><DiffuseReflectance>0 0 0</DiffuseReflectance><SpecularReflectance>0 0 0</SpecularReflectance></Material>'
    _, hdr, st = render(make(tmp_path, m))
    assert tuple(hdr[0, 0]) == (1.0, 2.0, 3.0)          # corner misses -> BackgroundColor
    assert tuple(hdr[4, 4]) == (10.0, 10.0, 10.0)       # ambient only (no diffuse/specular)


def test_material_object_is_reused(tmp_path):
    """parser.cpp:1115: one Material object for all <Material> elements -- a material
    without <DiffuseReflectance> inherits the previous one's."""
    mats = ('<Material id="1"><AmbientReflectance>0 0 0</AmbientReflectance><DiffuseReflectance>0.5 0.5 0.5</DiffuseReflectance>'
            '<SpecularReflectance>0 0 0</SpecularReflectance></Material>'
            '<Material id="2"><AmbientReflectance>0 0 0</AmbientReflectance></Material>')
    _, a, _ = render(make(tmp_path, mats, 1))
    _, b, _ = render(make(tmp_path, mats, 2))
    assert np.array_equal(a, b) and a[4, 4, 0] > 0


def test_camera_object_is_reused(tmp_path):
    """parser.cpp:1504: a Tonemap on camera 1 carries over to camera 2."""
    cam1_tm = BASE.replace("<ImageName>a.png</ImageName>",
                           "<ImageName>a.png</ImageName><Tonemap><TMO>Photographic</TMO></Tonemap>")
    cam2 = ('<Camera id="2"><Position>0 0 0</Position><Gaze>0 0 -1</Gaze><Up>0 1 0</Up>'
            '<NearPlane>-1 1 -1 1</NearPlane><NearDistance>1</NearDistance><ImageResolution>4 4</ImageResolution>'
            '<ImageName>b.png</ImageName><NumSamples>4</NumSamples></Camera>')
    m = '<Material id="1"><AmbientReflectance>1 1 1</AmbientReflectance></Material>'
    p = _scene(tmp_path, cam1_tm.replace("MATS", m).replace("<Material>MAT</Material>", "<Material>1</Material>").replace("CAM2", cam2))
    hs = rtgpu.HostScene(p)
    assert hs.num_cameras() == 2
    assert hs.camera(0)["tonemapped"] and hs.camera(1)["tonemapped"]
    assert hs.camera(1)["spp"] == 4 and hs.camera(1)["width"] == 4


def test_stream_leftovers_carry_over(tmp_path):
    """parser.cpp shares one stringstream: an extra token in <BackgroundColor> is read as
    the ShadowRayEpsilon (here 5 -> the shadow origin moves 5 units along the normal)."""
    m = '<Material id="1"><AmbientReflectance>0 0 0</AmbientReflectance><DiffuseReflectance>1 1 1</DiffuseReflectance><SpecularReflectance>0 0 0</SpecularReflectance></Material>'
    good = make(tmp_path, m)
    s = open(good).read().replace("<BackgroundColor>1 2 3</BackgroundColor>",
                                  "<BackgroundColor>1 2 3 5</BackgroundColor><ShadowRayEpsilon>0.001</ShadowRayEpsilon>")
    bad = _scene(tmp_path, s, "leftover.xml")
    _, a, _ = render(good)
    _, b, _ = render(bad)
    assert not np.array_equal(a, b)


def test_missing_ply_and_empty_texcoords_fail(tmp_path):
    s = open(os.path.join(SCENES, "ply_quads.xml")).read().replace("quads.ply", "nope.ply")
    with pytest.raises(rtgpu.RTGError) as e:
        rtgpu.HostScene(_scene(tmp_path, s))
    assert e.value.code == -2
    s2 = BASE.replace("MATS", '<Material id="1"></Material>').replace("<Material>MAT</Material>", "<Material>1</Material>")
    s2 = s2.replace("CAM2", "").replace("<Objects>", "<TexCoordData />\n    <Objects>")
    with pytest.raises(rtgpu.RTGError):
        rtgpu.HostScene(_scene(tmp_path, s2, "tc.xml"))


def test_unsupported_rotation_axis(tmp_path, monkeypatch):
    monkeypatch.chdir(SCENES)     # image paths resolve as inputs/<name> from the cwd
    s = open(os.path.join(SCENES, "transforms_textures.xml")).read().replace(
        '<Rotation id="1">30 0 1 0</Rotation>', '<Rotation id="1">30 0.7 0.7 0</Rotation>')
    with pytest.raises(rtgpu.RTGError) as e:
        rtgpu.HostScene(_scene(tmp_path, s))
    assert e.value.code == -6


def test_synthetic_scene_counts(tmp_path):
    xml = scenes.synthetic_heightfield(str(tmp_path), K=2000, width=64, height=36)
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        hs = rtgpu.HostScene(xml)
        c = hs.counts()
        assert c["objects"] == 1 and c["faces"] == 2 * 32 * 32 and c["lights"] == 1
        _, _, st = ob.render(hs)
        assert st["camera_rays"] == 64 * 36 and st["shadow_rays"] == 64 * 36   # every camera ray hits
    finally:
        os.chdir(old)


def test_comments_entities_and_whitespace(tmp_path):
    m = '<Material id="1"><AmbientReflectance>1 1 1</AmbientReflectance></Material>'
    s = make(tmp_path, m)
    t = open(s).read()
    t = t.replace("<Gaze>0 0 -1</Gaze>", "<Gaze>\n   0 0 -1   </Gaze><!-- comment -->")
    t = t.replace("<ImageName>a.png</ImageName>", "<ImageName> a&amp;b.png </ImageName>")
    _, a, _ = render(s)
    _, b, _ = render(_scene(tmp_path, t, "ws.xml"))
    assert np.array_equal(a, b)


def test_sphere_normal_map_is_rejected(tmp_path, monkeypatch):
    """A sphere normal map leaves the hit normal unset in the reference (sphere.cpp:95-113):
    the device scene refuses it instead of inventing a normal (checked before any GPU call)."""
    monkeypatch.chdir(SCENES)
    s = open(os.path.join(SCENES, "bump_normal.xml")).read().replace(
        "<Textures>4</Textures>", "<Textures>1</Textures>")
    hs = rtgpu.HostScene(_scene(tmp_path, s))
    with pytest.raises(rtgpu.RTGError) as e:
        rtgpu.DeviceScene(hs, 0)
    assert e.value.code == -6


def test_instances_take_base_mesh_bump_map(tmp_path, monkeypatch):
    """IntersectFace reads the BASE mesh's bump map for an instance (mesh.cpp:263-358 with
    `this` = baseMesh): dropping the instance's own (ignored) texture list changes nothing,
    dropping the base mesh's bump map changes the instance's pixels."""
    monkeypatch.chdir(SCENES)
    s = open(os.path.join(SCENES, "bump_normal.xml")).read()
    _, ref, _ = render("bump_normal.xml")
    inst = s.replace('<MeshInstance id="10" baseMeshId="2">\n            <Material>1</Material>',
                     '<MeshInstance id="10" baseMeshId="2">\n            <Material>1</Material>\n'
                     '            <Textures>3</Textures>')
    _, a, _ = render(_scene(tmp_path, inst, "a.xml"))
    assert np.array_equal(a.view(np.uint32), ref.view(np.uint32))
    nob = s.replace("<Textures>2</Textures>", "")
    _, b, _ = render(_scene(tmp_path, nob, "b.xml"))
    assert (np.abs(b - ref).max(-1) > 1e-3).mean() > 0.01


def test_recursion_deeper_than_the_frame_stack_is_rejected(tmp_path, monkeypatch):
    """MaxRecursionDepth beyond the kernels' 32-frame ray-tree stack is refused with
    RTG_ERR_UNSUPPORTED (before any device work), never silently truncated."""
    monkeypatch.chdir(SCENES)
    s = open(os.path.join(SCENES, "spheres_mirror.xml")).read()
    import re
    s = re.sub(r"<MaxRecursionDepth>[^<]*</MaxRecursionDepth>", "<MaxRecursionDepth>40</MaxRecursionDepth>", s)
    hs = rtgpu.HostScene(_scene(tmp_path, s))
    with pytest.raises(rtgpu.RTGError) as e:
        rtgpu.DeviceScene(hs, 0)
    assert e.value.code == -6


def test_device_bvh_load_flag(tmp_path, monkeypatch):
    """RTG_LOAD_DEVICE_BVH: same faces, parse order, no nodes; the oracle refuses such a
    description (it has no BVH to walk) and so does a GPU-less rtg_scene_create."""
    monkeypatch.chdir(SCENES)
    a = rtgpu.HostScene("c5_dragon.xml")
    b = rtgpu.HostScene("c5_dragon.xml", device_bvh=True)
    ca, cb = a.counts(), b.counts()
    assert cb["nodes"] == 0 and ca["nodes"] > 0 and ca["faces"] == cb["faces"]
    with pytest.raises(RuntimeError):
        ob.render(b)
    if rtgpu.device_count() == 0:
        with pytest.raises(rtgpu.RTGError) as e:
            rtgpu.DeviceScene(b, 0)
        assert e.value.code == -4
