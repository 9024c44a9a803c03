"""Image decoders of the host loader against the reference's own image classes.

Fixtures (tests/golden/make_images.py): small OpenEXR files written by that script's own EXR
writer (NONE / RLE / ZIPS / ZIP, HALF / FLOAT, RGB / RGBA / one channel / extra channels, a
decreasing line order, incompressible chunks stored raw) and JPEGs written by PIL (4:4:4, 4:2:2,
4:2:0, greyscale, restart markers, progressive).  Goldens: the texels HDRImage (tinyexr
LoadEXR, HDRImage.h:45-72) and LDRImage (stbi_load, LDRImage.h:37-44) read from them, dumped by
`oracle/_ref/refdriver imgdump` (the reference compiled here).  The loader must reproduce them
bit for bit, seen through the scene description a parsed <Images> entry produces."""
import ctypes
import os
import shutil

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu

IMAGES = os.path.join(ob.GOLDEN, "images")
GOLD = np.load(os.path.join(IMAGES, "decoded.npz"))
EXR = sorted(f for f in os.listdir(IMAGES) if f.endswith(".exr"))
JPG = sorted(f for f in os.listdir(IMAGES) if f.endswith(".jpg"))

SCENE = """<Scene>
    <Cameras><Camera id="1"><Position>0 0 0</Position><Gaze>0 0 -1</Gaze><Up>0 1 0</Up>
        <NearPlane>-1 1 -1 1</NearPlane><NearDistance>1</NearDistance>
        <ImageResolution>4 4</ImageResolution><ImageName>a.png</ImageName></Camera></Cameras>
    <Lights><AmbientLight>10 10 10</AmbientLight></Lights>
    <Materials><Material id="1"><DiffuseReflectance>1 1 1</DiffuseReflectance></Material></Materials>
    <Textures><Images><Image id="1">IMG</Image></Images></Textures>
    <VertexData>-1 -1 -2 1 -1 -2 0 1 -2</VertexData>
    <Objects><Triangle id="1"><Material>1</Material><Indices>1 2 3</Indices></Triangle></Objects>
</Scene>
"""


def _load(tmp_path, name):
    os.makedirs(tmp_path / "inputs", exist_ok=True)
    shutil.copy(os.path.join(IMAGES, name), tmp_path / "inputs" / name)
    (tmp_path / "s.xml").write_text(SCENE.replace("IMG", name))
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        return rtgpu.HostScene(str(tmp_path / "s.xml"))
    finally:
        os.chdir(old)


def _texels(hs):
    L = ob.lib()
    L.oracle_image.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    info = np.zeros(4, np.int32)
    assert L.oracle_image(hs.desc, 0, info.ctypes.data, None) == 0
    w, h, c, hdr = (int(x) for x in info)
    out = np.zeros((h, w, c), np.float32)
    L.oracle_image(hs.desc, 0, info.ctypes.data, out.ctypes.data)
    return info, out


@pytest.mark.parametrize("name", EXR + JPG)
def test_decoder_matches_reference(tmp_path, name):
    base = os.path.splitext(name)[0]
    hs = _load(tmp_path, name)
    info, tex = _texels(hs)
    assert list(info) == list(GOLD[base + "_info"]), (info, GOLD[base + "_info"])
    gold = GOLD[base]
    same = tex.view(np.uint32) == gold.view(np.uint32)
    assert same.all(), (name, int((~same).sum()), np.argwhere(~same)[:5])


def test_exr_fixture_semantics():
    """The goldens themselves carry LoadEXR's conventions: one channel -> grey, a decreasing
    line order comes out flipped, half specials widen exactly."""
    g = GOLD["exr_y_float_zip"]
    assert np.array_equal(g[..., 0], g[..., 1]) and np.array_equal(g[..., 1], g[..., 2])
    hz = GOLD["exr_half_zips"]
    assert hz[0, 0, 0] == np.float32(np.float16(6.0e-8)) and np.isinf(hz[0, 5, 0])
    assert np.signbit(hz[0, 3, 0]) and hz[0, 4, 0] == 65504.0
