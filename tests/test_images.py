"""Image decoders of the host loader against the reference's own image classes.

Fixtures (tests/golden/make_images.py): small PNGs written by that script's own encoder (grey at
1/2/4/8/16 bits, grey + alpha, RGB 8/16, RGBA, palette with and without tRNS; every row filter
type, split IDAT) and OpenEXR files from its own writer (HALF / FLOAT, NONE / RLE / ZIPS / ZIP,
increasing / decreasing line order, one channel, extra channels, half specials).  Goldens: the
texels LDRImage (stbi_load, LDRImage.h:37-44) and HDRImage (tinyexr LoadEXR, HDRImage.h:45-72)
read from them, dumped by `oracle/_ref/refdriver imgdump` (the reference compiled here).  The
loader must reproduce them bit for bit, seen through the scene description a parsed <Images>
entry produces.  JPEG is outside the loader (a parity gap): refused with
RTG_ERR_UNSUPPORTED."""
import ctypes
import os
import shutil

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu

IMAGES = os.path.join(ob.GOLDEN, "images")
GOLD = np.load(os.path.join(IMAGES, "decoded.npz"))
PNG = sorted(f for f in os.listdir(IMAGES) if f.endswith((".png", ".exr")))

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


@pytest.mark.parametrize("name", PNG)
def test_decoder_matches_reference(tmp_path, name):
    base = os.path.splitext(name)[0]
    hs = _load(tmp_path, name)
    info, tex = _texels(hs)
    assert list(info) == list(GOLD[base + "_info"]), (info, GOLD[base + "_info"])
    gold = GOLD[base]
    same = tex.view(np.uint32) == gold.view(np.uint32)
    assert same.all(), (name, int((~same).sum()), np.argwhere(~same)[:5])


@pytest.mark.parametrize("name,data", [("a.jpg", b"\xff\xd8\xff\xe0" + bytes(64)),
                                       ("b.exr", b"\x76\x2f\x31\x01" + b"\x02\x02\x00\x00" + bytes(64))])
def test_jpeg_and_tiled_exr_refused(tmp_path, name, data):
    os.makedirs(tmp_path / "inputs", exist_ok=True)
    (tmp_path / "inputs" / name).write_bytes(data)
    (tmp_path / "s.xml").write_text(SCENE.replace("IMG", name))
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        with pytest.raises(rtgpu.RTGError) as e:
            rtgpu.HostScene(str(tmp_path / "s.xml"))
    finally:
        os.chdir(old)
    assert e.value.code == -6, e.value


def _exr(attrs, offsets, tail=b""):
    """A scanline OpenEXR file from raw (name, type, value bytes, declared size) attributes."""
    import struct
    b = b"\x76\x2f\x31\x01" + b"\x02\x00\x00\x00"
    for name, typ, val, sz in attrs:
        b += name + b"\0" + typ + b"\0" + struct.pack("<I", len(val) if sz is None else sz) + val
    b += b"\0"
    start = len(b) + 8 * len(offsets)          # None: the chunk right after the offset table
    b += b"".join(struct.pack("<Q", start if o is None else o) for o in offsets)
    return b + tail


def _chans():
    import struct
    return b"".join(c + b"\0" + struct.pack("<iBBBBii", 2, 0, 0, 0, 0, 1, 1) for c in (b"B", b"G", b"R")) + b"\0"


def _malformed_exrs():
    import struct
    dw = struct.pack("<4i", 0, 0, 1, 0)           # 2 x 1 pixels
    ch = (b"channels", b"chlist", _chans(), None)
    good_chunk = struct.pack("<iI", 0, 24) + bytes(24)
    return {
        # a chunk offset near 2^64: off + 8 wraps to a small value
        "huge_offset": _exr([ch, (b"compression", b"compression", b"\0", None),
                             (b"dataWindow", b"box2i", dw, None), (b"lineOrder", b"lineOrder", b"\0", None)],
                            [2 ** 64 - 4], good_chunk),
        # a chunk length that runs past the file
        "long_chunk": _exr([ch, (b"compression", b"compression", b"\0", None),
                            (b"dataWindow", b"box2i", dw, None)], [None], struct.pack("<iI", 0, 2 ** 32 - 1)),
        # attributes declared shorter than the values read from them
        "short_datawindow": _exr([ch, (b"compression", b"compression", b"", 0), (b"dataWindow", b"box2i", b"", 4)],
                                 [0], bytes(32)),
        "short_compression": _exr([ch, (b"compression", b"compression", b"", 0)], [0], bytes(32)),
        # a data window whose size overflows 32 bits
        "huge_window": _exr([ch, (b"compression", b"compression", b"\0", None),
                             (b"dataWindow", b"box2i", struct.pack("<4i", -2 ** 31, 0, 2 ** 31 - 1, 0), None)],
                            [0], bytes(32)),
    }


@pytest.mark.parametrize("case", sorted(_malformed_exrs()))
def test_malformed_exr_refused(tmp_path, case):
    """Crafted EXR headers and offset tables are refused with an error, never read out of bounds
    (host_assets.cpp load_exr: offsets checked by subtraction, attribute sizes checked)."""
    os.makedirs(tmp_path / "inputs", exist_ok=True)
    (tmp_path / "inputs" / "m.exr").write_bytes(_malformed_exrs()[case])
    (tmp_path / "s.xml").write_text(SCENE.replace("IMG", "m.exr"))
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        with pytest.raises(rtgpu.RTGError) as e:
            rtgpu.HostScene(str(tmp_path / "s.xml"))
    finally:
        os.chdir(old)
    assert e.value.code == -2, e.value      # RTG_ERR_IO, as every unreadable image


def test_png_fixture_semantics():
    """The goldens carry stb's conventions: 16-bit samples keep the high byte, sub-byte grey
    is scaled to 0..255, a palette with tRNS expands to RGBA."""
    g16 = GOLD["png_grey16"]
    assert g16.max() <= 255 and g16.dtype == np.float32
    g1 = GOLD["png_grey1"]
    assert set(np.unique(g1)) <= {0.0, 255.0}
    assert GOLD["png_pal4_trns_info"][2] == 4
