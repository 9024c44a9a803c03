"""The C-ABI boundary: library loads, exports every function include/rtgpu.h declares,
reports errors through return codes + rtg_last_error (no exceptions, no crashes), and
refuses to run without a GPU instead of falling back to the CPU."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import rtgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtgpu.h")
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rtg_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_what_binding_uses():
    assert set(rtgpu.EXPORTED) == set(declared_functions())


def test_library_exports_every_declared_symbol():
    L = rtgpu.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", rtgpu.LIB_PATH], capture_output=True, text=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [n for n in declared_functions() if n not in syms]
    assert not missing, missing


def test_abi_version():
    assert rtgpu.lib().rtg_abi_version() == 6


def test_struct_layouts_are_plain_c(tmp_path):
    # the opts/stats structs Python mirrors must match the header's sizes (checked against a
    # C compiler's view of include/rtgpu.h)
    import shutil
    assert ctypes.sizeof(rtgpu.RenderOpts) == 40
    assert ctypes.sizeof(rtgpu.Stats) == 104
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    src = tmp_path / "sz.c"
    src.write_text('#include "rtgpu.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(void){printf("%zu %zu %zu %zu %zu %zu %zu\\n", '
                   'sizeof(rtg_render_opts), sizeof(rtg_stats), offsetof(rtg_render_opts, part_index), '
                   'sizeof(rtg_camera), offsetof(rtg_camera, tm_gamma), offsetof(rtg_scene_desc, cameras), '
                   'offsetof(rtg_scene_desc, num_cameras));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    opts, stats, part, cam, gamma, cams, ncams = map(
        int, subprocess.run([str(exe)], capture_output=True, text=True).stdout.split())
    assert (opts, stats) == (ctypes.sizeof(rtgpu.RenderOpts), ctypes.sizeof(rtgpu.Stats))
    assert part == rtgpu.RenderOpts.part_index.offset
    # the camera / description heads HostScene.tonemap_params reads
    assert cam == rtgpu.RTG_CAMERA_SIZE and gamma == rtgpu._Camera.tm_gamma.offset
    assert (cams, ncams) == (rtgpu._DescHead.cameras.offset, rtgpu._DescHead.num_cameras.offset)


def test_errors_are_codes_not_crashes(tmp_path):
    L = rtgpu.lib()
    h = ctypes.c_void_p()
    assert L.rtg_host_scene_load_xml(None, ctypes.byref(h)) == -1
    assert b"null" in L.rtg_last_error()
    with pytest.raises(rtgpu.RTGError) as e:
        rtgpu.HostScene(str(tmp_path / "missing.xml"))
    assert e.value.code == -2
    bad = tmp_path / "bad.xml"
    bad.write_text("<Scene><Cameras></Scene>")
    with pytest.raises(rtgpu.RTGError) as e:
        rtgpu.HostScene(str(bad))
    assert e.value.code == -3
    assert L.rtg_render(None, None, None, None) == -1
    assert L.rtg_desc_camera_info(None, 0, None, None, None, None) == -1


@pytest.mark.skipif(rtgpu.device_count() > 0, reason="checks the no-GPU path")
def test_no_gpu_is_an_error_not_a_fallback():
    hs = rtgpu.HostScene(os.path.join(SCENES, "simple.xml"))
    with pytest.raises(rtgpu.RTGError) as e:
        rtgpu.DeviceScene(hs, 0)
    assert e.value.code == -4


def test_png_writer_roundtrip(tmp_path):
    import struct
    import zlib
    img = (np.arange(7 * 5 * 3) % 256).astype(np.uint8).reshape(5, 7, 3)
    p = tmp_path / "x.png"
    rtgpu.write_png(str(p), img)
    data = p.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        typ = data[pos + 4:pos + 8]
        if typ == b"IHDR":
            w, h = struct.unpack(">II", data[pos + 8:pos + 16])
            assert (w, h) == (7, 5)
        if typ == b"IDAT":
            idat += data[pos + 8:pos + 8 + n]
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(5, 1 + 7 * 3)
    assert (rows[:, 0] == 0).all()
    assert np.array_equal(rows[:, 1:].reshape(5, 7, 3), img)


def test_resolve_accum_matches_reference_clamp():
    import oracle_bind as ob
    acc = np.zeros((2, 3, 4), np.float32)
    acc[..., :3] = np.array([[-5, 0.5, 254.9], [255.0, 1e12, np.nan]], np.float32)[..., None] * 2.0
    acc[..., 3] = 2.0
    hdr, ldr = rtgpu.resolve_accum(acc)
    assert np.array_equal(ldr, ob.clamp_ldr(hdr))
    assert ldr[1, 1, 0] == 0     # x86 cvttss2si overflow -> INT_MIN -> clamp 0
    assert ldr[1, 2, 0] == 0     # NaN -> 0


def _desc_layout(tmp_path):
    import shutil
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    src = tmp_path / "lay.c"
    src.write_text('#include "rtgpu.h"\n#include <stdio.h>\n#include <stddef.h>\nint main(void){printf("%zu %zu %zu %zu\\n", '
                   'sizeof(rtg_scene_desc), offsetof(rtg_scene_desc, faces), offsetof(rtg_scene_desc, num_faces), '
                   'sizeof(rtg_face));return 0;}\n')
    exe = tmp_path / "lay"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    return map(int, subprocess.run([str(exe)], capture_output=True, text=True).stdout.split())


def test_face_limit_refused(tmp_path):
    """rtg_scene_create refuses descriptions of more than 2^25 faces with RTG_ERR_INVALID
    before touching a device (rtg_api.cpp: the packet walks address node and face records by
    32-bit byte offsets, rtg_common.hpp rec_at).  The description is a real one with its face
    list replaced by 2^25 + 1 zeroed faces (calloc'd: untouched pages cost nothing)."""
    size, off_faces, off_num, face_size = _desc_layout(tmp_path)
    assert face_size == 80
    hs = rtgpu.HostScene(os.path.join(SCENES, "simple.xml"))
    buf = (ctypes.c_char * size)()
    ctypes.memmove(buf, hs.desc, size)
    n = (1 << 25) + 1
    faces = np.zeros(n * face_size, np.uint8)
    ctypes.c_void_p.from_buffer(buf, off_faces).value = faces.ctypes.data
    ctypes.c_int64.from_buffer(buf, off_num).value = n
    s = ctypes.c_void_p()
    rc = rtgpu.lib().rtg_scene_create(ctypes.addressof(buf), 0, ctypes.byref(s))
    assert rc == -1 and not s.value, rc
    assert b"2^25" in rtgpu.lib().rtg_last_error()
    # at the limit the count is accepted (what follows needs a device)
    ctypes.c_int64.from_buffer(buf, off_num).value = n - 1
    if rtgpu.device_count() == 0:
        rc = rtgpu.lib().rtg_scene_create(ctypes.addressof(buf), 0, ctypes.byref(s))
        assert rc == -4, (rc, rtgpu.lib().rtg_last_error())
