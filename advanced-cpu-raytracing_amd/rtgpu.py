"""ctypes binding of the rtgpu C-ABI (include/rtgpu.h).

Mirrors the reference's render interface for Python callers (tests, bench.py):

* ``HostScene(xml)``          -- ``DorkTracer::Scene::loadFromXml`` (src/parser.cpp:26-577)
* ``DeviceScene(host, dev)``  -- ``Raytracer::Raytracer(Scene&)`` (src/raytracer.cpp:7-16),
                                 a device-resident replica on HIP device ``dev``
* ``DeviceScene.render(cam)`` -- the per-camera block of ``main()`` (src/main.cpp:142-196):
                                 every pixel through ``RenderPixel`` (raytracer.hpp:19),
                                 returning the float image (main.cpp:114-116) and the
                                 ``clamp((int)c)`` LDR image (main.cpp:121)

The product path is librtgpu.so only; importing this module fails loudly when the
library has not been built.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RTGPU_LIB: an alternative in-tree build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("RTGPU_LIB") or os.path.join(HERE, "librtgpu.so")

RTG_RENDER_COUNT_STATS = 1
RTG_RENDER_ACCUM_ONLY = 2
RTG_RENDER_FUSED = 4
RTG_RENDER_TIMING = 8
RTG_RENDER_TREE = 16
RTG_RENDER_EXACT_SHADOW = 32
RTG_RENDER_ORDERED = 64
RTG_RENDER_SAMPLE_PASSES = 128
RTG_LOAD_DEVICE_BVH = 1
RTG_CAMERA_SIZE = 392   # sizeof(rtg_camera), checked against the C compiler by tests/test_abi.py


class RTGError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rtgpu error {code}: {msg}")
        self.code = code


class TonemapParams(ctypes.Structure):
    _fields_ = [("key", ctypes.c_float), ("burn_percent", ctypes.c_float), ("saturation", ctypes.c_float),
                ("gamma", ctypes.c_float)]


class _Camera(ctypes.Structure):
    """Head of rtg_camera (include/rtgpu.h) up to the tonemapper parameters."""
    _fields_ = [("f3", ctypes.c_float * 15), ("ext", ctypes.c_float * 5), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("spp", ctypes.c_int32), ("focus_distance", ctypes.c_float),
                ("aperture", ctypes.c_float), ("has_tonemapper", ctypes.c_int32), ("tm_key", ctypes.c_float),
                ("tm_burn", ctypes.c_float), ("tm_saturation", ctypes.c_float), ("tm_gamma", ctypes.c_float)]


class _DescHead(ctypes.Structure):
    """Head of rtg_scene_desc (include/rtgpu.h) up to the camera list."""
    _fields_ = [("background", ctypes.c_int32 * 3), ("shadow_epsilon", ctypes.c_float),
                ("max_recursion_depth", ctypes.c_int32), ("bg_texture", ctypes.c_int32),
                ("ambient_light", ctypes.c_float * 3), ("cameras", ctypes.c_void_p), ("num_cameras", ctypes.c_int32)]


class RenderOpts(ctypes.Structure):
    _fields_ = [
        ("camera", ctypes.c_int32),
        ("sample_begin", ctypes.c_int32),
        ("sample_count", ctypes.c_int32),
        ("row_begin", ctypes.c_int32),
        ("row_end", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("part_index", ctypes.c_int32),
        ("part_count", ctypes.c_int32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "camera_rays", "secondary_rays", "shadow_rays", "node_visits", "tri_tests",
        "sphere_tests", "object_tests", "shadow_node_visits", "shadow_tri_tests", "shadow_wide_visits",
        "shadow_fallbacks", "extend_wide_visits", "extend_fallbacks")]

    def as_dict(self) -> dict:
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


# every symbol include/rtgpu.h declares
EXPORTED = [
    "rtg_host_scene_load_xml", "rtg_host_scene_load_xml_ex", "rtg_host_scene_desc", "rtg_host_scene_free",
    "rtg_scene_export_bvh",
    "rtg_desc_camera_info", "rtg_desc_counts", "rtg_desc_anyhit_check", "rtg_scene_create", "rtg_scene_destroy",
    "rtg_device_count", "rtg_render", "rtg_render_device", "rtg_resolve_accum",
    "rtg_scene_stats", "rtg_scene_reset_stats", "rtg_scene_timings", "rtg_scene_timed_samples", "rtg_tonemap_device", "rtg_tonemap",
    "rtg_tonemap_log_average",
    "rtg_write_png", "rtg_write_hdr",
    "rtg_last_error", "rtg_abi_version",
    "rtg_scene_create_multi", "rtg_scene_num_devices", "rtg_part_runs", "rtg_copy_part_to_host",
    "rtg_host_alloc", "rtg_host_free", "rtg_host_register", "rtg_host_unregister",
]

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RTGError(-1, f"{LIB_PATH} not built: run `make -C {HERE}` (or __graft_entry__.build())")
    # One HIP runtime per process: torch's ROCm wheel ships its own libamdhip64.so.7.  If
    # torch is loaded first, librtgpu's NEEDED libamdhip64.so.7 binds to that same copy
    # (shared streams, events, allocations); loaded the other way round, two runtimes
    # end up in the process and torch's fails to initialise.  So load torch first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, P = ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER
    L.rtg_last_error.restype = ctypes.c_char_p
    L.rtg_abi_version.restype = ctypes.c_int
    L.rtg_host_scene_load_xml.argtypes = [ctypes.c_char_p, P(vp)]
    L.rtg_host_scene_load_xml_ex.argtypes = [ctypes.c_char_p, ctypes.c_uint32, P(vp)]
    L.rtg_scene_export_bvh.argtypes = [vp, vp, ctypes.c_int64, vp, ctypes.c_int64, P(ctypes.c_int64),
                                       P(ctypes.c_int64)]
    L.rtg_host_scene_desc.argtypes = [vp]
    L.rtg_host_scene_desc.restype = vp
    L.rtg_host_scene_free.argtypes = [vp]
    L.rtg_host_scene_free.restype = None
    L.rtg_desc_camera_info.argtypes = [vp, ctypes.c_int, P(i32), P(i32), P(i32), P(i32)]
    L.rtg_desc_counts.argtypes = [vp] + [P(ctypes.c_int64)] * 4
    L.rtg_desc_anyhit_check.argtypes = [vp, i32, P(ctypes.c_int64), i32]
    L.rtg_scene_create.argtypes = [vp, ctypes.c_int, P(vp)]
    L.rtg_scene_destroy.argtypes = [vp]
    L.rtg_scene_destroy.restype = None
    L.rtg_device_count.argtypes = [P(i32)]
    L.rtg_render.argtypes = [vp, P(RenderOpts), vp, vp]
    L.rtg_render_device.argtypes = [vp, P(RenderOpts), vp, vp, vp, vp]
    L.rtg_resolve_accum.argtypes = [vp, i32, i32, vp, vp]
    L.rtg_scene_stats.argtypes = [vp, P(Stats)]
    L.rtg_scene_reset_stats.argtypes = [vp]
    L.rtg_scene_timings.argtypes = [vp, P(ctypes.c_float), P(ctypes.c_char_p), i32, P(i32)]
    L.rtg_scene_timed_samples.argtypes = [vp, P(i32)]
    L.rtg_tonemap_device.argtypes = [vp, i32, i32, P(TonemapParams), vp, i32, vp]
    L.rtg_tonemap.argtypes = [vp, i32, i32, P(TonemapParams), vp, i32]
    L.rtg_tonemap_log_average.argtypes = [vp, i32, i32, i32, P(ctypes.c_double), i32]
    L.rtg_write_png.argtypes = [ctypes.c_char_p, i32, i32, vp]
    L.rtg_write_hdr.argtypes = [ctypes.c_char_p, i32, i32, vp]
    L.rtg_scene_create_multi.argtypes = [vp, P(i32), i32, P(vp)]
    L.rtg_scene_num_devices.argtypes = [vp, P(i32)]
    L.rtg_part_runs.argtypes = [i32, i32, i32, i32, vp, i32, P(i32)]
    L.rtg_copy_part_to_host.argtypes = [vp, P(RenderOpts), vp, vp, vp, vp, vp]
    L.rtg_host_alloc.argtypes = [ctypes.c_size_t, P(vp)]
    L.rtg_host_free.argtypes = [vp]
    L.rtg_host_register.argtypes = [vp, ctypes.c_size_t]
    L.rtg_host_unregister.argtypes = [vp]
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        raise RTGError(rc, lib().rtg_last_error().decode(errors="replace"))


def device_count() -> int:
    n = ctypes.c_int32()
    _check(lib().rtg_device_count(ctypes.byref(n)))
    return n.value


class HostScene:
    """Parsed + flattened scene (rtg_host_scene).  Paths inside the XML resolve like the
    reference's: PLY relative to the current directory, images as ``inputs/<name>``."""

    def __init__(self, xml_path: str, device_bvh: bool = False):
        """device_bvh: RTG_LOAD_DEVICE_BVH -- no host BVH build; DeviceScene builds it on the GPU."""
        h = ctypes.c_void_p()
        _check(lib().rtg_host_scene_load_xml_ex(os.fsencode(xml_path), RTG_LOAD_DEVICE_BVH if device_bvh else 0,
                                                ctypes.byref(h)))
        self._h = h
        self.desc = lib().rtg_host_scene_desc(h)

    def camera(self, idx: int = 0) -> dict:
        w, h, s, t = (ctypes.c_int32() for _ in range(4))
        _check(lib().rtg_desc_camera_info(self.desc, idx, ctypes.byref(w), ctypes.byref(h),
                                          ctypes.byref(s), ctypes.byref(t)))
        return {"width": w.value, "height": h.value, "spp": s.value, "tonemapped": bool(t.value)}

    def tonemap_params(self, idx: int = 0):
        """(key, burn %, saturation, gamma) of camera idx's <Tonemap> (tonemapper.h:18-25), or
        None for a camera without one."""
        head = _DescHead.from_address(self.desc)
        if not 0 <= idx < head.num_cameras:
            raise RTGError(-1, "camera index out of range")
        cam = _Camera.from_address(head.cameras + idx * RTG_CAMERA_SIZE)
        if not cam.has_tonemapper:
            return None
        return (cam.tm_key, cam.tm_burn, cam.tm_saturation, cam.tm_gamma)

    def counts(self) -> dict:
        v = [ctypes.c_int64() for _ in range(4)]
        _check(lib().rtg_desc_counts(self.desc, *[ctypes.byref(x) for x in v]))
        return dict(zip(("objects", "faces", "nodes", "lights"), (x.value for x in v)))

    def anyhit_check(self, mode: int = 1) -> dict:
        """Host-only build + structural check of the shadow rays' any-hit trees
        (rtg_desc_anyhit_check; mode 0 reference collapse, 1 SAH over leaves (default), 2 split)."""
        out = (ctypes.c_int64 * 8)()
        _check(lib().rtg_desc_anyhit_check(self.desc, mode, out, 8))
        keys = ("nodes", "entries", "depth", "leaf_prims", "face_prims", "exact_faces", "violations", "built")
        return dict(zip(keys, (int(x) for x in out)))

    def num_cameras(self) -> int:
        n = 0
        while True:
            try:
                self.camera(n)
            except RTGError:
                return n
            n += 1

    def close(self):
        if getattr(self, "_h", None):
            lib().rtg_host_scene_free(self._h)
            self._h = None
            self.desc = None

    def __del__(self):
        try:
            self.close()
        except Exception:      # interpreter shutdown: ctypes may already be torn down
            pass


class DeviceScene:
    """Device-resident scene replica (rtg_scene) on HIP device ``device``, or -- with
    ``devices=[d0, d1, ...]`` -- one replica per listed device (rtg_scene_create_multi),
    among which ``render()`` deals the frame's parts (multigpu.py)."""

    def __init__(self, host: HostScene, device: int = 0, devices=None):
        s = ctypes.c_void_p()
        if devices:
            arr = (ctypes.c_int32 * len(devices))(*devices)
            _check(lib().rtg_scene_create_multi(host.desc, arr, len(devices), ctypes.byref(s)))
            device = devices[0]
        else:
            _check(lib().rtg_scene_create(host.desc, device, ctypes.byref(s)))
        self._s = s
        self.host = host
        self.device = device
        self.devices = list(devices) if devices else [device]

    @staticmethod
    def opts(camera=0, sample_begin=0, sample_count=-1, rows=(0, 0), flags=0, seed=0x5EED, part=(0, 1)) -> RenderOpts:
        return RenderOpts(camera, sample_begin, sample_count, rows[0], rows[1], flags, seed, part[0], part[1])

    def render(self, camera: int = 0, rows=(0, 0), flags: int = 0, seed: int = 0x5EED, part=(0, 1), out=None):
        """Host-buffer render of one camera -> (hdr float32 HxWx3, ldr uint8 HxWx3).  With
        ``part=(i, n)`` only part i's rows are rendered and written (zeros elsewhere, or
        what ``out=(hdr, ldr)`` already holds)."""
        c = self.host.camera(camera)
        if out is None:
            hdr = np.zeros((c["height"], c["width"], 3), np.float32)
            ldr = np.zeros((c["height"], c["width"], 3), np.uint8)
        else:
            hdr, ldr = out
        o = self.opts(camera, 0, -1, rows, flags, seed, part)
        _check(lib().rtg_render(self._s, ctypes.byref(o), hdr.ctypes.data if hdr is not None else None,
                                ldr.ctypes.data if ldr is not None else None))
        return hdr, ldr

    def render_device(self, hdr_ptr: int, ldr_ptr: int, stream: int = 0, camera: int = 0, flags: int = 0,
                      seed: int = 0x5EED, accum_ptr: int = 0, sample_begin: int = 0, sample_count: int = -1,
                      rows=(0, 0), part=(0, 1)):
        """Asynchronous render into device buffers (e.g. torch tensor data_ptr()s) on ``stream``;
        ``part=(i, n)``: part i of n of the frame (multigpu.py)."""
        o = self.opts(camera, sample_begin, sample_count, rows, flags, seed, part)
        _check(lib().rtg_render_device(self._s, ctypes.byref(o), hdr_ptr or None, ldr_ptr or None,
                                       accum_ptr or None, stream or None))

    def copy_part_to_host(self, d_hdr: int, d_ldr: int, h_hdr: int, h_ldr: int, stream: int = 0, camera: int = 0,
                          rows=(0, 0), part=(0, 1)):
        """Enqueue the DMA of part ``part``'s rows from full-frame device buffers to the same
        offsets of full-frame host buffers (the host framebuffer gather)."""
        o = self.opts(camera, 0, -1, rows, 0, 0, part)
        _check(lib().rtg_copy_part_to_host(self._s, ctypes.byref(o), d_hdr or None, d_ldr or None, h_hdr or None,
                                           h_ldr or None, stream or None))

    def export_bvh(self):
        """(nodes (N, 8) float32, tris (F, 12) float32): the device's walk records."""
        nn, nf = ctypes.c_int64(), ctypes.c_int64()
        _check(lib().rtg_scene_export_bvh(self._s, None, 0, None, 0, ctypes.byref(nn), ctypes.byref(nf)))
        nodes = np.zeros((nn.value, 8), np.float32)
        tris = np.zeros((nf.value, 12), np.float32)
        _check(lib().rtg_scene_export_bvh(self._s, nodes.ctypes.data, nn.value, tris.ctypes.data, nf.value,
                                          ctypes.byref(nn), ctypes.byref(nf)))
        return nodes, tris

    def stats(self) -> dict:
        st = Stats()
        _check(lib().rtg_scene_stats(self._s, ctypes.byref(st)))
        return st.as_dict()

    def reset_stats(self):
        _check(lib().rtg_scene_reset_stats(self._s))

    def timings(self) -> dict:
        """{kernel: ms} of the last render issued with RTG_RENDER_TIMING (synchronises)."""
        ms = (ctypes.c_float * 8)()
        names = (ctypes.c_char_p * 8)()
        n = ctypes.c_int32()
        _check(lib().rtg_scene_timings(self._s, ms, names, 8, ctypes.byref(n)))
        return {names[k].decode(): float(ms[k]) for k in range(n.value)}

    def timed_samples(self) -> int:
        """Samples per pixel the stages of timings() covered (the last pass of a multi-sample
        render carries several, RTG_RENDER_SAMPLE_PASSES)."""
        n = ctypes.c_int32()
        _check(lib().rtg_scene_timed_samples(self._s, ctypes.byref(n)))
        return n.value

    def close(self):
        if getattr(self, "_s", None):
            lib().rtg_scene_destroy(self._s)
            self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedArray:
    """Page-locked host array (rtg_host_alloc): the frame buffer of the drop-in host path
    (the CLI allocates its frames the same way), so the device-to-host copy is one DMA."""

    def __init__(self, shape, dtype):
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = ctypes.c_void_p()
        _check(lib().rtg_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr = p.value
        self.array = np.frombuffer((ctypes.c_char * nbytes).from_address(self.ptr), dtype).reshape(shape)

    def close(self):
        if getattr(self, "ptr", None):
            self.array = None
            lib().rtg_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def resolve_accum(accum: np.ndarray):
    """(sum w*c, sum w) per pixel -> (hdr, ldr); host side (samples split across devices)."""
    h, w, _ = accum.shape
    accum = np.ascontiguousarray(accum, np.float32)
    hdr = np.zeros((h, w, 3), np.float32)
    ldr = np.zeros((h, w, 3), np.uint8)
    _check(lib().rtg_resolve_accum(accum.ctypes.data, w, h, hdr.ctypes.data, ldr.ctypes.data))
    return hdr, ldr


def tonemap(hdr: np.ndarray, key=0.18, burn=1.0, saturation=1.0, gamma=2.2, device: int = 0) -> np.ndarray:
    """Photographic tonemapper (Tonemapper::Tonemap, tonemapper.h:28-60) on the GPU."""
    hdr = np.ascontiguousarray(hdr, np.float32)
    h, w, _ = hdr.shape
    ldr = np.zeros((h, w, 3), np.uint8)
    p = TonemapParams(key, burn, saturation, gamma)
    _check(lib().rtg_tonemap(hdr.ctypes.data, w, h, ctypes.byref(p), ldr.ctypes.data, device))
    return ldr


def tonemap_log_average(hdr: np.ndarray, mode: int = -1, device: int = 0) -> float:
    """Tonemapper::avgLuminance (tonemapper.h:35-48) on the GPU; mode as rtg_tonemap_log_average."""
    hdr = np.ascontiguousarray(hdr, np.float32)
    h, w, _ = hdr.shape
    out = ctypes.c_double()
    _check(lib().rtg_tonemap_log_average(hdr.ctypes.data, w, h, mode, ctypes.byref(out), device))
    return out.value


def write_png(path: str, ldr: np.ndarray):
    ldr = np.ascontiguousarray(ldr, np.uint8)
    _check(lib().rtg_write_png(os.fsencode(path), ldr.shape[1], ldr.shape[0], ldr.ctypes.data))
