"""Procedural scenes in the reference's own XML schema (src/parser.cpp) for benches and
parity tests.  Every generator writes an XML file plus a binary little-endian PLY
(read by the reference through happly, parser.cpp:1396-1444, and by rtgpu's loader), so
the same files can be rendered by oracle/_ref, by the CPU oracle and by the GPU path.

Paths inside the XML are relative (PLY: relative to the current directory, as
parser.cpp:1404 opens them), so render with ``cwd`` set to the output directory.
"""
from __future__ import annotations

import os

import numpy as np


def write_ply(path: str, verts: np.ndarray, faces: np.ndarray):
    """Binary little-endian PLY: float x,y,z; uchar-count int vertex_indices."""
    verts = np.ascontiguousarray(verts, np.float32)
    faces = np.ascontiguousarray(faces, np.int32)
    head = (
        "ply\nformat binary_little_endian 1.0\n"
        f"element vertex {len(verts)}\nproperty float x\nproperty float y\nproperty float z\n"
        f"element face {len(faces)}\nproperty list uchar int vertex_indices\nend_header\n"
    ).encode()
    rec = np.zeros(len(faces), dtype=[("n", "u1"), ("i", "<i4", (faces.shape[1],))])
    rec["n"] = faces.shape[1]
    rec["i"] = faces
    with open(path, "wb") as f:
        f.write(head)
        f.write(verts.tobytes())
        f.write(rec.tobytes())


def _f(v) -> str:
    return " ".join(f"{float(x):.6f}" for x in np.atleast_1d(v))


def _camera_default(pos, gaze, up, near_plane, near_dist, res, name, spp=1) -> str:
    extra = f"\n            <NumSamples>{spp}</NumSamples>" if spp > 1 else ""
    return f"""    <Cameras>
        <Camera id="1">
            <Position>{_f(pos)}</Position>
            <Gaze>{_f(gaze)}</Gaze>
            <Up>{_f(up)}</Up>
            <NearPlane>{_f(near_plane)}</NearPlane>
            <NearDistance>{near_dist}</NearDistance>
            <ImageResolution>{res[0]} {res[1]}</ImageResolution>
            <ImageName>{name}</ImageName>{extra}
        </Camera>
    </Cameras>
"""


def heightfield_mesh(K: int, extent, seed: int = 1234, amp: float = 0.05):
    """Displaced grid with ~K triangles over extent = (x0, x1, y0, y1)."""
    n = max(1, int(round(np.sqrt(K / 2.0))))
    rng = np.random.default_rng(seed)
    x0, x1, y0, y1 = extent
    xs = np.linspace(x0, x1, n + 1, dtype=np.float64)
    ys = np.linspace(y0, y1, n + 1, dtype=np.float64)
    X, Y = np.meshgrid(xs, ys, indexing="ij")
    Z = amp * (np.sin(2.1 * X + 0.3) * np.cos(1.7 * Y) + 0.5 * np.sin(5.3 * X * Y + 1.0)
               + 0.35 * np.sin(11.0 * X + 7.0 * Y)) + 0.15 * amp * rng.standard_normal(X.shape)
    verts = np.stack([X, Y, Z], -1).reshape(-1, 3)
    verts = np.round(verts, 6).astype(np.float32)          # "vertices float with 6 decimals"
    idx = np.arange((n + 1) * (n + 1)).reshape(n + 1, n + 1)
    v00, v10, v01, v11 = idx[:-1, :-1], idx[1:, :-1], idx[:-1, 1:], idx[1:, 1:]
    t1 = np.stack([v00, v10, v11], -1).reshape(-1, 3)
    t2 = np.stack([v00, v11, v01], -1).reshape(-1, 3)
    faces = np.stack([t1, t2], 1).reshape(-1, 3)
    return verts, faces


def synthetic_heightfield(out_dir: str, K: int = 100352, width: int = 1920, height: int = 1080, seed: int = 1234,
                          spp: int = 1, depth: int = 0, name: str | None = None) -> str:
    """BASELINE headline scene: a seeded K-triangle height field filling a 16:9 frame, one
    point light, default Blinn-Phong material (exponent 20), primary + shadow rays.
    Returns the XML path."""
    os.makedirs(out_dir, exist_ok=True)
    name = name or f"synth_{K}"
    pos = np.array([0.0, -1.2, 1.3])
    look = np.array([0.0, 0.9, -0.05])
    gaze = look - pos
    gaze /= np.linalg.norm(gaze)
    up = np.array([0.0, 0.0, 1.0])
    aspect = width / height
    near, half_w = 0.6, 0.45
    half_h = half_w / aspect
    # frustum footprint on the lowest possible surface, plus margin -> every camera ray hits
    right = np.cross(up, -gaze)
    right /= np.linalg.norm(right)
    upo = np.cross(-gaze, right)
    amp = 0.05
    zmin = -2.5 * amp
    pts = []
    for sx in (-1, 1):
        for sy in (-1, 1):
            d = gaze * near + right * sx * half_w + upo * sy * half_h
            t = (zmin - pos[2]) / d[2]
            pts.append(pos + t * d)
    pts = np.array(pts)
    mx = 0.08 * (pts[:, 0].max() - pts[:, 0].min())
    my = 0.08 * (pts[:, 1].max() - pts[:, 1].min())
    extent = (pts[:, 0].min() - mx, pts[:, 0].max() + mx, pts[:, 1].min() - my, pts[:, 1].max() + my)
    verts, faces = heightfield_mesh(K, extent, seed, amp)
    ply = f"{name}.ply"
    write_ply(os.path.join(out_dir, ply), verts, faces)
    xml = f"""<Scene>
    <MaxRecursionDepth>{depth}</MaxRecursionDepth>
    <BackgroundColor>10 10 30</BackgroundColor>
    <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
{_camera_default(pos, gaze, up, (-half_w, half_w, -half_h, half_h), near, (width, height), name + '.png', spp)}
    <Lights>
        <AmbientLight>20 20 20</AmbientLight>
        <PointLight id="1">
            <Position>1.6 -0.4 1.1</Position>
            <Intensity>420 400 380</Intensity>
        </PointLight>
    </Lights>
    <Materials>
        <Material id="1">
            <AmbientReflectance>1 1 1</AmbientReflectance>
            <DiffuseReflectance>0.75 0.6 0.45</DiffuseReflectance>
            <SpecularReflectance>0.35 0.35 0.35</SpecularReflectance>
            <PhongExponent>20</PhongExponent>
        </Material>
    </Materials>
    <VertexData>0 0 0</VertexData>
    <Objects>
        <Mesh id="1">
            <Material>1</Material>
            <Faces plyFile="{ply}"/>
        </Mesh>
    </Objects>
</Scene>
"""
    path = os.path.join(out_dir, name + ".xml")
    with open(path, "w") as f:
        f.write(xml)
    return path


def with_resolution(src_xml: str, dst_xml: str, width: int, height: int, spp: int | None = None) -> str:
    """Copy a scene with a different <ImageResolution> (and optionally <NumSamples>)."""
    import re
    s = open(src_xml).read()
    s = re.sub(r"<ImageResolution>[^<]*</ImageResolution>", f"<ImageResolution>{width} {height}</ImageResolution>", s)
    if spp is not None:
        if "<NumSamples>" in s:
            s = re.sub(r"<NumSamples>[^<]*</NumSamples>", f"<NumSamples>{spp}</NumSamples>", s)
        else:
            s = s.replace("</ImageName>", f"</ImageName>\n            <NumSamples>{spp}</NumSamples>", 1)
    with open(dst_xml, "w") as f:
        f.write(s)
    return dst_xml


def with_depth(src_xml: str, dst_xml: str, depth: int) -> str:
    """Copy a scene with a different <MaxRecursionDepth> (0 = no ray-tree children)."""
    import re
    s = open(src_xml).read()
    if "<MaxRecursionDepth>" in s:
        s = re.sub(r"<MaxRecursionDepth>[^<]*</MaxRecursionDepth>", f"<MaxRecursionDepth>{depth}</MaxRecursionDepth>", s)
    else:
        s = s.replace("<Scene>", f"<Scene>\n    <MaxRecursionDepth>{depth}</MaxRecursionDepth>", 1)
    with open(dst_xml, "w") as f:
        f.write(s)
    return dst_xml
