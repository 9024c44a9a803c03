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


# ---------------------------------------------------------------------------
# BASELINE.json configurations C2-C5, as procedural scenes
# ---------------------------------------------------------------------------

def blob_mesh(K: int, center=(0.0, 0.0, 0.0), radius: float = 1.0, seed: int = 1234, bumps: float = 0.12):
    """Closed, displaced UV sphere with ~K triangles ("bunny / dragon class" stand-in)."""
    n = max(4, int(round(np.sqrt(K / 2.0))))
    n_lat, n_lon = n, n
    rng = np.random.default_rng(seed)
    ph = rng.uniform(0, 2 * np.pi, 6)
    th = np.linspace(0.0, np.pi, n_lat + 1)[1:-1]
    lo = np.linspace(0.0, 2 * np.pi, n_lon, endpoint=False)
    T, L = np.meshgrid(th, lo, indexing="ij")
    r = radius * (1 + bumps * (np.sin(3 * T + ph[0]) * np.cos(4 * L + ph[1]) + 0.5 * np.sin(9 * T + ph[2])
                               * np.sin(7 * L + ph[3]) + 0.25 * np.cos(17 * T + 13 * L + ph[4])))
    x = r * np.sin(T) * np.cos(L)
    y = r * np.cos(T)
    z = r * np.sin(T) * np.sin(L)
    ring = np.stack([x, y, z], -1).reshape(-1, 3)
    verts = np.concatenate([[[0, radius, 0]], ring, [[0, -radius, 0]]]) + np.asarray(center)
    verts = np.round(verts, 6).astype(np.float32)
    idx = 1 + np.arange((n_lat - 1) * n_lon).reshape(n_lat - 1, n_lon)
    nxt = np.roll(idx, -1, axis=1)
    faces = [np.stack([np.zeros(n_lon, int), nxt[0], idx[0]], -1)]                       # north cap
    a, b, c, d = idx[:-1], nxt[:-1], idx[1:], nxt[1:]
    faces.append(np.stack([a, b, d], -1).reshape(-1, 3))
    faces.append(np.stack([a, d, c], -1).reshape(-1, 3))
    south = len(verts) - 1
    faces.append(np.stack([idx[-1], nxt[-1], np.full(n_lon, south)], -1))                 # south cap
    return verts, np.concatenate(faces).astype(np.int32)


def torus_mesh(K: int, center=(0.0, 0.0, 0.0), R: float = 1.0, r: float = 0.45, seed: int = 1234,
               bumps: float = 0.08):
    """Displaced torus with ~K triangles, tilted 30 degrees about x: a dense closed mesh with
    no poles (a UV sphere's pole fans share centroid coordinates, which the reference's
    midpoint split cannot separate; scanned meshes have no such fans)."""
    nv = max(3, int(round(np.sqrt(K / 4.0))))
    nu = max(3, int(round(K / (2.0 * nv))))
    rng = np.random.default_rng(seed)
    ph = rng.uniform(0, 2 * np.pi, 4)
    u = np.linspace(0.0, 2 * np.pi, nu, endpoint=False)
    v = np.linspace(0.0, 2 * np.pi, nv, endpoint=False)
    U, Vv = np.meshgrid(u, v, indexing="ij")
    rr = r * (1 + bumps * (np.sin(7 * U + ph[0]) * np.cos(5 * Vv + ph[1]) + 0.5 * np.sin(23 * U + 3 * Vv + ph[2])
                           + 0.25 * np.cos(61 * U + 11 * Vv + ph[3])))
    x = (R + rr * np.cos(Vv)) * np.cos(U)
    z = (R + rr * np.cos(Vv)) * np.sin(U)
    y = rr * np.sin(Vv)
    a = np.radians(30.0)
    y, z = y * np.cos(a) - z * np.sin(a), y * np.sin(a) + z * np.cos(a)
    verts = np.round(np.stack([x, y, z], -1).reshape(-1, 3) + np.asarray(center), 6).astype(np.float32)
    idx = np.arange(nu * nv).reshape(nu, nv)
    i1 = np.roll(idx, -1, axis=0)
    j1 = np.roll(idx, -1, axis=1)
    ij1 = np.roll(i1, -1, axis=1)
    faces = np.concatenate([np.stack([idx, i1, ij1], -1).reshape(-1, 3), np.stack([idx, ij1, j1], -1).reshape(-1, 3)])
    return verts, faces.astype(np.int32)


def _lookat_camera(pos, gaze_point, up, fovy, res, name, spp=1) -> str:
    extra = f"\n            <NumSamples>{spp}</NumSamples>" if spp > 1 else ""
    return f"""    <Cameras>
        <Camera id="1" type="lookAt">
            <Position>{_f(pos)}</Position>
            <GazePoint>{_f(gaze_point)}</GazePoint>
            <Up>{_f(up)}</Up>
            <FovY>{fovy}</FovY>
            <NearDistance>1</NearDistance>
            <ImageResolution>{res[0]} {res[1]}</ImageResolution>
            <ImageName>{name}</ImageName>{extra}
        </Camera>
    </Cameras>
"""


def _write(out_dir, name, xml):
    path = os.path.join(out_dir, name + ".xml")
    with open(path, "w") as f:
        f.write(xml)
    return path


def _ground(size: float, y: float = 0.0):
    """VertexData block (4 corners) and the 1-based faces of a ground quad."""
    s = size
    v = f"{-s} {y} {-s}\n        {s} {y} {-s}\n        {s} {y} {s}\n        {-s} {y} {s}"
    return v, "1 3 2\n                1 4 3"


def write_ppm(path: str, img: np.ndarray):
    img = np.ascontiguousarray(np.clip(img, 0, 255).astype(np.uint8))
    with open(path, "wb") as f:
        f.write(f"P6\n{img.shape[1]} {img.shape[0]}\n255\n".encode())
        f.write(img.tobytes())


def config_c2(out_dir: str, src_xml: str, width: int = 800, height: int = 800, brdf: bool = True) -> str:
    """C2: the conductor Cornell box at 800x800, 1 spp; with ``brdf`` an OriginalPhong BRDF on
    the diffuse materials."""
    import re
    os.makedirs(out_dir, exist_ok=True)
    s = open(src_xml).read()
    s = re.sub(r"<ImageResolution>[^<]*</ImageResolution>", f"<ImageResolution>{width} {height}</ImageResolution>", s)
    if brdf:
        s = s.replace("<Materials>", "<BRDFs>\n        <OriginalPhong id=\"1\">\n            <Exponent>25</Exponent>\n"
                      "        </OriginalPhong>\n    </BRDFs>\n    <Materials>", 1)
        for mid in ("1", "2", "3", "4"):
            s = s.replace(f'<Material id="{mid}">', f'<Material id="{mid}" BRDF="1">', 1)
    return _write(out_dir, "c2_cornell", s)


def config_c3(out_dir: str, K: int = 70000, width: int = 1920, height: int = 1080, spp: int = 4) -> str:
    """C3: ~70k-triangle closed mesh + area light, OriginalBlinnPhong, 4 spp, 1920x1080."""
    os.makedirs(out_dir, exist_ok=True)
    v, f = blob_mesh(K, center=(0, 1.0, 0), radius=1.0, seed=7)
    write_ply(os.path.join(out_dir, "c3_blob.ply"), v, f)
    gv, gf = _ground(6.0)
    xml = f"""<Scene>
    <MaxRecursionDepth>1</MaxRecursionDepth>
    <BackgroundColor>5 5 10</BackgroundColor>
    <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
{_lookat_camera((0, 1.6, 4.2), (0, 0.9, 0), (0, 1, 0), 38, (width, height), 'c3.png', spp)}
    <Lights>
        <AmbientLight>8 8 8</AmbientLight>
        <AreaLight id="1">
            <Position>0.5 4 1</Position>
            <Normal>0 -1 0</Normal>
            <Radiance>1500 1400 1300</Radiance>
            <Size>1.5</Size>
        </AreaLight>
    </Lights>
    <BRDFs>
        <OriginalBlinnPhong id="1">
            <Exponent>40</Exponent>
        </OriginalBlinnPhong>
    </BRDFs>
    <Materials>
        <Material id="1" BRDF="1">
            <AmbientReflectance>0.3 0.3 0.3</AmbientReflectance>
            <DiffuseReflectance>0.7 0.55 0.4</DiffuseReflectance>
            <SpecularReflectance>0.4 0.4 0.4</SpecularReflectance>
        </Material>
        <Material id="2">
            <AmbientReflectance>0.3 0.3 0.3</AmbientReflectance>
            <DiffuseReflectance>0.5 0.5 0.55</DiffuseReflectance>
            <SpecularReflectance>0 0 0</SpecularReflectance>
        </Material>
    </Materials>
    <VertexData>
        {gv}
    </VertexData>
    <Objects>
        <Mesh id="1">
            <Material>1</Material>
            <Faces plyFile="c3_blob.ply"/>
        </Mesh>
        <Mesh id="2">
            <Material>2</Material>
            <Faces>
                {gf}
            </Faces>
        </Mesh>
    </Objects>
</Scene>
"""
    return _write(out_dir, "c3_blob", xml)


def config_defer_gate(out_dir: str, pad_objects: int = 0, pad_faces: int = 0, K: int = 20000, width: int = 320,
                      height: int = 180) -> str:
    """The reduced C3 blob (large leaves: pole fans) at depth 0, with padding meshes placed
    BEFORE it in object order, behind the camera: ``pad_objects`` one-face meshes and one mesh of
    ``pad_faces`` faces (a height field).  They push the blob's object index and its faces'
    record indices up to the limits of the deferred-leaf key (12 object bits, 20 face bits;
    rtg_common.hpp obj_key, gate in rtg_wave.hpp) without changing the image."""
    os.makedirs(out_dir, exist_ok=True)
    v, f = blob_mesh(K, center=(0, 1.0, 0), radius=1.0, seed=7)
    write_ply(os.path.join(out_dir, "gate_blob.ply"), v, f)
    pads = []
    if pad_faces > 0:
        n = int(np.ceil(np.sqrt(pad_faces / 2.0)))
        pv, pf = heightfield_mesh(2 * n * n, (-40.0, 40.0, -40.0, 40.0), seed=3)
        pv = pv[:, [0, 2, 1]] + np.array([0.0, -1.0, 60.0], np.float32)     # a floor patch behind the camera
        write_ply(os.path.join(out_dir, "gate_pad.ply"), pv, pf[:pad_faces])
        pads.append('        <Mesh id="{id}">\n            <Material>2</Material>\n'
                    '            <Faces plyFile="gate_pad.ply"/>\n        </Mesh>')
    gv, gf = _ground(6.0)
    # one-face pads: vertices 5.. (after the ground's 4), small triangles behind the camera
    pv_lines = []
    for k in range(pad_objects):
        x, z = (k % 64) * 0.5 - 16.0, 40.0 + (k // 64) * 0.5
        pv_lines.append(f"{x} 0 {z}\n        {x + 0.3} 0 {z}\n        {x} 0.3 {z}")
        b = 5 + 3 * k
        pads.append(f'        <Mesh id="{{id}}">\n            <Material>2</Material>\n'
                    f'            <Faces>{b} {b + 1} {b + 2}</Faces>\n        </Mesh>')
    objs = "\n".join(p.format(id=i + 1) for i, p in enumerate(pads))
    nid = len(pads)
    xml = f"""<Scene>
    <MaxRecursionDepth>0</MaxRecursionDepth>
    <BackgroundColor>5 5 10</BackgroundColor>
    <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
{_lookat_camera((0, 1.6, 4.2), (0, 0.9, 0), (0, 1, 0), 38, (width, height), 'gate.png', 1)}
    <Lights>
        <AmbientLight>8 8 8</AmbientLight>
        <PointLight id="1">
            <Position>0.5 4 3</Position>
            <Intensity>30000 28000 26000</Intensity>
        </PointLight>
    </Lights>
    <Materials>
        <Material id="1">
            <AmbientReflectance>0.3 0.3 0.3</AmbientReflectance>
            <DiffuseReflectance>0.7 0.55 0.4</DiffuseReflectance>
            <SpecularReflectance>0.4 0.4 0.4</SpecularReflectance>
            <PhongExponent>30</PhongExponent>
        </Material>
        <Material id="2">
            <AmbientReflectance>0.3 0.3 0.3</AmbientReflectance>
            <DiffuseReflectance>0.5 0.5 0.55</DiffuseReflectance>
            <SpecularReflectance>0 0 0</SpecularReflectance>
        </Material>
    </Materials>
    <VertexData>
        {gv}
        {chr(10).join(pv_lines)}
    </VertexData>
    <Objects>
{objs}
        <Mesh id="{nid + 1}">
            <Material>2</Material>
            <Faces>
                {gf}
            </Faces>
        </Mesh>
        <Mesh id="{nid + 2}">
            <Material>1</Material>
            <Faces plyFile="gate_blob.ply"/>
        </Mesh>
    </Objects>
</Scene>
"""
    return _write(out_dir, "gate", xml)


def config_c3_ton(out_dir: str, ply_dir: str, width: int = 1920, height: int = 1080, spp: int = 4) -> str:
    """C3 on a real mesh (SURVEY §8d's stand-in for the missing bunny): the reference's own
    archive/hw1_inputs/akif_uslu/ton_Roosendaal_smooth scene (62 160-triangle mesh_2.ply plus
    mesh_1 / mesh_3; camera, materials as shipped, the empty <TexCoordData /> dropped), with its
    point light replaced by an AreaLight of the same power at the same place, the materials on
    an OriginalBlinnPhong BRDF, 4 spp, 16:9 at 1920x1080.  `ply_dir` holds the three PLYs
    (tests/golden/scenes/ton_Roosendaal_smooth_ply); they are linked next to the XML."""
    os.makedirs(out_dir, exist_ok=True)
    dst = os.path.join(out_dir, "ton_Roosendaal_smooth_ply")
    if not os.path.exists(dst):
        os.symlink(os.path.abspath(ply_dir), dst)
    aspect = width / height
    xml = f"""<Scene>
    <BackgroundColor>25 76 113</BackgroundColor>
    <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
    <Cameras>
        <Camera id="1">
            <Position>-3.916900157928467 -16.159503936767578 -1.0512659549713135</Position>
            <Gaze>0.22766843438148499 0.971221923828125 -0.06996545195579529</Gaze>
            <Up>-7.450580596923828e-09 0.07185239344835281 0.99741530418396</Up>
            <NearPlane>{-aspect:.6f} {aspect:.6f} -1.0 1.0</NearPlane>
            <NearDistance>3</NearDistance>
            <ImageResolution>{width} {height}</ImageResolution>
            <ImageName>c3_ton.png</ImageName>
            <NumSamples>{spp}</NumSamples>
        </Camera>
    </Cameras>
    <Lights>
        <AmbientLight>0 0 0</AmbientLight>
        <AreaLight id="1">
            <Position>-6.154719352722168 -47.027748107910156 16.88732147216797</Position>
            <Normal>0.07 0.93 -0.36</Normal>
            <Radiance>5000 5000 5000</Radiance>
            <Size>10</Size>
        </AreaLight>
    </Lights>
    <BRDFs>
        <OriginalBlinnPhong id="1">
            <Exponent>30</Exponent>
        </OriginalBlinnPhong>
    </BRDFs>
    <Materials>
        <Material id="1" BRDF="1"><AmbientReflectance>1 1 1</AmbientReflectance><DiffuseReflectance>0.800000011920929 0.800000011920929 0.800000011920929</DiffuseReflectance><SpecularReflectance>0.5 0.5 0.5</SpecularReflectance><PhongExponent>1</PhongExponent></Material>
        <Material id="2" BRDF="1"><AmbientReflectance>1 1 1</AmbientReflectance><DiffuseReflectance>0.8000000715255737 0.3557424247264862 0.04346328601241112</DiffuseReflectance><SpecularReflectance>0.5 0.5 0.5</SpecularReflectance><PhongExponent>1</PhongExponent></Material>
        <Material id="3" BRDF="1"><AmbientReflectance>1 1 1</AmbientReflectance><DiffuseReflectance>0.8000000715255737 0.3774781823158264 0.04441830515861511</DiffuseReflectance><SpecularReflectance>0.5 0.5 0.5</SpecularReflectance><PhongExponent>1</PhongExponent></Material>
    </Materials>
    <VertexData>0 0 0</VertexData>
    <Objects>
        <Mesh id="1"><Material>2</Material><Faces plyFile="ton_Roosendaal_smooth_ply/mesh_1.ply" /></Mesh>
        <Mesh id="2"><Material>1</Material><Faces plyFile="ton_Roosendaal_smooth_ply/mesh_2.ply" /></Mesh>
        <Mesh id="3"><Material>3</Material><Faces plyFile="ton_Roosendaal_smooth_ply/mesh_3.ply" /></Mesh>
    </Objects>
</Scene>
"""
    return _write(out_dir, "c3_ton", xml)


def octasphere_mesh(level: int, center=(0.0, 0.0, 0.0), radius: float = 1.0, seed: int = 11,
                    bumps: float = 0.2):
    """Displaced sphere from a subdivided octahedron: 8 * 4**level triangles, no pole fans."""
    n = 1 << level
    rng = np.random.default_rng(seed)
    ph = rng.uniform(0, 2 * np.pi, 3)
    corners = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]], np.float64)
    octa = [(0, 1, 2), (1, 3, 2), (3, 4, 2), (4, 0, 2), (1, 0, 5), (3, 1, 5), (4, 3, 5), (0, 4, 5)]
    verts, faces = [], []
    for a, b, c in octa:
        A, B, Cc = corners[a], corners[b], corners[c]
        base = len(verts)
        idx = {}
        for i in range(n + 1):
            for j in range(n + 1 - i):
                idx[(i, j)] = len(verts)
                verts.append(A + (B - A) * (i / n) + (Cc - A) * (j / n))
        for i in range(n):
            for j in range(n - i):
                faces.append((idx[(i, j)], idx[(i + 1, j)], idx[(i, j + 1)]))
                if j < n - i - 1:
                    faces.append((idx[(i + 1, j)], idx[(i + 1, j + 1)], idx[(i, j + 1)]))
        del base
    V = np.array(verts)
    V /= np.linalg.norm(V, axis=1, keepdims=True)
    th = np.arccos(np.clip(V[:, 1], -1, 1))
    lo = np.arctan2(V[:, 2], V[:, 0])
    rad = radius * (1 + bumps * (np.sin(3 * th + ph[0]) * np.cos(4 * lo + ph[1]) + 0.4 * np.sin(9 * th + 7 * lo + ph[2])))
    V = V * rad[:, None] + np.asarray(center)
    return np.round(V, 6).astype(np.float32), np.array(faces, np.int32)


def tree_mesh(K: int = 10000, seed: int = 11):
    """Trunk (open cylinder) + crown (displaced octasphere, 8*4^level faces close to K) in
    one mesh, base at y=0."""
    level = max(1, int(round(np.log(max(K, 8) / 8.0) / np.log(4.0))))
    # base geometry in the positive octant (x, z in [0.3, 1.7]); the instances translate it
    # back.  The reference's node bboxes start from max = FLT_MIN (parser.cpp:1393,
    # mesh.cpp RecomputeBoundingBox), so a node whose faces all lie at negative
    # coordinates gets a box reaching 0, its midpoint falls outside every centroid and
    # the split gives up: leaves of thousands of faces.
    cv, cf = octasphere_mesh(level, center=(1.0, 1.6, 1.0), radius=0.7, seed=seed)
    # trunk: 12 rings (short triangles: a long sliver widens its node's box past every
    # centroid and the reference's midpoint split gives up, mesh.cpp:105-106)
    m, rings = 48, 12
    a = np.linspace(0, 2 * np.pi, m, endpoint=False)
    hs = np.linspace(0.0, 1.0, rings + 1)
    rad = 0.12 - 0.03 * hs
    tv = np.concatenate([np.stack([1.0 + rr * np.cos(a), np.full(m, h), 1.0 + rr * np.sin(a)], -1)
                         for h, rr in zip(hs, rad)])
    tv = np.round(tv, 6).astype(np.float32)
    i0 = np.arange(m)
    i1 = np.roll(i0, -1)
    tf = np.concatenate([np.concatenate([np.stack([i0, i1, i1 + m], -1), np.stack([i0, i1 + m, i0 + m], -1)]) + k * m
                         for k in range(rings)])
    verts = np.concatenate([cv, tv])
    faces = np.concatenate([cf, tf + len(cv)]).astype(np.int32)
    return verts, faces


def config_c4(out_dir: str, n_side: int = 10, K_tree: int = 10000, width: int = 1920, height: int = 1080,
              spp: int = 16) -> str:
    """C4: a ~10k-triangle tree x n_side^2 MeshInstances (~1M effective triangles) with
    placements composed from single-digit transform ids (parser.cpp:663,689,699): x and
    z offsets are binary sums of t1-t4 / t5-t8, orientation r1-r9, scale s1-s3;
    SphericalDirectionalLight with a synthetic sky (inputs/c4_sky.ppm), TorranceSparrow
    with kdfresnel, 16 spp.  The reference itself cannot render it: CastShadowRay reads the
    uninitialised Shape::material_id of every InstancedMesh (tests/golden/make_goldens.py)."""
    os.makedirs(os.path.join(out_dir, "inputs"), exist_ok=True)
    v, f = tree_mesh(K_tree)
    write_ply(os.path.join(out_dir, "c4_tree.ply"), v, f)
    # sky: vertical gradient + a sun blob (LDR, 0..255)
    H, W = 128, 256
    yy, xx = np.mgrid[0:H, 0:W]
    sky = np.stack([60 + 120 * (1 - yy / H), 90 + 110 * (1 - yy / H), 140 + 100 * (1 - yy / H)], -1)
    sun = np.exp(-(((xx - 0.3 * W) / 9.0) ** 2 + ((yy - 0.25 * H) / 9.0) ** 2))[..., None] * 255
    write_ppm(os.path.join(out_dir, "inputs", "c4_sky.ppm"), sky + sun)
    step = 2.0
    trans = "\n".join([f'        <Translation id="{k + 1}">{step * (1 << k)} 0 0</Translation>' for k in range(4)] +
                      [f'        <Translation id="{k + 5}">0 0 {-step * (1 << k)}</Translation>' for k in range(4)] +
                      [f'        <Translation id="9">{-step * (n_side - 1) / 2 - 1.0} 0 {step * 2 - 1.0}</Translation>'])
    rots = "\n".join(f'        <Rotation id="{k + 1}">{40 * k} 0 1 0</Rotation>' for k in range(9))
    scls = ('        <Scaling id="1">1 1 1</Scaling>\n        <Scaling id="2">1.15 1.25 1.15</Scaling>\n'
            '        <Scaling id="3">0.85 0.8 0.85</Scaling>')
    inst = []
    for i in range(n_side):
        for j in range(n_side):
            k = i * n_side + j
            ts = [f"t{b + 1}" for b in range(4) if (j >> b) & 1] + [f"t{b + 5}" for b in range(4) if (i >> b) & 1]
            tr = " ".join([f"s{1 + k % 3}", f"r{1 + (7 * k) % 9}"] + ts + ["t9"])
            inst.append(f'        <MeshInstance id="{100 + k}" baseMeshId="1">\n'
                        f'            <Material>{1 + k % 2}</Material>\n'
                        f'            <Transformations>{tr}</Transformations>\n'
                        f'        </MeshInstance>')
    gv, gf = _ground(60.0)
    xml = f"""<Scene>
    <MaxRecursionDepth>1</MaxRecursionDepth>
    <BackgroundColor>0 0 0</BackgroundColor>
    <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
{_lookat_camera((0, 6.0, 8.0), (0, 0.5, -8.0), (0, 1, 0), 50, (width, height), 'c4.png', spp)}
    <Lights>
        <AmbientLight>10 10 10</AmbientLight>
        <PointLight id="1">
            <Position>10 30 10</Position>
            <Intensity>250000 240000 230000</Intensity>
        </PointLight>
        <SphericalDirectionalLight id="1">
            <ImageId>1</ImageId>
        </SphericalDirectionalLight>
    </Lights>
    <Textures>
        <Images>
            <Image id="1">c4_sky.ppm</Image>
        </Images>
    </Textures>
    <BRDFs>
        <TorranceSparrow id="1" kdfresnel="true">
            <Exponent>30</Exponent>
        </TorranceSparrow>
    </BRDFs>
    <Materials>
        <Material id="1" BRDF="1">
            <AmbientReflectance>0.1 0.1 0.1</AmbientReflectance>
            <DiffuseReflectance>0.2 0.45 0.15</DiffuseReflectance>
            <SpecularReflectance>0.2 0.2 0.2</SpecularReflectance>
            <RefractionIndex>1.4</RefractionIndex>
        </Material>
        <Material id="2" BRDF="1">
            <AmbientReflectance>0.1 0.1 0.1</AmbientReflectance>
            <DiffuseReflectance>0.35 0.4 0.1</DiffuseReflectance>
            <SpecularReflectance>0.2 0.2 0.2</SpecularReflectance>
            <RefractionIndex>1.4</RefractionIndex>
        </Material>
        <Material id="3">
            <AmbientReflectance>0.1 0.1 0.1</AmbientReflectance>
            <DiffuseReflectance>0.3 0.25 0.2</DiffuseReflectance>
            <SpecularReflectance>0 0 0</SpecularReflectance>
        </Material>
    </Materials>
    <Transformations>
{trans}
{rots}
{scls}
    </Transformations>
    <VertexData>
        {gv}
    </VertexData>
    <Objects>
        <Mesh id="1">
            <Material>1</Material>
            <Faces plyFile="c4_tree.ply"/>
        </Mesh>
        <Mesh id="2">
            <Material>3</Material>
            <Faces>
                {gf}
            </Faces>
        </Mesh>
{chr(10).join(inst)}
    </Objects>
</Scene>
"""
    return _write(out_dir, "c4_forest", xml)


def config_c5(out_dir: str, K: int = 870000, width: int = 3840, height: int = 2160, spp: int = 64,
              depth: int = 5) -> str:
    """C5: ~870k-triangle closed mesh ("dragon" stand-in: a displaced, tilted torus) as a
    dielectric, a mirror sphere, a Perlin replace_kd ground, reflect/refract depth 5,
    3840x2160, 64 spp.  No area light, roughness or DOF: deterministic."""
    os.makedirs(out_dir, exist_ok=True)
    v, f = torus_mesh(K, center=(0, 1.1, 0), R=1.0, r=0.42, seed=5)
    write_ply(os.path.join(out_dir, "c5_dragon.ply"), v, f)
    gv, gf = _ground(12.0)
    xml = f"""<Scene>
    <MaxRecursionDepth>{depth}</MaxRecursionDepth>
    <BackgroundColor>20 25 40</BackgroundColor>
    <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
{_lookat_camera((0, 2.0, 5.0), (0, 0.9, 0), (0, 1, 0), 40, (width, height), 'c5.png', spp)}
    <Lights>
        <AmbientLight>15 15 15</AmbientLight>
        <PointLight id="1">
            <Position>3 6 4</Position>
            <Intensity>3000 2900 2800</Intensity>
        </PointLight>
        <PointLight id="2">
            <Position>-4 5 -2</Position>
            <Intensity>1500 1600 1800</Intensity>
        </PointLight>
    </Lights>
    <Materials>
        <Material id="1" type="dielectric">
            <AmbientReflectance>0 0 0</AmbientReflectance>
            <DiffuseReflectance>0 0 0</DiffuseReflectance>
            <SpecularReflectance>0 0 0</SpecularReflectance>
            <AbsorptionCoefficient>0.01 0.05 0.1</AbsorptionCoefficient>
            <RefractionIndex>1.5</RefractionIndex>
        </Material>
        <Material id="2" type="mirror">
            <AmbientReflectance>0 0 0</AmbientReflectance>
            <DiffuseReflectance>0.05 0.05 0.05</DiffuseReflectance>
            <SpecularReflectance>0 0 0</SpecularReflectance>
            <MirrorReflectance>0.85 0.85 0.9</MirrorReflectance>
        </Material>
        <Material id="3">
            <AmbientReflectance>0.5 0.5 0.5</AmbientReflectance>
            <DiffuseReflectance>0.6 0.6 0.6</DiffuseReflectance>
            <SpecularReflectance>0.2 0.2 0.2</SpecularReflectance>
            <PhongExponent>10</PhongExponent>
        </Material>
    </Materials>
    <Textures>
        <TextureMap id="1" type="perlin">
            <DecalMode>replace_kd</DecalMode>
            <NoiseConversion>absval</NoiseConversion>
            <NoiseScale>1.5</NoiseScale>
        </TextureMap>
    </Textures>
    <VertexData>
        {gv}
        -2.2 0.8 -1.5
    </VertexData>
    <Objects>
        <Mesh id="1">
            <Material>1</Material>
            <Faces plyFile="c5_dragon.ply"/>
        </Mesh>
        <Mesh id="2">
            <Material>3</Material>
            <Textures>1</Textures>
            <Faces>
                {gf}
            </Faces>
        </Mesh>
        <Sphere id="1">
            <Material>2</Material>
            <Center>5</Center>
            <Radius>0.8</Radius>
        </Sphere>
    </Objects>
</Scene>
"""
    return _write(out_dir, "c5_dragon", xml)
