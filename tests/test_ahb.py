"""The shadow rays' any-hit trees (rtg_ahb.cpp), built on the host exactly as rtg_scene_create
builds them, checked structurally on every fixture scene in the three modes (0: the reference's
BVH collapsed, 1: the default, binned SAH over its leaves, 2: opt-in, large leaves split into single
faces): every face of a mesh reached by exactly one leaf entry naming its reference leaf, child
boxes nested in their parent slot's box, every entry's triangle inside its leaf slot's box
(rtg_desc_anyhit_check).  The traversal answer against the reference walk is the GPU test
tests/test_gpu_shadow.py."""
import os

import pytest

import oracle_bind as ob
import rtgpu

SCENES = os.path.join(ob.GOLDEN, "scenes")
NAMES = sorted(ob.manifest())


@pytest.fixture(scope="module", autouse=True)
def _cwd():
    old = os.getcwd()
    os.chdir(SCENES)
    yield
    os.chdir(old)


@pytest.mark.parametrize("name", NAMES)
def test_anyhit_tree_structure(name):
    hs = rtgpu.HostScene(name + ".xml")
    faces = hs.counts()["faces"]
    res = [hs.anyhit_check(mode) for mode in (0, 1, 2)]
    for mode, r in enumerate(res):
        assert r["built"] == 1 and r["violations"] == 0, (mode, r)
        assert r["entries"] == faces, (mode, r)
    # the SAH trees are no larger than the collapsed reference; only mode 2 splits leaves
    assert res[1]["nodes"] <= res[0]["nodes"] and res[0]["face_prims"] == res[1]["face_prims"] == 0


def test_anyhit_splits_pole_fans():
    """ton_Roosendaal's mesh has the reference's large leaves (pole fans): split into faces,
    their slivers (kappa > 64) kept on their leaf box."""
    hs = rtgpu.HostScene("ton_roosendaal.xml")
    r = hs.anyhit_check(2)
    assert r["face_prims"] > 1000 and 0 < r["exact_faces"] < r["face_prims"] and r["violations"] == 0


def test_anyhit_headline_size(tmp_path):
    import scenes
    xml = scenes.synthetic_heightfield(str(tmp_path), K=100352)
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        hs = rtgpu.HostScene(xml)
        r = hs.anyhit_check(2)
    finally:
        os.chdir(old)
    assert r["built"] == 1 and r["violations"] == 0 and r["entries"] == 100352
