"""Ordered closest hit (RTG_RENDER_ORDERED: rtg_common.hpp trace_closest_pk on the any-hit tree
as wave packets) against the
reference-order walk it replaces for camera rays of plain mesh scenes.

The reference's IntersectObjects (raytracer.cpp:625-643) walks each BVH left child first
(bvh.cpp:5-30) with minT shrinking.  The ordered walk visits the 4-wide BVH nearest child first
and keeps the minimum (t, object, face) key; its result is checked (the winner's leaf box must
pass the exact slab test at t*, nothing culled within 2^-16 of t*) and the reference walk answers
where the check fails.  The check is not a proof, so these tests MEASURE the
agreement: every golden scene, the shipped scenes' fixtures and the headline at full size must
come out bit-identical, and the number of differing pixels (n_fail) is printed per scene."""
import os

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu

pytestmark = pytest.mark.gpu

SCENES = os.path.join(ob.GOLDEN, "scenes")
NAMES = sorted(ob.manifest())


@pytest.fixture(scope="module", autouse=True)
def _cwd():
    old = os.getcwd()
    os.chdir(SCENES)
    yield
    os.chdir(old)


def _diff(a, b):
    """Pixels whose float RGB bits differ."""
    a = np.ascontiguousarray(a).view(np.uint32).reshape(-1, 3)
    b = np.ascontiguousarray(b).view(np.uint32).reshape(-1, 3)
    return int(np.any(a != b, axis=1).sum())


def _stats(ds, flags):
    ds.reset_stats()
    ds.render(0, flags=flags | rtgpu.RTG_RENDER_COUNT_STATS)
    return ds.stats()


def _check(ds, name):
    hdr, ldr = ds.render(0, seed=5)
    ohdr, oldr = ds.render(0, seed=5, flags=rtgpu.RTG_RENDER_ORDERED)
    n_fail = _diff(hdr, ohdr)
    s = _stats(ds, rtgpu.RTG_RENDER_ORDERED)
    e = _stats(ds, 0)
    print(f"{name}: n_fail {n_fail} of {hdr.size // 3} pixels; camera rays {s['camera_rays']}, "
          f"wide visits/ray {s['extend_wide_visits'] / max(s['camera_rays'], 1):.2f} "
          f"(reference walk: {e['node_visits'] / max(e['camera_rays'], 1):.2f} nodes/ray), "
          f"checked-out rays {s['extend_fallbacks']}")
    assert n_fail == 0 and np.array_equal(ldr, oldr), (name, n_fail)
    return s, e


@pytest.mark.parametrize("name", NAMES)
def test_ordered_equals_reference_order(name):
    hs = rtgpu.HostScene(name + ".xml")
    ds = rtgpu.DeviceScene(hs, 0)
    _check(ds, name)


def test_ordered_headline_full_size(tmp_path):
    """The ordered walk (the any-hit tree as wave packets) on the full headline."""
    import scenes
    xml = scenes.synthetic_heightfield(str(tmp_path), K=100352)
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        hs = rtgpu.HostScene(xml)
        ds = rtgpu.DeviceScene(hs, 0)
        s, e = _check(ds, "headline K=100352 1920x1080")
        # the ordered walk ran (wide nodes counted) and left almost every ray to itself
        assert s["extend_wide_visits"] > 0 and e["extend_wide_visits"] == 0
        assert s["extend_fallbacks"] < 0.02 * s["camera_rays"]
    finally:
        os.chdir(old)
