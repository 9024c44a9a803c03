"""The CPU restatement (oracle) against the reference itself at the 15 shipped scenes' native
resolutions (tests/golden/native, tests/golden/make_native.py): bit for bit -- the float
frame's SHA-256, every 8-bit value, the sampled float pixels.  Pins the oracle the GPU tests
compare against at full size (tests/test_gpu_shipped.py), not only at the reduced golden
sizes."""
import hashlib
import os
import re

import numpy as np
import pytest

import oracle_bind as ob
import rtgpu
from test_gpu_shipped import NATIVE

SCENES = os.path.join(ob.GOLDEN, "scenes")


@pytest.mark.parametrize("name", sorted(NATIVE))
def test_oracle_matches_reference_at_native_resolution(tmp_path, name):
    for f in os.listdir(SCENES):
        if not f.endswith(".xml"):
            os.symlink(os.path.join(SCENES, f), tmp_path / f)
    w, h = NATIVE[name]
    src = open(os.path.join(SCENES, name + ".xml")).read()
    src = re.sub(r"<ImageResolution>[^<]*</ImageResolution>", f"<ImageResolution>{w} {h}</ImageResolution>", src)
    (tmp_path / "native.xml").write_text(src)
    old = os.getcwd()
    os.chdir(tmp_path)
    try:
        hs = rtgpu.HostScene("native.xml")
        hdr, ldr, _ = ob.render(hs)
    finally:
        os.chdir(old)
    g = ob.load_native(name)
    assert hashlib.sha256(hdr.tobytes()).digest() == g["sha256"].tobytes(), ob.compare_native(hdr, ldr, g)
    assert np.array_equal(ldr, g["ldr"])
