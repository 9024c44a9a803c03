"""Native-resolution goldens of the 15 shipped scenes (tests/test_gpu_shipped.py NATIVE): the
reference itself (oracle/_ref/refdriver dump: Raytracer::RenderPixel per pixel, the reference's
own sources compiled here) at each scene's shipped <ImageResolution> -- up to 1080x1920.

A full float frame is 25 MB, too big to keep per scene, so each golden stores
  * ldr: the whole 8-bit frame clamp((int)c) (main.cpp:121), compressed -- every pixel;
  * the float frame at a fixed pseudo-random sample of 8192 pixels (sample_idx, sample_hdr):
    the parity bound |gpu - ref| <= 1e-4 max(1, |ref|) is checked there at full precision;
  * row_sums: the float frame's per-row sums (float64) -- a checksum of the whole frame;
  * sha256 of the float frame.
Written to tests/golden/native/<name>.npz.  Runs only where /root/reference is (refdriver).

    python tests/golden/make_native.py [name ...]
"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SCENES = os.path.join(HERE, "scenes")
OUT = os.path.join(HERE, "native")
DRIVER = os.path.join(ROOT, "oracle", "_ref", "refdriver")
sys.path.insert(0, os.path.join(ROOT, "tests"))
NSAMPLE = 8192


def native_sizes():
    src = open(os.path.join(ROOT, "tests", "test_gpu_shipped.py")).read()
    body = src[src.index("NATIVE = {"):src.index("}", src.index("NATIVE = {")) + 1]
    return {k: (int(w), int(h)) for k, w, h in re.findall(r'"(\w+)": \((\d+), (\d+)\)', body)}


def clamp_ldr(hdr):
    # x86 cvttss2si + clamp (helperMath.cpp:140-152): NaN / out of range -> INT_MIN -> 0
    x = np.where(np.isfinite(hdr) & (hdr > -2147483904.0) & (hdr < 2147483648.0), hdr, -1.0)
    return np.clip(np.trunc(x), 0, 255).astype(np.uint8)


def sample_indices(h, w):
    rng = np.random.default_rng(20261017)
    return np.sort(rng.choice(h * w, size=min(NSAMPLE, h * w), replace=False)).astype(np.int64)


def make(name, w, h):
    with tempfile.TemporaryDirectory() as td:
        for f in os.listdir(SCENES):
            if not f.endswith(".xml"):
                os.symlink(os.path.join(SCENES, f), os.path.join(td, f))
        src = open(os.path.join(SCENES, name + ".xml")).read()
        src = re.sub(r"<ImageResolution>[^<]*</ImageResolution>", f"<ImageResolution>{w} {h}</ImageResolution>", src)
        open(os.path.join(td, "native.xml"), "w").write(src)
        out = os.path.join(td, "o.bin")
        subprocess.run([DRIVER, "dump", "native.xml", out], cwd=td, check=True, stdout=subprocess.DEVNULL)
        raw = open(out, "rb").read()
    assert raw[:4] == b"RTGF"
    ww, hh = np.frombuffer(raw[4:12], np.int32)
    assert (ww, hh) == (w, h), (name, ww, hh)
    hdr = np.frombuffer(raw[12:], np.float32).reshape(h, w, 3)
    idx = sample_indices(h, w)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), ldr=clamp_ldr(hdr), sample_idx=idx,
                        sample_hdr=hdr.reshape(-1, 3)[idx].copy(), row_sums=hdr.astype(np.float64).sum(axis=(1, 2)),
                        sha256=np.frombuffer(hashlib.sha256(hdr.tobytes()).digest(), np.uint8))
    return name, os.path.getsize(os.path.join(OUT, name + ".npz"))


def main():
    if not os.path.exists(DRIVER):
        sys.exit(f"{DRIVER} missing: make -C oracle (needs /root/reference)")
    os.makedirs(OUT, exist_ok=True)
    sizes = native_sizes()
    names = sys.argv[1:] or sorted(sizes)
    with ThreadPoolExecutor(max_workers=6) as ex:
        for name, nbytes in ex.map(lambda n: make(n, *sizes[n]), names):
            print(name, sizes[name], nbytes, "bytes", flush=True)


if __name__ == "__main__":
    main()
