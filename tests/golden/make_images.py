"""Image-decoder fixtures: small PNG files and the texels the reference's own LDRImage
(stbi_load, LDRImage.h:37-44) reads from them, through `oracle/_ref/refdriver imgdump` (the
reference compiled here, oracle/Makefile).  Writes tests/golden/images/<name>.png and
tests/golden/images/decoded.npz (per fixture: "<name>" texels, "<name>_info" = w, h, c, is_hdr).

The PNG writer below is this script's own: it chooses the scanline filter per row (all five
filter types appear in every fixture), so the loader's unfiltering is exercised whatever zlib
makes of the data.  Colour types: grey (1/2/4/8/16 bit), grey + alpha, RGB (8/16 bit), RGBA,
palette with and without tRNS.  JPEG and OpenEXR are outside the loader (refused
with RTG_ERR_UNSUPPORTED).

    python tests/golden/make_images.py        (needs oracle/_ref/refdriver: make -C oracle)
"""
import os
import struct
import subprocess
import sys
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "images")
REFDRIVER = os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle", "_ref", "refdriver")


def _chunk(typ, body):
    return struct.pack(">I", len(body)) + typ + body + struct.pack(">I", zlib.crc32(typ + body) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = np.abs(p - a), np.abs(p - b), np.abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def _filter_rows(rows, bpp):
    """rows: list of raw scanline byte arrays; filter type of row y = y % 5."""
    out = bytearray()
    prev = np.zeros(len(rows[0]), np.int32)
    for y, r in enumerate(rows):
        cur = np.frombuffer(bytes(r), np.uint8).astype(np.int32)
        a = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]]) if bpp < len(cur) else np.zeros_like(cur)
        c = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]]) if bpp < len(cur) else np.zeros_like(cur)
        f = y % 5
        pred = [np.zeros_like(cur), a, prev, (a + prev) // 2, _paeth(a, prev, c)][f]
        out += bytes([f]) + ((cur - pred) & 255).astype(np.uint8).tobytes()
        prev = cur
    return bytes(out)


def write_png(path, w, h, depth, ctype, rows, palette=None, trns=None):
    samples = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    bpp = max(1, samples * depth // 8)
    body = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 0))
    if palette is not None:
        body += _chunk(b"PLTE", palette)
    if trns is not None:
        body += _chunk(b"tRNS", trns)
    data = zlib.compress(_filter_rows(rows, bpp), 9)
    # two IDAT chunks: the decoder must concatenate them
    body += _chunk(b"IDAT", data[: len(data) // 2]) + _chunk(b"IDAT", data[len(data) // 2:])
    body += _chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(body)


def _pack_bits(vals, depth):
    """One row of sub-byte samples, MSB first."""
    per = 8 // depth
    n = (len(vals) + per - 1) // per
    out = bytearray(n)
    for i, v in enumerate(vals):
        out[i // per] |= int(v) << (8 - depth * (i % per + 1))
    return bytes(out)


def png_fixtures():
    rng = np.random.default_rng(11)
    H, W = 23, 37
    yy, xx = np.mgrid[0:H, 0:W]
    rgb = np.stack([(xx * 255 // W), (yy * 255 // H), ((xx + yy) * 7) % 256], -1).astype(np.uint8)
    rgb[5:12, 10:25] = rng.integers(0, 256, (7, 15, 3), dtype=np.uint8)
    alpha = ((xx * 11 + yy * 5) % 256).astype(np.uint8)
    out = []

    def save(name, w, h, depth, ctype, rows, **kw):
        write_png(os.path.join(OUT, name + ".png"), w, h, depth, ctype, rows, **kw)
        out.append(name + ".png")

    save("png_rgb8", W, H, 8, 2, [rgb[y].tobytes() for y in range(H)])
    save("png_rgba8", W, H, 8, 6, [np.dstack([rgb, alpha])[y].tobytes() for y in range(H)])
    save("png_grey8", W, H, 8, 0, [rgb[y, :, 0].tobytes() for y in range(H)])
    save("png_greya8", W, H, 8, 4, [np.dstack([rgb[..., 1], alpha])[y].tobytes() for y in range(H)])
    rgb16 = (rgb.astype(np.uint16) * 257 + rng.integers(0, 256, rgb.shape)).astype(">u2")
    save("png_rgb16", W, H, 16, 2, [rgb16[y].tobytes() for y in range(H)])
    save("png_grey16", W, H, 16, 0, [rgb16[y, :, 2].tobytes() for y in range(H)])
    for d in (1, 2, 4):
        g = (rgb[..., 0].astype(np.int32) >> (8 - d))
        save(f"png_grey{d}", W, H, d, 0, [_pack_bits(g[y], d) for y in range(H)])
    pal = rng.integers(0, 256, (16, 3), dtype=np.uint8)
    idx = ((xx // 3 + yy // 2) % 16).astype(np.uint8)
    save("png_pal8", W, H, 8, 3, [idx[y].tobytes() for y in range(H)], palette=pal.tobytes())
    save("png_pal4_trns", W, H, 4, 3, [_pack_bits(idx[y], 4) for y in range(H)], palette=pal.tobytes(),
         trns=bytes(range(0, 160, 16)))
    return out


def decode_with_reference(files):
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            b = os.path.join(td, "o.bin")
            subprocess.run([REFDRIVER, "imgdump", os.path.join(OUT, f), b], check=True, stdout=subprocess.DEVNULL)
            raw = open(b, "rb").read()
            assert raw[:4] == b"RTGI"
            w, h, c, hdr = struct.unpack("<4i", raw[4:20])
            res[os.path.splitext(f)[0]] = np.frombuffer(raw[20:], np.float32).reshape(h, w, c).copy()
            res[os.path.splitext(f)[0] + "_info"] = np.array([w, h, c, hdr], np.int32)
    return res


def main():
    os.makedirs(OUT, exist_ok=True)
    for f in os.listdir(OUT):
        if f.endswith((".png", ".jpg", ".exr")):
            os.remove(os.path.join(OUT, f))
    files = png_fixtures()
    np.savez_compressed(os.path.join(OUT, "decoded.npz"), **decode_with_reference(files))
    print("wrote", len(files), "fixtures to", OUT)


if __name__ == "__main__":
    sys.exit(main())
