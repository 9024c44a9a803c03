"""Image-decoder fixtures: small PNG and OpenEXR files and the texels the reference's own image
classes read from them -- LDRImage (stbi_load, LDRImage.h:37-44) and HDRImage (tinyexr LoadEXR,
HDRImage.h:45-72) -- through `oracle/_ref/refdriver imgdump` (the reference compiled here,
oracle/Makefile).  Writes tests/golden/images/<name>.{png,exr} and
tests/golden/images/decoded.npz (per fixture: "<name>" texels, "<name>_info" = w, h, c, is_hdr).

The EXR writer below is this script's own (single-part scanline files, NONE / RLE / ZIPS / ZIP,
HALF / FLOAT channels, OpenEXR's byte reordering + delta predictor).

The PNG writer below is this script's own: it chooses the scanline filter per row (all five
filter types appear in every fixture), so the loader's unfiltering is exercised whatever zlib
makes of the data.  Colour types: grey (1/2/4/8/16 bit), grey + alpha, RGB (8/16 bit), RGBA,
palette with and without tRNS.  JPEG is outside the loader (refused with RTG_ERR_UNSUPPORTED).

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


def _attr(name, typ, data):
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def _predict(raw):
    """OpenEXR's ZIP / RLE pre-pass: split even / odd bytes, then byte deltas (+128)."""
    b = np.frombuffer(raw, np.uint8)
    t = np.concatenate([b[0::2], b[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128 + 256) & 255
    return d.astype(np.uint8).tobytes()


def _rle(data):
    out = bytearray()
    i, n = 0, len(data)
    while i < n:
        j = i
        while j + 1 < n and data[j + 1] == data[i] and j - i < 127:
            j += 1
        run = j - i + 1
        if run >= 3:
            out += struct.pack("<b", run - 1) + bytes([data[i]])
            i = j + 1
            continue
        k = i
        while k < n and k - i < 127:
            if k + 2 < n and data[k] == data[k + 1] == data[k + 2]:
                break
            k += 1
        out += struct.pack("<b", -(k - i)) + bytes(data[i:k])
        i = k
    return bytes(out)


def write_exr(path, channels, comp=3, line_order=0):
    """channels: {name: (HxW float array, 1 = HALF / 2 = FLOAT)}; comp 0 NONE, 1 RLE, 2 ZIPS, 3 ZIP."""
    names = sorted(channels)
    h, w = next(iter(channels.values()))[0].shape
    chl = b"".join(n.encode() + b"\0" + struct.pack("<iB3xii", channels[n][1], 0, 1, 1) for n in names) + b"\0"
    hdr = (_attr("channels", "chlist", chl) + _attr("compression", "compression", bytes([comp])) +
           _attr("dataWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)) +
           _attr("displayWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)) +
           _attr("lineOrder", "lineOrder", bytes([line_order])) +
           _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0)) +
           _attr("screenWindowCenter", "v2f", struct.pack("<2f", 0.0, 0.0)) +
           _attr("screenWindowWidth", "float", struct.pack("<f", 1.0)) + b"\0")
    lines = 16 if comp == 3 else 1
    chunks = []
    for y0 in range(0, h, lines):
        raw = b""
        for y in range(y0, min(h, y0 + lines)):
            for n in names:
                a, t = channels[n]
                raw += a[y].astype(np.float16 if t == 1 else np.float32).astype("<f2" if t == 1 else "<f4").tobytes()
        if comp in (2, 3):
            data = zlib.compress(_predict(raw), 9)
        elif comp == 1:
            data = _rle(_predict(raw))
        else:
            data = raw
        if len(data) >= len(raw):        # stored when it does not compress (OpenEXR / tinyexr)
            data = raw
        chunks.append(struct.pack("<ii", y0, len(data)) + data)
    head = struct.pack("<Ii", 20000630, 2) + hdr
    off = len(head) + 8 * len(chunks)
    table = b""
    for c in chunks:
        table += struct.pack("<Q", off)
        off += len(c)
    with open(path, "wb") as f:
        f.write(head + table + b"".join(chunks))


def exr_fixtures():
    rng = np.random.default_rng(7)
    H, W = 37, 29
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    smooth = {c: (np.sin(xx * (0.2 + 0.1 * k)) * np.cos(yy * 0.15) * 4.0 + 2.0 * k).astype(np.float32)
              for k, c in enumerate("RGB")}
    noise = {c: (rng.standard_normal((H, W)) * 10 ** rng.uniform(-6, 4, (H, W))).astype(np.float32) for c in "RGBA"}
    # half specials: subnormals, zero, -0, large, inf
    spec = noise["R"].copy()
    spec[0, :6] = [6.0e-8, -6.0e-8, 0.0, -0.0, 65504.0, np.inf]
    fx = {
        "exr_half_zip": ({c: (smooth[c], 1) for c in "RGB"}, 3, 0),
        "exr_float_none_rgba_decreasing": ({c: (noise[c], 2) for c in "RGBA"}, 0, 1),
        "exr_half_zips": ({"R": (spec, 1), "G": (smooth["G"], 1), "B": (noise["B"], 1)}, 2, 0),
        "exr_half_rle": ({c: (np.round(smooth[c]), 1) for c in "RGB"}, 1, 0),
        "exr_float_zip_noise": ({c: (noise[c], 2) for c in "RGB"}, 3, 0),     # incompressible: stored chunks
        "exr_y_float_zip": ({"Y": (smooth["G"], 2)}, 3, 0),                   # one channel -> grey
        "exr_mixed_extra": ({"R": (smooth["R"], 1), "G": (smooth["G"], 2), "B": (smooth["B"], 1),
                             "A": (noise["A"], 1), "Z": (noise["R"], 2)}, 3, 0),
    }
    for name, (ch, comp, lo) in fx.items():
        write_exr(os.path.join(OUT, name + ".exr"), ch, comp, lo)
    return [n + ".exr" for n in fx]


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
    files = png_fixtures() + exr_fixtures()
    np.savez_compressed(os.path.join(OUT, "decoded.npz"), **decode_with_reference(files))
    print("wrote", len(files), "fixtures to", OUT)


if __name__ == "__main__":
    sys.exit(main())
