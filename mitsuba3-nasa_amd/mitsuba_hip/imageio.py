"""Film / bitmap file formats (src/core/bitmap.cpp,
src/films/hdrfilm.cpp:407-590, src/python/python/util.py write_bitmap).

  * OpenEXR: single-part scanline files, FLOAT or HALF channels,
    NO_COMPRESSION / ZIPS / ZIP (zlib with the OpenEXR byte interleave and
    delta predictor).  Channels are stored in alphabetical order as the
    format requires; the channel names follow hdrfilm (R,G,B / Y / X,Y,Z).
  * PFM: 'PF' / 'Pf', little endian (negative scale), bottom-to-top rows.
  * PNG (8-bit, sRGB transfer curve, written with zlib) for previews.
Readers exist for the three so that renders round-trip and bitmap textures
can be loaded from files.
"""
from __future__ import annotations

import os
import struct
import zlib
from typing import Optional, Sequence

import numpy as np

_EXR_MAGIC = 20000630
_COMP = {"none": 0, "zips": 2, "zip": 3}
_LINES = {0: 1, 2: 1, 3: 16}


def _default_channels(c: int):
    return {1: ["Y"], 2: ["Y", "A"], 3: ["R", "G", "B"], 4: ["R", "G", "B", "A"]}.get(c) or \
        [f"ch{i}" for i in range(c)]


# ---------------------------------------------------------------------------
# OpenEXR
# ---------------------------------------------------------------------------
def _attr(name: str, ty: str, payload: bytes) -> bytes:
    return name.encode() + b"\0" + ty.encode() + b"\0" + struct.pack("<i", len(payload)) + payload


def _zip_encode(raw: bytes) -> bytes:
    a = np.frombuffer(raw, np.uint8)
    t = np.concatenate([a[0::2], a[1::2]])
    d = t.astype(np.int16)
    d[1:] = (t[1:].astype(np.int16) - t[:-1].astype(np.int16) + 128 + 256) & 0xFF
    return zlib.compress(d.astype(np.uint8).tobytes())


def _zip_decode(data: bytes, n: int) -> bytes:
    t = np.frombuffer(zlib.decompress(data), np.uint8).astype(np.int32)
    if len(t) != n:
        raise RuntimeError("read_exr: corrupt ZIP block")
    t = (np.cumsum(np.concatenate([t[:1], t[1:] - 128])) & 0xFF).astype(np.uint8)
    half = (n + 1) // 2
    out = np.empty(n, np.uint8)
    out[0::2] = t[:half]
    out[1::2] = t[half:]
    return out.tobytes()


def write_exr(path, img, channels: Optional[Sequence[str]] = None, half: bool = False,
              compression: str = "zip"):
    img = np.asarray(img, np.float32)
    if img.ndim == 2:
        img = img[..., None]
    H, W, C = img.shape
    names = list(channels) if channels is not None else _default_channels(C)
    if len(names) != C:
        raise ValueError("write_exr: channel name count mismatch")
    comp = _COMP[compression]
    order = sorted(range(C), key=lambda i: names[i])
    ptype, dt = (1, "<f2") if half else (2, "<f4")
    chl = b"".join(names[i].encode() + b"\0" + struct.pack("<iB3xii", ptype, 0, 1, 1) for i in order) + b"\0"
    box = struct.pack("<iiii", 0, 0, W - 1, H - 1)
    header = (struct.pack("<ii", _EXR_MAGIC, 2) +
              _attr("channels", "chlist", chl) + _attr("compression", "compression", bytes([comp])) +
              _attr("dataWindow", "box2i", box) + _attr("displayWindow", "box2i", box) +
              _attr("lineOrder", "lineOrder", b"\0") + _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0)) +
              _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0)) +
              _attr("screenWindowWidth", "float", struct.pack("<f", 1.0)) + b"\0")
    planes = img[..., order].astype(dt)                 # (H, W, C) in file channel order
    lines = _LINES[comp]
    chunks = []
    for y0 in range(0, H, lines):
        blk = planes[y0:y0 + lines]                      # (l, W, C) -> per line, per channel
        raw = np.ascontiguousarray(blk.transpose(0, 2, 1)).tobytes()
        data = raw
        if comp:
            z = _zip_encode(raw)
            data = z if len(z) < len(raw) else raw
        chunks.append(struct.pack("<ii", y0, len(data)) + data)
    off = len(header) + 8 * len(chunks)
    table = []
    for c in chunks:
        table.append(struct.pack("<Q", off))
        off += len(c)
    with open(path, "wb") as f:
        f.write(header + b"".join(table) + b"".join(chunks))


def read_exr(path):
    """Returns (image (H, W, C) float32, channel names in file order)."""
    b = open(path, "rb").read()
    magic, ver = struct.unpack_from("<ii", b, 0)
    if magic != _EXR_MAGIC or (ver & 0xFF) != 2 or ver & 0x200:
        raise RuntimeError(f'read_exr: "{os.path.basename(str(path))}" is not a single-part scanline OpenEXR file')
    p = 8
    attrs = {}
    while b[p] != 0:
        e = b.index(b"\0", p)
        name = b[p:e].decode()
        e2 = b.index(b"\0", e + 1)
        ty = b[e + 1:e2].decode()
        (n,) = struct.unpack_from("<i", b, e2 + 1)
        attrs[name] = (ty, b[e2 + 5:e2 + 5 + n])
        p = e2 + 5 + n
    p += 1
    chl = attrs["channels"][1]
    chans, q = [], 0
    while chl[q] != 0:
        e = chl.index(b"\0", q)
        ptype, _, xs, ys = struct.unpack_from("<iB3xii", chl, e + 1)
        if xs != 1 or ys != 1 or ptype not in (1, 2):
            raise RuntimeError("read_exr: only FLOAT/HALF channels without subsampling are supported")
        chans.append((chl[q:e].decode(), ptype))
        q = e + 17
    comp = attrs["compression"][1][0]
    if comp not in _LINES:
        raise RuntimeError(f"read_exr: unsupported compression {comp}")
    x0, y0, x1, y1 = struct.unpack("<iiii", attrs["dataWindow"][1])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    lines = _LINES[comp]
    n_chunks = (H + lines - 1) // lines
    offs = struct.unpack_from(f"<{n_chunks}Q", b, p)
    img = np.zeros((H, W, len(chans)), np.float32)
    bpp = [2 if t == 1 else 4 for _, t in chans]
    for o in offs:
        y, n = struct.unpack_from("<ii", b, o)
        nl = min(lines, y1 - y + 1)
        size = nl * W * sum(bpp)
        data = b[o + 8:o + 8 + n]
        if comp and n < size:
            data = _zip_decode(data, size)
        a = 0
        for li in range(nl):
            for ci, (_, t) in enumerate(chans):
                k = W * bpp[ci]
                img[y - y0 + li, :, ci] = np.frombuffer(data[a:a + k], "<f2" if t == 1 else "<f4")
                a += k
    return img, [c for c, _ in chans]


# ---------------------------------------------------------------------------
# PFM
# ---------------------------------------------------------------------------
def write_pfm(path, img):
    img = np.asarray(img, np.float32)
    if img.ndim == 3 and img.shape[2] == 1:
        img = img[..., 0]
    color = img.ndim == 3
    if color and img.shape[2] != 3:
        raise ValueError("write_pfm: 1 or 3 channels")
    H, W = img.shape[:2]
    with open(path, "wb") as f:
        f.write(b"PF\n" if color else b"Pf\n")
        f.write(f"{W} {H}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(img[::-1]).astype("<f4").tobytes())


def read_pfm(path):
    with open(path, "rb") as f:
        tag = f.readline().strip()
        W, H = (int(x) for x in f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4")
    c = 3 if tag == b"PF" else 1
    return data.reshape(H, W, c)[::-1].astype(np.float32).copy()


# ---------------------------------------------------------------------------
# PNG (8-bit sRGB)
# ---------------------------------------------------------------------------
def linear_to_srgb(x):
    """spectrum.h linear_to_srgb (IEC 61966-2-1)."""
    x = np.asarray(x, np.float64)
    return np.where(x <= 0.0031308, 12.92 * x, 1.055 * np.power(np.maximum(x, 0), 1 / 2.4) - 0.055)


def srgb_to_linear(x):
    x = np.asarray(x, np.float64)
    return np.where(x <= 0.04045, x / 12.92, np.power((x + 0.055) / 1.055, 2.4))


def write_png(path, img, srgb: bool = True):
    img = np.asarray(img, np.float32)
    if img.ndim == 2:
        img = img[..., None]
    H, W, C = img.shape
    v = linear_to_srgb(img) if srgb else img
    q = np.clip(np.round(v * 255.0), 0, 255).astype(np.uint8)
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[C]
    raw = b"".join(b"\0" + q[y].tobytes() for y in range(H))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, ctype, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b""))


# ---------------------------------------------------------------------------
# dispatch (util.py write_bitmap / Bitmap(filename))
# ---------------------------------------------------------------------------
def write_bitmap(path, img, channels=None):
    ext = os.path.splitext(str(path))[1].lower()
    if hasattr(img, "detach"):
        img = img.detach().cpu().numpy()
    if ext == ".exr":
        write_exr(path, img, channels)
    elif ext == ".pfm":
        write_pfm(path, img)
    elif ext == ".png":
        write_png(path, img)
    elif ext == ".npy":
        np.save(path, np.asarray(img, np.float32))
    else:
        raise RuntimeError(f'write_bitmap: unsupported file format "{ext}"')


def read_bitmap(path, raw: bool = False):
    """Image as float32 (H, W, C); 8-bit sRGB images are linearised unless raw."""
    ext = os.path.splitext(str(path))[1].lower()
    if ext == ".exr":
        img, names = read_exr(path)
        for want in (["R", "G", "B", "A"], ["R", "G", "B"], ["X", "Y", "Z"], ["Y", "A"], ["Y"]):
            if set(want) <= set(names):
                return img[..., [names.index(c) for c in want]]
        return img
    if ext == ".pfm":
        return read_pfm(path)
    if ext == ".npy":
        return np.load(path, allow_pickle=False).astype(np.float32)
    if ext in (".png", ".jpg", ".jpeg", ".bmp", ".tga"):
        from PIL import Image
        a = np.asarray(Image.open(path)).astype(np.float64) / 255.0
        if a.ndim == 2:
            a = a[..., None]
        if not raw:
            a[..., :3] = srgb_to_linear(a[..., :3])
        return a.astype(np.float32)
    raise RuntimeError(f'read_bitmap: unsupported file format "{ext}"')
