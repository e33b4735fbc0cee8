"""Volume grids: the binary `.vol` format of src/render/volumegrid.cpp:29-125
(reader and writer) and the deterministic fBm density used by the
heterogeneous-medium configuration."""
from __future__ import annotations

import struct

import numpy as np


class VolumeGrid:
    """mi.VolumeGrid: data (z, y, x, channels) float32 + bounding box."""

    def __init__(self, data, bbox_min=(0.0, 0.0, 0.0), bbox_max=(1.0, 1.0, 1.0)):
        arr = np.asarray(data, dtype=np.float32)
        if arr.ndim == 3:
            arr = arr[..., None]
        if arr.ndim != 4:
            raise RuntimeError("VolumeGrid: expected a (z, y, x[, channels]) array")
        self.data = np.ascontiguousarray(arr)
        self.bbox_min = np.asarray(bbox_min, np.float32)
        self.bbox_max = np.asarray(bbox_max, np.float32)

    def size(self):
        z, y, x, _ = self.data.shape
        return (x, y, z)

    def channel_count(self):
        return self.data.shape[3]

    def max(self) -> float:
        return float(self.data.max()) if self.data.size else float("-inf")

    def write(self, path):
        """VolumeGrid::write (volumegrid.cpp:96-121): 'VOL', version 3,
        type 1 (float32), x, y, z, channels, bbox (6 floats), data."""
        x, y, z = self.size()
        with open(path, "wb") as f:
            f.write(b"VOL")
            f.write(struct.pack("<B", 3))
            f.write(struct.pack("<iiiii", 1, x, y, z, self.channel_count()))
            f.write(struct.pack("<6f", *self.bbox_min.tolist(), *self.bbox_max.tolist()))
            f.write(self.data.astype("<f4").tobytes())

    @staticmethod
    def read(path) -> "VolumeGrid":
        """VolumeGrid::read (volumegrid.cpp:29-78)."""
        with open(path, "rb") as f:
            hdr = f.read(3)
            if hdr != b"VOL":
                raise RuntimeError("Invalid volume file!")
            (version,) = struct.unpack("<B", f.read(1))
            if version != 3:
                raise RuntimeError(f"Invalid version, currently only version 3 is supported (found {version})")
            (dtype,) = struct.unpack("<i", f.read(4))
            if dtype != 1:
                raise RuntimeError("Wrong type, currently only type == 1 (Float32) data is "
                                   f"supported (found type = {dtype})")
            x, y, z, c = struct.unpack("<iiii", f.read(16))
            dims = struct.unpack("<6f", f.read(24))
            data = np.frombuffer(f.read(4 * x * y * z * c), dtype="<f4").astype(np.float32)
        if data.size != x * y * z * c:
            raise RuntimeError("Invalid volume file: truncated data")
        return VolumeGrid(data.reshape(z, y, x, c), dims[:3], dims[3:])


def fbm_grid(res: int = 256, seed: int = 1234, octaves: int = 5) -> np.ndarray:
    """Deterministic fractional-Brownian-motion density in [0, 1], shape
    (res, res, res) float32: a sum of `octaves` trilinearly upsampled value-
    noise lattices (numpy default_rng(seed)), amplitude halving per octave,
    normalised to [0, 1], times a smooth spherical falloff."""
    rng = np.random.default_rng(seed)
    acc = np.zeros((res, res, res), np.float64)
    amp, total = 1.0, 0.0
    coords = (np.arange(res) + 0.5) / res
    for o in range(octaves):
        n = 4 * 2 ** o + 1
        lat = rng.random((n, n, n))
        f = coords * (n - 1)
        i0 = np.minimum(np.floor(f).astype(np.int64), n - 2)
        w = f - i0
        # separable trilinear upsampling
        a = lat[i0] * (1 - w)[:, None, None] + lat[i0 + 1] * w[:, None, None]
        a = a[:, i0] * (1 - w)[None, :, None] + a[:, i0 + 1] * w[None, :, None]
        a = a[:, :, i0] * (1 - w)[None, None, :] + a[:, :, i0 + 1] * w[None, None, :]
        acc += amp * a
        total += amp
        amp *= 0.5
    acc /= total
    acc = (acc - acc.min()) / max(acc.max() - acc.min(), 1e-12)
    c = coords * 2 - 1
    r2 = c[:, None, None] ** 2 + c[None, :, None] ** 2 + c[None, None, :] ** 2
    falloff = np.clip(1.25 - r2, 0.0, 1.0)
    return np.clip(acc * falloff, 0.0, 1.0).astype(np.float32)
