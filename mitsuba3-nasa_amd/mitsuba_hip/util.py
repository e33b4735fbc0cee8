"""`mi.util` on the hot path (src/python/python/util.py).

The reference's `mi.util` namespace gathers the scene-parameter map
(`SceneParameters`, `traverse`, util.py:23-292), the differentiable render
entry points (`render`, `render_1`, util.py:512-670), the image helpers
(`convert_to_bitmap`, `write_bitmap`, util.py:719-755), the Cornell box
dictionary (util.py:757) and `variant_context` (util.py:895).  Here they are
the same objects the package exports; the two helpers with no other home are
defined below.
"""
import contextlib

import numpy as np

from .imageio import linear_to_srgb, read_bitmap, write_bitmap  # noqa: F401
from .render import SceneParameters, render, render_1, traverse  # noqa: F401
from .scene import cornell_box  # noqa: F401


def convert_to_bitmap(data, uint8_srgb: bool = True):
    """Film tensor -> HxWxC array (util.py:719-736).

    `uint8_srgb` applies the sRGB curve and quantises to uint8 as the
    reference's `Bitmap.convert(..., srgb_gamma=True)` does; otherwise the
    linear float32 values are returned.  Accepts torch tensors (any device)
    and numpy arrays.
    """
    if hasattr(data, "detach"):
        data = data.detach().float().cpu().numpy()
    img = np.asarray(data, dtype=np.float32)
    if img.ndim == 2:
        img = img[:, :, None]
    if img.ndim != 3:
        raise ValueError(f"convert_to_bitmap(): expected an HxW or HxWxC image, got shape {img.shape}")
    if not uint8_srgb:
        return img
    return np.clip(np.rint(linear_to_srgb(img) * 255.0), 0, 255).astype(np.uint8)


@contextlib.contextmanager
def variant_context(*names):
    """Temporarily switch variant (util.py:895-915); restores the previous one."""
    import sys

    pkg = sys.modules[__package__]
    prev = pkg.variant()
    pkg.set_variant(*names)
    try:
        yield
    finally:
        pkg._variant = prev
