"""mi.util namespace on the hot path (src/python/python/util.py:23-915): the
re-exported entry points are the package's own, convert_to_bitmap follows the
sRGB / uint8 rule, variant_context restores the previous variant.  CPU only."""
import numpy as np
import pytest

import mitsuba_hip as mi
from mitsuba_hip import util


def test_util_exports_are_the_package_objects():
    assert util.render is mi.render
    assert util.traverse is mi.traverse
    assert util.cornell_box is mi.cornell_box
    for name in ("SceneParameters", "render_1", "write_bitmap", "convert_to_bitmap", "variant_context"):
        assert callable(getattr(util, name))


def test_convert_to_bitmap_srgb_uint8():
    img = np.array([[[0.0, 0.0031308, 0.5], [1.0, 2.0, -1.0]]], np.float32)
    out = util.convert_to_bitmap(img)
    assert out.dtype == np.uint8 and out.shape == (1, 2, 3)
    # IEC 61966-2-1: 0.5 -> 0.7354 -> 188; clamped above 1 and below 0
    assert out[0, 0].tolist() == [0, 10, 188]
    assert out[0, 1].tolist() == [255, 255, 0]
    lin = util.convert_to_bitmap(img, uint8_srgb=False)
    assert lin.dtype == np.float32 and np.array_equal(lin, img)
    assert util.convert_to_bitmap(np.zeros((2, 3), np.float32)).shape == (2, 3, 1)
    with pytest.raises(ValueError):
        util.convert_to_bitmap(np.zeros(4, np.float32))


def test_variant_context_restores():
    prev = mi.variant()
    with util.variant_context("hip_ad_rgb"):
        assert mi.variant() == "hip_ad_rgb"
    assert mi.variant() == prev
    with pytest.raises(ImportError):
        with util.variant_context("cuda_ad_rgb"):
            pass
    assert mi.variant() == prev
