"""mitsuba_hip — the `hip_ad_rgb` variant of ksalesin/mitsuba3-nasa on MI355X.

A drop-in for the reference's Python entry points on the `path` / `volpath` /
`prb` hot path (src/python/__init__.py:71-318, src/python/python/util.py):

    import mitsuba_hip as mi
    mi.set_variant('hip_ad_rgb')
    scene = mi.load_dict(mi.cornell_box())
    img = mi.render(scene, spp=256)                  # torch tensor on the GPU
    params = mi.traverse(scene)
    params['white.reflectance.value'].requires_grad_()
    img = mi.render(scene, params, integrator=mi.load_dict({'type': 'prb', 'max_depth': 8}))
    img.mean().backward()                           # == dr.backward(dr.mean(img))

Only `hip_ad_rgb` is compiled into this package; `scalar_rgb` / `llvm_ad_rgb`
are the reference's own variants and are not provided (set_variant raises,
as the reference does for variants that were not compiled).
"""
from __future__ import annotations

from . import _abi
from ._abi import MitsubaHipError
from .render import (SceneParameters, develop, prb_weights, render, render_1, render_backward,
                     render_film, render_forward, sample_tea_32, traverse)
from .scene import Integrator, Scene, cornell_box, gaussian_coefficients, load_dict
from .transform import ScalarTransform4f, Transform4f
from .scenes import cornell_box_bitmap, volume_cube
from .volume import VolumeGrid, fbm_grid
from .xml import load_file, load_string
from . import meshio, imageio, util, ad
from .imageio import write_bitmap, read_bitmap

__version__ = "0.1.0"
MI_VERSION = "3.5.0"  # reference version this backend mirrors (include/mitsuba/mitsuba.h:11-13)

_VARIANTS = ["hip_ad_rgb"]
_variant = None


def variants():
    return list(_VARIANTS)


def set_variant(*names):
    """src/python/__init__.py:287-318 — first available variant wins."""
    global _variant
    for n in names:
        if n in _VARIANTS:
            _variant = n
            return
    raise ImportError(f"Requested an unsupported variant {names}. The following variants are "
                      f"available: {', '.join(_VARIANTS)}.")


def variant():
    return _variant


def is_available() -> bool:
    """True when the native library loads and a HIP device is present."""
    import ctypes
    try:
        n = ctypes.c_int(0)
        _abi.lib().mh_device_count(ctypes.byref(n))
        return n.value > 0
    except Exception:
        return False


__all__ = ["set_variant", "variant", "variants", "load_dict", "cornell_box", "render", "traverse",
           "render_backward", "render_forward", "render_film", "develop", "prb_weights", "SceneParameters", "Scene",
           "Integrator", "Transform4f", "ScalarTransform4f", "sample_tea_32", "MitsubaHipError",
           "gaussian_coefficients", "is_available", "volume_cube", "cornell_box_bitmap", "VolumeGrid", "fbm_grid",
           "load_file", "load_string", "meshio", "imageio",
           "write_bitmap", "read_bitmap", "ad", "render_1"]
