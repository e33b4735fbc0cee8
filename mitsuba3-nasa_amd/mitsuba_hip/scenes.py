"""Scene dictionaries of the benchmark configurations.

`volume_cube` is configuration 4, the NASA radiative-transfer case the
reference ships no scene for: a `null`-BSDF cube [-1, 1]^3 bounding a
heterogeneous medium (sigma_t = fBm `gridvolume`, scale 20, albedo 0.9,
Henyey-Greenstein g = 0.85) lit by a `constant` sky (0.2) and a
`directional` sun (irradiance 5 along (0, -1, -0.3)), seen from (0, 0, 4)."""
from __future__ import annotations

from typing import Optional

import numpy as np

from .scene import cornell_box
from .transform import Transform4f
from .volume import fbm_grid


def cornell_box_bitmap(tex_res: int = 64, width: int = 512, height: int = 512, spp: int = 64):
    """Configuration 3(b): cornell_box with white's
    reflectance replaced by a tex_res^2 x 3 `bitmap` initialised to the
    constant (0.885809, 0.698859, 0.666422); key 'white.reflectance.data'."""
    d = cornell_box()
    white = np.asarray(d["white"]["reflectance"]["value"], np.float32)
    d["white"]["reflectance"] = {"type": "bitmap", "data": np.tile(white, (tex_res, tex_res, 1)),
                                 "filter_type": "bilinear", "wrap_mode": "repeat", "raw": True}
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = width, height
    d["sensor"]["sampler"]["sample_count"] = spp
    return d


def volume_cube(width: int = 256, height: int = 256, spp: int = 64, grid: Optional[np.ndarray] = None,
                grid_res: int = 256, scale: float = 20.0, albedo=0.9, g: float = 0.85,
                max_depth: int = 64, rr_depth: int = 5, sky: float = 0.2, sun: Optional[float] = 5.0,
                sun_dir=(0.0, -1.0, -0.3), medium_type: str = "heterogeneous", sigma_t: float = 1.0,
                fov: float = 39.3077):
    T = Transform4f
    if medium_type == "heterogeneous":
        if grid is None:
            grid = fbm_grid(grid_res)
        med = {"type": "heterogeneous",
               "sigma_t": {"type": "gridvolume", "data": grid,
                           "to_world": T.translate([-1.0, -1.0, -1.0]) @ T.scale([2.0, 2.0, 2.0])},
               "scale": scale, "albedo": albedo, "phase": {"type": "hg", "g": g}}
    else:
        med = {"type": "homogeneous", "sigma_t": sigma_t, "scale": scale, "albedo": albedo,
               "phase": {"type": "hg", "g": g} if g != 0.0 else {"type": "isotropic"}}
    d = {
        "type": "scene",
        "integrator": {"type": "volpath", "max_depth": max_depth, "rr_depth": rr_depth},
        "sensor": {
            "type": "perspective", "fov_axis": "smaller", "fov": fov, "near_clip": 0.001, "far_clip": 100.0,
            "to_world": T.look_at(origin=[0, 0, 4], target=[0, 0, 0], up=[0, 1, 0]),
            "sampler": {"type": "independent", "sample_count": spp},
            "film": {"type": "hdrfilm", "width": width, "height": height, "rfilter": {"type": "gaussian"}},
        },
        "medium1": med,
        "cube": {"type": "cube", "bsdf": {"type": "null"}, "interior": {"type": "ref", "id": "medium1"}},
        "sky": {"type": "constant", "radiance": {"type": "rgb", "value": sky}},
    }
    if sun is not None:
        d["sun"] = {"type": "directional", "direction": list(sun_dir), "irradiance": {"type": "rgb", "value": sun}}
    return d
