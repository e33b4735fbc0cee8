"""Scene dictionary loader -> flattened ``mh_scene_desc``.

Restates, for the plugins on the hot path, what ``mi.load_dict`` does in the
reference (src/core/python/xml_v.cpp:112, plugin constructors) and then
flattens the result into the C-ABI description of include/mitsuba_hip.h.
Plugin names, property names and traverse() keys follow the reference:

  perspective  src/sensors/perspective.cpp:131-184, render/sensor.cpp:149-196
  hdrfilm      src/films/hdrfilm.cpp          gaussian  src/rfilters/gaussian.cpp:48-92
  independent  src/samplers/independent.cpp   rectangle src/shapes/rectangle.cpp:98-126
  cube         src/shapes/cube.cpp:104-160    diffuse   src/bsdfs/diffuse.cpp:90-99
  rgb          src/spectra/srgb.cpp:48-90     bitmap    src/textures/bitmap.cpp:156-310
  area         src/emitters/area.cpp:62-80    path/volpath/prb integrators
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Any, Dict, List, Optional

import numpy as np

from . import _abi as A
from .transform import Transform4f


def _f32(x):
    return np.asarray(x, dtype=np.float32)


def _normalize32(v):
    """dr::normalize in float32: v * rsqrt(dot(v, v)), dot as an fmadd chain."""
    v = _f32(v)
    d = np.float32(np.float64(v[2]) * np.float64(v[2]) +
                   np.float64(np.float32(np.float64(v[1]) * np.float64(v[1]) + np.float64(np.float32(v[0] * v[0])))))
    return (v * np.float32(np.float32(1.0) / np.sqrt(d, dtype=np.float32))).astype(np.float32)


# ---------------------------------------------------------------------------
# Integrators (integrator.cpp:22-28,1281-1298; ad/integrators/common.py:29-41)
# ---------------------------------------------------------------------------
class Integrator:
    TYPES = {"path": A.INTEGRATOR_PATH, "volpath": A.INTEGRATOR_VOLPATH, "prb": A.INTEGRATOR_PRB,
             "prbvolpath": A.INTEGRATOR_PRBVOLPATH}

    def __init__(self, type_: str, props: Dict[str, Any]):
        if type_ not in self.TYPES:
            raise RuntimeError(f'Plugin "{type_}" is not available in the hip_ad_rgb variant')
        self.type = type_
        default_depth = 6 if type_ in ("prb", "prbvolpath") else -1
        max_depth = int(props.get("max_depth", default_depth))
        if max_depth < 0 and max_depth != -1:
            raise RuntimeError('"max_depth" must be set to -1 (infinite) or a value >= 0')
        self.max_depth = 0xFFFFFFFF if max_depth == -1 else max_depth
        self.rr_depth = int(props.get("rr_depth", 5))
        if self.rr_depth <= 0:
            raise RuntimeError('"rr_depth" must be set to a value greater than zero!')
        self.hide_emitters = bool(props.get("hide_emitters", False))

    def c(self) -> A.Integrator:
        return A.Integrator(self.TYPES[self.type], self.max_depth & 0xFFFFFFFF, self.rr_depth,
                            int(self.hide_emitters))

    def __repr__(self):
        return (f"{type(self).__name__}[type={self.type}, max_depth={self.max_depth}, "
                f"rr_depth={self.rr_depth}]")


# ---------------------------------------------------------------------------
# Gaussian filter constants (gaussian.cpp:48-92) — restated in float32
# ---------------------------------------------------------------------------
_REMEZ = [9.992604880e-1, -4.977025247e-1, 1.222248550e-1, -1.932406282e-2,
          2.136713061e-3, -1.679873860e-4, 9.202145248e-6, -3.329417433e-7,
          7.128382794e-9, -6.821193280e-11]


def _fma32(a, b, c):
    return np.float32(np.float64(a) * np.float64(b) + np.float64(c))


def _estrin32(x, k):
    k = [np.float32(v) for v in k]
    x = np.float32(x)
    while len(k) > 1:
        nk = [_fma32(x, k[2 * i + 1], k[2 * i]) for i in range(len(k) // 2)]
        if len(k) % 2:
            nk.append(k[-1])
        k = nk
        x = np.float32(x * x)
    return k[0]


def gaussian_coefficients(stddev: float = 0.5):
    stddev = np.float32(stddev)
    radius = np.float32(4) * stddev
    coeff = []
    scale = 1.0
    for c in _REMEZ:
        coeff.append(np.float32(c * scale))
        scale /= float(stddev) ** 2
    coeff[0] = np.float32(coeff[0] - _estrin32(np.float32(radius * radius), coeff))
    return np.array(coeff, dtype=np.float32), float(radius)


def parse_fov(props: Dict[str, Any], aspect: float) -> float:
    """render/sensor.cpp:149-196"""
    if "fov" in props and "focal_length" in props:
        raise RuntimeError("Please specify either a focal length ('focal_length') or a field of view ('fov')!")
    if "fov" in props:
        fov = float(props["fov"])
        axis = str(props.get("fov_axis", "x")).lower()
        if axis == "smaller":
            axis = "y" if aspect > 1 else "x"
        elif axis == "larger":
            axis = "x" if aspect > 1 else "y"
    else:
        f = str(props.get("focal_length", "50mm"))
        if f.endswith("mm"):
            f = f[:-2]
        fov = 2.0 * math.degrees(math.atan(math.sqrt(36 * 36 + 24 * 24) / (2.0 * float(f))))
        axis = "diagonal"
    if axis == "x":
        return fov
    if axis == "y":
        return math.degrees(2.0 * math.atan(math.tan(0.5 * math.radians(fov)) * aspect))
    if axis == "diagonal":
        diagonal = 2.0 * math.tan(0.5 * math.radians(fov))
        width = diagonal / math.sqrt(1.0 + 1.0 / (aspect * aspect))
        return math.degrees(2.0 * math.atan(width * 0.5))
    raise RuntimeError(f"The 'fov_axis' parameter must be set to one of 'smaller', 'larger', 'diagonal', 'x', or 'y'!")


def perspective_projection(film_size, crop_size, crop_offset, fov_x, near, far) -> Transform4f:
    """render/sensor.h:227-263"""
    fs = np.asarray(film_size, dtype=np.float64)
    rel_size = np.asarray(crop_size, dtype=np.float64) / fs
    rel_offset = np.asarray(crop_offset, dtype=np.float64) / fs
    aspect = fs[0] / fs[1]
    return (Transform4f.scale([1.0 / rel_size[0], 1.0 / rel_size[1], 1.0])
            @ Transform4f.translate([-rel_offset[0], -rel_offset[1], 0.0])
            @ Transform4f.scale([-0.5, -0.5 * aspect, 1.0])
            @ Transform4f.translate([-1.0, -1.0 / aspect, 0.0])
            @ Transform4f.perspective(fov_x, near, far))


# ---------------------------------------------------------------------------
# cube geometry (shapes/cube.cpp:104-130)
# ---------------------------------------------------------------------------
_CUBE_V = [[1, -1, -1], [1, -1, 1], [-1, -1, 1], [-1, -1, -1], [1, 1, -1], [-1, 1, -1],
           [-1, 1, 1], [1, 1, 1], [1, -1, -1], [1, 1, -1], [1, 1, 1], [1, -1, 1],
           [1, -1, 1], [1, 1, 1], [-1, 1, 1], [-1, -1, 1], [-1, -1, 1], [-1, 1, 1],
           [-1, 1, -1], [-1, -1, -1], [1, 1, -1], [1, -1, -1], [-1, -1, -1], [-1, 1, -1]]
_CUBE_N = [[0, -1, 0]] * 4 + [[0, 1, 0]] * 4 + [[1, 0, 0]] * 4 + [[0, 0, 1]] * 4 + \
          [[-1, 0, 0]] * 4 + [[0, 0, -1]] * 4
_CUBE_UV = [[0, 1], [1, 1], [1, 0], [0, 0]] * 6
_CUBE_F = [[0, 1, 2], [3, 0, 2], [4, 5, 6], [7, 4, 6], [8, 9, 10], [11, 8, 10], [12, 13, 14],
           [15, 12, 14], [16, 17, 18], [19, 16, 18], [20, 21, 22], [23, 20, 22]]


def _to_transform(v) -> Transform4f:
    if v is None:
        return Transform4f()
    if isinstance(v, Transform4f):
        return v
    return Transform4f(np.asarray(v, dtype=np.float64).reshape(4, 4))


class _Builder:
    """Accumulates flattened plugin records."""

    def __init__(self):
        self.shapes: List[A.Shape] = []
        self.shape_names: List[str] = []
        self.bsdfs: List[A.Bsdf] = []
        self.textures: List[A.Texture] = []
        self.emitters: List[A.Emitter] = []
        self.positions: List[np.ndarray] = []
        self.normals: List[np.ndarray] = []
        self.texcoords: List[np.ndarray] = []
        self.faces: List[np.ndarray] = []
        self.texels: List[np.ndarray] = []
        self.n_vertices = 0
        self.n_faces = 0
        self.n_texels = 0
        self.bsdf_ids: Dict[str, int] = {}
        self.params: Dict[str, Any] = {}   # key -> ("rgb"|"bitmap", texture index)
        self.any_normals = False
        self.any_texcoords = False
        self.media: List[A.Medium] = []
        self.medium_ids: Dict[str, int] = {}
        self.grids: List[np.ndarray] = []
        self.n_grid = 0
        self.environment = A.INVALID
        self.bbox_min = np.full(3, np.inf, np.float32)   # Scene::bbox() over the shapes
        self.bbox_max = np.full(3, -np.inf, np.float32)

    # -- textures ---------------------------------------------------------------
    def texture(self, spec, key_prefix: str, bounded=True) -> int:
        t = A.Texture()
        t.to_uv[:] = [1, 0, 0, 0, 1, 0]
        if isinstance(spec, (int, float)):
            spec = {"type": "rgb", "value": [float(spec)] * 3}
        elif isinstance(spec, (list, tuple, np.ndarray)) and not isinstance(spec, dict):
            spec = {"type": "rgb", "value": list(np.asarray(spec, dtype=np.float64).reshape(-1))}
        ty = spec.get("type")
        idx = len(self.textures)
        if ty in ("rgb", "srgb"):
            v = spec.get("value", spec.get("color"))
            v = np.broadcast_to(np.asarray(v, dtype=np.float64).reshape(-1), (3,))
            if bounded and (np.any(v < 0) or np.any(v > 1)) and not spec.get("unbounded", False):
                raise RuntimeError(f"Invalid RGB reflectance value {v.tolist()}, must be in the range [0, 1]!")
            t.type = A.TEX_RGB
            t.value[:] = [float(x) for x in v]
            self.params[key_prefix + ".value"] = ("rgb", idx)
        elif ty == "bitmap":
            data = spec.get("data")
            if data is None and "filename" in spec:   # bitmap.cpp: file images (mitsuba_hip/imageio.py)
                from .imageio import read_bitmap
                data = read_bitmap(spec["filename"], raw=bool(spec.get("raw", False)))
                if data.shape[2] == 4:
                    data = data[..., :3]
                elif data.shape[2] == 2:
                    data = data[..., :1]
            if data is None:
                raise RuntimeError("bitmap: specify 'data' or 'filename'")
            arr = np.asarray(data, dtype=np.float32)
            if arr.ndim == 2:
                arr = arr[:, :, None]
            if arr.ndim != 3 or arr.shape[2] not in (1, 3):
                raise RuntimeError("Bitmap raw tensor has dimension %d, expected 3" % arr.ndim)
            filt = spec.get("filter_type", "bilinear")
            wrap = spec.get("wrap_mode", "repeat")
            if filt not in ("nearest", "bilinear"):
                raise RuntimeError('Invalid filter type "%s", must be one of: "nearest", or "bilinear"!' % filt)
            if wrap not in ("repeat", "mirror", "clamp"):
                raise RuntimeError('Invalid wrap mode "%s", must be one of: "repeat", "mirror", or "clamp"!' % wrap)
            t.type = A.TEX_BITMAP
            t.height, t.width, t.channels = arr.shape
            t.data_offset = self.n_texels
            t.filter = 0 if filt == "nearest" else 1
            t.wrap = {"repeat": 0, "mirror": 1, "clamp": 2}[wrap]
            if "to_uv" in spec:
                m = _to_transform(spec["to_uv"]).matrix
                t.to_uv[:] = [m[0, 0], m[0, 1], m[0, 3], m[1, 0], m[1, 1], m[1, 3]]
            self.texels.append(np.ascontiguousarray(arr.reshape(-1)))
            self.n_texels += arr.size
            self.params[key_prefix + ".data"] = ("bitmap", idx)
        else:
            raise RuntimeError(f'Texture plugin "{ty}" is not available in the hip_ad_rgb variant')
        self.textures.append(t)
        return idx

    # -- BSDFs --------------------------------------------------------------------
    def bsdf(self, spec, name: str) -> int:
        if spec.get("type") == "ref":
            ref = spec["id"]
            if ref not in self.bsdf_ids:
                raise RuntimeError(f'Reference "{ref}" not found')
            return self.bsdf_ids[ref]
        ty = spec.get("type")
        b = A.Bsdf()
        if ty == "diffuse":
            b.type = A.BSDF_DIFFUSE
            b.reflectance = self.texture(spec.get("reflectance", 0.5), name + ".reflectance")
        elif ty == "null":
            b.type = A.BSDF_NULL
            b.reflectance = A.INVALID
        else:
            raise RuntimeError(f'BSDF plugin "{ty}" is not available in the hip_ad_rgb variant')
        self.bsdfs.append(b)
        idx = len(self.bsdfs) - 1
        self.bsdf_ids[name] = idx
        return idx

    def default_bsdf(self) -> int:
        if "__default__" not in self.bsdf_ids:
            return self.bsdf({"type": "diffuse"}, "__default__")
        return self.bsdf_ids["__default__"]

    # -- media (heterogeneous.cpp, homogeneous.cpp, grid.cpp, hg.cpp, isotropic.cpp) ----
    def medium(self, spec, name: str) -> int:
        if isinstance(spec, str):
            spec = {"type": "ref", "id": spec}
        if spec.get("type") == "ref":
            ref = spec["id"]
            if ref not in self.medium_ids:
                raise RuntimeError(f'Reference "{ref}" not found')
            return self.medium_ids[ref]
        if name in self.medium_ids:
            return self.medium_ids[name]
        ty = spec.get("type")
        m = A.Medium()
        m.grid_offset = 0
        m.scale = float(np.float32(spec.get("scale", 1.0)))
        alb = spec.get("albedo", 0.75)
        if isinstance(alb, dict):
            if alb.get("type") not in ("rgb", "constvolume"):
                raise RuntimeError("hip_ad_rgb: only constant albedo volumes are supported")
            alb = alb.get("value", alb.get("color"))
        m.albedo[:] = [float(x) for x in _f32(np.broadcast_to(np.asarray(alb, np.float64).reshape(-1), (3,)))]
        ph = spec.get("phase", {"type": "isotropic"})
        if ph.get("type") == "hg":
            g = float(ph.get("g", 0.8))
            if g >= 1.0 or g <= -1.0:
                raise RuntimeError("The asymmetry parameter must lie in the interval (-1, 1)!")
            m.phase, m.g = A.PHASE_HG, float(np.float32(g))
        elif ph.get("type") == "isotropic":
            m.phase, m.g = A.PHASE_ISOTROPIC, 0.0
        else:
            raise RuntimeError(f'Phase function plugin "{ph.get("type")}" is not available in the hip_ad_rgb variant')
        m.flags = ((0 if spec.get("sample_emitters", True) else A.MEDIUM_NO_EMITTER_SAMPLING) |
                   (0 if spec.get("has_spectral_extinction", True) else A.MEDIUM_NO_SPECTRAL_EXTINCTION))
        st = spec.get("sigma_t", 1.0)
        if ty == "homogeneous":
            if isinstance(st, dict):
                st = st.get("value", st.get("color"))
            v = np.asarray(st, np.float64).reshape(-1)
            if v.size != 1 and not np.all(v == v[0]):
                raise RuntimeError("hip_ad_rgb: spectrally varying sigma_t is not supported")
            m.type = A.MEDIUM_HOMOGENEOUS
            m.sigma_t_const = float(np.float32(v[0]))
            self.params[name + ".sigma_t.value"] = ("medium_sigma_t", len(self.media))
        elif ty == "heterogeneous":
            if not isinstance(st, dict) or st.get("type") != "gridvolume":
                raise RuntimeError("hip_ad_rgb: heterogeneous media need a 'gridvolume' sigma_t")
            from .volume import VolumeGrid
            if "filename" in st:
                grid = VolumeGrid.read(st["filename"])
            elif "data" in st:
                grid = VolumeGrid(st["data"])
            elif "grid" in st:
                grid = st["grid"]
            else:
                raise RuntimeError("gridvolume: specify 'filename', 'data' or 'grid'")
            if grid.channel_count() != 1:
                raise RuntimeError("hip_ad_rgb: sigma_t grids must have one channel")
            if st.get("filter_type", "trilinear") != "trilinear" or st.get("wrap_mode", "clamp") != "clamp":
                raise RuntimeError("hip_ad_rgb: gridvolume supports filter_type='trilinear', wrap_mode='clamp'")
            T = _to_transform(st.get("to_world"))
            if st.get("use_grid_bbox", False):
                lo, hi = grid.bbox_min.astype(np.float64), grid.bbox_max.astype(np.float64)
                T = T @ Transform4f.translate(lo) @ Transform4f.scale(hi - lo)
            x, y, z = grid.size()
            m.type = A.MEDIUM_HETEROGENEOUS
            m.grid_res[:] = [x, y, z]
            m.grid_offset = self.n_grid
            inv = np.linalg.inv(T.matrix)
            m.grid_to_local[:] = [float(v) for v in _f32(inv[:3, :].reshape(-1))]
            corners = np.array([[i, j, k] for i in (0, 1) for j in (0, 1) for k in (0, 1)], np.float64)
            wc = np.array([T.transform_point(c) for c in corners], np.float64).astype(np.float32)
            m.bbox_min[:] = [float(v) for v in wc.min(0)]
            m.bbox_max[:] = [float(v) for v in wc.max(0)]
            m.max_density = float(np.float32(st["max_value"])) if "max_value" in st else grid.max()
            flat = np.ascontiguousarray(grid.data.reshape(-1))
            self.grids.append(flat)
            self.n_grid += flat.size
            self.params[name + ".sigma_t.data"] = ("grid", len(self.media))
        else:
            raise RuntimeError(f'Medium plugin "{ty}" is not available in the hip_ad_rgb variant')
        self.params[name + ".albedo.value"] = ("medium_albedo", len(self.media))
        self.media.append(m)
        idx = len(self.media) - 1
        self.medium_ids[name] = idx
        return idx

    # -- infinite emitters (constant.cpp, directional.cpp) ---------------------------
    def infinite_emitter(self, spec, name: str):
        ty = spec.get("type")
        e = A.Emitter()
        e.shape = A.INVALID
        key = "radiance" if ty == "constant" else "irradiance"
        v = spec.get(key, 1.0)
        if isinstance(v, dict):
            v = v.get("value", v.get("color"))
        e.radiance[:] = [float(x) for x in _f32(np.broadcast_to(np.asarray(v, np.float64).reshape(-1), (3,)))]
        if ty == "constant":
            if self.environment != A.INVALID:
                raise RuntimeError("Only one environment emitter can be specified per scene.")
            e.type = A.EMITTER_CONSTANT
            self.environment = len(self.emitters)
        elif ty == "directional":
            if "to_world" in spec:
                raise RuntimeError("hip_ad_rgb: directional emitters take 'direction' (not 'to_world')")
            d = _normalize32(_normalize32(_f32(spec.get("direction", [0.0, 0.0, 1.0]))))
            e.type = A.EMITTER_DIRECTIONAL
            e.direction[:] = [float(x) for x in d]
        else:
            raise RuntimeError(f'Emitter plugin "{ty}" is not available in the hip_ad_rgb variant')
        self.params[f"{name}.{key}.value"] = ("emitter_radiance", len(self.emitters))
        self.emitters.append(e)

    def _expand_bbox(self, pts):
        pts = _f32(pts).reshape(-1, 3)
        self.bbox_min = np.minimum(self.bbox_min, pts.min(0))
        self.bbox_max = np.maximum(self.bbox_max, pts.max(0))

    def finalize(self):
        """Emitter::set_scene (constant.cpp:76-85, directional.cpp:100-110):
        bounding sphere of Scene::bbox(), radius = max(RayEps, r (1 + RayEps))."""
        ray_eps = np.float32(1500.0) * np.float32(2.0 ** -24)
        if np.all(self.bbox_min <= self.bbox_max):
            c = (self.bbox_max + self.bbox_min) * np.float32(0.5)
            dd = (c - self.bbox_max).astype(np.float32)
            r = np.sqrt(np.float32(dd[2] * dd[2]) + np.float32(dd[1] * dd[1]) + np.float32(dd[0] * dd[0]), dtype=np.float32)
            r = max(ray_eps, np.float32(r * np.float32(1 + ray_eps)))
        else:
            c, r = np.zeros(3, np.float32), np.float32(1.0)
        for e in self.emitters:
            if e.type in (A.EMITTER_CONSTANT, A.EMITTER_DIRECTIONAL):
                e.scene_center[:] = [float(x) for x in c]
                e.scene_radius = float(r)

    # -- shapes ---------------------------------------------------------------------
    def shape(self, spec, name: str):
        ty = spec.get("type")
        T = _to_transform(spec.get("to_world"))
        if spec.get("flip_normals", False) and ty in ("rectangle", "cube"):
            T = T @ Transform4f.scale([1.0, 1.0, -1.0])
        s = A.Shape()
        s.emitter = A.INVALID
        s.interior_medium = s.exterior_medium = A.INVALID
        if spec.get("interior") is not None:
            s.interior_medium = self.medium(spec["interior"], name + ".interior_medium")
        if spec.get("exterior") is not None:
            s.exterior_medium = self.medium(spec["exterior"], name + ".exterior_medium")
        bspec = spec.get("bsdf")
        s.bsdf = self.bsdf(bspec, name + ".bsdf") if bspec is not None else self.default_bsdf()
        if ty == "rectangle":
            s.type = A.SHAPE_RECTANGLE
            s.face_count = 1
            M = T.matrix
            inv = np.linalg.inv(M)
            s.to_world[:] = [float(x) for x in _f32(M[:3, :].reshape(-1))]
            s.to_object[:] = [float(x) for x in _f32(inv[:3, :].reshape(-1))]
            dp_du = M[:3, :3] @ np.array([2.0, 0, 0])
            dp_dv = M[:3, :3] @ np.array([0, 2.0, 0])
            n = T.transform_normal([0, 0, 1.0])
            n /= np.linalg.norm(n)
            s.frame_s[:] = [float(x) for x in _f32(dp_du)]
            s.frame_t[:] = [float(x) for x in _f32(dp_dv)]
            s.frame_n[:] = [float(x) for x in _f32(n)]
            area = np.linalg.norm(np.cross(_f32(dp_du).astype(np.float64), _f32(dp_dv).astype(np.float64)))
            s.inv_area = float(np.float32(1.0 / area))
            self._expand_bbox([T.transform_point([x, y, 0.0]) for x in (-1.0, 1.0) for y in (-1.0, 1.0)])
        elif ty in ("cube", "mesh", "obj", "ply"):
            M = T.matrix
            xp = lambda P: (np.asarray(P, np.float64).reshape(-1, 3) @ M[:3, :3].T + M[:3, 3])
            IT = T.inverse_transpose[:3, :3]

            def xn(Nn):
                n = np.asarray(Nn, np.float64).reshape(-1, 3) @ IT.T
                with np.errstate(invalid="ignore", divide="ignore"):
                    return n / np.linalg.norm(n, axis=1, keepdims=True)
            if ty == "cube":
                V = np.array([T.transform_point(p) for p in _CUBE_V])
                N = np.array([T.transform_normal(n) / np.linalg.norm(T.transform_normal(n)) for n in _CUBE_N])
                UV = np.array(_CUBE_UV, dtype=np.float64)
                F = np.array(_CUBE_F, dtype=np.uint32)
            elif ty == "mesh":  # in-memory mesh: {'type': 'mesh', 'vertex_positions', 'faces', ...}
                V = xp(spec["vertex_positions"])
                F = np.asarray(spec["faces"], dtype=np.uint32).reshape(-1, 3)
                N = spec.get("vertex_normals")
                if N is not None:   # stored as given unless a to_world is applied
                    N = xn(N) if "to_world" in spec else np.asarray(N, np.float32).reshape(-1, 3)
                UV = spec.get("vertex_texcoords")
                if UV is not None:
                    UV = np.asarray(UV, dtype=np.float64).reshape(-1, 2)
            else:  # obj.cpp / ply.cpp (mitsuba_hip/meshio.py)
                from . import meshio
                fn = spec.get("filename")
                if fn is None:
                    raise RuntimeError(f'"{ty}" shape: property "filename" is required')
                face_normals = bool(spec.get("face_normals", False))
                rd = meshio.read_obj if ty == "obj" else meshio.read_ply
                m = rd(fn, flip_tex_coords=bool(spec.get("flip_tex_coords", ty == "obj")), face_normals=face_normals)
                V = _f32(xp(m["positions"])).astype(np.float64)
                F = m["faces"]
                if F.size and F.max() >= len(V):
                    raise RuntimeError(f'Error while loading {ty.upper()} file: face index out of range')
                N = xn(m["normals"]) if m["normals"] is not None else None
                if m["recompute_normals"] and len(F):
                    N = meshio.recompute_vertex_normals(V, F).astype(np.float64)
                UV = m["texcoords"]
                if spec.get("flip_normals", False):
                    # Mesh::m_flip_normals: reversed winding flips the geometric
                    # normal; shading normals are negated
                    F = F[:, [0, 2, 1]].copy()
                    if N is not None:
                        N = -N
            s.type = A.SHAPE_MESH
            s.face_offset = self.n_faces
            s.face_count = len(F)
            s.vertex_offset = self.n_vertices
            s.vertex_count = len(V)
            s.has_normals = int(N is not None)
            s.has_texcoords = int(UV is not None)
            self.positions.append(_f32(V))
            self._expand_bbox(V)
            self.normals.append(_f32(N) if N is not None else np.zeros((len(V), 3), np.float32))
            self.texcoords.append(_f32(UV) if UV is not None else np.zeros((len(V), 2), np.float32))
            self.faces.append(F)
            self.any_normals |= N is not None
            self.any_texcoords |= UV is not None
            self.n_vertices += len(V)
            self.n_faces += len(F)
            s.inv_area = 0.0
        else:
            raise RuntimeError(f'Shape plugin "{ty}" is not available in the hip_ad_rgb variant')
        shape_idx = len(self.shapes)
        em = spec.get("emitter")
        if em is not None:
            if em.get("type") != "area":
                raise RuntimeError("Only 'area' emitters can be attached to shapes")
            if "to_world" in em:
                raise RuntimeError("Found a 'to_world' transformation -- this is not allowed. "
                                   "The area light inherits this transformation from its parent shape.")
            e = A.Emitter()
            e.type = A.EMITTER_AREA
            e.shape = shape_idx
            rad = em.get("radiance", 1.0)
            tex_key = name + ".emitter.radiance"
            if isinstance(rad, dict):
                v = rad.get("value", rad.get("color"))
            else:
                v = rad
            v = np.broadcast_to(np.asarray(v, dtype=np.float64).reshape(-1), (3,))
            e.radiance[:] = [float(x) for x in v]
            s.emitter = len(self.emitters)
            self.emitters.append(e)
            self.params[tex_key + ".value"] = ("emitter_radiance", s.emitter)
        self.shapes.append(s)
        self.shape_names.append(name)


class Scene:
    """A loaded scene: flattened host description + lazily created device handles."""

    def __init__(self, sensor: A.Sensor, builder: _Builder, integrator: Optional[Integrator],
                 spec: Dict[str, Any]):
        self.integrator_ = integrator
        self.spec = spec
        self.params = builder.params
        self.shape_names = builder.shape_names
        b = builder
        b.finalize()
        self._shapes = (A.Shape * max(len(b.shapes), 1))(*b.shapes)
        self._bsdfs = (A.Bsdf * max(len(b.bsdfs), 1))(*b.bsdfs)
        self._textures = (A.Texture * max(len(b.textures), 1))(*b.textures)
        self._emitters = (A.Emitter * max(len(b.emitters), 1))(*b.emitters)
        self._media = (A.Medium * max(len(b.media), 1))(*b.media)
        cat = lambda xs, w, dt: (np.ascontiguousarray(np.concatenate(xs).reshape(-1)).astype(dt)
                                 if xs else np.zeros(w, dt))
        self.positions = cat(b.positions, 3, np.float32)
        self.normals = cat(b.normals, 3, np.float32)
        self.texcoords = cat(b.texcoords, 2, np.float32)
        self.faces = cat(b.faces, 3, np.uint32)
        self.texels = cat(b.texels, 1, np.float32)
        self.grid = cat(b.grids, 1, np.float32)
        d = A.SceneDesc()
        d.abi_version = A.ABI_VERSION
        d.sensor = sensor
        d.n_shapes, d.n_bsdfs, d.n_textures = len(b.shapes), len(b.bsdfs), len(b.textures)
        d.n_emitters, d.n_media = len(b.emitters), len(b.media)
        d.n_vertices, d.n_faces = b.n_vertices, b.n_faces
        d.shapes = C.cast(self._shapes, C.POINTER(A.Shape))
        d.bsdfs = C.cast(self._bsdfs, C.POINTER(A.Bsdf))
        d.textures = C.cast(self._textures, C.POINTER(A.Texture))
        d.emitters = C.cast(self._emitters, C.POINTER(A.Emitter))
        d.media = C.cast(self._media, C.POINTER(A.Medium))
        d.positions = self.positions.ctypes.data_as(A.PF)
        d.normals = self.normals.ctypes.data_as(A.PF) if b.any_normals else None
        d.texcoords = self.texcoords.ctypes.data_as(A.PF) if b.any_texcoords else None
        d.faces = self.faces.ctypes.data_as(A.PU)
        d.texels = self.texels.ctypes.data_as(A.PF)
        d.n_texels = b.n_texels
        d.grid_data = self.grid.ctypes.data_as(A.PF)
        d.n_grid = b.n_grid
        d.environment = b.environment
        self.desc = d
        self._handles: Dict[int, C.c_void_p] = {}
        self._streams: Dict[int, Any] = {}

    # -- reference-like accessors -----------------------------------------------------
    @property
    def width(self):
        return self.desc.sensor.width

    @property
    def height(self):
        return self.desc.sensor.height

    def integrator(self):
        return self.integrator_

    def sample_count(self):
        return self.desc.sensor.sample_count

    def texture(self, idx: int) -> A.Texture:
        return self._textures[idx]

    def medium(self, idx: int) -> A.Medium:
        return self._media[idx]

    def grid_data(self, idx: int) -> np.ndarray:
        m = self._media[idx]
        n = m.grid_res[0] * m.grid_res[1] * m.grid_res[2]
        return self.grid[m.grid_offset:m.grid_offset + n]

    def texture_data(self, idx: int) -> np.ndarray:
        t = self._textures[idx]
        n = t.width * t.height * t.channels
        return self.texels[t.data_offset:t.data_offset + n]

    # -- device handle (product path; no fallback) ---------------------------------------
    def handle(self, device: int = 0, stream=None) -> C.c_void_p:
        """Device copy of the scene.  `stream` (an int hipStream_t, 0 = the
        null stream) makes the scene's kernels run on the caller's stream;
        None keeps the scene's own stream."""
        h = self._handles.get(device)
        if h is None:
            L = A.lib()
            h = C.c_void_p()
            A.check(L.mh_scene_create(C.byref(self.desc), device, None, C.byref(h)))
            self._handles[device] = h
            self._streams[device] = None
        if stream is not None and self._streams.get(device) != stream:
            A.check(A.lib().mh_scene_set_stream(h, C.c_void_p(stream) if stream else None))
            self._streams[device] = stream
        return h

    def release(self):
        if self._handles:
            L = A.lib()
            for h in self._handles.values():
                L.mh_scene_destroy(h)
            self._handles.clear()

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    def __repr__(self):
        return (f"Scene[shapes={self.desc.n_shapes}, bsdfs={self.desc.n_bsdfs}, "
                f"emitters={self.desc.n_emitters}, film={self.width}x{self.height}]")


def _sensor(spec: Dict[str, Any]) -> A.Sensor:
    ty = spec.get("type", "perspective")
    if ty != "perspective":
        raise RuntimeError(f'Sensor plugin "{ty}" is not available in the hip_ad_rgb variant')
    film = spec.get("film", {"type": "hdrfilm"})
    if film.get("type", "hdrfilm") != "hdrfilm":
        raise RuntimeError(f'Film plugin "{film.get("type")}" is not available in the hip_ad_rgb variant')
    W, H = int(film.get("width", 768)), int(film.get("height", 576))
    pf = film.get("pixel_format", "rgb").lower()
    # hdrfilm.cpp:160-188
    pix = {"rgb": A.PIXEL_RGB, "luminance": A.PIXEL_Y, "xyz": A.PIXEL_XYZ, "rgba": A.PIXEL_RGBA,
           "luminance_alpha": A.PIXEL_YA, "xyza": A.PIXEL_XYZA}.get(pf)
    if pix is None:
        raise RuntimeError('The "pixel_format" parameter must either be equal to "luminance", '
                           f'"luminance_alpha", "rgb", "rgba",  "xyz", "xyza". Found {pf}.')
    if "crop_offset_x" in film or "crop_width" in film:
        raise RuntimeError("hdrfilm: crop windows are not available in the hip_ad_rgb variant")
    rf = film.get("rfilter", {"type": "gaussian"})
    s = A.Sensor()
    s.pixel_format = pix
    if rf.get("type", "gaussian") == "gaussian":
        coeff, radius = gaussian_coefficients(float(rf.get("stddev", 0.5)))
        s.rfilter = A.RFILTER_GAUSSIAN
        s.rfilter_radius = radius
        s.filter_coeff[:] = [float(c) for c in coeff]
    elif rf.get("type") == "box":
        s.rfilter = A.RFILTER_BOX
        s.rfilter_radius = 0.5
    else:
        raise RuntimeError(f'Reconstruction filter "{rf.get("type")}" is not available in the hip_ad_rgb variant')
    smp = spec.get("sampler", {"type": "independent"})
    if smp.get("type", "independent") != "independent":
        raise RuntimeError(f'Sampler plugin "{smp.get("type")}" is not available in the hip_ad_rgb variant')
    s.sample_count = int(smp.get("sample_count", 4))
    s.sampler_seed = int(smp.get("seed", 0))
    near = float(spec.get("near_clip", 1e-2))
    far = float(spec.get("far_clip", 1e4))
    if near <= 0:
        raise RuntimeError("The 'near_clip' parameter must be greater than zero!")
    if near >= far:
        raise RuntimeError("The 'near_clip' parameter must be smaller than the 'far_clip' parameter!")
    to_world = _to_transform(spec.get("to_world"))
    if to_world.has_scale():
        raise RuntimeError("Scale factors in the camera-to-world transformation are not allowed!")
    fov_x = parse_fov(spec, W / H)
    cam_to_sample = perspective_projection([W, H], [W, H], [0, 0], fov_x, near, far)
    sample_to_camera = cam_to_sample.inverse()
    s.to_world[:] = [float(x) for x in _f32(to_world.matrix.reshape(-1))]
    s.sample_to_camera[:] = [float(x) for x in _f32(sample_to_camera.matrix.reshape(-1))]
    s.near_clip, s.far_clip = near, far
    s.width, s.height = W, H
    s.medium = A.INVALID
    return s


def load_dict(d: Dict[str, Any]):
    """mi.load_dict (core/python/xml_v.cpp:112) for the hot-path plugins."""
    ty = d.get("type")
    if ty in Integrator.TYPES:
        return Integrator(ty, d)
    if ty != "scene":
        raise RuntimeError(f'load_dict(): top-level plugin "{ty}" is not supported by the hip_ad_rgb variant')
    b = _Builder()
    integrator = None
    sensor = None
    # BSDFs and textures declared at the top level first (so that refs resolve)
    for k, v in d.items():
        if k == "type" or not isinstance(v, dict):
            continue
        if v.get("type") in ("diffuse", "null"):
            b.bsdf(v, k)
        elif v.get("type") in ("heterogeneous", "homogeneous"):
            b.medium(v, k)
    for k, v in d.items():
        if k == "type" or not isinstance(v, dict):
            continue
        vt = v.get("type")
        if vt in Integrator.TYPES:
            integrator = Integrator(vt, v)
        elif vt == "perspective" or k == "sensor":
            if sensor is not None:
                raise RuntimeError("hip_ad_rgb: multiple sensors are not supported")
            sensor = _sensor(v)
            if v.get("medium") is not None:
                sensor.medium = b.medium(v["medium"], k + ".medium")
        elif vt in ("rectangle", "cube", "mesh", "obj", "ply"):
            b.shape(v, k)
        elif vt in ("constant", "directional"):
            b.infinite_emitter(v, k)
        elif vt in ("diffuse", "null", "heterogeneous", "homogeneous"):
            pass
        else:
            raise RuntimeError(f'Plugin "{vt}" is not available in the hip_ad_rgb variant')
    if sensor is None:
        sensor = _sensor({"type": "perspective"})
    if integrator is None:
        integrator = Integrator("path", {})
    return Scene(sensor, b, integrator, d)


def cornell_box():
    """src/python/python/util.py:757-891 (same dictionary)."""
    T = Transform4f
    return {
        "type": "scene",
        "integrator": {"type": "path", "max_depth": 8},
        "sensor": {
            "type": "perspective", "fov_axis": "smaller", "near_clip": 0.001, "far_clip": 100.0,
            "focus_distance": 1000, "fov": 39.3077,
            "to_world": T.look_at(origin=[0, 0, 3.90], target=[0, 0, 0], up=[0, 1, 0]),
            "sampler": {"type": "independent", "sample_count": 64},
            "film": {"type": "hdrfilm", "width": 256, "height": 256, "rfilter": {"type": "gaussian"},
                     "pixel_format": "rgb", "component_format": "float32"},
        },
        "white": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.885809, 0.698859, 0.666422]}},
        "green": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.105421, 0.37798, 0.076425]}},
        "red": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.570068, 0.0430135, 0.0443706]}},
        "light": {
            "type": "rectangle",
            "to_world": T.translate([0.0, 0.99, 0.01]).rotate([1, 0, 0], 90).scale([0.23, 0.19, 0.19]),
            "bsdf": {"type": "ref", "id": "white"},
            "emitter": {"type": "area", "radiance": {"type": "rgb", "value": [18.387, 13.9873, 6.75357]}},
        },
        "floor": {"type": "rectangle", "to_world": T.translate([0.0, -1.0, 0.0]).rotate([1, 0, 0], -90),
                  "bsdf": {"type": "ref", "id": "white"}},
        "ceiling": {"type": "rectangle", "to_world": T.translate([0.0, 1.0, 0.0]).rotate([1, 0, 0], 90),
                    "bsdf": {"type": "ref", "id": "white"}},
        "back": {"type": "rectangle", "to_world": T.translate([0.0, 0.0, -1.0]),
                 "bsdf": {"type": "ref", "id": "white"}},
        "green-wall": {"type": "rectangle", "to_world": T.translate([1.0, 0.0, 0.0]).rotate([0, 1, 0], -90),
                       "bsdf": {"type": "ref", "id": "green"}},
        "red-wall": {"type": "rectangle", "to_world": T.translate([-1.0, 0.0, 0.0]).rotate([0, 1, 0], 90),
                     "bsdf": {"type": "ref", "id": "red"}},
        "small-box": {"type": "cube", "to_world": T.translate([0.335, -0.7, 0.38]).rotate([0, 1, 0], -17).scale(0.3),
                      "bsdf": {"type": "ref", "id": "white"}},
        "large-box": {"type": "cube",
                      "to_world": T.translate([-0.33, -0.4, -0.28]).rotate([0, 1, 0], 18.25).scale([0.3, 0.61, 0.3]),
                      "bsdf": {"type": "ref", "id": "white"}},
    }
