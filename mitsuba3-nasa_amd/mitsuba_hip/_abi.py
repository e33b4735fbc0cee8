"""ctypes mirror of ``include/mitsuba_hip.h`` and the product library loader.

The product library is ``libmitsuba_hip.so`` next to this file (built in-tree
by ``__graft_entry__.build()``).  There is deliberately no fallback: if the
library is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 2
INVALID = 0xFFFFFFFF

# status codes
MH_OK = 0
MH_ERR_INVALID_ARGUMENT, MH_ERR_HIP, MH_ERR_OUT_OF_MEMORY, MH_ERR_UNSUPPORTED, MH_ERR_NO_DEVICE = 1, 2, 3, 4, 5
ERRORS = {1: "invalid argument", 2: "HIP error", 3: "out of memory", 4: "unsupported", 5: "no device"}

SHAPE_RECTANGLE, SHAPE_MESH = 0, 1
BSDF_DIFFUSE, BSDF_NULL = 0, 1
TEX_RGB, TEX_BITMAP = 0, 1
EMITTER_AREA, EMITTER_CONSTANT, EMITTER_DIRECTIONAL = 0, 1, 2
RFILTER_BOX, RFILTER_GAUSSIAN = 0, 1
PIXEL_RGB, PIXEL_Y, PIXEL_XYZ, PIXEL_RGBA, PIXEL_YA, PIXEL_XYZA = 0, 1, 2, 3, 4, 5


def pixel_has_alpha(fmt: int) -> bool:
    return fmt in (PIXEL_RGBA, PIXEL_YA, PIXEL_XYZA)


def film_channels(fmt: int) -> int:
    """Channels of the film storage: RGBW, or RGBAW with alpha (hdrfilm.cpp:327-330)."""
    return 5 if pixel_has_alpha(fmt) else 4


def image_channels(fmt: int) -> int:
    """Channels of the developed image: colour (1 or 3) + alpha."""
    return (1 if fmt in (PIXEL_Y, PIXEL_YA) else 3) + (1 if pixel_has_alpha(fmt) else 0)


def image_channel_names(fmt: int):
    """Bitmap channel names of hdrfilm's output (EXR layers)."""
    return {PIXEL_RGB: ["R", "G", "B"], PIXEL_Y: ["Y"], PIXEL_XYZ: ["X", "Y", "Z"],
            PIXEL_RGBA: ["R", "G", "B", "A"], PIXEL_YA: ["Y", "A"], PIXEL_XYZA: ["X", "Y", "Z", "A"]}[fmt]
MEDIUM_HETEROGENEOUS, MEDIUM_HOMOGENEOUS = 0, 1
PHASE_ISOTROPIC, PHASE_HG = 0, 1
MEDIUM_NO_EMITTER_SAMPLING, MEDIUM_NO_SPECTRAL_EXTINCTION = 1, 2
INTEGRATOR_PATH, INTEGRATOR_VOLPATH, INTEGRATOR_PRB, INTEGRATOR_PRBVOLPATH = 0, 1, 2, 3
# differentiable parameter ids of mh_render_backward (texture index, or kind | medium)
PARAM_KIND_MASK = 0xF0000000
PARAM_MEDIUM_SIGMA_T = 0x10000000
PARAM_MEDIUM_ALBEDO = 0x20000000

FLAG_DEVICE_POINTERS = 1 << 0
FLAG_ACCUMULATE = 1 << 1
FLAG_NO_SYNC = 1 << 2
FLAG_MEGAKERNEL = 1 << 3
FLAG_WAVEFRONT = 1 << 4
FLAG_PRB_REPLAY = 1 << 5
FLAG_DETERMINISTIC = 1 << 6
FLAG_REDUCE = 1 << 7
FLAG_REDUCE_ROOT = 1 << 8
FLAG_LOCAL_WEIGHTS = 1 << 9
FLAG_SHARED_DEVICE = 1 << 10  # performance hint: another call runs on the device at the same time
COMM_ID_BYTES = 128

u32, u64, f32, f64 = C.c_uint32, C.c_uint64, C.c_float, C.c_double
PF = C.POINTER(C.c_float)
PU = C.POINTER(C.c_uint32)


class Shape(C.Structure):
    _fields_ = [("type", u32), ("bsdf", u32), ("emitter", u32), ("interior_medium", u32),
                ("exterior_medium", u32), ("face_offset", u32), ("face_count", u32),
                ("vertex_offset", u32), ("vertex_count", u32), ("has_normals", u32),
                ("has_texcoords", u32), ("pad0", u32), ("to_world", f32 * 12),
                ("to_object", f32 * 12), ("frame_s", f32 * 3), ("frame_t", f32 * 3),
                ("frame_n", f32 * 3), ("inv_area", f32)]


class Texture(C.Structure):
    _fields_ = [("type", u32), ("width", u32), ("height", u32), ("channels", u32),
                ("data_offset", u64), ("filter", u32), ("wrap", u32), ("value", f32 * 3),
                ("to_uv", f32 * 6), ("pad1", f32)]


class Bsdf(C.Structure):
    _fields_ = [("type", u32), ("reflectance", u32)]


class Emitter(C.Structure):
    _fields_ = [("type", u32), ("shape", u32), ("pad0", u32), ("pad1", u32),
                ("radiance", f32 * 3), ("direction", f32 * 3), ("scene_center", f32 * 3),
                ("scene_radius", f32)]


class Medium(C.Structure):
    _fields_ = [("type", u32), ("phase", u32), ("g", f32), ("scale", f32), ("albedo", f32 * 3),
                ("sigma_t_const", f32), ("grid_res", u32 * 3), ("flags", u32),
                ("grid_offset", u64), ("grid_to_local", f32 * 12), ("bbox_min", f32 * 3),
                ("bbox_max", f32 * 3), ("max_density", f32), ("pad1", f32)]


class Sensor(C.Structure):
    _fields_ = [("to_world", f32 * 16), ("sample_to_camera", f32 * 16), ("near_clip", f32),
                ("far_clip", f32), ("width", u32), ("height", u32), ("rfilter", u32),
                ("rfilter_radius", f32), ("filter_coeff", f32 * 10), ("sample_count", u32),
                ("sampler_seed", u32), ("medium", u32), ("pixel_format", u32)]


class SceneDesc(C.Structure):
    _fields_ = [("abi_version", u32), ("pad0", u32), ("sensor", Sensor), ("n_shapes", u32),
                ("n_bsdfs", u32), ("n_textures", u32), ("n_emitters", u32), ("n_media", u32),
                ("n_vertices", u32), ("n_faces", u32), ("pad1", u32),
                ("shapes", C.POINTER(Shape)), ("bsdfs", C.POINTER(Bsdf)),
                ("textures", C.POINTER(Texture)), ("emitters", C.POINTER(Emitter)),
                ("media", C.POINTER(Medium)), ("positions", PF), ("normals", PF),
                ("texcoords", PF), ("faces", PU), ("texels", PF), ("n_texels", u64),
                ("grid_data", PF), ("n_grid", u64), ("environment", u32), ("pad2", u32)]


class Integrator(C.Structure):
    _fields_ = [("type", u32), ("max_depth", u32), ("rr_depth", u32), ("hide_emitters", u32)]


class Stats(C.Structure):
    _fields_ = [("samples", u64), ("rays_closest", u64), ("rays_shadow", u64), ("bounces", u64),
                ("ms_total", f64), ("ms_kernel", f64), ("ms_trace", f64), ("n_trace_launches", u64),
                ("mode", u32), ("invalid_samples", u32), ("grid_lookups", u64), ("aux_items", u64),
                ("ms_aux", f64), ("n_aux_launches", u64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# Every symbol include/mitsuba_hip.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "mh_last_error", "mh_abi_version", "mh_device_count", "mh_scene_create", "mh_scene_destroy",
    "mh_scene_set_stream", "mh_scene_update_rgb", "mh_scene_update_texture", "mh_render",
    "mh_develop", "mh_prb_weights", "mh_render_backward", "mh_trace_closest", "mh_trace_shadow",
    "mh_scene_bvh_info", "mh_render_samples", "mh_scene_update_medium", "mh_trace_preliminary",
    "mh_render_forward", "mh_comm_unique_id", "mh_comm_create", "mh_comm_create_all", "mh_comm_destroy",
    "mh_comm_info", "mh_comm_reduce", "mh_scene_set_comm", "mh_scene_synchronize", "mh_render_sharded",
    "mh_render_backward_sharded",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# MH_LIB selects an alternative build of the same library (A/B experiments, tools/)
LIB_PATH = os.environ.get("MH_LIB") or os.path.join(_HERE, "libmitsuba_hip.so")
_lib = None


class MitsubaHipError(RuntimeError):
    pass


def lib():
    """Load ``libmitsuba_hip.so`` (raises if it was not built — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MitsubaHipError(
            f"mitsuba_hip: native library not found at {LIB_PATH}; run "
            "__graft_entry__.build() (hip_ad_rgb has no CPU fallback)")
    # One HIP runtime per process: when torch (ROCm) is installed, load it
    # first so that libmitsuba_hip.so's DT_NEEDED libamdhip64.so.7 binds to
    # the runtime torch already mapped (same soname) instead of a second copy.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.mh_last_error.restype = C.c_char_p
    L.mh_abi_version.restype = u32
    L.mh_device_count.argtypes = [C.POINTER(C.c_int)]
    L.mh_scene_create.argtypes = [C.POINTER(SceneDesc), C.c_int, vp, C.POINTER(vp)]
    L.mh_scene_destroy.argtypes = [vp]
    L.mh_scene_set_stream.argtypes = [vp, vp]
    L.mh_scene_update_rgb.argtypes = [vp, u32, PF]
    L.mh_scene_update_texture.argtypes = [vp, u32, PF, u64]
    L.mh_scene_update_medium.argtypes = [vp, u32, vp, vp, vp, u64, u32]
    L.mh_render.argtypes = [vp, C.POINTER(Integrator), u32, u32, u32, u32, vp, u32, C.POINTER(Stats)]
    L.mh_develop.argtypes = [vp, vp, vp, u32]
    L.mh_render_samples.argtypes = [vp, C.POINTER(Integrator), u32, u32, u32, u32, vp, u32]
    L.mh_prb_weights.argtypes = [vp, u32, u32, u32, u32, vp, u32]
    L.mh_render_backward.argtypes = [vp, C.POINTER(Integrator), u32, u32, u32, u32, vp, vp, u32,
                                     PU, C.POINTER(vp), u32, C.POINTER(Stats)]
    L.mh_render_forward.argtypes = [vp, C.POINTER(Integrator), u32, u32, u32, u32, u32, PU, C.POINTER(vp), vp,
                                    u32, C.POINTER(Stats)]
    L.mh_trace_closest.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, u32, C.POINTER(Stats)]
    L.mh_trace_shadow.argtypes = [vp, u64, vp, vp, u32, C.POINTER(Stats)]
    L.mh_trace_preliminary.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, vp, u32, C.POINTER(Stats)]
    L.mh_scene_bvh_info.argtypes = [vp, PU, PU, PU]
    pi = C.POINTER(C.c_int)
    L.mh_comm_unique_id.argtypes = [C.c_char_p]
    L.mh_comm_create.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
    L.mh_comm_create_all.argtypes = [C.c_int, pi, C.POINTER(vp)]
    L.mh_comm_destroy.argtypes = [vp]
    L.mh_comm_info.argtypes = [vp, pi, pi, pi]
    L.mh_comm_reduce.argtypes = [C.POINTER(vp), C.c_int, C.POINTER(vp), u64, C.POINTER(vp), C.c_int]
    L.mh_scene_set_comm.argtypes = [vp, vp]
    L.mh_scene_synchronize.argtypes = [vp]
    L.mh_render_sharded.argtypes = [C.POINTER(vp), u32, C.POINTER(Integrator), u32, u32, C.POINTER(vp), u32,
                                    C.POINTER(Stats)]
    L.mh_render_backward_sharded.argtypes = [C.POINTER(vp), u32, C.POINTER(Integrator), u32, u32, C.POINTER(vp),
                                             u32, PU, C.POINTER(vp), u32, C.POINTER(Stats)]
    for name in EXPORTS:
        if name not in ("mh_last_error", "mh_abi_version"):
            getattr(L, name).restype = C.c_int
    if L.mh_abi_version() != ABI_VERSION:
        raise MitsubaHipError("mitsuba_hip: ABI version mismatch between Python and libmitsuba_hip.so")
    _lib = L
    return L


def check(rc: int):
    """Raise RuntimeError with the library's message (mirrors the reference's Throw)."""
    if rc != MH_OK:
        msg = lib().mh_last_error().decode(errors="replace")
        raise MitsubaHipError(msg or ERRORS.get(rc, f"error {rc}"))
