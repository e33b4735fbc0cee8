"""ctypes binding of the CPU oracle (oracle/libmh_oracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "libmh_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    from mitsuba_hip import _abi as A
    L = C.CDLL(LIB)
    vp = C.c_void_p
    L.oracle_tea32.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.oracle_tea_float32.argtypes = [C.c_uint32, C.c_uint32, C.c_int]
    L.oracle_tea_float32.restype = C.c_float
    L.oracle_tea_float64.argtypes = [C.c_uint32, C.c_uint32, C.c_int]
    L.oracle_tea_float64.restype = C.c_double
    L.oracle_pcg32_stream.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, vp]
    L.oracle_sampler_floats.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, vp]
    L.oracle_gaussian_eval.argtypes = [vp, C.c_float]
    L.oracle_gaussian_eval.restype = C.c_float
    L.oracle_sincos.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    L.oracle_log.argtypes = [C.c_float]
    L.oracle_log.restype = C.c_float
    L.oracle_diffuse_eval_pdf.argtypes = [vp, vp, vp, vp, C.POINTER(C.c_float)]
    L.oracle_square_to_cosine_hemisphere.argtypes = [vp, vp]
    L.oracle_trace_closest.argtypes = [C.POINTER(A.SceneDesc), C.c_uint64, vp, vp, vp, vp, vp, vp]
    L.oracle_trace_shadow.argtypes = [C.POINTER(A.SceneDesc), C.c_uint64, vp, vp]
    L.oracle_camera_ray.argtypes = [C.POINTER(A.SceneDesc), vp, vp, vp, C.POINTER(C.c_float)]
    L.oracle_sample_range.argtypes = [C.POINTER(A.SceneDesc), C.POINTER(A.Integrator), C.c_uint32,
                                      C.c_uint32, C.c_uint64, C.c_uint64, vp, vp, vp]
    L.oracle_render.argtypes = [C.POINTER(A.SceneDesc), C.POINTER(A.Integrator), C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_uint32, C.c_int, vp]
    L.oracle_develop.argtypes = [C.c_uint32, C.c_uint32, vp, vp]
    L.oracle_develop_format.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, vp, vp]
    L.oracle_prb_weights.argtypes = [C.POINTER(A.SceneDesc), C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_uint32, C.c_int, vp]
    L.oracle_prb_weights_rows.argtypes = [C.POINTER(A.SceneDesc), C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_uint32, C.c_int, vp]
    L.oracle_render_backward.argtypes = [C.POINTER(A.SceneDesc), C.POINTER(A.Integrator), C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, C.c_uint32,
                                         vp, C.POINTER(C.c_void_p), C.c_int]
    L.oracle_render_forward.argtypes = [C.POINTER(A.SceneDesc), C.POINTER(A.Integrator), C.c_uint32,
                                        C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp,
                                        C.POINTER(C.c_void_p), C.c_int, vp]
    L.oracle_render_scalar.argtypes = [C.POINTER(A.SceneDesc), C.POINTER(A.Integrator), C.c_uint32, C.c_uint32,
                                       C.c_uint32, C.c_int, vp]
    L.oracle_spiral_order.restype = C.c_uint32
    L.oracle_spiral_order.argtypes = [C.c_uint32, C.c_uint32, vp, vp]
    L.oracle_last_error.restype = C.c_char_p
    L.oracle_grid_lookups.restype = C.c_uint64
    L.oracle_grid_lookups.argtypes = [C.c_int]
    _lib = L
    return L


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def check(rc):
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())


def nthreads():
    """Host threads of the oracle: the CPUs this process may run on, capped by
    OMP_NUM_THREADS where it is set (the GPU box's share is 16 of a larger
    machine) and by 64."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 64
    return max(1, min(n, cap, 64))


def render(scene, integrator=None, seed=0, spp=0, spp_begin=0, spp_end=0, threads=None):
    integrator = integrator or scene.integrator()
    from mitsuba_hip import _abi as A
    film = np.zeros((scene.height, scene.width, A.film_channels(scene.desc.sensor.pixel_format)), np.float32)
    ic = integrator.c()
    check(lib().oracle_render(C.byref(scene.desc), C.byref(ic), seed, spp or scene.sample_count(),
                              spp_begin, spp_end, threads or nthreads(), _p(film)))
    return film


def render_scalar(scene, integrator=None, seed=0, spp=0, block_size=32, threads=None):
    """scalar_rgb render (config 1): spiral blocks, per-pixel Morton-order
    PCG32 seeding and the scalar `path` control flow
    (integrator.cpp:189-275, 1099-1124; path.cpp:179-196)."""
    integrator = integrator or scene.integrator()
    film = np.zeros((scene.height, scene.width, 4), np.float32)
    ic = integrator.c()
    check(lib().oracle_render_scalar(C.byref(scene.desc), C.byref(ic), seed, spp or scene.sample_count(),
                                     block_size, threads or nthreads(), _p(film)))
    return film


def spiral_order(bw, bh):
    bx = np.zeros(bw * bh, np.uint32)
    by = np.zeros(bw * bh, np.uint32)
    n = lib().oracle_spiral_order(bw, bh, _p(bx), _p(by))
    return list(zip(bx[:n].tolist(), by[:n].tolist()))


def develop(film, pixel_format=0):
    from mitsuba_hip import _abi as A
    h, w = film.shape[:2]
    out = np.zeros((h, w, A.image_channels(pixel_format)), np.float32)
    lib().oracle_develop_format(w, h, pixel_format, _p(np.ascontiguousarray(film)), _p(out))
    return out


def sample_range(scene, integrator, seed, spp, begin, end):
    n = end - begin
    L = np.zeros((n, 3), np.float32)
    pos = np.zeros((n, 2), np.float32)
    valid = np.zeros(n, np.uint32)
    ic = integrator.c()
    check(lib().oracle_sample_range(C.byref(scene.desc), C.byref(ic), seed, spp, begin, end,
                                    _p(L), _p(pos), _p(valid)))
    return L, pos, valid


def trace_closest(scene, rays):
    rays = np.ascontiguousarray(rays, np.float32)
    n = rays.shape[1]
    t, u, v = (np.zeros(n, np.float32) for _ in range(3))
    prim, shape = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
    check(lib().oracle_trace_closest(C.byref(scene.desc), n, _p(rays), _p(t), _p(u), _p(v), _p(prim), _p(shape)))
    return t, u, v, prim, shape


def trace_shadow(scene, rays):
    rays = np.ascontiguousarray(rays, np.float32)
    n = rays.shape[1]
    occ = np.zeros(n, np.uint32)
    check(lib().oracle_trace_shadow(C.byref(scene.desc), n, _p(rays), _p(occ)))
    return occ


def prb_weights(scene, seed, spp, spp_begin=0, spp_end=0, threads=None):
    w = np.zeros((scene.height, scene.width), np.float32)
    check(lib().oracle_prb_weights(C.byref(scene.desc), seed, spp, spp_begin, spp_end,
                                   threads or nthreads(), _p(w)))
    return w


def prb_weights_rows(scene, seed, spp, row_lo, row_hi, threads=None):
    """W image from the samples of pixel rows [row_lo, row_hi) only: exact on
    rows [row_lo + 2, row_hi - 2) and on image-border rows inside the range."""
    w = np.zeros((scene.height, scene.width), np.float32)
    check(lib().oracle_prb_weights_rows(C.byref(scene.desc), seed, spp, row_lo, row_hi, threads or nthreads(),
                                        _p(w)))
    return w


def render_backward(scene, integrator, seed, spp, grad_in, textures, shapes, weights=None,
                    spp_begin=0, spp_end=0, threads=None):
    grads = [np.zeros(s, np.float32) for s in shapes]
    ptrs = (C.c_void_p * len(grads))(*[g.ctypes.data for g in grads])
    tex = np.asarray(textures, np.uint32)
    ic = integrator.c()
    check(lib().oracle_render_backward(
        C.byref(scene.desc), C.byref(ic), seed, spp, spp_begin, spp_end,
        _p(np.ascontiguousarray(grad_in, np.float32)),
        _p(np.ascontiguousarray(weights, np.float32)) if weights is not None else None,
        len(grads), _p(tex), ptrs, threads or nthreads()))
    return grads


def render_forward(scene, integrator, seed, spp, param_ids, tangents, spp_begin=0, spp_end=0, threads=None):
    """RBIntegrator.render_forward (common.py:696-826): the film of the
    per-sample tangent radiance (develop it with develop())."""
    from mitsuba_hip import _abi as A
    film = np.zeros((scene.height, scene.width, A.film_channels(scene.desc.sensor.pixel_format)), np.float32)
    tans = [np.ascontiguousarray(t, np.float32) for t in tangents]
    ptrs = (C.c_void_p * max(len(tans), 1))(*[t.ctypes.data for t in tans])
    ids = np.asarray(param_ids, np.uint32)
    ic = integrator.c()
    check(lib().oracle_render_forward(C.byref(scene.desc), C.byref(ic), seed, spp, spp_begin, spp_end,
                                      len(tans), _p(ids), ptrs, threads or nthreads(), _p(film)))
    return film


def grid_lookups(reset=True):
    """Density-grid lookups of the oracle's renders since the last reset
    (the check of mh_stats.grid_lookups)."""
    return int(lib().oracle_grid_lookups(1 if reset else 0))
