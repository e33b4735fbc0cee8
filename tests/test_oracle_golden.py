"""CPU: the oracle (oracle/libmh_oracle.so) against the reference's own
known-answer vectors (tests/golden/known_answers.json, provenance per entry)
and the committed oracle regression fixtures; plus the reference's linearity
(test_ad.py:6-92) and finite-difference (test_ad_integrators.py:917-962)
methodologies applied to the restated PRB."""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

import oracle_py as O

HERE = os.path.dirname(os.path.abspath(__file__))
KA = json.load(open(os.path.join(HERE, "golden", "known_answers.json")))
REG = np.load(os.path.join(HERE, "golden", "oracle_regression.npz"))


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


# ---- RNG ---------------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["float32", "float64"])
def test_tea_known_answers(kind):
    L = O.lib()
    fn = L.oracle_tea_float32 if kind == "float32" else L.oracle_tea_float64
    assert len(KA["tea"][kind]) == 8
    for e in KA["tea"][kind]:
        assert fn(e["v0"], e["v1"], e["rounds"]) == e["value"], e["source"]


def test_pcg32_demo_stream():
    e = KA["pcg32_demo"]
    out = np.zeros(len(e["values"]), np.uint32)
    O.lib().oracle_pcg32_stream(e["initstate"], e["initseq"], len(out), out.ctypes.data_as(C.c_void_p))
    assert out.tolist() == e["values"]


def test_sample_tea_32_host_matches_oracle():
    mi = _mi()
    L = O.lib()
    rng = np.random.default_rng(3)
    for v0, v1 in rng.integers(0, 2**32, size=(200, 2), dtype=np.uint64):
        a, b = C.c_uint32(), C.c_uint32()
        L.oracle_tea32(int(v0), int(v1), 4, C.byref(a), C.byref(b))
        assert mi.sample_tea_32(int(v0), int(v1)) == (a.value, b.value)


def test_sampler_float_construction():
    """next_float = bits((u >> 9) | 0x3f800000) - 1 over the PCG32 stream seeded
    with TEA(seed_value, lane) (sampler.cpp:115-134)."""
    L = O.lib()
    for lane in (0, 5, 1000):
        v0, v1 = C.c_uint32(), C.c_uint32()
        L.oracle_tea32(17, lane, 4, C.byref(v0), C.byref(v1))
        u = np.zeros(6, np.uint32)
        L.oracle_pcg32_stream(v0.value, v1.value, 6, u.ctypes.data_as(C.c_void_p))
        f = np.zeros(6, np.float32)
        L.oracle_sampler_floats(17, lane, 6, f.ctypes.data_as(C.c_void_p))
        exp = ((u >> 9) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1)
        assert np.array_equal(f, exp)


# ---- filter / BSDF / warps -----------------------------------------------------------
def test_gaussian_filter_known_answers():
    mi = _mi()
    coeff, radius = mi.gaussian_coefficients(0.5)
    assert radius == 2.0
    for e in KA["gaussian"]:
        v = O.lib().oracle_gaussian_eval(coeff.ctypes.data_as(C.c_void_p), e["x"])
        if e["atol"] == 0.0:
            assert v == e["value"], e["source"]
        else:
            assert abs(v - e["value"]) <= e["atol"], e["source"]
    # radius 2: f(r) = 0 exactly, non-negative inside
    xs = np.linspace(0, 2.5, 101, dtype=np.float32)
    vals = [O.lib().oracle_gaussian_eval(coeff.ctypes.data_as(C.c_void_p), float(x)) for x in xs]
    assert all(v >= 0 for v in vals) and vals[-1] == 0.0


def test_diffuse_eval_pdf_known_answers():
    e = KA["diffuse"]
    wi = np.array(e["wi"], np.float32)
    rho = np.full(3, e["reflectance"], np.float32)
    for i in range(e["n"]):
        th = i / 19.0 * (math.pi / 2)
        wo = np.array([math.sin(th), 0, math.cos(th)], np.float32)
        val = np.zeros(3, np.float32)
        pdf = C.c_float()
        O.lib().oracle_diffuse_eval_pdf(wi.ctypes.data_as(C.c_void_p), wo.ctypes.data_as(C.c_void_p),
                                        rho.ctypes.data_as(C.c_void_p), val.ctypes.data_as(C.c_void_p),
                                        C.byref(pdf))
        assert np.isclose(pdf.value, wo[2] / math.pi, rtol=1e-5, atol=1e-7), e["source"]
        assert np.isclose(val[0], 0.5 * wo[2] / math.pi, rtol=1e-5, atol=1e-7), e["source"]


def test_cosine_hemisphere_warp():
    rng = np.random.default_rng(1)
    for s in rng.random((200, 2), dtype=np.float32):
        out = np.zeros(3, np.float32)
        O.lib().oracle_square_to_cosine_hemisphere(s.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p))
        assert abs(np.linalg.norm(out) - 1) < 1e-5 and out[2] >= 0


# ---- shapes / ray queries --------------------------------------------------------------
def _scene_with(shape):
    mi = _mi()
    return mi.load_dict({"type": "scene", "foo": shape})


def test_rectangle_known_answers():
    mi = _mi()
    e = KA["rectangle"]
    scene = _scene_with({"type": "rectangle", "to_world": mi.Transform4f.scale(e["scale"])})
    a = np.linspace(-1, 1, e["n"]).astype(np.float32)
    rays = np.zeros((7, e["n"]), np.float32)
    rays[0], rays[1], rays[2] = a, a, e["origin_z"]
    rays[3:6] = np.asarray(e["dir"], np.float32)[:, None]
    rays[6] = np.finfo(np.float32).max
    occ = O.trace_shadow(scene, rays)
    t, u, v, prim, shape = O.trace_closest(scene, rays)
    expect = np.abs(a) <= 0.5
    assert np.array_equal(occ.astype(bool), expect), e["source"]
    assert np.array_equal(shape != 0xFFFFFFFF, expect)
    assert int(expect.sum()) == e["valid_count"]
    assert np.all(t[expect] == 5.0) and np.all(np.isinf(t[~expect]))


def test_cube_known_answers():
    mi = _mi()
    e = KA["cube"]
    c = np.asarray(e["coords"], np.float32)
    X, Y = np.meshgrid(c, c, indexing="ij")
    X, Y = X.ravel(), Y.ravel()
    n = X.size
    for sx, sy, sz in e["scales"]:
        scene = _scene_with({"type": "cube", "to_world": mi.Transform4f.scale([sx, sy, sz])})
        rays = np.zeros((7, n), np.float32)
        rays[0], rays[1], rays[2] = X, Y, e["origin_z"]
        rays[3:6] = np.asarray(e["dir"], np.float32)[:, None]
        rays[6] = np.finfo(np.float32).max
        expect = (np.abs(X) <= sx) & (np.abs(Y) <= sy)
        assert np.array_equal(O.trace_shadow(scene, rays).astype(bool), expect), e["source"]
        t, *_ = O.trace_closest(scene, rays)
        assert np.allclose(t[expect], 8.0 - sz, rtol=1e-6)
    scene = _scene_with({"type": "cube"})
    for o, d, nrm in e["faces"]:
        rays = np.array([[o[0]], [o[1]], [o[2]], [d[0]], [d[1]], [d[2]], [np.finfo(np.float32).max]], np.float32)
        t, u, v, prim, shape = O.trace_closest(scene, rays)
        assert shape[0] == 0 and abs(t[0] - 7.0) < 1e-6
        # the hit triangle's geometric normal is the face normal (test_cube.py test05)
        f = scene.faces.reshape(-1, 3)[prim[0]]
        p = scene.positions.reshape(-1, 3)[f].astype(np.float64)
        gn = np.cross(p[1] - p[0], p[2] - p[0])
        assert np.allclose(gn / np.linalg.norm(gn), nrm, atol=1e-6)


# ---- regression fixtures (oracle pinned against drift) ----------------------------------
def test_oracle_regression_fixtures():
    mi = _mi()
    L = O.lib()
    sf = np.zeros((64, 8), np.float32)
    for lane in range(64):
        L.oracle_sampler_floats(0, lane * 16, 8, sf[lane].ctypes.data_as(C.c_void_p))
    assert np.array_equal(sf, REG["sampler_floats_seed0"])
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 32
    scene = mi.load_dict(d)
    t, u, v, prim, shape = O.trace_closest(scene, REG["trace_rays"])
    assert np.array_equal(t, REG["trace_t"]) and np.array_equal(prim, REG["trace_prim"])
    assert np.array_equal(shape, REG["trace_shape"])
    film = O.render(scene, mi.load_dict({"type": "path", "max_depth": 8}), seed=1, spp=16, threads=4)
    assert np.array_equal(film, REG["film_32_spp16_seed1"])


# ---- PRB methodology tests ---------------------------------------------------------------
def _linear_scene(mi, spp):
    T = mi.Transform4f
    return mi.load_dict({
        "type": "scene",
        "integrator": {"type": "prb", "max_depth": 2},
        "sensor": {"type": "perspective", "near_clip": 0.1, "far_clip": 1000.0,
                   "to_world": T.look_at(origin=[0, 0, 4], target=[0, 0, 0], up=[0, 1, 0]),
                   "film": {"type": "hdrfilm", "rfilter": {"type": "box"}, "width": 1, "height": 1},
                   "sampler": {"type": "independent", "sample_count": spp}},
        "rect": {"type": "rectangle", "bsdf": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.6, 0.6, 0.6]}}},
        "light": {"type": "rectangle", "to_world": T.look_at(origin=[2, 0, 2], target=[0, 0, 0], up=[0, 1, 0]) @ T.scale([0.5, 0.5, 1]),
                  "bsdf": {"type": "null"},
                  "emitter": {"type": "area", "radiance": {"type": "rgb", "value": [10.0, 10.0, 10.0]}}},
    })


@pytest.mark.parametrize("spp", [1, 4, 44])
def test_prb_linearity(spp):
    """test_ad.py:6-92: loss(rho + lr) == loss(rho) + lr * dloss/drho for a
    scene whose radiance is linear in rho (one diffuse bounce)."""
    mi = _mi()
    scene = _linear_scene(mi, spp)
    integ = scene.integrator()
    key = "rect.bsdf.reflectance.value" if "rect.bsdf.reflectance.value" in scene.params else \
        [k for k in scene.params if k.endswith("reflectance.value")][0]
    tex = scene.params[key][1]
    loss1 = float(O.develop(O.render(scene, integ, seed=0, spp=spp)).sum())
    g = O.render_backward(scene, integ, 0, spp, np.ones((1, 1, 3), np.float32), [tex], [(3,)])[0]
    lr = 0.01
    scene.texture(tex).value[0] += lr
    loss2 = float(O.develop(O.render(scene, integ, seed=0, spp=spp)).sum())
    assert loss1 > 0
    assert np.isclose(loss1, loss2 - lr * g[0], rtol=1e-5, atol=1e-7)


def test_prb_gradient_vs_finite_differences():
    """test_ad_integrators.py:917-962 methodology: central differences at the
    same seed (no RR: max_depth 3 < rr_depth) vs render_backward."""
    mi = _mi()
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 16
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "prb", "max_depth": 3})
    key = "white.reflectance.value"
    tex = scene.params[key][1]
    spp, seed = 16, 3
    gi = np.full((16, 16, 3), 1.0 / (16 * 16 * 3), np.float32)
    g = O.render_backward(scene, integ, seed, spp, gi, [tex], [(3,)])[0]
    base = np.array(scene.texture(tex).value[:], np.float64)
    eps = 1e-3
    for c in range(3):
        vals = []
        for s in (+1, -1):
            v = base.copy()
            v[c] += s * eps
            scene.texture(tex).value[:] = [float(x) for x in v]
            vals.append(float(O.develop(O.render(scene, integ, seed=seed, spp=spp)).astype(np.float64).mean()))
        scene.texture(tex).value[:] = [float(x) for x in base]
        fd = (vals[0] - vals[1]) / (2 * eps)
        assert np.isclose(g[c], fd, rtol=2e-2), (c, g[c], fd)
