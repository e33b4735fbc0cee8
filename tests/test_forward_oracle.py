"""CPU checks of the oracle's render_forward (common.py:696-826), the checker
of tests/test_gpu_forward.py.  Parity with the reference is unpinned (it ships
no forward-mode images); the oracle's forward mode is pinned by two
properties of an exact derivative of the same seeded render:

  adjoint   <g_in, dI/dpi . t> == <dloss/dpi, t> against the oracle's
            render_backward (itself checked by the reference's linearity and
            FD tests, tests/test_oracle_golden.py) -- prb and prbvolpath
  FD        with Russian roulette off (rr_depth > max_depth) the prb image is
            smooth in the reflectance: central differences at eps = 1e-3
            (test_ad_integrators.py:917-962's methodology) match per pixel
"""
import numpy as np
import pytest
import torch

import oracle_py as O


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


def _cbox(mi, w=24, h=16, spp=16):
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = w
    d["sensor"]["film"]["height"] = h
    d["sensor"]["sampler"]["sample_count"] = spp
    return mi.load_dict(d)


def _fwd(scene, params, integ, tans, seed, spp):
    film = O.render_forward(scene, integ, seed, spp, [params.param_id(k) for k in tans],
                            [np.asarray(v, np.float32) for v in tans.values()], threads=4)
    return O.develop(film, scene.desc.sensor.pixel_format)


def test_oracle_forward_adjoint_identity_prb():
    mi = _mi()
    scene = _cbox(mi)
    prb = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    rng = np.random.default_rng(0)
    tans = {"white.reflectance.value": np.array([1.0, 0.5, -0.25], np.float32),
            "green.reflectance.value": np.array([0.1, 0.4, 0.2], np.float32)}
    img = _fwd(scene, params, prb, tans, 5, 16)
    gi = rng.random(img.shape).astype(np.float32)
    grads = O.render_backward(scene, prb, 5, 16, gi, [params.param_id(k) for k in tans], [(3,), (3,)], threads=4)
    lhs = float((gi.astype(np.float64) * img).sum())
    rhs = sum(float((g.astype(np.float64) * t).sum()) for g, t in zip(grads, tans.values()))
    assert abs(lhs - rhs) <= 1e-4 * abs(rhs), (lhs, rhs)


def test_oracle_forward_adjoint_identity_bitmap():
    mi = _mi()
    scene = mi.load_dict(mi.cornell_box_bitmap(tex_res=8, width=24, height=16, spp=8))
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    key = "white.reflectance.data"
    rng = np.random.default_rng(1)
    t = rng.standard_normal(tuple(params[key].shape)).astype(np.float32)
    img = _fwd(scene, params, prb, {key: t}, 3, 8)
    gi = rng.random(img.shape).astype(np.float32)
    g = O.render_backward(scene, prb, 3, 8, gi, [params.param_id(key)], [tuple(params[key].shape)], threads=4)[0]
    lhs = float((gi.astype(np.float64) * img).sum())
    rhs = float((g.astype(np.float64) * t).sum())
    assert abs(lhs - rhs) <= 1e-4 * abs(rhs), (lhs, rhs)


def test_oracle_forward_adjoint_identity_prbvolpath():
    mi = _mi()
    d = mi.volume_cube(16, 12, 4, grid=mi.fbm_grid(8), scale=4.0)
    d["integrator"] = {"type": "prbvolpath", "max_depth": 6, "rr_depth": 5}
    scene = mi.load_dict(d)
    integ = scene.integrator()
    params = mi.traverse(scene)
    rng = np.random.default_rng(2)
    tans = {"medium1.sigma_t.data": rng.random(tuple(params["medium1.sigma_t.data"].shape)).astype(np.float32),
            "medium1.albedo.value": np.array([0.3, -0.1, 0.2], np.float32)}
    img = _fwd(scene, params, integ, tans, 9, 4)
    gi = rng.standard_normal(img.shape).astype(np.float32)
    grads = O.render_backward(scene, integ, 9, 4, gi, [params.param_id(k) for k in tans],
                              [tuple(params[k].shape) for k in tans], threads=4)
    lhs = float((gi.astype(np.float64) * img).sum())
    rhs = sum(float((g.astype(np.float64) * t).sum()) for g, t in zip(grads, tans.values()))
    assert abs(lhs - rhs) <= 1e-3 * max(abs(rhs), 1e-6), (lhs, rhs)


def test_oracle_forward_finite_differences():
    mi = _mi()
    scene = _cbox(mi, 16, 12, 8)
    prb = mi.load_dict({"type": "prb", "max_depth": 6, "rr_depth": 100})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    t = np.array([1.0, 0.5, 0.25], np.float32)
    img = _fwd(scene, params, prb, {key: t}, 4, 8)
    v0 = params[key].clone()
    eps = 1e-3

    def render(v):
        params[key] = torch.as_tensor(v)
        params.update()
        return O.develop(O.render(scene, prb, 4, 8, threads=4))

    fd = (render(v0.numpy() + eps * t) - render(v0.numpy() - eps * t)) / (2 * eps)
    render(v0.numpy())
    np.testing.assert_allclose(img, fd, rtol=2e-2, atol=2e-3 * np.abs(img).max())


def test_oracle_forward_rejects_path():
    mi = _mi()
    scene = _cbox(mi, 8, 8, 4)
    params = mi.traverse(scene)
    with pytest.raises(RuntimeError, match="render_forward"):
        _fwd(scene, params, mi.load_dict({"type": "path"}), {"white.reflectance.value": np.ones(3)}, 0, 4)
