"""CPU: mi.ad.SGD / Adam (ad/optimizers.py) against
a numpy restatement of the reference's update rules."""
import numpy as np
import pytest
import torch


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


def _grads(n, shape, seed=0):
    r = np.random.default_rng(seed)
    gs = r.standard_normal((n,) + shape).astype(np.float32)
    gs[1, 0] = 0.0    # an unobserved entry (mask_updates)
    return gs


@pytest.mark.parametrize("mask_updates", [False, True])
@pytest.mark.parametrize("uniform", [False, True])
def test_adam_matches_reference_rule(mask_updates, uniform):
    mi = _mi()
    shape = (5, 3)
    p0 = np.random.default_rng(1).random(shape).astype(np.float32)
    gs = _grads(4, shape)
    opt = mi.ad.Adam(lr=0.05, mask_updates=mask_updates, uniform=uniform)
    opt["x"] = torch.from_numpy(p0)
    b1, b2, eps = 0.9, 0.999, 1e-8
    p, m, v = p0.astype(np.float64), np.zeros(shape), np.zeros(shape)
    for t, g in enumerate(gs, 1):
        opt["x"].grad = torch.from_numpy(g)
        opt.step()
        lr_t = 0.05 * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        m_t, v_t = b1 * m + (1 - b1) * g, b2 * v + (1 - b2) * g.astype(np.float64) ** 2
        nz = g != 0
        if mask_updates:
            m_t, v_t = np.where(nz, m_t, m), np.where(nz, v_t, v)
        m, v = m_t, v_t
        step = lr_t * m / ((np.sqrt(v.max()) if uniform else np.sqrt(v)) + eps)
        if mask_updates:
            step = np.where(nz, step, 0)
        p = p - step
        np.testing.assert_allclose(opt["x"].detach().numpy(), p, rtol=1e-5, atol=1e-6)
        assert opt["x"].requires_grad and opt["x"].grad is None


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_sgd_matches_reference_rule(momentum):
    """Momentum SGD steps with the *previous* state (optimizers.py:160-168)."""
    mi = _mi()
    shape = (7,)
    p0 = np.linspace(0, 1, 7).astype(np.float32)
    gs = _grads(3, shape, 2)
    opt = mi.ad.SGD(lr=0.1, momentum=momentum)
    opt["x"] = torch.from_numpy(p0)
    p, s = p0.astype(np.float64), np.zeros(shape)
    for g in gs:
        opt["x"].grad = torch.from_numpy(g)
        opt.step()
        if momentum:
            step = 0.1 * s
            s = momentum * s + g
        else:
            step = 0.1 * g
        p = p - step
        np.testing.assert_allclose(opt["x"].detach().numpy(), p, rtol=1e-6, atol=1e-7)


def test_optimizer_container_semantics():
    mi = _mi()
    opt = mi.ad.Adam(lr={"a": 0.1} if False else 0.1)
    opt["a"] = torch.ones(3)
    opt["a"].grad = torch.ones(3)
    opt.step()
    assert opt.t["a"] == 1
    opt["a"] = torch.zeros(3)            # same shape: state kept
    assert opt.t["a"] == 1
    opt["a"] = torch.zeros(4)            # new shape: state reset
    assert opt.t["a"] == 0
    with pytest.raises(Exception, match="differentiable"):
        opt["b"] = torch.zeros(3, dtype=torch.int32)
    opt.set_learning_rate({"a": 0.5})
    assert opt.lr["a"] == 0.5 and "a" in opt and len(opt) == 1


def test_render_1_is_rejected_in_rgb_variants():
    mi = _mi()
    sc = mi.load_dict(mi.cornell_box())
    with pytest.raises(RuntimeError, match="monochromatic and spectral"):
        mi.render_1(sc)


def test_render_1_prb_returns_zero_spectrum_in_rgb(monkeypatch):
    """ADIntegrator.render_1 (ad/integrators/common.py:113-196), which prb and
    prbvolpath inherit, renders the primal and returns Spectrum(0) * nf in RGB
    modes instead of raising as the C++ SamplingIntegrator::render_1 of path /
    volpath does (integrator.cpp:398-411)."""
    import importlib
    import torch
    mi = _mi()
    R = importlib.import_module("mitsuba_hip.render")  # the module (the package exports the render function)
    sc = mi.load_dict(mi.cornell_box())
    calls = []

    def fake_film(scene, integrator=None, seed=0, spp=0, **kw):  # the primal pass (no device here)
        calls.append((integrator.type, seed, spp))
        return torch.zeros((scene.height, scene.width, 4))
    monkeypatch.setattr(R, "render_film", fake_film)
    for t in ("prb", "prbvolpath"):
        out = mi.render_1(sc, seed=3, spp=4, integrator=mi.load_dict({"type": t}))
        assert out.shape == (3,) and out.dtype == torch.float32 and float(out.abs().sum()) == 0.0
    assert calls[:2] == [("prb", 3, 4), ("prbvolpath", 3, 4)]
    # mi.render_1's own signature (util.py:627-634): params second, positionally
    params = mi.traverse(sc)
    out = mi.render_1(sc, params, 0, mi.load_dict({"type": "prb"}), 5, 0, 8, 8)
    assert out.shape == (3,) and float(out.abs().sum()) == 0.0
    assert calls[-1] == ("prb", 5, 8)
    out = mi.render_1(sc, params=params, integrator=mi.load_dict({"type": "prb"}), seed=1, seed_grad=2, spp_grad=4)
    assert calls[-1] == ("prb", 1, sc.sample_count())
    with pytest.raises(RuntimeError, match="should be different"):
        mi.render_1(sc, params, integrator=mi.load_dict({"type": "prb"}), seed=3, seed_grad=3)
    with pytest.raises(RuntimeError, match="SceneParameter"):
        mi.render_1(sc, {"a": 1}, integrator=mi.load_dict({"type": "prb"}))
    with pytest.raises(RuntimeError, match="monochromatic and spectral"):  # path keeps the C++ behaviour
        mi.render_1(sc, integrator=mi.load_dict({"type": "path"}))
    with pytest.raises(RuntimeError, match="monochromatic and spectral"):
        mi.render_1(sc, integrator=mi.load_dict({"type": "volpath"}))
