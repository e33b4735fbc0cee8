"""GPU parity of render_forward (RBIntegrator.render_forward, common.py:696-826):
the forward-mode gradient image of `prb` / `prbvolpath` through the C-ABI
(mh_render_forward) vs the CPU oracle, whose forward mode is the reference's
primal + forward replay (prb.py:244-248 `δL += dr.forward_to(Lo)`), run once
per colour channel through the adjoint sinks.  The HIP prb path is the
single-traversal regrouping (prb_forward), so the two differ by fp association
only.

Criteria:
  image     |d| <= 1e-4 + 2e-3 |ref| for >= 99.5 % of the pixel channels and
            mean |d| / mean |ref| < 1e-3 (splat atomics, the oracle's
            L_total - P_k cancellation on deep vertices)
  adjoint   <g_in, dI/dpi . t> == <dloss/dpi, t>: the forward image against
            render_backward at the same seed, rtol 2e-3 -- size independent,
            checked at config 3's own size (512^2 @ 64)
"""
import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def _mi():
    import mitsuba_hip as mi
    if not mi.is_available():
        pytest.fail("no HIP device / native library: the GPU tests need an MI355X")
    mi.set_variant("hip_ad_rgb")
    return mi


def _cbox(mi, w, h, spp, fmt=None):
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = w
    d["sensor"]["film"]["height"] = h
    d["sensor"]["sampler"]["sample_count"] = spp
    if fmt:
        d["sensor"]["film"]["pixel_format"] = fmt
    return mi.load_dict(d)


def _close(img, ref):
    d = np.abs(img - ref)
    ok = d <= 1e-4 + 2e-3 * np.abs(ref)
    assert ok.mean() >= 0.995, f"{(~ok).sum()} of {ok.size} channels off, max {d.max():.3e}"
    assert d.mean() / max(np.abs(ref).mean(), 1e-12) < 1e-3


def _gpu_forward(mi, scene, params, tans, integ, seed, spp, **kw):
    import torch
    t = {k: torch.as_tensor(v).cuda() for k, v in tans.items()}
    return mi.render_forward(scene, params, t, integ, seed=seed, spp=spp, **kw).cpu().numpy()


def _oracle_forward(scene, params, tans, integ, seed, spp):
    film = O.render_forward(scene, integ, seed, spp, [params.param_id(k) for k in tans],
                            [np.asarray(v, np.float32) for v in tans.values()])
    return O.develop(film, scene.desc.sensor.pixel_format)


@pytest.mark.parametrize("mode", ["auto", "mega"])
@pytest.mark.parametrize("fmt", [None, "rgba", "luminance"])
def test_render_forward_rgb_parity(fmt, mode, monkeypatch):
    """auto: the fused forward-mode wavefront (k_wf_bounce_fwd); mega: the
    per-sample kernel (k_render_forward, prb_forward)."""
    if mode == "mega":
        monkeypatch.setenv("MH_MODE", "mega")
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _cbox(mi, 40, 32, 16, fmt)
    integ = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    tans = {"white.reflectance.value": np.array([1.0, -0.5, 0.25], np.float32),
            "red.reflectance.value": np.array([0.3, 0.2, 0.1], np.float32)}
    st = A.Stats()
    img = _gpu_forward(mi, scene, params, tans, integ, 11, 16, stats=st)
    assert st.mode == (2 if mode == "auto" else 0)
    ref = _oracle_forward(scene, params, tans, integ, 11, 16)
    assert img.shape == ref.shape
    _close(img, ref)
    if fmt == "rgba":  # film.develop()'s alpha channel: the coverage (common.py:799-824)
        assert np.allclose(img[..., 3], ref[..., 3], atol=1e-5)


@pytest.mark.parametrize("mode", ["auto", "mega"])
@pytest.mark.parametrize("channels", [3, 1])
def test_render_forward_bitmap_parity(channels, mode, monkeypatch):
    if mode == "mega":
        monkeypatch.setenv("MH_MODE", "mega")
    mi = _mi()
    d = mi.cornell_box_bitmap(tex_res=8, width=32, height=24, spp=16)
    if channels == 1:
        d["white"]["reflectance"]["data"] = np.full((8, 8, 1), 0.7, np.float32)
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    key = "white.reflectance.data"
    rng = np.random.default_rng(3)
    tans = {key: rng.standard_normal(tuple(params[key].shape)).astype(np.float32),
            "green.reflectance.value": np.array([0.2, 0.9, -0.1], np.float32)}
    img = _gpu_forward(mi, scene, params, tans, integ, 5, 16)
    ref = _oracle_forward(scene, params, tans, integ, 5, 16)
    _close(img, ref)


def _pvp_scene(mi, w=24, h=20, spp=8, **kw):
    kw.setdefault("grid", mi.fbm_grid(16))
    kw.setdefault("scale", 4.0)
    d = mi.volume_cube(w, h, spp, **kw)
    d["integrator"] = {"type": "prbvolpath", "max_depth": 6, "rr_depth": 5}
    T = mi.Transform4f
    d["floor"] = {"type": "rectangle",
                  "to_world": T.translate([0, -1.2, 0]) @ T.rotate([1, 0, 0], -90) @ T.scale([3, 3, 3]),
                  "bsdf": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.6, 0.5, 0.4]}}}
    return mi.load_dict(d)


@pytest.mark.parametrize("homogeneous", [False, True])
def test_render_forward_prbvolpath_parity(homogeneous):
    mi = _mi()
    kw = {"medium_type": "homogeneous", "sigma_t": 0.8, "scale": 1.0} if homogeneous else {}
    scene = _pvp_scene(mi, **kw)
    integ = scene.integrator()
    params = mi.traverse(scene)
    sig = "medium1.sigma_t." + ("value" if homogeneous else "data")
    rng = np.random.default_rng(9)
    tans = {sig: rng.random(tuple(params[sig].shape)).astype(np.float32),
            "medium1.albedo.value": np.array([0.1, -0.2, 0.3], np.float32),
            "floor.bsdf.reflectance.value": np.array([0.5, 0.5, 0.5], np.float32)}
    img = _gpu_forward(mi, scene, params, tans, integ, 7, 8)
    ref = _oracle_forward(scene, params, tans, integ, 7, 8)
    d = np.abs(img - ref)
    # grid taps summed in float (GPU) vs double (oracle) along long walks
    ok = d <= 1e-4 + 5e-3 * np.abs(ref)
    assert ok.mean() >= 0.99, f"{(~ok).sum()} of {ok.size} off, max {d.max():.3e}"


def test_render_forward_adjoint_identity_config3():
    """BASELINE config 3 size (512^2 @ 64, prb max_depth 8): the forward image
    dotted with grad_in equals the backward gradient dotted with the tangent
    (both exact derivatives of the same seeded render)."""
    mi = _mi()
    import torch
    scene = _cbox(mi, 512, 512, 64)
    integ = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    tan = np.array([0.7, -0.3, 1.1], np.float32)
    img = _gpu_forward(mi, scene, params, {key: tan}, integ, 3, 64)
    gi = np.random.default_rng(1).random((512, 512, 3)).astype(np.float32) / (512 * 512 * 3)
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), [key], integ, seed=3, spp=64)[0]
    lhs = float((gi.astype(np.float64) * img).sum())
    rhs = float((g.cpu().numpy().astype(np.float64) * tan).sum())
    assert abs(lhs - rhs) <= 2e-3 * abs(rhs), (lhs, rhs)


def test_render_forward_adjoint_identity_config3b():
    """Config 3(b)'s size (64^2 x 3 bitmap, 512^2 @ 64): the tangent texels are
    gathered by tex_eval's bilinear taps, the backward scatters through the
    same taps -- the two are adjoint."""
    mi = _mi()
    import torch
    scene = mi.load_dict(mi.cornell_box_bitmap(64, 512, 512, 64))
    integ = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    key = "white.reflectance.data"
    t = np.random.default_rng(5).standard_normal(tuple(params[key].shape)).astype(np.float32)
    img = _gpu_forward(mi, scene, params, {key: t}, integ, 4, 64)
    gi = np.random.default_rng(6).random((512, 512, 3)).astype(np.float32) / (512 * 512 * 3)
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), [key], integ, seed=4, spp=64)[0]
    lhs = float((gi.astype(np.float64) * img).sum())
    rhs = float((g.cpu().numpy().astype(np.float64) * t).sum())
    assert abs(lhs - rhs) <= 2e-3 * max(abs(rhs), 1e-12), (lhs, rhs)


def test_render_forward_sample_slabs_add_up():
    """Sample-slab sharding of the forward-mode film: the
    films of slabs [0, 8) and [8, 16) sum to the one-call film."""
    mi = _mi()
    import torch
    scene = _cbox(mi, 48, 40, 16)
    integ = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    t = {"white.reflectance.value": torch.tensor([1.0, 2.0, 0.5], device="cuda")}
    full = mi.render_forward(scene, params, t, integ, seed=9, spp=16, develop_image=False).cpu().numpy()
    parts = [mi.render_forward(scene, params, t, integ, seed=9, spp=16, spp_begin=b, spp_end=e,
                               develop_image=False).cpu().numpy() for b, e in ((0, 8), (8, 16))]
    np.testing.assert_allclose(parts[0] + parts[1], full, rtol=1e-5, atol=1e-6)


def test_render_forward_torch_forward_ad():
    """mi.render under torch.autograd.forward_ad: _RenderOp.jvp runs
    render_forward at (seed_grad, spp_grad), as _RenderOp.forward does
    (util.py:386-395)."""
    mi = _mi()
    import torch
    import torch.autograd.forward_ad as fwAD
    scene = _cbox(mi, 32, 24, 8)
    integ = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    tan = torch.tensor([1.0, 0.5, 0.25])
    with fwAD.dual_level():
        params[key] = fwAD.make_dual(params[key].detach(), tan.to(params[key].device))
        img = mi.render(scene, params, integrator=integ, spp=8, seed=2)
        primal, jvp = fwAD.unpack_dual(img)
    assert jvp is not None
    ref = mi.render_forward(scene, params, {key: tan}, integ, seed=mi.sample_tea_32(2, 1)[0], spp=8)
    np.testing.assert_allclose(jvp.cpu().numpy(), ref.cpu().numpy(), rtol=1e-6, atol=1e-7)
    assert primal.shape == (24, 32, 3)


def test_render_forward_errors():
    mi = _mi()
    import torch
    scene = _cbox(mi, 16, 16, 4)
    params = mi.traverse(scene)
    path = mi.load_dict({"type": "path"})
    with pytest.raises(mi.MitsubaHipError, match="render_forward"):
        mi.render_forward(scene, params, {"white.reflectance.value": torch.ones(3)}, path)
    prb = mi.load_dict({"type": "prb"})
    with pytest.raises(mi.MitsubaHipError, match="shape"):
        mi.render_forward(scene, params, {"white.reflectance.value": torch.ones(4)}, prb)
