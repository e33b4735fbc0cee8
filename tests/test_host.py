"""CPU: host-side mirror of the reference interface (mi.load_dict / traverse
/ render argument handling / transforms / camera constants).  No GPU."""
import math

import numpy as np
import pytest


@pytest.fixture(scope="module")
def mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


def test_variants(mi):
    assert "hip_ad_rgb" in mi.variants()
    assert mi.variant() == "hip_ad_rgb"
    with pytest.raises(Exception):
        mi.set_variant("cuda_ad_rgb")


def test_integrator_properties(mi):
    """integrator.cpp:22-28,1281-1298; common.py:29-41"""
    p = mi.load_dict({"type": "path"})
    assert (p.max_depth, p.rr_depth, p.hide_emitters) == (0xFFFFFFFF, 5, False)  # -1 = infinite
    q = mi.load_dict({"type": "prb", "max_depth": 8, "rr_depth": 3, "hide_emitters": True})
    assert (q.max_depth, q.rr_depth, q.hide_emitters) == (8, 3, True)
    with pytest.raises(RuntimeError, match="rr_depth"):
        mi.load_dict({"type": "path", "rr_depth": 0})
    with pytest.raises(RuntimeError, match="max_depth"):
        mi.load_dict({"type": "path", "max_depth": -2})


def test_unsupported_plugins_raise(mi):
    with pytest.raises(RuntimeError, match="not available"):
        mi.load_dict({"type": "scene", "s": {"type": "sphere"}})
    with pytest.raises(RuntimeError):
        mi.load_dict({"type": "scene", "r": {"type": "rectangle",
                                              "bsdf": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [1.5, 0, 0]}}}})


def test_cornell_box_description(mi):
    scene = mi.load_dict(mi.cornell_box())
    assert (scene.width, scene.height, scene.sample_count()) == (256, 256, 64)
    d = scene.desc
    assert d.n_shapes == 8 and d.n_emitters == 1 and d.n_faces == 24
    keys = set(scene.params)
    for k in ("white.reflectance.value", "red.reflectance.value", "green.reflectance.value",
              "light.emitter.radiance.value"):
        assert k in keys
    params = mi.traverse(scene)
    assert np.allclose(params["white.reflectance.value"].numpy(), [0.885809, 0.698859, 0.666422], atol=1e-6)
    assert np.allclose(params["light.emitter.radiance.value"].numpy() if "light.emitter.radiance.value" in params
                       else [18.387, 13.9873, 6.75357], [18.387, 13.9873, 6.75357], atol=1e-4)
    s = d.sensor
    assert s.rfilter == 1 and abs(s.rfilter_radius - 2.0) < 1e-7  # gaussian sigma 0.5
    assert abs(s.near_clip - 0.001) < 1e-9 and abs(s.far_clip - 100.0) < 1e-5


def test_scene_parameters_update_without_device(mi):
    scene = mi.load_dict(mi.cornell_box())
    params = mi.traverse(scene)
    params["red.reflectance.value"] = [0.25, 0.5, 0.75]
    params.update()
    tex = scene.params["red.reflectance.value"][1]
    assert list(scene.texture(tex).value) == pytest.approx([0.25, 0.5, 0.75])
    with pytest.raises(KeyError):
        params["nope"] = 1.0


def test_transforms(mi):
    T = mi.Transform4f
    t = T.look_at(origin=[0, 0, 3.9], target=[0, 0, 0], up=[0, 1, 0])
    R = t.matrix[:3, :3]
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
    assert np.allclose(t.matrix[:3, 3], [0, 0, 3.9])
    assert np.allclose(t.matrix[:3, 2], [0, 0, -1])  # looks down -z
    c = T.translate([1, 2, 3]).rotate([0, 0, 1], 90).scale([2, 2, 2])
    p = c @ np.array([1.0, 0, 0])
    assert np.allclose(p, [1, 4, 3], atol=1e-12)
    assert np.allclose((c.inverse() @ c).matrix, np.eye(4), atol=1e-12)


def test_fov_axis(mi):
    from mitsuba_hip.scene import parse_fov
    assert parse_fov({"fov": 40, "fov_axis": "x"}, 2.0) == 40
    y = parse_fov({"fov": 40, "fov_axis": "y"}, 2.0)
    assert math.isclose(math.tan(math.radians(y) / 2), 2 * math.tan(math.radians(20)))
    assert parse_fov({"fov": 40, "fov_axis": "smaller"}, 2.0) == y
    with pytest.raises(RuntimeError):
        parse_fov({"fov": 40, "fov_axis": "bad"}, 1.0)


def test_render_argument_checks(mi):
    scene = mi.load_dict(mi.cornell_box())
    with pytest.raises(RuntimeError, match="SceneParameter"):
        mi.render(scene, params={"a": 1})
    params = mi.traverse(scene)
    params["white.reflectance.value"].requires_grad_()
    with pytest.raises(RuntimeError, match="seed"):
        mi.render(scene, params, seed=3, seed_grad=3)


def test_seed_grad_default(mi):
    # util.py:614-622: seed_grad = sample_tea_32(seed, 1)[0]
    assert mi.sample_tea_32(0, 1)[0] != 0
    assert mi.sample_tea_32(5, 1) == mi.sample_tea_32(5, 1)


def test_bitmap_texture_params(mi):
    data = np.full((4, 8, 3), 0.5, np.float32)
    scene = mi.load_dict({"type": "scene",
                          "r": {"type": "rectangle", "bsdf": {"type": "diffuse", "reflectance": {"type": "bitmap", "data": data}}}})
    key = [k for k in scene.params if k.endswith("reflectance.data")][0]
    params = mi.traverse(scene)
    assert tuple(params[key].shape) == (4, 8, 3)
    params[key] = np.full((4, 8, 3), 0.25, np.float32)
    params.update()
    assert np.allclose(scene.texture_data(scene.params[key][1]), 0.25)


def test_hdrfilm_pixel_formats():
    """hdrfilm.cpp:160-188: the six pixel formats, their film / image
    channel counts, and the reference's error for anything else."""
    import mitsuba_hip as mi
    from mitsuba_hip import _abi as A
    want = {"rgb": (A.PIXEL_RGB, 4, 3), "luminance": (A.PIXEL_Y, 4, 1), "xyz": (A.PIXEL_XYZ, 4, 3),
            "rgba": (A.PIXEL_RGBA, 5, 4), "luminance_alpha": (A.PIXEL_YA, 5, 2), "xyza": (A.PIXEL_XYZA, 5, 4)}
    for pf, (fmt, fch, ich) in want.items():
        d = mi.cornell_box()
        d["sensor"]["film"]["pixel_format"] = pf.upper() if pf == "rgba" else pf
        s = mi.load_dict(d)
        assert s.desc.sensor.pixel_format == fmt
        assert (A.film_channels(fmt), A.image_channels(fmt)) == (fch, ich)
    d = mi.cornell_box()
    d["sensor"]["film"]["pixel_format"] = "rgbe"
    with pytest.raises(RuntimeError, match="luminance_alpha"):
        mi.load_dict(d)


def test_oracle_alpha_develop():
    """oracle develop of R G B A W films: colour / w, then alpha / w."""
    import numpy as np
    import oracle_py as O
    from mitsuba_hip import _abi as A
    rng = np.random.default_rng(0)
    f = rng.random((3, 4, 5)).astype(np.float32) + 0.1
    f[0, 0, 4] = 0.0
    rgba = O.develop(f, A.PIXEL_RGBA)
    d = np.where(f[..., 4:] == 0, 1, f[..., 4:])
    np.testing.assert_allclose(rgba[..., :3], f[..., :3] / d, rtol=1e-6)
    np.testing.assert_allclose(rgba[..., 3], f[..., 3] / d[..., 0], rtol=1e-6)
    ya = O.develop(f, A.PIXEL_YA)
    y = O.develop(np.concatenate([f[..., :3], f[..., 4:]], -1), A.PIXEL_Y)
    np.testing.assert_array_equal(ya[..., :1], y)
    np.testing.assert_array_equal(ya[..., 1], rgba[..., 3])
    xyza = O.develop(f, A.PIXEL_XYZA)
    xyz = O.develop(np.concatenate([f[..., :3], f[..., 4:]], -1), A.PIXEL_XYZ)
    np.testing.assert_array_equal(xyza[..., :3], xyz)
