"""The two-stream chunk pipeline of the fused wavefront (mh_api.hip
fork_stream): odd chunks of mh_render / mh_render_backward run on a second
stream with their own workspace, and a single-chunk call of >= 2^19 samples
is split in two.  The samples are the same as on one stream (the chunking
changes which launch renders a pixel, not its lanes), so the film, the rgb
gradient and the bitmap gradient equal the one-stream call up to float
summation order (MH_WF_STREAMS=1 keeps one stream; MH_FLAG_SHARED_DEVICE
calls keep one too)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mi():
    import mitsuba_hip as mi
    if not mi.is_available():
        pytest.fail("no HIP device / native library: the GPU tests need an MI355X")
    mi.set_variant("hip_ad_rgb")
    return mi


def _both(fn):
    """fn() with the two-stream pipeline (default) and with one stream."""
    old = os.environ.pop("MH_WF_STREAMS", None)
    try:
        a = fn()
        os.environ["MH_WF_STREAMS"] = "1"
        b = fn()
    finally:
        os.environ.pop("MH_WF_STREAMS", None)
        if old is not None:
            os.environ["MH_WF_STREAMS"] = old
    return a, b


def test_forward_two_streams_equal_one():
    mi = _mi()
    from mitsuba_hip import _abi as A
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = 256, 255  # odd pixel count: unequal halves
    s = mi.load_dict(d)
    integ = mi.load_dict({"type": "path", "max_depth": 6})

    def run():
        st = A.Stats()
        f = mi.render_film(s, integ, seed=5, spp=16, stats=st).cpu().numpy()
        return f, st.n_aux_launches, st.rays_closest

    (f2, n2, r2), (f1, n1, r1) = _both(run)
    assert (n2, n1) == (2, 1) and r2 == r1  # 256 * 255 * 16 >= 2^19 samples: split in two, the same paths
    np.testing.assert_allclose(f2, f1, rtol=2e-5, atol=1e-6)


def test_rgb_prb_two_streams_equal_one():
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = 192, 160
    s = mi.load_dict(d)
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(s)
    keys = ["white.reflectance.value", "red.reflectance.value"]
    gi = torch.full((160, 192, 3), 1.0 / (160 * 192 * 3), device="cuda")

    def run():
        st = A.Stats()
        g = mi.render_backward(s, params, gi, keys, integ, seed=9, spp=32, stats=st)
        return [x.cpu().numpy() for x in g], st.n_trace_launches, st.rays_closest

    (g2, n2, r2), (g1, n1, r1) = _both(run)
    assert (n2, n1) == (2 * 6, 6) and r2 == r1
    for a, b in zip(g2, g1):
        assert np.abs(b).min() > 0
        np.testing.assert_allclose(a, b, rtol=1e-4)


def test_bitmap_two_streams_equal_one():
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    s = mi.load_dict(mi.cornell_box_bitmap(16, 160, 128, 32))
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(s)
    key = "white.reflectance.data"
    gi = torch.full((128, 160, 3), 1.0 / (128 * 160 * 3), device="cuda")

    def run():
        st = A.Stats()
        (g,) = mi.render_backward(s, params, gi, [key], integ, seed=4, spp=32, stats=st)
        return g.cpu().numpy(), st.n_aux_launches, st.aux_items

    (g2, n2, a2), (g1, n1, a1) = _both(run)
    assert (n2, n1) == (2, 1) and a2 == a1  # the same vertex records, in two scatters
    assert np.abs(g1).max() > 0
    np.testing.assert_allclose(g2, g1, rtol=1e-4, atol=1e-6 * np.abs(g1).max())


def test_shared_device_flag_keeps_one_stream():
    mi = _mi()
    from mitsuba_hip import _abi as A
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = 256, 255
    s = mi.load_dict(d)
    integ = mi.load_dict({"type": "path", "max_depth": 6})
    st, st2 = A.Stats(), A.Stats()
    f = mi.render_film(s, integ, seed=5, spp=16, stats=st, shared=True).cpu().numpy()
    g = mi.render_film(s, integ, seed=5, spp=16, stats=st2).cpu().numpy()
    assert (st.n_aux_launches, st2.n_aux_launches) == (1, 2)  # the hint: another call runs beside, one stream
    np.testing.assert_allclose(f, g, rtol=2e-5, atol=1e-6)


def _blob(mi, n_tri=6000, w=256, h=256):
    # a displaced UV sphere in the box: a BVH in global memory, traced by the
    # per-lane stream engine (unfused trace / shade / shadow kernels)
    m = max(8, int(np.sqrt(n_tri / 4)))
    th = np.linspace(0, np.pi, m + 1)
    ph = np.linspace(0, 2 * np.pi, 2 * m + 1)
    T_, P_ = np.meshgrid(th, ph, indexing="ij")
    r = 1.0 + 0.08 * np.sin(7 * T_) * np.cos(9 * P_)
    V = np.stack([r * np.sin(T_) * np.cos(P_), r * np.cos(T_), r * np.sin(T_) * np.sin(P_)], -1).reshape(-1, 3)
    a = (np.arange(m)[:, None] * (2 * m + 1) + np.arange(2 * m)[None, :]).reshape(-1)
    F = np.concatenate([np.stack([a, a + 2 * m + 1, a + 1], 1), np.stack([a + 1, a + 2 * m + 1, a + 2 * m + 2], 1)])
    d = mi.cornell_box()
    d["sensor"]["film"].update(width=w, height=h)
    T = mi.Transform4f
    d["blob"] = {"type": "mesh", "vertex_positions": V.astype(np.float32), "faces": F.astype(np.uint32),
                 "to_world": T.translate([0, -0.45, 0]) @ T.scale(0.45), "bsdf": {"type": "ref", "id": "white"}}
    return mi.load_dict(d)


@pytest.mark.parametrize("stack", ["20", "4"])
def test_stream_engine_two_streams_equal_one(stack, monkeypatch):
    # "4": a 4-entry LDS stack, so most rays use the global overflow columns,
    # which the second stream's launches have their own copy of
    monkeypatch.setenv("MH_STREAM_STACK", stack)
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    s = _blob(mi)
    integ = mi.load_dict({"type": "path", "max_depth": 6})

    def run():
        st = A.Stats()
        f = mi.render_film(s, integ, seed=3, spp=16, stats=st).cpu().numpy()
        return f, st.n_aux_launches, st.rays_closest, st.mode

    (f2, n2, r2, m2), (f1, n1, r1, m1) = _both(run)
    assert (m2, m1) == (1, 1)  # the unfused stream-engine pipeline
    assert (n2, n1) == (2, 1) and r2 == r1
    np.testing.assert_allclose(f2, f1, rtol=2e-5, atol=1e-6)
    # the PRB gradient of the same scene (unfused k_wf_shade_prb / k_wf_shadow_prb)
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(s)
    gi = torch.full((256, 256, 3), 1.0 / (256 * 256 * 3), device="cuda")

    def runb():
        st = A.Stats()
        (g,) = mi.render_backward(s, params, gi, ["white.reflectance.value"], prb, seed=7, spp=16, stats=st)
        return g.cpu().numpy(), st.n_trace_launches, st.rays_closest

    (g2, t2, q2), (g1, t1, q1) = _both(runb)
    assert (t2, t1) == (2 * 6, 6) and q2 == q1
    assert np.abs(g1).min() > 0
    np.testing.assert_allclose(g2, g1, rtol=1e-4)
