"""SURVEY.md §5 auxiliaries on the device path.

* invalid-sample counter: the test of ImageBlock::put's warn_invalid /
  warn_negative (src/render/imageblock.cpp:180-204: a channel < -1e-5 or not
  finite) evaluated in the splat kernels and returned as
  mh_stats.invalid_samples -- checked against the per-sample radiance the
  same render produces (mh_render_samples, bit-identical per sample);
* deterministic splat (MH_FLAG_DETERMINISTIC, the ordered-reduction build
  to diff the float-atomic build against): bit-identical films from run to
  run, equal to the atomic film within the splat's float-order tolerance and
  to the oracle, over several wavefront chunks and with an alpha film
  (gradients are not covered: the wavefront queues are compacted by
  wave-ballot atomics, so the order in which a thread's registers
  accumulate paths varies from run to run);
* roctx ranges: the library links the roctx API (the ScopedPhase ranges);
* asynchronous entry points (MH_FLAG_NO_SYNC): same results once the stream
  drains.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def _mi():
    import mitsuba_hip as mi
    if not mi.is_available():
        pytest.fail("no HIP device / native library: the GPU tests need an MI355X")
    return mi


def _cbox(mi, w, h, spp, light=None):
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = w, h
    d["sensor"]["sampler"]["sample_count"] = spp
    if light is not None:
        d["light"]["emitter"]["radiance"]["value"] = light
    return d


def _samples(mi, scene, integ, seed, spp, flags=0):
    from mitsuba_hip import _abi as A
    n = scene.width * scene.height * spp
    out = np.zeros(5 * n, np.float32)
    ic = integ.c()
    A.check(A.lib().mh_render_samples(scene.handle(0), C.byref(ic), seed, spp, 0, 0,
                                      out.ctypes.data_as(C.c_void_p), flags))
    return out[:3 * n].reshape(3, n).T


@pytest.mark.parametrize("light,mode", [(None, "auto"), ([-1.0, 2.0, 3.0], "auto"), ([-1.0, 2.0, 3.0], "mega"),
                                        ([float("inf"), 1.0, 1.0], "auto")])
def test_invalid_sample_counter(light, mode):
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = mi.load_dict(_cbox(mi, 40, 32, 16, light))
    integ = mi.load_dict({"type": "path", "max_depth": 6})
    st = A.Stats()
    mi.render_film(scene, integ, seed=3, spp=16, stats=st, mode=mode)
    L = _samples(mi, scene, integ, 3, 16, A.FLAG_MEGAKERNEL if mode == "mega" else 0)
    expect = int(np.sum(np.any(~(L >= -1e-5) | ~np.isfinite(L), axis=1)))
    assert st.invalid_samples == expect
    assert (expect == 0) == (light is None)


@pytest.mark.parametrize("sky", [0.2, -0.2])
def test_invalid_sample_counter_volpath(sky):
    """volpath (the phase-scheduled kernel, whose work head shares the
    counter block): a negative sky gives negative samples."""
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = mi.load_dict(mi.volume_cube(24, 20, 8, grid=mi.fbm_grid(16), scale=4.0, sky=sky, max_depth=8))
    integ = scene.integrator()
    st = A.Stats()
    mi.render_film(scene, integ, seed=2, spp=8, stats=st)
    assert st.mode == 3
    L = _samples(mi, scene, integ, 2, 8, A.FLAG_WAVEFRONT)
    expect = int(np.sum(np.any(~(L >= -1e-5) | ~np.isfinite(L), axis=1)))
    assert st.invalid_samples == expect
    assert (expect == 0) == (sky > 0)


@pytest.mark.parametrize("chunk", [None, "4096"])
def test_deterministic_film_bit_reproducible(chunk, monkeypatch):
    if chunk:
        monkeypatch.setenv("MH_WF_CHUNK", chunk)
    mi = _mi()
    scene = mi.load_dict(_cbox(mi, 48, 40, 16))
    integ = scene.integrator()
    a = mi.render_film(scene, integ, seed=4, spp=16, deterministic=True).cpu().numpy()
    b = mi.render_film(scene, integ, seed=4, spp=16, deterministic=True).cpu().numpy()
    assert np.array_equal(a, b)
    atomic = mi.render_film(scene, integ, seed=4, spp=16).cpu().numpy()
    np.testing.assert_allclose(a, atomic, rtol=1e-5, atol=1e-6)
    ref = O.render(scene, integ, seed=4, spp=16)
    ok = np.all(np.abs(a - ref) <= 1e-4 * np.maximum(1.0, np.abs(ref)), axis=-1)
    assert ok.mean() >= 0.995


def test_deterministic_weights_and_alpha():
    mi = _mi()
    d = _cbox(mi, 36, 28, 8)
    d["sensor"]["film"]["pixel_format"] = "rgba"
    scene = mi.load_dict(d)
    integ = scene.integrator()
    a = mi.render_film(scene, integ, seed=9, spp=8, deterministic=True).cpu().numpy()
    b = mi.render_film(scene, integ, seed=9, spp=8, deterministic=True).cpu().numpy()
    assert a.shape[-1] == 5 and np.array_equal(a, b)
    np.testing.assert_allclose(a, mi.render_film(scene, integ, seed=9, spp=8).cpu().numpy(), rtol=1e-5, atol=1e-6)
    w1 = mi.prb_weights(scene, 9, 8, deterministic=True).cpu().numpy()
    w2 = mi.prb_weights(scene, 9, 8, deterministic=True).cpu().numpy()
    assert np.array_equal(w1, w2)
    np.testing.assert_allclose(w1, mi.prb_weights(scene, 9, 8).cpu().numpy(), rtol=1e-5)
    np.testing.assert_allclose(w1, a[..., 4], rtol=1e-5)  # the film's W channel is the same sum


@pytest.mark.parametrize("chunk,keys", [(None, ["white.reflectance.value"]),
                                        ("65536", ["white.reflectance.value", "red.reflectance.value"])])
def test_deterministic_prb_gradient_bit_reproducible(chunk, keys, monkeypatch):
    """MH_FLAG_DETERMINISTIC on the fused PRB wavefront: every path carries
    its own gradient sum and the sums are reduced in path-id order, so
    repeated runs give the same bits (also over several wavefront chunks and
    with two rgb slots); equal to the atomic-order build and to the oracle
    within the float-order tolerance (prb.py:245-246 scatter)."""
    if chunk:
        monkeypatch.setenv("MH_WF_CHUNK", chunk)
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    scene = mi.load_dict(_cbox(mi, 64, 48, 32))
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    gi = torch.full((48, 64, 3), 1.0 / (48 * 64 * 3), device="cuda:0")
    st = A.Stats()
    runs = [mi.render_backward(scene, params, gi, keys, prb, seed=5, spp=32, deterministic=True, stats=st)
            for _ in range(3)]
    assert st.mode == 1  # the fused wavefront
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    atomic = mi.render_backward(scene, params, gi, keys, prb, seed=5, spp=32)
    ref = O.render_backward(scene, prb, 5, 32, gi.cpu().numpy(), [params.texture_of(k) for k in keys],
                            [(3,)] * len(keys))
    for a, b, r in zip(runs[0], atomic, ref):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-5)
        np.testing.assert_allclose(a.cpu().numpy(), r, rtol=1e-3)


@pytest.mark.parametrize("chunk", [None, "4096"])
def test_deterministic_prb_bitmap_gradient_bit_reproducible(chunk, monkeypatch):
    """MH_FLAG_DETERMINISTIC with bitmap parameters on the fused PRB
    wavefront: the texel scatter runs as a max pass and an int64 fixed-point
    pass per chunk (exact sums, folded into the float gradient in chunk
    order), the rgb slot beside it by per-path sums; repeated runs give the
    same bits, equal to the float build and to the oracle within tolerance."""
    if chunk:
        monkeypatch.setenv("MH_WF_CHUNK", chunk)
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    scene = mi.load_dict(mi.cornell_box_bitmap(tex_res=8, width=48, height=40, spp=16))
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    keys = ["white.reflectance.data", "red.reflectance.value"]
    gi = torch.from_numpy(np.random.default_rng(9).random((40, 48, 3)).astype(np.float32) / (40 * 48 * 3)).cuda()
    st = A.Stats()
    runs = [mi.render_backward(scene, params, gi, keys, prb, seed=7, spp=16, deterministic=True, stats=st)
            for _ in range(3)]
    assert st.mode == 1
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    flt = mi.render_backward(scene, params, gi, keys, prb, seed=7, spp=16)
    ref = O.render_backward(scene, prb, 7, 16, gi.cpu().numpy(), [params.texture_of(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for k, a, b, r in zip(keys, runs[0], flt, ref):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6 * np.abs(r).max(), err_msg=k)
        np.testing.assert_allclose(a, r, rtol=2e-3, atol=1e-9 + 2e-4 * np.abs(r).max(), err_msg=k)


def test_async_entry_points_match_synchronous():
    """MH_FLAG_DEVICE_POINTERS | MH_FLAG_NO_SYNC without stats: mh_render,
    mh_prb_weights and mh_render_backward return with their work enqueued on
    the scene's stream; once the stream drains, the film, W image and
    gradient equal the synchronous calls' (deterministic splat: bitwise)."""
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    scene = mi.load_dict(_cbox(mi, 64, 48, 16))
    path = mi.load_dict({"type": "path", "max_depth": 8})
    prb = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    st = torch.cuda.current_stream()
    h = scene.handle(0, st.cuda_stream)
    lib = A.lib()
    P = lambda t: C.c_void_p(t.data_ptr())
    results = []
    for flags in (A.FLAG_DEVICE_POINTERS | A.FLAG_DETERMINISTIC,
                  A.FLAG_DEVICE_POINTERS | A.FLAG_DETERMINISTIC | A.FLAG_NO_SYNC):
        film = torch.full((48, 64, 4), -1.0, device="cuda")
        w = torch.full((48, 64), -1.0, device="cuda")
        gi = torch.full((48, 64, 3), 1.0 / (48 * 64 * 3), device="cuda")
        g = torch.zeros(3, device="cuda")
        ic_f, ic_b = path.c(), prb.c()
        A.check(lib.mh_render(h, C.byref(ic_f), 3, 16, 0, 0, P(film), flags, None))
        A.check(lib.mh_prb_weights(h, 5, 16, 0, 0, P(w), flags))
        ids = (C.c_uint32 * 1)(params.param_id(key))
        ptrs = (C.c_void_p * 1)(g.data_ptr())
        A.check(lib.mh_render_backward(h, C.byref(ic_b), 5, 16, 0, 0, P(gi), P(w), 1, ids, ptrs, flags, None))
        torch.cuda.synchronize()
        results.append((film.cpu().numpy(), w.cpu().numpy(), g.cpu().numpy()))
    (f0, w0, g0), (f1, w1, g1) = results
    assert np.array_equal(f0, f1) and np.array_equal(w0, w1)
    assert f0.min() >= 0.0 and w0.min() > 0.0
    np.testing.assert_allclose(g1, g0, rtol=1e-5)


@pytest.mark.parametrize("case", ["bitmap_replay", "bitmap_replay_global", "rgb_mega"])
def test_deterministic_prb_replay_bit_reproducible(case, monkeypatch):
    """MH_FLAG_DETERMINISTIC on the replay kernel (the bitmap path of scenes
    the fused wavefront does not take; MH_PRB_REPLAY=1 forces it here) and on
    the rgb megakernel (MH_MODE=mega): a max pass and an int64 fixed-point
    pass, bitmap texels into an int64 mirror of the slot block, the lanes'
    small-slot sums folded exactly; repeated runs give the same bits, equal
    to the float build and to the oracle within tolerance (prb.py:245-246)."""
    if case == "rgb_mega":
        monkeypatch.setenv("MH_MODE", "mega")
    else:
        monkeypatch.setenv("MH_PRB_REPLAY", "1")
    if case == "bitmap_replay_global":
        monkeypatch.setenv("MH_PRB_LDS_TEX", "0")
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    if case == "rgb_mega":
        scene = mi.load_dict(_cbox(mi, 40, 32, 16))
        keys = ["white.reflectance.value", "red.reflectance.value"]
    else:
        scene = mi.load_dict(mi.cornell_box_bitmap(tex_res=8, width=40, height=32, spp=16))
        keys = ["white.reflectance.data", "red.reflectance.value"]
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    gi = torch.from_numpy(np.random.default_rng(4).random((32, 40, 3)).astype(np.float32) / (32 * 40 * 3)).cuda()
    st = A.Stats()
    runs = [mi.render_backward(scene, params, gi, keys, prb, seed=3, spp=16, deterministic=True, stats=st)
            for _ in range(3)]
    assert st.mode == 0  # the replay / megakernel, not the wavefront
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    flt = mi.render_backward(scene, params, gi, keys, prb, seed=3, spp=16)
    ref = O.render_backward(scene, prb, 3, 16, gi.cpu().numpy(), [params.texture_of(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for k, a, b, r in zip(keys, runs[0], flt, ref):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.abs(r).max() > 0, k
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6 * np.abs(r).max(), err_msg=k)
        np.testing.assert_allclose(a, r, rtol=2e-3, atol=1e-9 + 2e-4 * np.abs(r).max(), err_msg=k)


@pytest.mark.parametrize("size,chunk", [((37, 29), None), ((37, 29), "3136"), ((64, 9), "1200"), ((5, 70), None)])
def test_tiled_film_splat_matches_gather(size, chunk, monkeypatch):
    """The film splat on 4 x 4 source tiles with an LDS film block
    (k_splat_tile): film sizes that are not multiples of the tile, chunks
    that start and end inside a row (MH_WF_CHUNK, in samples) -- equal to the
    fixed-order gather (MH_FLAG_DETERMINISTIC) up to float summation order,
    and to the oracle (imageblock.cpp:418-531)."""
    if chunk:
        monkeypatch.setenv("MH_WF_CHUNK", chunk)
    mi = _mi()
    w, h = size
    scene = mi.load_dict(_cbox(mi, w, h, 16))
    integ = scene.integrator()
    tiled = mi.render_film(scene, integ, seed=6, spp=16).cpu().numpy()
    gather = mi.render_film(scene, integ, seed=6, spp=16, deterministic=True).cpu().numpy()
    assert tiled.shape == (h, w, 4) and np.abs(gather).max() > 0
    np.testing.assert_allclose(tiled, gather, rtol=1e-5, atol=1e-6)
    ref = O.render(scene, integ, seed=6, spp=16)
    ok = np.all(np.abs(tiled - ref) <= 1e-4 * np.maximum(1.0, np.abs(ref)), axis=-1)
    assert ok.mean() >= 0.995
