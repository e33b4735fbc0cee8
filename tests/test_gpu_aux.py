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
* roctx ranges: the library links the roctx API (the ScopedPhase ranges).
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
