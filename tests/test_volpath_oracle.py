"""CPU: the volpath restatement (oracle) — plugin known answers and
unbiasedness checks.  The reference ships no
volpath image fixtures, so beyond these analytic properties the volpath
oracle is "parity unpinned" against llvm_ad_rgb."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import oracle_py as O


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


def test_exp_restatement_accuracy():
    L = O.lib()
    L.oracle_exp.argtypes = [C.c_float]
    L.oracle_exp.restype = C.c_float
    xs = np.concatenate([np.linspace(-87, 88, 2001), [-100.0, 100.0, 0.0]]).astype(np.float32)
    for x in xs:
        v = L.oracle_exp(float(x))
        if x < -88.3762626647949:
            assert v == 0.0
        elif x > 88.3762626647949:
            assert math.isinf(v)
        else:
            assert abs(v - math.exp(float(x))) <= 2e-7 * math.exp(float(x)) + 1e-38, (x, v)


def test_log_restatement_accuracy():
    for x in np.geomspace(1e-30, 1e30, 500).astype(np.float32):
        v = O.lib().oracle_log(float(x))
        assert abs(v - math.log(float(x))) <= 2e-7 * max(1.0, abs(math.log(float(x))))


def test_vol_file_roundtrip(tmp_path):
    mi = _mi()
    g = mi.fbm_grid(16)
    vg = mi.VolumeGrid(g, (-1, -1, -1), (1, 1, 1))
    p = tmp_path / "grid.vol"
    vg.write(p)
    raw = open(p, "rb").read()
    assert raw[:3] == b"VOL" and raw[3] == 3 and len(raw) == 4 + 4 * 5 + 24 + 4 * g.size
    r = mi.VolumeGrid.read(p)
    assert r.size() == (16, 16, 16) and r.channel_count() == 1
    assert np.array_equal(r.data[..., 0], g)
    assert np.allclose(r.bbox_min, -1) and np.allclose(r.bbox_max, 1)
    # the scene loader reads .vol files (gridvolume 'filename')
    d = mi.volume_cube(8, 8, 4, grid=g)
    d["medium1"]["sigma_t"] = {"type": "gridvolume", "filename": str(p),
                               "to_world": d["medium1"]["sigma_t"]["to_world"]}
    a = O.render(mi.load_dict(d), seed=1, spp=4)
    b = O.render(mi.load_dict(mi.volume_cube(8, 8, 4, grid=g)), seed=1, spp=4)
    assert np.array_equal(a, b)


def test_fbm_grid_deterministic():
    mi = _mi()
    a, b = mi.fbm_grid(24), mi.fbm_grid(24)
    assert np.array_equal(a, b) and a.dtype == np.float32
    assert a.min() >= 0 and a.max() <= 1 and a.max() > 0.5


def test_white_furnace():
    """Non-absorbing medium (albedo 1) inside a null cube under a unit
    constant sky: every pixel's expectation is exactly 1."""
    mi = _mi()
    s = mi.load_dict(mi.volume_cube(16, 16, 64, grid=mi.fbm_grid(32), albedo=1.0, sky=1.0, sun=None,
                                    scale=5.0, max_depth=-1))
    img = O.develop(O.render(s, seed=0, spp=256))
    assert abs(img.mean() - 1.0) < 0.01 and img.std() < 0.05


@pytest.mark.parametrize("phase_g", [0.0, 0.7])
def test_homogeneous_absorber_transmittance(phase_g):
    """Pure absorber (albedo 0): the centre pixel sees exp(-sigma_t * 2)."""
    mi = _mi()
    s = mi.load_dict(mi.volume_cube(9, 9, 4096, medium_type="homogeneous", sigma_t=0.5, scale=1.0,
                                    albedo=0.0, g=phase_g, sky=1.0, sun=None, max_depth=-1))
    img = O.develop(O.render(s, seed=0, spp=4096))
    assert abs(img[4, 4, 0] - math.exp(-1.0)) < 0.02


def test_sun_contributes_unattenuated_like_the_reference():
    """The directional emitter's shadow ray is spawned toward p - d * inf,
    whose NaN components end the transmittance loop at once
    (volpath.cpp:361-375): the sun is never attenuated by the medium in the
    reference.  Reproduced, not corrected."""
    mi = _mi()
    g = mi.fbm_grid(16)
    with_sun = O.develop(O.render(mi.load_dict(mi.volume_cube(8, 8, 64, grid=g, sky=0.0, sun=5.0)), seed=2, spp=64))
    assert np.isfinite(with_sun).all() and with_sun.mean() > 0


def test_per_sample_determinism_and_threads():
    mi = _mi()
    s = mi.load_dict(mi.volume_cube(12, 10, 8, grid=mi.fbm_grid(16)))
    a = O.render(s, seed=3, spp=8, threads=1)
    b = O.render(s, seed=3, spp=8, threads=4)
    c = O.render(s, seed=3, spp=8, threads=4)
    assert np.array_equal(b, c)
    # band partitions change the splat summation order only
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
