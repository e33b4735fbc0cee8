"""The shadow rays' division-free rectangle pretest (rect_separated,
mitsuba3-nasa_amd/csrc/mh_shading.hpp) must be conservative: whenever it
calls a lane separated, the exact test of rect_pair / rect_one -- the plane
distance tt = -lz / ldz in IEEE float32, hit iff 0 <= tt <= bound -- rejects
the lane too.  Checked here in float32 arithmetic on random and adversarial
(lz, ldz, bound) triples, the fmas emulated exactly in float64 (a float32
product is exact in float64; the sum is rounded once to float32, as an fma
is, except in double-rounding ties that the margin dwarfs)."""
import numpy as np
import pytest

F = np.float32


def fma32(a, b, c):
    with np.errstate(invalid="ignore", over="ignore"):
        return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F)


def separated(lz, ldz, bound):
    s1 = fma32(ldz, bound, lz)
    m = fma32(fma32(np.abs(ldz), np.maximum(bound, F(2.0 ** -126)), np.abs(lz)), np.full_like(lz, 2.0 ** -20),
              np.full_like(lz, 1e-30))
    return ((lz > m) & (s1 > m)) | ((lz < -m) & (s1 < -m))


def exact_hit(lz, ldz, bound):
    with np.errstate(divide="ignore", invalid="ignore", over="ignore", under="ignore"):
        tt = (-lz / ldz).astype(F)
    return (tt >= F(0)) & (tt <= bound)


def _check(lz, ldz, bound):
    lz, ldz, bound = (np.asarray(x, F) for x in (lz, ldz, bound))
    sep = separated(lz, ldz, bound)
    bad = sep & exact_hit(lz, ldz, bound)
    assert not bad.any(), (lz[bad][:5], ldz[bad][:5], bound[bad][:5])
    return sep


def test_random_triples_over_wide_exponents():
    rng = np.random.default_rng(5)
    n = 2_000_000
    mag = lambda lo, hi: F(10.0) ** rng.uniform(lo, hi, n).astype(F)
    lz = (rng.choice([-1, 1], n) * mag(-30, 6)).astype(F)
    ldz = (rng.choice([-1, 1], n) * mag(-8, 8)).astype(F)
    bound = mag(-6, 6)
    sep = _check(lz, ldz, bound)
    assert 0.2 < sep.mean() < 0.9  # the test is not vacuous


def test_subnormal_and_tiny_bounds():
    rng = np.random.default_rng(7)
    n = 1_000_000
    mag = lambda lo, hi: F(10.0) ** rng.uniform(lo, hi, n).astype(F)
    lz = (rng.choice([-1, 1], n) * mag(-38, 0)).astype(F)
    ldz = (rng.choice([-1, 1], n) * mag(0, 38)).astype(F)
    bound = mag(-45, -30)
    _check(lz, ldz, bound)


def test_segments_ending_just_short_of_the_plane():
    # t = -lz / ldz just above bound: the adversarial side of the pretest
    rng = np.random.default_rng(6)
    n = 1_000_000
    ldz = (-(F(10.0) ** rng.uniform(-4, 4, n))).astype(F)
    t = (F(10.0) ** rng.uniform(-3, 3, n)).astype(F)
    lz = (-t * ldz).astype(F)
    for rel in (0.0, 1e-7, 2e-7, 1e-6, 4e-6, 1e-5, 1e-4):
        bound = (t * F(1.0 - rel)).astype(F)
        _check(lz, ldz, bound)
        _check(-lz, -ldz, bound)


@pytest.mark.parametrize("lz,ldz,bound", [
    (1e-30, 1e8, 1.0), (1.5e-30, 1e8, 1.0), (1e-38, 1.0, 1.0), (1.0, 0.0, 1.0), (-1.0, 0.0, 1.0),
    (1.0, -0.0, np.inf), (1.0, -1.0, np.inf), (np.nan, 1.0, 1.0), (1.0, np.nan, 1.0), (0.0, 1.0, 1.0),
    (-0.0, -1.0, 1.0), (1.0, -1.0, 1.0), (1.0, -1.0000001, 1.0), (3.0, -1.0, 3.0000002),
    # subnormal bounds: -lz / ldz underflows to -0, which the exact test accepts
    (1e-12, 3e38, 1.4e-45), (-1e-12, -3e38, 1.4e-45), (1e-30, 1e20, 1e-40), (1e-25, 3e38, 2 ** -126),
])
def test_edge_values(lz, ldz, bound):
    _check([lz], [ldz], [bound])
