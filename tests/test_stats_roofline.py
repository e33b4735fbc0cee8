"""CPU: the measurement plumbing behind bench.py's roofline lines (VERDICT r5
item 2).  The oracle's density-grid lookup counter (the check of
mh_stats.grid_lookups) is deterministic and independent of the thread count;
the roofline helpers compute frac = algorithmic bytes per launch / average
launch time / HBM peak from nothing but the mh_stats fields, so a line can be
recomputed by hand; and the PMC counters of the profiled config-2 launches are
attached to config-2 lines only."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import oracle_py as O  # noqa: E402


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


def test_oracle_grid_lookups_deterministic_over_threads():
    mi = _mi()
    s = mi.load_dict(mi.volume_cube(12, 10, 8, grid=mi.fbm_grid(16)))
    O.grid_lookups(reset=True)
    O.render(s, seed=3, spp=8, threads=1)
    a = O.grid_lookups(reset=True)
    O.render(s, seed=3, spp=8, threads=4)
    b = O.grid_lookups(reset=True)
    assert a == b and a > 12 * 10 * 8  # several lookups per sample
    O.render(s, seed=4, spp=8, threads=4)
    assert O.grid_lookups(reset=True) != a  # another seed, other paths


def test_oracle_grid_lookups_zero_without_heterogeneous_media():
    mi = _mi()
    s = mi.load_dict(mi.volume_cube(9, 9, 16, medium_type="homogeneous", sigma_t=0.5, scale=1.0))
    O.grid_lookups(reset=True)
    O.render(s, seed=1, spp=16, threads=2)
    assert O.grid_lookups(reset=True) == 0


class _St:  # the mh_stats fields the helpers read
    def __init__(self, **kw):
        self.__dict__.update(dict(rays_closest=0, ms_trace=0.0, n_trace_launches=0, grid_lookups=0, aux_items=0,
                                  ms_aux=0.0, n_aux_launches=0), **kw)


def test_volsched_roofline_from_stats():
    st = _St(grid_lookups=152_225_810, ms_trace=16.5, n_trace_launches=1)
    r = bench.volsched_roofline(st, 4_194_304)
    alg = 32 * 152_225_810 + 20 * 4_194_304
    assert r["algorithmic_bytes_per_launch"] == alg
    assert r["kernel_avg_us"] == 16500.0
    assert abs(r["frac"] - alg / 16.5e-3 / 8e12) < 1e-4
    assert r["lookups_per_sample"] == round(152_225_810 / 4_194_304, 3)


def test_bitmap_rooflines_from_stats():
    N, R, V = 16_777_216, 69_000_000, 36_782_641
    st = _St(rays_closest=R, ms_trace=8 * 0.8, n_trace_launches=8, aux_items=V, ms_aux=1.33, n_aux_launches=1)
    bounce, scat = bench.bitmap_rooflines(st, N, 64 * 64 * 3)
    assert bounce["algorithmic_bytes_per_launch"] == round((2 * 100 * (R - N) + 48 * N + 48 * V) / 8)
    assert abs(bounce["kernel_avg_us"] - 800.0) < 1e-6
    assert scat["algorithmic_bytes_per_launch"] == round(32 * N + 48 * V + 4 * 64 * 64 * 3)
    assert abs(scat["frac"] - scat["algorithmic_bytes_per_launch"] / 1.33e-3 / 8e12) < 1e-4


def test_splat_roofline_from_stats():
    st = _St(aux_items=67_108_864, ms_aux=0.63, n_aux_launches=2)
    r = bench.splat_roof(st, 512 * 512)
    assert r["kernel"] == "k_splat_tile<0>"
    assert r["algorithmic_bytes_per_launch"] == round((20 * 67_108_864 + 16 * 512 * 512 * 2) / 2)
    assert abs(r["kernel_avg_us"] - 315.0) < 1e-6


@pytest.mark.parametrize("argv,applies", [([], True), (["--config", "5"], False), (["--res", "1024"], False),
                                          (["--spp", "64"], False), (["--max-depth", "6"], False)])
def test_pmc_counters_attach_to_the_profiled_workload_only(argv, applies):
    a = bench.parse(argv)
    assert bench.pmc_applies(a) == applies


def test_overlapped_roofline_recomputes_from_the_line():
    # the round-6 final line's figures (profiles/r6_bench_line_2.txt): the
    # PRB bounce's timed-region launches and both families' serial rooflines
    timed = {"kernel": "k_wf_bounce_prb", "achieved": 1502.0, "frac": 0.1877, "kernel_avg_us": 1922.2,
             "launches_per_step": 16, "algorithmic_bytes_per_launch": 2887105140, "traffic": None}
    prb = {"algorithmic_bytes_per_launch": 2887130263, "launches_per_step": 16}
    fwd = {"algorithmic_bytes_per_launch": 2041861558, "launches_per_step": 16}
    r = bench.overlapped_roofline(timed, (prb, fwd), 32.392)
    assert r["kernel"] == "k_wf_bounce_prb" and r["kernel_avg_us"] == 1922.2 and "traffic" not in r
    chip = 16 * (2887130263 + 2041861558)
    assert r["chip_bounce_bytes_per_step"] == chip == 78863869136  # the line's value
    assert (r["chip_achieved"], r["chip_frac"]) == (2434.7, 0.3043)
    assert r["chip_achieved"] == pytest.approx(chip / 32.392e-3 / 1e9, abs=0.1)
    assert r["chip_frac"] == pytest.approx(r["chip_achieved"] / bench.HBM_PEAK_GBS, abs=1e-4)
    assert 0.29 < r["chip_frac"] < 0.31
    # a missing second family (forward-only rooflines) counts nothing
    assert bench.overlapped_roofline(timed, (prb, None), 32.392)["chip_bounce_bytes_per_step"] == 16 * 2887130263
