"""mh_stats version 2 on the device (the fields bench.py's roofline lines are
computed from):

* grid_lookups: k_vol_sched's device-counted density-grid lookups equal the
  oracle's count at the same seed (per-sample bit-exact paths take the same
  medium samples), deterministic from run to run;
* the bitmap texel scatter of a prb backward: aux_items (the vertex records
  it read) deterministic and non-zero, its HIP-event time and launch count;
* the film splat of mh_render: one launch per chunk, aux_items = samples.
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


@pytest.mark.parametrize("seed,spp", [(3, 8), (11, 16)])
def test_grid_lookups_equal_the_oracles(seed, spp):
    mi = _mi()
    from mitsuba_hip import _abi as A
    s = mi.load_dict(mi.volume_cube(12, 10, spp, grid=mi.fbm_grid(16)))
    st = A.Stats()
    mi.render_film(s, seed=seed, spp=spp, stats=st)
    assert st.mode == 3 and st.n_trace_launches >= 1 and st.ms_trace > 0
    O.grid_lookups(reset=True)
    O.render(s, seed=seed, spp=spp, threads=4)
    ref = O.grid_lookups(reset=True)
    assert ref > 12 * 10 * spp
    assert st.grid_lookups == ref, (st.grid_lookups, ref)
    st2 = A.Stats()
    mi.render_film(s, seed=seed, spp=spp, stats=st2)
    assert st2.grid_lookups == st.grid_lookups


def test_bitmap_scatter_stats():
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    s = mi.load_dict(mi.cornell_box_bitmap(16, 64, 48, 16))
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(s)
    key = "white.reflectance.data"
    gi = torch.full((48, 64, 3), 1.0 / (48 * 64 * 3), device="cuda")
    st, st2 = A.Stats(), A.Stats()
    mi.render_backward(s, params, gi, [key], integ, seed=5, spp=16, stats=st)
    mi.render_backward(s, params, gi, [key], integ, seed=5, spp=16, stats=st2)
    assert st.mode == 1 and st.n_aux_launches >= 1 and st.ms_aux > 0
    assert 0 < st.aux_items and st.aux_items == st2.aux_items  # the record set is a function of the seed
    # records: at most one per path and bitmap depth, and the camera vertex
    # of most paths lands on a white surface of the box
    n = 48 * 64 * 16
    assert st.aux_items <= n * 5
    assert st.ms_trace > 0 and st.n_trace_launches == st.n_aux_launches * 6


def test_film_splat_stats():
    mi = _mi()
    from mitsuba_hip import _abi as A
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = 64, 48
    s = mi.load_dict(d)
    st = A.Stats()
    mi.render_film(s, s.integrator(), seed=2, spp=16, stats=st)
    assert st.mode == 2 and st.n_aux_launches == 1 and st.aux_items == 64 * 48 * 16 and st.ms_aux > 0
    assert st.grid_lookups == 0
