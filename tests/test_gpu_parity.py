"""GPU parity: HIP product path (through the C-ABI) vs the CPU oracle.

Criteria:
  traversal   identical (t, prim, shape) for >= 99.99 % of rays
  per-sample  L identical bit-for-bit for >= 99.9 % of samples (the rest are
              BVH-vs-brute-force ties); |dL| <= 1e-4 * max(1, |L|) otherwise
  film        |d| <= 1e-4 * max(1, |ref|) for >= 99.5 % of pixels (atomic order)
  gradient    relative error < 1e-3 vs the oracle
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


def cbox(mi, w=32, h=32, spp=16):
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = w
    d["sensor"]["film"]["height"] = h
    d["sensor"]["sampler"]["sample_count"] = spp
    return mi.load_dict(d)


def random_rays(scene, n, seed=1):
    """Camera rays + rays from random interior points in random directions."""
    rng = np.random.default_rng(seed)
    o = np.zeros((3, n), np.float32)
    o[0] = rng.uniform(-0.95, 0.95, n)
    o[1] = rng.uniform(-0.95, 0.95, n)
    o[2] = rng.uniform(-0.95, 3.5, n)
    d = rng.normal(size=(3, n)).astype(np.float32)
    d /= np.linalg.norm(d, axis=0)
    maxt = np.where(rng.random(n) < 0.5, np.float32(3.4028235e38), rng.uniform(0.1, 5, n)).astype(np.float32)
    return np.concatenate([o, d, maxt[None]], 0).astype(np.float32)


def gpu_trace(mi, scene, rays):
    from mitsuba_hip import _abi as A
    n = rays.shape[1]
    t, u, v = (np.zeros(n, np.float32) for _ in range(3))
    prim, shape, occ = (np.zeros(n, np.uint32) for _ in range(3))
    h = scene.handle(0)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    rays = np.ascontiguousarray(rays)
    A.check(A.lib().mh_trace_closest(h, n, p(rays), p(t), p(u), p(v), p(prim), p(shape), 0, None))
    A.check(A.lib().mh_trace_shadow(h, n, p(rays), p(occ), 0, None))
    return t, u, v, prim, shape, occ


def test_trace_parity():
    mi = _mi()
    scene = cbox(mi)
    rays = random_rays(scene, 1 << 18)
    t, u, v, prim, shape, occ = gpu_trace(mi, scene, rays)
    rt, ru, rv, rprim, rshape = O.trace_closest(scene, rays)
    rocc = O.trace_shadow(scene, rays)
    same = (shape == rshape) & (prim == rprim) & ((t == rt) | (np.isinf(t) & np.isinf(rt)))
    assert same.mean() >= 0.9999, f"closest-hit mismatch fraction {1 - same.mean()}"
    assert (occ == rocc).mean() >= 0.9999
    hit = rshape != 0xFFFFFFFF
    assert hit.mean() > 0.3
    np.testing.assert_array_equal(u[same & hit], ru[same & hit])
    np.testing.assert_array_equal(v[same & hit], rv[same & hit])
    # the OptiX payload (scene_optix.inl:602-657): rectangles report
    # prim_index 0 (rectangle.cuh:42); a miss leaves prim_index 0, prim_uv
    # (0, 0), t = +inf and a null shape (optix_rt.cu:9-17)
    is_rect = np.isin(shape, [i for i in range(scene.desc.n_shapes)
                              if scene.desc.shapes[i].type == 0])
    assert is_rect.sum() > 1000 and (~is_rect & hit).sum() > 1000
    assert np.all(prim[is_rect & hit] == 0)
    miss = shape == 0xFFFFFFFF
    assert miss.sum() > 0
    assert np.all(prim[miss] == 0) and np.all(u[miss] == 0) and np.all(v[miss] == 0) and np.all(np.isinf(t[miss]))
    # instance payload: null for every ray (no shapegroups, scene_optix.inl:607-608)
    from mitsuba_hip import _abi as A
    n = rays.shape[1]
    t2, u2, v2 = (np.zeros(n, np.float32) for _ in range(3))
    prim2, shape2, inst = (np.zeros(n, np.uint32) for _ in range(3))
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    A.check(A.lib().mh_trace_preliminary(scene.handle(0), n, p(np.ascontiguousarray(rays)), p(t2), p(u2), p(v2),
                                         p(prim2), p(shape2), p(inst), 0, None))
    assert np.all(inst == 0xFFFFFFFF)
    np.testing.assert_array_equal(prim2, prim)
    np.testing.assert_array_equal(shape2, shape)


def _gpu_samples(mi, scene, integrator, seed, spp, flags=0):
    from mitsuba_hip import _abi as A
    n = scene.width * scene.height * spp
    out = np.zeros(5 * n, np.float32)
    ic = integrator.c()
    A.check(A.lib().mh_render_samples(scene.handle(0), C.byref(ic), seed, spp, 0, 0,
                                      out.ctypes.data_as(C.c_void_p), flags))
    return out[:3 * n].reshape(3, n).T, out[3 * n:].reshape(2, n).T


@pytest.mark.parametrize("itype,mode", [("path", "mega"), ("prb", "mega"), ("path", "wavefront"),
                                        ("path", "wavefront-lane"), ("path", "wavefront-unfused")])
def test_per_sample_parity(itype, mode, monkeypatch):
    """wavefront: fused bounce kernel with the packet engine (small-BVH default);
    wavefront-unfused: trace / shade / shadow kernels with the packet engine;
    wavefront-lane: trace / shade / shadow kernels with the per-lane engine."""
    if mode == "wavefront-lane":
        monkeypatch.setenv("MH_TRAVERSAL", "lane")
        mode = "wavefront"
    if mode == "wavefront-unfused":
        monkeypatch.setenv("MH_WF_FUSED", "0")
        mode = "wavefront"
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = cbox(mi, 24, 24, 8)
    integ = mi.load_dict({"type": itype, "max_depth": 8})
    L, pos = _gpu_samples(mi, scene, integ, 3, 8, A.FLAG_WAVEFRONT if mode == "wavefront" else 0)
    n = L.shape[0]
    rL, rpos, _ = O.sample_range(scene, integ, 3, 8, 0, n)
    np.testing.assert_array_equal(pos, rpos)
    exact = np.all(L == rL, axis=1)
    assert exact.mean() >= 0.999, f"bit-exact fraction {exact.mean()}"
    close = np.all(np.abs(L - rL) <= 1e-4 * np.maximum(1, np.abs(rL)), axis=1)
    assert close.mean() >= 0.999


def _film_close(a, b, frac=0.995):
    ok = np.all(np.abs(a - b) <= 1e-4 * np.maximum(1.0, np.abs(b)), axis=-1)
    return ok.mean() >= frac, ok.mean()


@pytest.mark.parametrize("spp,mode", [(1, "auto"), (2, "auto"), (16, "mega"), (16, "wavefront"), (64, "auto")])
def test_render_film_parity(spp, mode):
    mi = _mi()
    scene = cbox(mi, 40, 32, spp)
    integ = scene.integrator()
    film = mi.render_film(scene, integ, seed=5, spp=spp, mode=mode).cpu().numpy()
    ref = O.render(scene, integ, seed=5, spp=spp)
    ok, frac = _film_close(film, ref)
    assert ok, f"film parity {frac}"
    img = mi.develop(scene, mi.render_film(scene, integ, seed=5, spp=spp)).cpu().numpy()
    ok, frac = _film_close(img, O.develop(ref))
    assert ok, f"image parity {frac}"


def test_sample_slabs_sum_to_full():
    """Multi-GPU sample-slab sharding: slabs sum to the full film."""
    mi = _mi()
    scene = cbox(mi, 32, 32, 16)
    integ = scene.integrator()
    full = mi.render_film(scene, integ, seed=0, spp=16).cpu().numpy()
    acc = np.zeros_like(full)
    for b in range(0, 16, 4):
        acc += mi.render_film(scene, integ, seed=0, spp=16, spp_begin=b, spp_end=b + 4).cpu().numpy()
    ok, frac = _film_close(acc, full)
    assert ok, frac


def test_prb_weights_parity():
    mi = _mi()
    scene = cbox(mi, 32, 24, 16)
    w = mi.prb_weights(scene, seed=7, spp=16).cpu().numpy()
    rw = O.prb_weights(scene, 7, 16)
    np.testing.assert_allclose(w, rw, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("spp,mode", [(4, "replay"), (16, "replay"), (4, "mega"), (16, "auto"), (4, "auto")])
def test_prb_backward_rgb_parity(spp, mode):
    mi = _mi()
    import torch
    scene = cbox(mi, 32, 32, spp)
    integ = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    keys = ["white.reflectance.value", "red.reflectance.value"]
    H, W = scene.height, scene.width
    grad_in = np.full((H, W, 3), 1.0 / (H * W * 3), np.float32)
    g = mi.render_backward(scene, params, torch.from_numpy(grad_in).cuda(), keys, integ, seed=11, spp=spp,
                           mode=mode)
    g = [x.cpu().numpy() for x in g]
    ref = O.render_backward(scene, integ, 11, spp, grad_in, [params.texture_of(k) for k in keys], [(3,), (3,)])
    for a, b in zip(g, ref):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-7)


@pytest.mark.gpu
def test_prb_backward_fused_vs_replay_random_grad():
    """The fused single-traversal gradient equals the primal+adjoint replay
    (same RNG stream) for a non-uniform upstream gradient."""
    mi = _mi()
    import torch
    scene = cbox(mi, 48, 40, 8)
    integ = mi.load_dict({"type": "prb", "max_depth": 6, "rr_depth": 2})
    params = mi.traverse(scene)
    keys = ["white.reflectance.value", "red.reflectance.value", "green.reflectance.value"]
    rng = np.random.default_rng(5)
    gi = torch.from_numpy(rng.standard_normal((40, 48, 3)).astype(np.float32)).cuda()
    a = mi.render_backward(scene, params, gi, keys, integ, seed=4, spp=8, mode="replay")
    for mode in ("mega", "auto"):
        b = mi.render_backward(scene, params, gi, keys, integ, seed=4, spp=8, mode=mode)
        for x, y in zip(a, b):
            np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=2e-3, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["packet", "lane", "packet-unfused"])
def test_prb_backward_wavefront_chunked(monkeypatch, engine):
    """Multi-chunk wavefront backward (lane maps offset per chunk, partials
    accumulated across chunks) equals the single-chunk run."""
    mi = _mi()
    import torch
    scene = cbox(mi, 40, 24, 16)
    integ = mi.load_dict({"type": "prb", "max_depth": 5, "hide_emitters": True})
    params = mi.traverse(scene)
    keys = ["white.reflectance.value", "green.reflectance.value"]
    gi = torch.full((24, 40, 3), 1.0 / (24 * 40 * 3), dtype=torch.float32, device="cuda")
    monkeypatch.setenv("MH_TRAVERSAL", engine.split("-")[0])
    if engine.endswith("unfused"):
        monkeypatch.setenv("MH_WF_FUSED", "0")
    a = mi.render_backward(scene, params, gi, keys, integ, seed=9, spp=16)
    monkeypatch.setenv("MH_WF_CHUNK", "2048")
    b = mi.render_backward(scene, params, gi, keys, integ, seed=9, spp=16)
    ref = O.render_backward(scene, integ, 9, 16, gi.cpu().numpy(), [params.texture_of(k) for k in keys],
                            [(3,), (3,)])
    for x, y, r in zip(a, b, ref):
        np.testing.assert_allclose(x.cpu().numpy(), y.cpu().numpy(), rtol=1e-4, atol=1e-8)
        np.testing.assert_allclose(x.cpu().numpy(), r, rtol=1e-3, atol=1e-7)


# ---------------------------------------------------------------------------
# volpath: heterogeneous grid medium, HG phase,
# null-BSDF boundary, constant + directional emitters
# ---------------------------------------------------------------------------
def _vol_scene(mi, w=24, h=20, spp=8, **kw):
    kw.setdefault("grid", mi.fbm_grid(32))
    return mi.load_dict(mi.volume_cube(w, h, spp, **kw))


def _vol_floor_scene(mi, w=24, h=20, spp=8, **kw):
    """volume_cube + a diffuse floor below it: surface NEE walks through the
    medium (suspended surface paths carry their interaction through HBM)."""
    kw.setdefault("grid", mi.fbm_grid(16))
    kw.setdefault("scale", 4.0)
    d = mi.volume_cube(w, h, spp, **kw)
    T = mi.Transform4f
    d["floor"] = {"type": "rectangle",
                  "to_world": T.translate([0, -1.2, 0]) @ T.rotate([1, 0, 0], -90) @ T.scale([3, 3, 3]),
                  "bsdf": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.6, 0.5, 0.4]}}}
    return mi.load_dict(d)


VOL_CASES = [{}, {"medium_type": "homogeneous", "sigma_t": 0.8, "scale": 1.0},
             {"max_depth": 8, "g": -0.3, "albedo": [0.9, 0.5, 0.2]}, {"floor": True}, {"floor": True, "max_depth": 3},
             {"max_depth": 1}, {"max_depth": 0}]


@pytest.mark.parametrize("mode", ["mega", "wavefront", "wavefront-rounds", "wavefront-finish1", "wavefront-rounds100"])
@pytest.mark.parametrize("kw", VOL_CASES)
def test_volpath_per_sample_parity(kw, mode, monkeypatch):
    """mega: k_render<VOLPATH>; wavefront: the phase-scheduled persistent
    kernel k_vol_sched (mh_volwave.hip); -rounds: k_vw_main / k_vw_walk
    rounds then k_vw_finish; -rounds100: rounds only; -finish1: one round,
    then the finish kernel.  Bit-identical per sample."""
    mi = _mi()
    from mitsuba_hip import _abi as A
    if mode != "wavefront" and mode != "mega":
        monkeypatch.setenv("MH_VOL_MODE", "rounds")
    if mode == "wavefront-rounds100":
        monkeypatch.setenv("MH_VW_ROUNDS", "100000")
    if mode == "wavefront-finish1":
        monkeypatch.setenv("MH_VW_ROUNDS", "1")
    mode = mode.split("-")[0]
    kw = dict(kw)
    scene = _vol_floor_scene(mi, **kw) if kw.pop("floor", False) else _vol_scene(mi, **kw)
    integ = scene.integrator()
    L, pos = _gpu_samples(mi, scene, integ, 3, 8, A.FLAG_WAVEFRONT if mode == "wavefront" else 0)
    rL, rpos, _ = O.sample_range(scene, integ, 3, 8, 0, L.shape[0])
    np.testing.assert_array_equal(pos, rpos)
    exact = np.all(L == rL, axis=1)
    assert exact.mean() >= 0.999, f"bit-exact fraction {exact.mean()}"
    close = np.all(np.abs(L - rL) <= 1e-4 * np.maximum(1, np.abs(rL)), axis=1)
    assert close.mean() >= 0.999


@pytest.mark.parametrize("mode", ["mega", "wavefront"])
def test_volpath_film_parity(mode):
    mi = _mi()
    scene = _vol_scene(mi, 40, 32, 16)
    film = mi.render_film(scene, seed=5, spp=16, mode=mode).cpu().numpy()
    ref = O.render(scene, seed=5, spp=16)
    ok, frac = _film_close(film, ref)
    assert ok, f"film parity {frac}"


def test_volpath_wavefront_matches_megakernel_stats():
    """The two execution modes trace the same rays (closest / shadow counts)
    and produce the same samples on a 64^3 grid at 64 x 48 @ 16 spp."""
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _vol_scene(mi, 64, 48, 16, grid=mi.fbm_grid(64))
    sm, sw = A.Stats(), A.Stats()
    fm = mi.render_film(scene, seed=9, spp=16, mode="mega", stats=sm).cpu().numpy()
    fw = mi.render_film(scene, seed=9, spp=16, mode="wavefront", stats=sw).cpu().numpy()
    assert sw.mode == 3 and sm.mode == 0
    assert (sw.rays_closest, sw.rays_shadow) == (sm.rays_closest, sm.rays_shadow)
    ok, frac = _film_close(fw, fm, 0.999)
    assert ok, f"film agreement {frac}"


def test_volpath_white_furnace_gpu():
    mi = _mi()
    scene = _vol_scene(mi, 32, 32, 256, albedo=1.0, sky=1.0, sun=None, scale=5.0, max_depth=-1)
    img = mi.develop(scene, mi.render_film(scene, seed=0, spp=256)).cpu().numpy()
    assert abs(img.mean() - 1.0) < 0.01


# ---------------------------------------------------------------------------
# prbvolpath (prbvolpath.py): primal per sample and
# the adjoint wrt the sigma_t grid, the albedo and a surface reflectance
# ---------------------------------------------------------------------------
def _pvp_scene(mi, w=24, h=20, spp=8, floor=True, pixel_format=None, **kw):
    kw.setdefault("grid", mi.fbm_grid(16))
    kw.setdefault("scale", 4.0)
    d = mi.volume_cube(w, h, spp, **kw)
    if pixel_format:
        d["sensor"]["film"]["pixel_format"] = pixel_format
    d["integrator"] = {"type": "prbvolpath", "max_depth": kw.get("max_depth", 6), "rr_depth": 5}
    if floor:
        T = mi.Transform4f
        d["floor"] = {"type": "rectangle",
                      "to_world": T.translate([0, -1.2, 0]) @ T.rotate([1, 0, 0], -90) @ T.scale([3, 3, 3]),
                      "bsdf": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.6, 0.5, 0.4]}}}
    return mi.load_dict(d)


PVP_CASES = [{}, {"medium_type": "homogeneous", "sigma_t": 0.8, "scale": 1.0},
             {"max_depth": 8, "g": -0.3, "albedo": [0.9, 0.5, 0.2], "floor": False},
             {"max_depth": 3}, {"max_depth": 1}, {"max_depth": 0}, {"scale": 12.0, "max_depth": 12}]


@pytest.mark.parametrize("mode", ["mega", "wavefront"])
@pytest.mark.parametrize("kw", PVP_CASES)
def test_prbvolpath_per_sample_parity(kw, mode):
    """The primal per sample (prbvolpath.py:91-431, mode primal).  mega:
    k_render<PRBVOLPATH>; wavefront: the phase-scheduled persistent kernel
    (k_vol_sched<PvMachine>: the loop trip cut at its closest-hit queries
    and at every step of the NEE walk).  Bit-identical per sample."""
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _pvp_scene(mi, **kw)
    integ = scene.integrator()
    assert integ.type == "prbvolpath"
    L, pos = _gpu_samples(mi, scene, integ, 3, 8, A.FLAG_WAVEFRONT if mode == "wavefront" else 0)
    rL, rpos, _ = O.sample_range(scene, integ, 3, 8, 0, L.shape[0])
    np.testing.assert_array_equal(pos, rpos)
    # max_depth <= 1: nothing is added (emitter hits are not counted in the
    # fork, prbvolpath.py:216-234, and NEE needs depth + 1 < max_depth)
    assert (np.abs(rL).max() > 0) == (kw.get("max_depth", 6) > 1)
    exact = np.all(L == rL, axis=1)
    assert exact.mean() >= 0.999, f"bit-exact fraction {exact.mean()}"
    close = np.all(np.abs(L - rL) <= 1e-4 * np.maximum(1, np.abs(rL)), axis=1)
    assert close.mean() >= 0.999


@pytest.mark.parametrize("nee", ["single", "main4", "sched_nee2", "sched_off", "twopass", "cap2", "replay"])
@pytest.mark.parametrize("kw", [{}, {"medium_type": "homogeneous", "sigma_t": 0.8, "scale": 1.0}])
def test_prbvolpath_backward_parity(kw, nee, monkeypatch):
    """Gradients (sigma_t, albedo, floor reflectance) vs the oracle: same
    samples, float vs double accumulation and atomic order -> 2e-3.
      single     one traversal on the phase scheduler (k_vol_sched<PvBwdMachine>):
                 the L-dependent terms logged per lane (MainLog) and charged
                 once L_total is known, NEE walks logged (NeeLog) -- the default
      main4      4 MainLog entries: most paths overflow, and their adjoint is
                 replayed from the overflow list (k_pvb_replay_paths) without
                 the NEE terms already charged
      sched_nee2 2 NeeLog entries on the scheduler: most walks overflow and are
                 replayed from the overflow list (k_pvb_replay_walks)
      sched_off  the same single pass on the per-sample kernel (k_prbvol_backward)
      twopass    primal + adjoint replay, NEE walks logged (MH_PVP_SINGLE=0)
      cap2       two-pass with 2 NeeLog entries: most walks replay
      replay     the reference's structure: two passes, NEE walks replayed"""
    if nee == "sched_nee2":
        monkeypatch.setenv("MH_PVP_NEE_CAP", "2")
    elif nee == "sched_off":
        monkeypatch.setenv("MH_PVP_SCHED", "0")
    elif nee == "replay":
        monkeypatch.setenv("MH_PVP_NEE_LOG", "0")
    elif nee == "cap2":
        monkeypatch.setenv("MH_PVP_NEE_CAP", "2")
        monkeypatch.setenv("MH_PVP_SINGLE", "0")
    elif nee == "twopass":
        monkeypatch.setenv("MH_PVP_SINGLE", "0")
    elif nee == "main4":
        monkeypatch.setenv("MH_PVP_MAIN_CAP", "4")
    mi = _mi()
    import torch
    scene = _pvp_scene(mi, 24, 20, 8, **kw)
    integ = scene.integrator()
    params = mi.traverse(scene)
    keys = ["medium1.sigma_t." + ("value" if kw else "data"), "medium1.albedo.value",
            "floor.bsdf.reflectance.value"]
    H, W = scene.height, scene.width
    gi = np.random.default_rng(4).standard_normal((H, W, 3)).astype(np.float32)
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), keys, integ, seed=7, spp=8)
    ref = O.render_backward(scene, integ, 7, 8, gi, [params.param_id(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for k, a, b in zip(keys, g, ref):
        a = a.cpu().numpy()
        assert a.shape == b.shape, k
        assert np.abs(b).max() > 0, k
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-7 + 2e-4 * np.abs(b).max(), err_msg=k)


@pytest.mark.parametrize("shape", [(16, 16, 16), (7, 9, 5), (1, 3, 2)])
def test_prbvolpath_grid_corner_scatter(shape, monkeypatch):
    """The sigma_t grid gradient scattered per cell into corner blocks and
    gathered afterwards (corner_scatter / k_corner_gather, the default)
    equals the float atomics straight into the (z, y, x) gradient
    (MH_GRID_CORNER=0) up to the float order of the adds, and the oracle
    (heterogeneous.cpp:192 adjoint, prbvolpath.py:412-414 scatter).
    Non-cubic and one-texel-thin grids exercise the clamped boundary cells."""
    mi = _mi()
    import torch
    o = [(16 - n) // 2 for n in shape]  # the dense centre of the fBm cube
    grid = np.ascontiguousarray(mi.fbm_grid(16)[o[0]:o[0] + shape[0], o[1]:o[1] + shape[1], o[2]:o[2] + shape[2]])
    scene = _pvp_scene(mi, 24, 20, 8, grid=grid)
    integ = scene.integrator()
    params = mi.traverse(scene)
    key = "medium1.sigma_t.data"
    H, W = scene.height, scene.width
    gi = np.random.default_rng(5).standard_normal((H, W, 3)).astype(np.float32)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MH_GRID_CORNER", mode)
        out[mode] = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), [key], integ, seed=7,
                                       spp=8)[0].cpu().numpy()
    ref = O.render_backward(scene, integ, 7, 8, gi, [params.param_id(key)], [tuple(params[key].shape)])[0]
    assert out["1"].shape == ref.shape and np.abs(ref).max() > 0
    scale = np.abs(ref).max()
    np.testing.assert_allclose(out["1"], out["0"], rtol=1e-4, atol=1e-6 * scale)
    np.testing.assert_allclose(out["1"], ref, rtol=2e-3, atol=1e-7 + 2e-4 * scale)


@pytest.mark.parametrize("mode", ["sched", "sched_off", "replay"])
def test_prbvolpath_deterministic_grid_gradient(mode, monkeypatch):
    """MH_FLAG_DETERMINISTIC on prbvolpath: the grid gradient's corner blocks
    and the small slots (albedo, the floor's rgb reflectance) hold int64
    fixed point (a pre-pass finds each one's largest item, the real pass adds
    round(item * 2^S)), so repeated runs give the same bits whatever the order
    of the adds; equal to the float-atomic gradients up to float order and to
    the oracle at 2e-3.  On the scheduler (default), the per-sample kernel
    (MH_PVP_SCHED=0) and the NEE-replaying kernel (MH_PVP_NEE_LOG=0)."""
    if mode == "sched_off":
        monkeypatch.setenv("MH_PVP_SCHED", "0")
    elif mode == "replay":
        monkeypatch.setenv("MH_PVP_NEE_LOG", "0")
    mi = _mi()
    import torch
    scene = _pvp_scene(mi, 24, 20, 8)
    integ = scene.integrator()
    params = mi.traverse(scene)
    keys = ["medium1.sigma_t.data", "medium1.albedo.value", "floor.bsdf.reflectance.value"]
    H, W = scene.height, scene.width
    gi = torch.from_numpy(np.random.default_rng(6).standard_normal((H, W, 3)).astype(np.float32)).cuda()
    runs = [mi.render_backward(scene, params, gi, keys, integ, seed=3, spp=8, deterministic=True) for _ in range(3)]
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    flt = mi.render_backward(scene, params, gi, keys, integ, seed=3, spp=8)
    ref = O.render_backward(scene, integ, 3, 8, gi.cpu().numpy(), [params.param_id(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for k, a, b, r in zip(keys, runs[0], flt, ref):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        scale = np.abs(r).max()
        assert scale > 0, k
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-6 * scale, err_msg=k)
        np.testing.assert_allclose(a, r, rtol=2e-3, atol=1e-7 + 2e-4 * scale, err_msg=k)


@pytest.mark.parametrize("alpha", [False, True])
def test_prbvolpath_film_modes_agree(alpha):
    """mh_render of prbvolpath: the phase scheduler (default) against the
    megakernel and the oracle, films with and without the alpha channel
    (valid_ray, prbvolpath.py:128, 274, 327), and the same ray counts."""
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _pvp_scene(mi, 40, 32, 16, **({"pixel_format": "rgba"} if alpha else {}))
    integ = scene.integrator()
    sw, sm = A.Stats(), A.Stats()
    fw = mi.render_film(scene, integ, seed=5, spp=16, stats=sw).cpu().numpy()
    fm = mi.render_film(scene, integ, seed=5, spp=16, mode="mega", stats=sm).cpu().numpy()
    assert sw.mode == 3 and sm.mode == 0
    assert (sw.rays_closest, sw.rays_shadow) == (sm.rays_closest, sm.rays_shadow)
    ref = O.render(scene, integ, seed=5, spp=16)
    for f in (fw, fm):
        ok, frac = _film_close(f, ref)
        assert ok, f"film parity {frac}"


def test_prbvolpath_grid_update_changes_majorant():
    """SceneParameters.update of the grid (parameters_changed: majorant =
    scale * max) gives the same render as a scene built with that grid."""
    mi = _mi()
    g0 = mi.fbm_grid(16)
    scene = _pvp_scene(mi, 16, 16, 4, grid=g0)
    params = mi.traverse(scene)
    g1 = (g0 * 1.7 + 0.05).astype(np.float32)
    params["medium1.sigma_t.data"] = g1[..., None]
    params.update()
    a = mi.render_film(scene, seed=2, spp=4).cpu().numpy()
    b = mi.render_film(_pvp_scene(mi, 16, 16, 4, grid=g1), seed=2, spp=4).cpu().numpy()
    c = mi.render_film(_pvp_scene(mi, 16, 16, 4, grid=g0), seed=2, spp=4).cpu().numpy()
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)   # film splat: atomic order only
    assert np.abs(a - c).max() > 1e-3


# ---------------------------------------------------------------------------
# PRB wrt a bitmap texture (config 3(b)): texel gradients on the fused
# wavefront (vertex records + scatter pass) and on the replay megakernel
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mode", ["auto", "replay"])
@pytest.mark.parametrize("spp", [4, 16])
def test_prb_backward_bitmap_parity(spp, mode):
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    scene = mi.load_dict(mi.cornell_box_bitmap(tex_res=8, width=32, height=24, spp=spp))
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    keys = ["white.reflectance.data", "red.reflectance.value"]
    H, W = scene.height, scene.width
    rng = np.random.default_rng(2)
    gi = rng.random((H, W, 3)).astype(np.float32) / (H * W * 3)
    st = A.Stats()
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), keys, integ, seed=13, spp=spp,
                           mode=mode, stats=st)
    assert st.mode == (1 if mode == "auto" else 0), st.mode
    ref = O.render_backward(scene, integ, 13, spp, gi, [params.texture_of(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for a, b in zip(g, ref):
        a = a.cpu().numpy()
        assert a.shape == b.shape
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-9 + 2e-4 * np.abs(b).max())


@pytest.mark.parametrize("lds", ["1", "0"])
@pytest.mark.parametrize("channels,max_depth", [(3, 3), (1, 6), (3, 12)])
def test_prb_bitmap_wavefront_chunks(channels, max_depth, lds, monkeypatch):
    """Bitmap on the fused wavefront across several 4096-path chunks (the
    vertex records and L_total are per chunk), with two rgb slots beside it
    (the 4-slot kernel instance), a one-channel bitmap (adjoint summed over
    r, g, b) and shallow / deep max_depth (record count max_depth - 1); the
    texel scatter in LDS and as transposed global atomics (MH_PRB_LDS_TEX=0)."""
    monkeypatch.setenv("MH_WF_CHUNK", "4096")
    monkeypatch.setenv("MH_PRB_LDS_TEX", lds)
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    d = mi.cornell_box_bitmap(tex_res=8, width=40, height=32, spp=16)
    if channels == 1:
        d["white"]["reflectance"]["data"] = np.full((8, 8, 1), 0.7, np.float32)
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "prb", "max_depth": max_depth})
    params = mi.traverse(scene)
    keys = ["red.reflectance.value", "white.reflectance.data", "green.reflectance.value"]
    rng = np.random.default_rng(7)
    gi = rng.random((32, 40, 3)).astype(np.float32) / (32 * 40 * 3)
    st = A.Stats()
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), keys, integ, seed=21, spp=16, stats=st)
    assert st.mode == 1
    ref = O.render_backward(scene, integ, 21, 16, gi, [params.texture_of(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for k, a, b in zip(keys, g, ref):
        a = a.cpu().numpy()
        assert a.shape == b.shape and np.abs(b).max() > 0, k
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-9 + 2e-4 * np.abs(b).max(), err_msg=k)


@pytest.mark.parametrize("tex_res", [73, 74])
def test_prb_bitmap_lds_accumulator_limit(tex_res, monkeypatch):
    """The largest bitmap the texel scatter accumulates in LDS: 73^2 x 3 =
    15,987 floats, a 128-KB double accumulator (one 1,024-thread workgroup
    per CU; round 5), and the first size past it (74^2 x 3: the transposed
    global atomics).  Gradients vs the oracle over several 4096-path chunks."""
    monkeypatch.setenv("MH_WF_CHUNK", "4096")
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    d = mi.cornell_box_bitmap(tex_res=tex_res, width=40, height=32, spp=16)
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "prb", "max_depth": 5})
    params = mi.traverse(scene)
    keys = ["white.reflectance.data"]
    gi = np.random.default_rng(9).random((32, 40, 3)).astype(np.float32) / (32 * 40 * 3)
    st = A.Stats()
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), keys, integ, seed=29, spp=16, stats=st)
    assert st.mode == 1
    ref = O.render_backward(scene, integ, 29, 16, gi, [params.texture_of(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    a, b = g[0].cpu().numpy(), ref[0]
    assert a.shape == b.shape == (tex_res, tex_res, 3) and np.abs(b).max() > 0
    np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-9 + 2e-4 * np.abs(b).max())


@pytest.mark.parametrize("lds", ["1", "0"])
@pytest.mark.parametrize("red_channels", [3, 1])
def test_prb_two_bitmaps_wavefront(red_channels, lds, monkeypatch):
    """Two bitmap parameters (white and red) plus an rgb slot: on the fused
    wavefront every bitmap vertex is recorded with its bitmap index and the
    scatter adds it to that bitmap's texels (LDS block of both, or transposed
    global atomics).  Bitmaps of different channel counts take the replay
    megakernel instead.  Gradients vs the oracle."""
    monkeypatch.setenv("MH_WF_CHUNK", "4096")
    monkeypatch.setenv("MH_PRB_LDS_TEX", lds)
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    d = mi.cornell_box_bitmap(tex_res=8, width=40, height=32, spp=16)
    red = np.zeros((6, 5, red_channels), np.float32)
    red[..., 0] = 0.57
    if red_channels == 3:
        red[..., 1], red[..., 2] = 0.04, 0.04
    d["red"]["reflectance"] = {"type": "bitmap", "data": red, "filter_type": "bilinear", "wrap_mode": "repeat",
                               "raw": True}
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    keys = ["white.reflectance.data", "red.reflectance.data", "green.reflectance.value"]
    gi = np.random.default_rng(8).random((32, 40, 3)).astype(np.float32) / (32 * 40 * 3)
    st = A.Stats()
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), keys, integ, seed=23, spp=16, stats=st)
    assert st.mode == (1 if red_channels == 3 else 0), st.mode
    ref = O.render_backward(scene, integ, 23, 16, gi, [params.texture_of(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for k, a, b in zip(keys, g, ref):
        a = a.cpu().numpy()
        assert a.shape == b.shape and np.abs(b).max() > 0, k
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-9 + 2e-4 * np.abs(b).max(), err_msg=k)


# ---------------------------------------------------------------------------
# Config 5: W*H*spp > 2^32 -> passes of spp_per_pass samples, each lane's RNG
# continuing across passes (integrator.cpp:281-295, 353-357)
# ---------------------------------------------------------------------------
@pytest.mark.slow
@pytest.mark.parametrize("b,e", [(0, 2), (510, 512)])
def test_multipass_config5_slab_parity(b, e):
    """Config 5's forward as measured (tools/bench_config5.py: max_depth 8):
    2048^2 * 1024 = 2^32 > 2^32 - 1 samples, so two passes of 512 spp
    (integrator.cpp:281-295).  Lanes [b, e) of every pass-pixel run both
    passes; pass 2 seeds from each lane's carried PCG32 state, continuing
    pass 1's stream (integrator.cpp:353-357), at bounces 1..8.  [510, 512)
    holds the last lanes of every pass-pixel (lane 2^32 - 2 .. 2^32 - 1 of
    the last pixel sits at the pass's end)."""
    mi = _mi()
    scene = cbox(mi, 2048, 2048, 1024)
    integ = mi.load_dict({"type": "path", "max_depth": 8})
    from mitsuba_hip import _abi as A
    st = A.Stats()
    film = mi.render_film(scene, integ, seed=2, spp=1024, spp_begin=b, spp_end=e, stats=st).cpu().numpy()
    # the single chunk is split in two for the two-stream chunk pipeline
    # (mh_api.hip fork_stream): 2 chunks x 2 passes x 8 bounces
    assert st.mode == 2 and st.n_trace_launches == 2 * 2 * 8
    ref = O.render(scene, integ, seed=2, spp=1024, spp_begin=b, spp_end=e)
    assert ref[..., 3].sum() > 0
    ok, frac = _film_close(film, ref)
    assert ok, f"film parity {frac}"


@pytest.mark.slow
def test_config5_prb_gradient_slab_parity():
    """Config 5's gradient leg: 2048^2 @ 1024 = 2^32 samples is ONE AD
    wavefront (ADIntegrator.prepare raises only above 2^32, common.py:571-578;
    lane indices [0, 2^32) in uint32).  The W image sums all 2^32 jitters; the
    gradient of the top slab [1022, 1024) of every pixel (the last lane is
    2^32 - 1) vs the oracle with the same W."""
    mi = _mi()
    import torch
    scene = cbox(mi, 2048, 2048, 1024)
    integ = mi.load_dict({"type": "prb", "max_depth": 8})  # as tools/bench_config5.py measures it
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    seed = mi.sample_tea_32(2, 1)[0]
    w = mi.prb_weights(scene, seed, 1024)
    wn = w.cpu().numpy()
    top = O.prb_weights_rows(scene, seed, 1024, 0, 6)
    bot = O.prb_weights_rows(scene, seed, 1024, 2042, 2048)
    np.testing.assert_allclose(wn[:4], top[:4], rtol=1e-4)
    np.testing.assert_allclose(wn[-4:], bot[-4:], rtol=1e-4)
    gi = np.full((2048, 2048, 3), 1.0 / (2048 * 2048 * 3), np.float32)
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), [key], integ, seed=seed, spp=1024,
                           spp_begin=1022, spp_end=1024, weights=w)[0].cpu().numpy()
    ref = O.render_backward(scene, integ, seed, 1024, gi, [params.texture_of(key)], [(3,)], weights=wn,
                            spp_begin=1022, spp_end=1024)[0]
    assert np.abs(ref).max() > 0
    np.testing.assert_allclose(g, ref, rtol=1e-3, atol=1e-9)


def test_ad_wavefront_limit():
    """prepare() raises above 2^32 samples (common.py:571-578); the C++
    SamplingIntegrator (path) splits into passes instead."""
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = cbox(mi, 2048, 2048, 1536)   # 1.5 * 2^32 samples
    with pytest.raises(A.MitsubaHipError, match="exceeds 2\\^32"):
        mi.prb_weights(scene, 1, 1536)
    with pytest.raises(A.MitsubaHipError, match="exceeds 2\\^32"):
        mi.render_film(scene, mi.load_dict({"type": "prb"}), seed=0, spp=1536, spp_begin=0, spp_end=1)
    st = A.Stats()
    film = mi.render_film(scene, mi.load_dict({"type": "path", "max_depth": 2}), seed=0, spp=1536,
                          spp_begin=0, spp_end=1, stats=st)   # 2 passes of 768
    assert float(film[..., 3].sum()) > 0 and st.samples == 2048 * 2048 * 2
    # integrator.cpp:281-295 + the spp_per_pass divisibility error
    with pytest.raises(A.MitsubaHipError, match="multiple of samples_per_wavefront"):
        mi.render_film(scene, mi.load_dict({"type": "path"}), seed=0, spp=2048, spp_begin=0, spp_end=1)


def test_multipass_wavefront_matches_megakernel():
    """The fused wavefront runs the passes of a > 2^32-sample render back to
    back, carrying each lane's PCG32 state (integrator.cpp:353-357); the
    megakernel runs every pass of a lane in one thread.  Same samples."""
    mi = _mi()
    scene = cbox(mi, 2048, 2048, 1024)
    integ = mi.load_dict({"type": "path", "max_depth": 8})
    from mitsuba_hip import _abi as A
    st = A.Stats()
    wf = mi.render_film(scene, integ, seed=3, spp=1024, spp_begin=4, spp_end=6, mode="wavefront",
                        stats=st).cpu().numpy()
    assert st.mode == 2 and st.n_trace_launches == 2 * 2 * 8  # two chunks (two-stream split), two passes of 8 bounces
    mega = mi.render_film(scene, integ, seed=3, spp=1024, spp_begin=4, spp_end=6, mode="mega").cpu().numpy()
    assert mega[..., 3].sum() > 0
    ok, frac = _film_close(wf, mega)
    assert ok, f"film parity {frac}"


# ---------------------------------------------------------------------------
# path / prb with several emitters of different kinds (uniform emitter
# selection, scene.cpp:227-250; constant environment; delta directional)
# ---------------------------------------------------------------------------
def _cbox_lights(mi, w=24, h=20, spp=8):
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = w, h
    d["sensor"]["sampler"]["sample_count"] = spp
    d["sky"] = {"type": "constant", "radiance": {"type": "rgb", "value": [0.3, 0.4, 0.5]}}
    d["sun"] = {"type": "directional", "direction": [0.2, -0.5, -1.0], "irradiance": {"type": "rgb", "value": 2.0}}
    return mi.load_dict(d)


@pytest.mark.parametrize("itype,mode", [("path", "mega"), ("path", "wavefront"), ("prb", "mega")])
def test_multi_emitter_per_sample_parity(itype, mode):
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _cbox_lights(mi)
    assert scene.desc.n_emitters == 3 and scene.desc.environment != A.INVALID
    integ = mi.load_dict({"type": itype, "max_depth": 6})
    L, pos = _gpu_samples(mi, scene, integ, 5, 8, A.FLAG_WAVEFRONT if mode == "wavefront" else 0)
    rL, rpos, _ = O.sample_range(scene, integ, 5, 8, 0, L.shape[0])
    exact = np.all(L == rL, axis=1)
    assert exact.mean() >= 0.999, f"bit-exact fraction {exact.mean()}"
    assert rL.mean() > 0


@pytest.mark.parametrize("mode", ["wavefront", "mega", "wavefront-unfused"])
def test_hide_emitters_path_parity(mode, monkeypatch):
    """path with hide_emitters and an environment: camera rays that escape
    return 0 (valid_ray, path.cpp:115, 256, 284); later escapes still see the
    environment."""
    if mode == "wavefront-unfused":
        monkeypatch.setenv("MH_WF_FUSED", "0")
        mode = "wavefront"
    mi = _mi()
    from mitsuba_hip import _abi as A
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = 24, 20
    d.pop("back")   # open box: camera rays escape
    d["sky"] = {"type": "constant", "radiance": {"type": "rgb", "value": [0.3, 0.4, 0.5]}}
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "path", "max_depth": 6, "hide_emitters": True})
    L, pos = _gpu_samples(mi, scene, integ, 5, 8, A.FLAG_WAVEFRONT if mode == "wavefront" else 0)
    rL, rpos, _ = O.sample_range(scene, integ, 5, 8, 0, L.shape[0])
    exact = np.all(L == rL, axis=1)
    assert exact.mean() >= 0.999, f"bit-exact fraction {exact.mean()}"
    assert (rL.sum(1) == 0).mean() > 0.05 and rL.mean() > 0


def test_multi_emitter_prb_backward_parity():
    mi = _mi()
    import torch
    scene = _cbox_lights(mi, 32, 24, 8)
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    keys = ["white.reflectance.value", "green.reflectance.value"]
    gi = np.full((24, 32, 3), 1.0 / (24 * 32 * 3), np.float32)
    ref = O.render_backward(scene, integ, 21, 8, gi, [params.texture_of(k) for k in keys], [(3,), (3,)])
    for mode in ("auto", "mega", "replay"):
        g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), keys, integ, seed=21, spp=8, mode=mode)
        for a, b in zip(g, ref):
            np.testing.assert_allclose(a.cpu().numpy(), b, rtol=1e-3, atol=1e-7)


# ---------------------------------------------------------------------------
# hdrfilm pixel formats: luminance / xyz develop,
# and the PRB adjoint through the colour conversion
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("pf", ["rgb", "luminance", "xyz"])
def test_develop_pixel_format_parity(pf):
    mi = _mi()
    d = mi.cornell_box()
    d["sensor"]["film"].update(width=24, height=20, pixel_format=pf)
    scene = mi.load_dict(d)
    film = mi.render_film(scene, seed=1, spp=8)
    img = mi.develop(scene, film).cpu().numpy()
    ref = O.develop(film.cpu().numpy(), scene.desc.sensor.pixel_format)
    assert img.shape == ref.shape
    np.testing.assert_array_equal(img, ref)


def test_prb_backward_luminance_film():
    """d(sum Y)/d rho through a luminance film == the rgb adjoint with
    grad_rgb = [0.212671, 0.715160, 0.072169] per pixel."""
    mi = _mi()
    import torch
    d = mi.cornell_box()
    d["sensor"]["film"].update(width=24, height=20, pixel_format="luminance")
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    gy = torch.ones((20, 24, 1), device="cuda")
    g = mi.render_backward(scene, params, gy, ["white.reflectance.value"], integ, seed=3, spp=8)[0].cpu().numpy()
    grgb = np.broadcast_to(np.array([0.212671, 0.715160, 0.072169], np.float32), (20, 24, 3)).copy()
    ref = O.render_backward(scene, integ, 3, 8, grgb, [params.texture_of("white.reflectance.value")], [(3,)])[0]
    np.testing.assert_allclose(g, ref, rtol=1e-3)


# ---------------------------------------------------------------------------
# The optimisation loop around the path:
# mi.render -> loss.backward (PRB render_backward) -> mi.ad.Adam -> update
# ---------------------------------------------------------------------------
def test_inverse_rendering_loop_recovers_albedo():
    mi = _mi()
    import torch
    d = mi.cornell_box()
    d["sensor"]["film"].update(width=32, height=32)
    d["integrator"] = {"type": "prb", "max_depth": 4}
    scene = mi.load_dict(d)
    key = "red.reflectance.value"
    params = mi.traverse(scene, device="cuda")
    target = params[key].clone()
    ref = mi.render(scene, seed=100, spp=128)
    params[key] = torch.tensor([0.2, 0.2, 0.2], device="cuda")
    params.update()
    opt = mi.ad.Adam(lr=0.05)
    opt[key] = params[key]
    params.update(opt)
    err0 = float((params[key].detach() - target).abs().max())
    losses = []
    for it in range(40):
        img = mi.render(scene, params, seed=it, spp=64)
        loss = ((img - ref) ** 2).mean()
        loss.backward()
        opt.step()
        opt[key] = opt[key].detach().clamp(0.0, 1.0)
        params.update(opt)
        losses.append(float(loss.detach()))
    err = float((params[key].detach() - target).abs().max())
    # the loss bottoms out at the Monte Carlo noise floor; the parameter converges
    assert np.mean(losses[-10:]) < np.mean(losses[:3]), losses
    assert err < 0.35 * err0, (err, err0, params[key])


# ---------------------------------------------------------------------------
# large meshes (BVH in HBM/L2, not LDS): the per-lane stream engine on the
# collapsed 4-wide BVH (mh_bvh.cpp collapse_bvh4) and on the binary BVH
# ---------------------------------------------------------------------------
def _blob_scene(mi, n_tri=6000, w=24, h=24, spp=8, max_depth=6):
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
    d["sensor"]["sampler"]["sample_count"] = spp
    d["integrator"]["max_depth"] = max_depth
    T = mi.Transform4f
    d["blob"] = {"type": "mesh", "vertex_positions": V.astype(np.float32), "faces": F.astype(np.uint32),
                 "to_world": T.translate([0, -0.45, 0]) @ T.scale(0.45), "bsdf": {"type": "ref", "id": "white"}}
    return mi.load_dict(d)


@pytest.mark.parametrize("bvh4", ["1", "q", "0", "1-ovf"])
def test_large_mesh_trace_parity(bvh4, monkeypatch):
    # the trace entry points run the wavefront's stream engine on a global-
    # memory BVH: float BVH4, quantised BVH4 (MH_BVH4Q=1) or BVH2; "-ovf": a
    # 4-entry LDS stack, so most rays take the global overflow region too
    monkeypatch.setenv("MH_BVH4", "0" if bvh4 == "0" else "1")
    monkeypatch.setenv("MH_BVH4Q", "1" if bvh4 == "q" else "0")
    if bvh4.endswith("-ovf"):
        monkeypatch.setenv("MH_STREAM_STACK", "4")
    mi = _mi()
    scene = _blob_scene(mi)
    rays = random_rays(scene, 1 << 16, seed=4)
    t, u, v, prim, shape, occ = gpu_trace(mi, scene, rays)
    rt, ru, rv, rprim, rshape = O.trace_closest(scene, rays)
    rocc = O.trace_shadow(scene, rays)
    same = (shape == rshape) & (prim == rprim) & ((t == rt) | (np.isinf(t) & np.isinf(rt)))
    assert same.mean() >= 0.9999, f"closest-hit mismatch fraction {1 - same.mean()}"
    assert (occ == rocc).mean() >= 0.9999
    assert (rshape == 8).mean() > 0.02      # the blob is hit


@pytest.mark.parametrize("bvh4,fused", [("1", "1"), ("1", "0"), ("q", "1"), ("q", "0"), ("0", "1"), ("1-ovf", "0")])
def test_large_mesh_per_sample_parity(bvh4, fused, monkeypatch):
    monkeypatch.setenv("MH_BVH4", "0" if bvh4 == "0" else "1")
    monkeypatch.setenv("MH_BVH4Q", "1" if bvh4 == "q" else "0")
    if bvh4.endswith("-ovf"):
        monkeypatch.setenv("MH_STREAM_STACK", "4")
    monkeypatch.setenv("MH_WF_FUSED", fused)
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _blob_scene(mi)
    integ = scene.integrator()
    L, pos = _gpu_samples(mi, scene, integ, 2, 8, A.FLAG_WAVEFRONT)
    rL, rpos, _ = O.sample_range(scene, integ, 2, 8, 0, L.shape[0])
    np.testing.assert_array_equal(pos, rpos)
    exact = np.all(L == rL, axis=1)
    assert exact.mean() >= 0.999, f"bit-exact fraction {exact.mean()}"


# ---------------------------------------------------------------------------
# smooth shading frames on the device: a height-field mesh with
# interpolated vertex normals (meshio.recompute_vertex_normals, the
# reference's angle-weighted normals) and uvs driving a bitmap texture
# (mesh.cpp:1368-1460 compute_surface_interaction: shading frame from the
# interpolated normal, uv from the texcoords)
# ---------------------------------------------------------------------------
def _smooth_mesh_scene(mi, n, w=32, h=28, spp=8):
    from mitsuba_hip import meshio
    x, y = np.meshgrid(np.linspace(-0.8, 0.8, n), np.linspace(-0.8, 0.8, n))
    z = 0.15 * np.sin(3 * x) * np.cos(2 * y)
    V = np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)
    UV = np.stack([(x + 0.8) / 1.6, (y + 0.8) / 1.6], -1).reshape(-1, 2).astype(np.float32)
    i = np.arange(n - 1)
    a = (i[:, None] * n + i[None, :]).reshape(-1)
    F = np.concatenate([np.stack([a, a + 1, a + n + 1], 1), np.stack([a, a + n + 1, a + n], 1)]).astype(np.uint32)
    T = mi.Transform4f
    to_world = T.translate([0, 0.1, 0]) @ T.rotate([1, 0, 0], -70)
    Vw = (V.astype(np.float64) @ to_world.matrix[:3, :3].T + to_world.matrix[:3, 3]).astype(np.float32)
    N = meshio.recompute_vertex_normals(Vw, F)
    tex = np.random.default_rng(5).uniform(0.2, 0.9, (8, 8, 3)).astype(np.float32)
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = w, h
    d["sensor"]["sampler"]["sample_count"] = spp
    d.pop("small-box")
    d.pop("large-box")
    d["bumpy"] = {"type": "mesh", "vertex_positions": Vw, "faces": F, "vertex_normals": N, "vertex_texcoords": UV,
                  "bsdf": {"type": "diffuse", "reflectance": {"type": "bitmap", "data": tex, "raw": True,
                                                              "filter_type": "bilinear"}}}
    return mi.load_dict(d)


@pytest.mark.parametrize("n,mode", [(5, "wavefront"), (5, "mega"), (12, "wavefront"), (12, "mega")])
def test_smooth_normals_per_sample_parity(n, mode):
    """n = 5: 32 triangles + 6 rectangles (packet engine, fused bounce);
    n = 12: 242 triangles (per-lane stream engine, unfused wavefront)."""
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _smooth_mesh_scene(mi, n)
    assert scene.desc.normals and scene.desc.texcoords
    integ = mi.load_dict({"type": "path", "max_depth": 6})
    L, pos = _gpu_samples(mi, scene, integ, 4, 8, A.FLAG_WAVEFRONT if mode == "wavefront" else 0)
    rL, rpos, _ = O.sample_range(scene, integ, 4, 8, 0, L.shape[0])
    np.testing.assert_array_equal(pos, rpos)
    exact = np.all(L == rL, axis=1)
    assert exact.mean() >= 0.999, f"bit-exact fraction {exact.mean()}"
    assert rL.mean() > 0


def test_smooth_normals_prb_gradient_parity():
    mi = _mi()
    import torch
    scene = _smooth_mesh_scene(mi, 5, 24, 20, 8)
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    keys = ["bumpy.bsdf.reflectance.data", "red.reflectance.value"]
    gi = np.random.default_rng(1).random((20, 24, 3)).astype(np.float32) / (20 * 24 * 3)
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), keys, integ, seed=6, spp=8)
    ref = O.render_backward(scene, integ, 6, 8, gi, [params.texture_of(k) for k in keys],
                            [tuple(params[k].shape) for k in keys])
    for k, a, b in zip(keys, g, ref):
        a = a.cpu().numpy()
        assert np.abs(b).max() > 0, k
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=1e-9 + 2e-4 * np.abs(b).max(), err_msg=k)


# ---------------------------------------------------------------------------
# alpha films (hdrfilm rgba / luminance_alpha / xyza, hdrfilm.cpp:160-188,
# 304-405): the film stores R G B A W, a sample's alpha is its ray validity
# (integrator.cpp:1229-1231; prb: depth != 0, prb.py:253-257)
# ---------------------------------------------------------------------------
def _open_box(mi, pf, w=32, h=24, spp=8, env=False):
    d = mi.cornell_box()
    d["sensor"]["film"].update(width=w, height=h, pixel_format=pf)
    d["sensor"]["sampler"]["sample_count"] = spp
    d.pop("back")   # camera rays escape through the back: alpha 0 there
    if env:
        d["sky"] = {"type": "constant", "radiance": {"type": "rgb", "value": [0.3, 0.4, 0.5]}}
    return mi.load_dict(d)


@pytest.mark.parametrize("pf,itype,mode", [("rgba", "path", "auto"), ("rgba", "path", "mega"),
                                           ("luminance_alpha", "path", "auto"), ("xyza", "prb", "auto"),
                                           ("rgba", "volpath", "auto")])
def test_alpha_film_parity(pf, itype, mode):
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _open_box(mi, pf)
    fmt = scene.desc.sensor.pixel_format
    assert A.pixel_has_alpha(fmt)
    integ = mi.load_dict({"type": itype, "max_depth": 6})
    film = mi.render_film(scene, integ, seed=2, spp=8, mode=mode).cpu().numpy()
    ref = O.render(scene, integ, seed=2, spp=8)
    assert film.shape == ref.shape == (24, 32, 5)
    ok, frac = _film_close(film, ref)
    assert ok, f"film parity {frac}"
    assert 0.05 < (ref[..., 3] / ref[..., 4]).mean() < 0.95       # partly transparent
    img = mi.develop(scene, mi.render_film(scene, integ, seed=2, spp=8, mode=mode)).cpu().numpy()
    rimg = O.develop(ref, fmt)
    assert img.shape == rimg.shape == (24, 32, A.image_channels(fmt))
    ok, frac = _film_close(img, rimg)
    assert ok, f"image parity {frac}"


@pytest.mark.parametrize("itype,mode", [("path", "wavefront"), ("path", "mega"), ("prb", "mega"),
                                        ("volpath", "mega"), ("volpath", "wavefront"), ("volpath", "wavefront-lane"),
                                        ("volpath", "wavefront-rounds")])
def test_alpha_per_sample_validity(itype, mode, monkeypatch):
    if mode == "wavefront-lane":
        monkeypatch.setenv("MH_TRAVERSAL", "lane")
    if mode == "wavefront-rounds":
        monkeypatch.setenv("MH_VOL_MODE", "rounds")
    mode = mode.split("-")[0]
    mi = _mi()
    from mitsuba_hip import _abi as A
    scene = _open_box(mi, "rgba", 24, 20, 8, env=(itype == "path"))
    integ = mi.load_dict({"type": itype, "max_depth": 6, "hide_emitters": itype == "path"})
    n = 24 * 20 * 8
    out = np.zeros(6 * n, np.float32)
    ic = integ.c()
    A.check(A.lib().mh_render_samples(scene.handle(0), C.byref(ic), 3, 8, 0, 0, out.ctypes.data_as(C.c_void_p),
                                      A.FLAG_WAVEFRONT if mode == "wavefront" else 0))
    rL, rpos, rvalid = O.sample_range(scene, integ, 3, 8, 0, n)
    alpha = out[5 * n:]
    np.testing.assert_array_equal(alpha, rvalid.astype(np.float32))
    assert 0.05 < alpha.mean() < 0.95
    exact = np.all(out[:3 * n].reshape(3, n).T == rL, axis=1)
    assert exact.mean() >= 0.999


def test_alpha_film_prb_backward():
    """d loss / d rho through an rgba film: the alpha channel carries no
    derivative, the colour channels are the rgb adjoint."""
    mi = _mi()
    import torch
    scene = _open_box(mi, "rgba", 24, 20, 8)
    integ = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    gi = np.random.default_rng(2).random((20, 24, 4)).astype(np.float32)
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), [key], integ, seed=5, spp=8)[0].cpu().numpy()
    ref = O.render_backward(scene, integ, 5, 8, np.ascontiguousarray(gi[..., :3]), [params.texture_of(key)],
                            [(3,)])[0]
    np.testing.assert_allclose(g, ref, rtol=1e-3)
