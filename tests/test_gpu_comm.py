"""Multi-GPU through the C ABI (include/mitsuba_hip.h "Multi-GPU", SURVEY.md
§8(e); the splice point is SamplingIntegrator::render,
src/render/integrator.cpp:276-390).

The 1-GPU box can run an RCCL communicator of one rank only (RCCL refuses
two ranks on one device), so:
  * world-1 communicators (mh_comm_create from a unique id, and
    mh_comm_create_all) check that the in-call reductions (MH_FLAG_REDUCE /
    MH_FLAG_REDUCE_ROOT) sit in the right place: results equal the plain
    calls bit for bit (deterministic films) or to float order (gradients);
  * the sharded entry points without communicators (2 and 3 scenes on
    cuda:0, summed by device copies) check the slab split itself: the
    union of the slabs equals one render of all samples to the float order
    of the sum, and the sharded gradient equals one render_backward.
The N-rank RCCL run is the driver's (bench.py over torch.distributed; its
rehearsal with gloo ranks is tests/test_gpu_multirank.py).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mi():
    import mitsuba_hip as mi
    if not mi.is_available():
        pytest.fail("no HIP device / native library: the GPU tests need an MI355X")
    return mi


def _scene(mi, res=48, spp=16):
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = res
    d["sensor"]["sampler"]["sample_count"] = spp
    return mi.load_dict(d)


def _film(scene, torch):
    return torch.zeros((scene.height, scene.width, 4), dtype=torch.float32, device="cuda:0")


def _render(A, scene, integ, seed, spp, film, flags):
    ic = integ.c()
    A.check(A.lib().mh_render(scene.handle(0), C.byref(ic), seed, spp, 0, 0, C.c_void_p(film.data_ptr()),
                              A.FLAG_DEVICE_POINTERS | flags, None))


def test_comm_world1_reduce_is_identity():
    mi = _mi()
    import torch
    from mitsuba_hip.comm import Comm
    uid = Comm.unique_id()
    assert len(uid) == 128
    c = Comm(uid, 1, 0, 0)
    assert c.info() == (1, 0, 0)
    x = torch.randn(1 << 16, device="cuda:0")
    ref = x.clone()
    c.reduce_(x)
    c.reduce_(x, root=0)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    (c1,) = Comm.create_all([0])
    assert c1.info() == (1, 0, 0)
    c1.reduce_(x)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    c.close()
    c1.close()
    del mi


def test_render_reduce_flags_world1_match_plain_calls():
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    from mitsuba_hip.comm import Comm, scene_set_comm
    scene = _scene(mi)
    integ = mi.load_dict({"type": "path", "max_depth": 6})
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    ref, red, root = _film(scene, torch), _film(scene, torch), _film(scene, torch)
    _render(A, scene, integ, 5, 16, ref, A.FLAG_DETERMINISTIC)
    with pytest.raises(A.MitsubaHipError, match="needs a communicator"):
        _render(A, scene, integ, 5, 16, red, A.FLAG_DETERMINISTIC | A.FLAG_REDUCE)
    scene_set_comm(scene, comm)
    _render(A, scene, integ, 5, 16, red, A.FLAG_DETERMINISTIC | A.FLAG_REDUCE)
    _render(A, scene, integ, 5, 16, root, A.FLAG_DETERMINISTIC | A.FLAG_REDUCE_ROOT)
    with pytest.raises(A.MitsubaHipError, match="ACCUMULATE"):
        _render(A, scene, integ, 5, 16, red, A.FLAG_REDUCE | A.FLAG_ACCUMULATE)
    torch.cuda.synchronize()
    assert torch.equal(red, ref) and torch.equal(root, ref)

    # render_backward: the slab W + all-reduce (1 rank: every sample) and the
    # all-reduced gradient equal the plain call; MH_FLAG_LOCAL_WEIGHTS too
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    gi = torch.full((scene.height, scene.width, 3), 1.0 / (scene.height * scene.width * 3), device="cuda:0")
    tex = (C.c_uint32 * 1)(params.param_id(key))

    def bwd(flags):
        g = torch.zeros(3, device="cuda:0")
        ptr = (C.c_void_p * 1)(g.data_ptr())
        ic = prb.c()
        A.check(A.lib().mh_render_backward(scene.handle(0), C.byref(ic), 9, 16, 0, 0, C.c_void_p(gi.data_ptr()),
                                           None, 1, tex, ptr, A.FLAG_DEVICE_POINTERS | flags, None))
        torch.cuda.synchronize()
        return g.cpu().numpy()

    g0 = bwd(0)
    np.testing.assert_allclose(bwd(A.FLAG_REDUCE), g0, rtol=1e-5)
    np.testing.assert_allclose(bwd(A.FLAG_REDUCE | A.FLAG_LOCAL_WEIGHTS), g0, rtol=1e-5)
    scene_set_comm(scene, None)
    comm.close()


def test_reduce_extents_with_scale_hook(monkeypatch):
    """Which extents the in-call reductions cover: with MH_TEST_COMM_SCALE a
    one-rank sum doubles its buffer (mh_comm.cpp comm_reduce_one), so the film
    (MH_FLAG_REDUCE and _ROOT), the W image and the gradients -- rgb, bitmap,
    and prbvolpath's grid (corner-gathered) + albedo -- must come out exactly
    twice the plain calls' (local W: no W reduction), and the backward with
    the in-call W reduction exactly equal to the plain one (2 W halves dL,
    the gradient sum doubles it back).  Deterministic mode: bit-comparable."""
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    from mitsuba_hip.comm import Comm, scene_set_comm
    D = A.FLAG_DETERMINISTIC
    tex = np.random.default_rng(1).uniform(0.2, 0.8, (8, 8, 3)).astype(np.float32)
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 32
    d["red"]["reflectance"] = {"type": "bitmap", "data": tex, "filter_type": "bilinear", "wrap_mode": "repeat",
                               "raw": True}
    scene = mi.load_dict(d)
    integ = mi.load_dict({"type": "path", "max_depth": 5})
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    scene_set_comm(scene, comm)
    monkeypatch.setenv("MH_TEST_COMM_SCALE", "1")
    plain, red, root = _film(scene, torch), _film(scene, torch), _film(scene, torch)
    _render(A, scene, integ, 5, 16, plain, D)
    _render(A, scene, integ, 5, 16, red, D | A.FLAG_REDUCE)
    _render(A, scene, integ, 5, 16, root, D | A.FLAG_REDUCE_ROOT)
    torch.cuda.synchronize()
    assert float(plain.abs().max()) > 0
    assert torch.equal(red, 2 * plain) and torch.equal(root, 2 * plain)
    # W image
    w0 = torch.zeros((32, 32), device="cuda:0")
    w1 = torch.zeros((32, 32), device="cuda:0")
    for w, f in ((w0, 0), (w1, A.FLAG_REDUCE)):
        A.check(A.lib().mh_prb_weights(scene.handle(0), 9, 16, 0, 0, C.c_void_p(w.data_ptr()),
                                       A.FLAG_DEVICE_POINTERS | D | f))
    torch.cuda.synchronize()
    assert torch.equal(w1, 2 * w0)
    # gradients: an rgb slot and a bitmap slot
    prb = mi.load_dict({"type": "prb", "max_depth": 5})
    params = mi.traverse(scene)
    keys = ["white.reflectance.value", "red.reflectance.data"]
    gi = torch.full((32, 32, 3), 1.0 / (32 * 32 * 3), device="cuda:0")

    def bwd(sc, ps, ks, integrator, flags, gin):
        tex_ids = (C.c_uint32 * len(ks))(*[ps.param_id(k) for k in ks])
        outs = [torch.zeros(ps[k].shape, dtype=torch.float32, device="cuda:0") for k in ks]
        ptr = (C.c_void_p * len(ks))(*[o.data_ptr() for o in outs])
        ic = integrator.c()
        A.check(A.lib().mh_render_backward(sc.handle(0), C.byref(ic), 9, 16, 0, 0, C.c_void_p(gin.data_ptr()),
                                           None, len(ks), tex_ids, ptr, A.FLAG_DEVICE_POINTERS | D | flags, None))
        torch.cuda.synchronize()
        return [o.cpu().numpy() for o in outs]

    g0 = bwd(scene, params, keys, prb, 0, gi)
    g_local = bwd(scene, params, keys, prb, A.FLAG_REDUCE | A.FLAG_LOCAL_WEIGHTS, gi)
    g_red = bwd(scene, params, keys, prb, A.FLAG_REDUCE, gi)
    for k, a, b, c in zip(keys, g0, g_local, g_red):
        assert np.abs(a).max() > 0, k
        np.testing.assert_allclose(b, 2 * a, rtol=1e-6, atol=0, err_msg=k)
        np.testing.assert_allclose(c, a, rtol=1e-6, atol=0, err_msg=k)
    scene_set_comm(scene, None)
    # prbvolpath: the grid sigma_t (corner blocks) and the albedo
    dv = mi.volume_cube(24, 20, 8, grid=mi.fbm_grid(16), scale=4.0, max_depth=6)
    dv["integrator"] = {"type": "prbvolpath", "max_depth": 6, "rr_depth": 5}
    vs = mi.load_dict(dv)
    scene_set_comm(vs, comm)
    vp = mi.traverse(vs)
    vkeys = ["medium1.sigma_t.data", "medium1.albedo.value"]
    gv = torch.from_numpy(np.random.default_rng(2).standard_normal((20, 24, 3)).astype(np.float32)).cuda()
    v0 = bwd(vs, vp, vkeys, vs.integrator(), 0, gv)
    v_local = bwd(vs, vp, vkeys, vs.integrator(), A.FLAG_REDUCE | A.FLAG_LOCAL_WEIGHTS, gv)
    for k, a, b in zip(vkeys, v0, v_local):
        assert np.abs(a).max() > 0, k
        np.testing.assert_allclose(b, 2 * a, rtol=1e-6, atol=0, err_msg=k)
    scene_set_comm(vs, None)
    comm.close()


def test_comm_destroy_refused_while_attached():
    mi = _mi()
    from mitsuba_hip import _abi as A
    from mitsuba_hip.comm import Comm, scene_set_comm
    scene = _scene(mi)
    c = Comm(Comm.unique_id(), 1, 0, 0)
    scene_set_comm(scene, c)
    assert scene._comms[0] is c  # the scene keeps the Comm alive
    with pytest.raises(A.MitsubaHipError, match="still attached"):
        c.close()
    scene_set_comm(scene, None)
    assert 0 not in scene._comms
    c.close()


@pytest.mark.parametrize("n", [2, 3])
def test_render_sharded_slabs_sum_to_one_render(n):
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    from mitsuba_hip.comm import render_sharded
    spp = 16
    scenes = [_scene(mi, spp=spp) for _ in range(n)]
    integ = mi.load_dict({"type": "path", "max_depth": 6})
    ref = _film(scenes[0], torch)
    _render(A, scenes[0], integ, 7, spp, ref, 0)
    films = [_film(s, torch) for s in scenes]
    stats = [None] * n
    render_sharded(scenes, integ, 7, spp, films, stats=stats)
    torch.cuda.synchronize()
    for f in films[1:]:
        assert torch.equal(f, films[0])  # the sum is copied to every scene
    assert sum(s.samples for s in stats) == scenes[0].width * scenes[0].height * spp
    tol = 1e-5 * float(ref.abs().max())
    assert float((films[0] - ref).abs().max()) <= tol
    # root-only: films[0] holds the sum
    films2 = [_film(s, torch) for s in scenes]
    render_sharded(scenes, integ, 7, spp, films2, reduce_all=False)
    torch.cuda.synchronize()
    assert float((films2[0] - ref).abs().max()) <= tol


def test_render_backward_sharded_matches_one_call():
    mi = _mi()
    import torch
    from mitsuba_hip.comm import render_backward_sharded
    spp = 16
    scenes = [_scene(mi, spp=spp) for _ in range(2)]
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    params = mi.traverse(scenes[0])
    key = "white.reflectance.value"
    gi = torch.full((scenes[0].height, scenes[0].width, 3), 1.0 / (48 * 48 * 3), device="cuda:0")
    (ref,) = mi.render_backward(scenes[0], params, gi, [key], prb, seed=3, spp=spp)
    outs = render_backward_sharded(scenes, params, gi, [key], prb, 3, spp)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    np.testing.assert_allclose(outs[0][0].cpu().numpy(), ref.cpu().numpy(), rtol=1e-4)


def test_render_backward_sharded_prbvolpath():
    """The sharded backward of prbvolpath (grid sigma_t through the per-scene
    corner blocks, albedo through the small slots): the slabs' gradients,
    summed by device copies, equal one render_backward to float order."""
    mi = _mi()
    import torch
    from mitsuba_hip.comm import render_backward_sharded
    spp = 8

    def vol():
        d = mi.volume_cube(24, 20, spp, grid=mi.fbm_grid(16), scale=4.0, max_depth=6)
        d["integrator"] = {"type": "prbvolpath", "max_depth": 6, "rr_depth": 5}
        return mi.load_dict(d)

    scenes = [vol() for _ in range(2)]
    integ = scenes[0].integrator()
    params = mi.traverse(scenes[0])
    keys = ["medium1.sigma_t.data", "medium1.albedo.value"]
    gi = torch.from_numpy(np.random.default_rng(2).standard_normal((20, 24, 3)).astype(np.float32)).cuda()
    ref = mi.render_backward(scenes[0], params, gi, keys, integ, seed=4, spp=spp)
    outs = render_backward_sharded(scenes, params, gi, keys, integ, 4, spp)
    torch.cuda.synchronize()
    for i, (k, r) in enumerate(zip(keys, ref)):
        a, r = outs[0][i].cpu().numpy(), r.cpu().numpy()
        assert np.abs(r).max() > 0, k
        np.testing.assert_allclose(a, r, rtol=1e-4, atol=1e-6 * np.abs(r).max(), err_msg=k)


def test_render_sharded_with_world1_comm_and_argument_checks():
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    from mitsuba_hip.comm import Comm, render_sharded, scene_set_comm
    scene = _scene(mi)
    integ = mi.load_dict({"type": "path", "max_depth": 6})
    ref = _film(scene, torch)
    _render(A, scene, integ, 2, 16, ref, A.FLAG_DETERMINISTIC)
    (c,) = Comm.create_all([0])
    scene_set_comm(scene, c)
    f = _film(scene, torch)
    render_sharded([scene], integ, 2, 16, [f], deterministic=True)
    torch.cuda.synchronize()
    assert torch.equal(f, ref)
    with pytest.raises(A.MitsubaHipError, match="appears twice"):
        render_sharded([scene, scene], integ, 2, 16, [f, f])
    other = _scene(mi)
    with pytest.raises(A.MitsubaHipError, match="every scene has a communicator or none"):
        render_sharded([scene, other], integ, 2, 16, [f, _film(other, torch)])
    scene_set_comm(scene, None)
    with pytest.raises(A.MitsubaHipError, match="spp must be >="):
        render_sharded([scene, other], integ, 2, 1, [f, _film(other, torch)])
    c.close()


def test_failed_collective_call_aborts_its_communicator(monkeypatch):
    """A MH_FLAG_REDUCE call that fails after it was issued aborts the scene's
    communicator (mh_api.hip abort_on_failure): its error says so, and every
    later reduce on that communicator fails at once with 'aborted' instead of
    pairing with a peer's different collective.  The failure is
    injected by the MH_TEST_FAIL_AFTER_ISSUE hook of mh_render."""
    mi = _mi()
    import torch
    from mitsuba_hip import _abi as A
    from mitsuba_hip.comm import Comm, scene_set_comm
    scene = _scene(mi)
    integ = mi.load_dict({"type": "path", "max_depth": 6})
    comm = Comm(Comm.unique_id(), 1, 0, 0)
    scene_set_comm(scene, comm)
    film = _film(scene, torch)
    _render(A, scene, integ, 5, 16, film, A.FLAG_REDUCE)  # healthy first
    monkeypatch.setenv("MH_TEST_FAIL_AFTER_ISSUE", "1")
    with pytest.raises(A.MitsubaHipError, match="injected failure.*communicator was aborted"):
        _render(A, scene, integ, 5, 16, film, A.FLAG_REDUCE)
    monkeypatch.delenv("MH_TEST_FAIL_AFTER_ISSUE")
    with pytest.raises(A.MitsubaHipError, match="aborted"):
        _render(A, scene, integ, 5, 16, film, A.FLAG_REDUCE)
    # without MH_FLAG_REDUCE the scene still renders
    ref = _film(scene, torch)
    _render(A, scene, integ, 5, 16, ref, 0)
    torch.cuda.synchronize()
    assert float(ref.sum()) > 0
    scene_set_comm(scene, None)
    comm.close()


_DEADLINE_SCRIPT = r"""
import ctypes as C, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "mitsuba3-nasa_amd"))
import torch
import mitsuba_hip as mi
from mitsuba_hip import _abi as A
from mitsuba_hip.comm import Comm, scene_set_comm
mi.set_variant("hip_ad_rgb")
d = mi.cornell_box()
d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 512
scene = mi.load_dict(d)
integ = mi.load_dict({"type": "path", "max_depth": 8})
comm = Comm(Comm.unique_id(), 1, 0, 0)
scene_set_comm(scene, comm)
film = torch.zeros((512, 512, 4), device="cuda:0")
ic = integ.c()
rc = A.lib().mh_render(scene.handle(0), C.byref(ic), 1, 256, 0, 0, C.c_void_p(film.data_ptr()),
                       A.FLAG_DEVICE_POINTERS | A.FLAG_REDUCE, None)
msg = A.lib().mh_last_error().decode()
torch.cuda.synchronize()
print("RC", rc)
print("MSG", msg)
"""


def test_collective_wait_deadline_aborts(tmp_path):
    """comm_wait's deadline (MH_COMM_TIMEOUT_S, read once per process): a
    REDUCE call whose stream has not drained within it aborts the
    communicator and returns an error naming the deadline instead of waiting
    (a peer that never issues its collective would otherwise hang the rank).
    Here the deadline (1 ms) is shorter than the render (~20 ms)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "deadline.py"
    script.write_text(_DEADLINE_SCRIPT)
    env = dict(os.environ, MH_COMM_TIMEOUT_S="0.001")
    r = subprocess.run([sys.executable, str(script), root], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = dict(l.split(" ", 1) for l in r.stdout.splitlines() if l.startswith(("RC ", "MSG ")))
    assert out["RC"] != "0"
    assert "did not complete within" in out["MSG"] and "aborted" in out["MSG"], out["MSG"]
