"""CPU, world_size 2 and 4 over gloo: the sample-slab sharding + all-reduce
orchestration that bench.py runs over RCCL (mitsuba_hip.distributed), with
the CPU oracle standing in for the HIP entry points.  The union of the two
ranks' slabs must reproduce the single-process render and PRB gradient."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(mi):
    d = mi.cornell_box()
    d["sensor"]["film"]["width"], d["sensor"]["film"]["height"] = 24, 16
    return mi.load_dict(d)


def _ops(mi, O, scene, torch):
    fwd = mi.load_dict({"type": "path", "max_depth": 6})
    prb = mi.load_dict({"type": "prb", "max_depth": 6})
    key = "white.reflectance.value"
    tex = scene.params[key][1]
    gi = np.full((scene.height, scene.width, 3), 1.0 / (scene.height * scene.width * 3), np.float32)
    from mitsuba_hip import distributed as D
    return D.StepOps(
        render_film=lambda seed, spp, b, e: torch.from_numpy(O.render(scene, fwd, seed, spp, b, e, threads=2)),
        develop=lambda f: torch.from_numpy(O.develop(f.numpy())),
        prb_weights=lambda seed, spp, b, e: torch.from_numpy(O.prb_weights(scene, seed, spp, b, e, threads=2)),
        render_backward=lambda seed, spp, b, e, w: [torch.from_numpy(
            O.render_backward(scene, prb, seed, spp, gi, [tex], [(3,)], weights=None if w is None else w.numpy(),
                              spp_begin=b, spp_end=e, threads=2)[0])],
        seed_grad=lambda seed: mi.sample_tea_32(seed, 1)[0])


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd"), os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist
    import mitsuba_hip as mi
    import oracle_py as O
    from mitsuba_hip import distributed as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = _scene(mi)
    slab = D.sample_slab(rank, world, 8 // world)
    img, grads = D.fwd_grad_step(_ops(mi, O, scene, torch), slab, seed=7)
    # the same step with the W image computed locally on every rank (no W
    # all-reduce) and the film summed onto rank 0 only
    img2, grads2 = D.fwd_grad_step(_ops(mi, O, scene, torch), slab, seed=7, local_weights=True, film_to_root=True)
    # packed: film and W summed in one all-reduce (bench.py's default step)
    # ... timed as bench.py times it at N > 1 (collective names, bytes, calls)
    timer = D.CollTimer()
    D.set_collective_timer(timer)
    img3, grads3 = D.fwd_grad_step(_ops(mi, O, scene, torch), slab, seed=7, packed=True)
    D.set_collective_timer(None)
    colls = timer.summary(1)
    # overlapped (bench.py's default): forward on a worker thread alongside
    # W + W all-reduce + backward, then film + gradient in one all-reduce
    ops = _ops(mi, O, scene, torch)
    ops.concurrent = D.PairRunner()
    D.set_collective_timer(timer)
    img4, grads4 = D.fwd_grad_step(ops, slab, seed=7, overlap=True)
    D.set_collective_timer(None)
    colls4 = timer.summary(1)
    t = D.max_over_ranks(float(rank) + 0.5)
    tmin = D.min_over_ranks(float(rank) + 0.5)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), img=img.numpy(), g=grads[0].numpy(), t=t, tmin=tmin,
             begin=slab.begin, end=slab.end, img2=img2.numpy(), g2=grads2[0].numpy(), img3=img3.numpy(),
             g3=grads3[0].numpy(), coll_names=np.array(sorted(colls)),
             coll_bytes=np.array([colls[k]["bytes"] for k in sorted(colls)]),
             coll_calls=np.array([colls[k]["calls_per_step"] for k in sorted(colls)]),
             coll_ms=np.array([colls[k]["ms_per_step"] for k in sorted(colls)]), img4=img4.numpy(),
             g4=grads4[0].numpy(), coll4_names=np.array(sorted(colls4)),
             coll4_bytes=np.array([colls4[k]["bytes"] for k in sorted(colls4)]))
    dist.barrier()
    dist.destroy_process_group()


def test_sample_slab():
    from mitsuba_hip import distributed as D
    s = [D.sample_slab(r, 4, 64) for r in range(4)]
    assert [(x.begin, x.end) for x in s] == [(0, 64), (64, 128), (128, 192), (192, 256)]
    assert all(x.spp_total == 256 for x in s)
    with pytest.raises(ValueError):
        D.sample_slab(4, 4, 64)


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_ranks_match_single_process(world, tmp_path):
    import torch
    import torch.multiprocessing as mp
    import mitsuba_hip as mi
    import oracle_py as O
    from mitsuba_hip import distributed as D
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    rs = [np.load(tmp_path / f"r{i}.npz") for i in range(world)]
    per = 8 // world
    assert [(int(r["begin"]), int(r["end"])) for r in rs] == [(i * per, (i + 1) * per) for i in range(world)]
    assert all(float(r["t"]) == world - 0.5 for r in rs)  # max over ranks
    assert all(float(r["tmin"]) == 0.5 for r in rs)  # min over ranks
    # the timed packed step: one film + W all-reduce (RGBW film + W image,
    # concatenated) and one gradient all-reduce (3 floats), once each
    for r in rs:
        assert list(r["coll_names"]) == ["film+W", "gradient"]
        assert list(r["coll_bytes"]) == [24 * 16 * 5 * 4, 12]
        assert list(r["coll_calls"]) == [1.0, 1.0] and np.all(r["coll_ms"] >= 0)
    r0, r1 = rs[0], rs[-1]
    for r in rs[1:]:
        assert np.array_equal(r0["img"], r["img"]) and np.array_equal(r0["g"], r["g"])
    # single process, all 8 samples per pixel
    scene = _scene(mi)
    img, grads = D.fwd_grad_step(_ops(mi, O, scene, torch), D.sample_slab(0, 1, 8), seed=7)
    np.testing.assert_allclose(r0["img"], img.numpy(), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(r0["g"], grads[0].numpy(), rtol=1e-5, atol=1e-9)
    # local W (no W all-reduce) + the film reduced onto rank 0 only: rank 0's
    # image and both ranks' gradients equal the single-process step
    np.testing.assert_allclose(r0["img2"], img.numpy(), rtol=2e-6, atol=1e-7)
    assert np.array_equal(r0["g2"], r1["g2"])
    np.testing.assert_allclose(r0["g2"], grads[0].numpy(), rtol=1e-5, atol=1e-9)
    # one packed film + W all-reduce: every rank's image and gradient equal the single-process step
    for r in rs:
        np.testing.assert_allclose(r["img3"], img.numpy(), rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(r["g3"], grads[0].numpy(), rtol=1e-5, atol=1e-9)
    # overlapped: W all-reduce, then film + gradient (4 + 16 B per pixel + 12 B) in one
    for r in rs:
        assert list(r["coll4_names"]) == ["W", "film+gradient"]
        assert list(r["coll4_bytes"]) == [24 * 16 * 4, 24 * 16 * 16 + 12]
        np.testing.assert_allclose(r["img4"], img.numpy(), rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(r["g4"], grads[0].numpy(), rtol=1e-5, atol=1e-9)


def test_pair_runner_runs_both_and_propagates_errors():
    import threading
    from mitsuba_hip import distributed as D
    run = D.PairRunner()
    names = []
    a, b = run(lambda: names.append(threading.current_thread().name) or 1,
               lambda: names.append(threading.current_thread().name) or 2)
    assert (a, b) == (1, 2) and len(set(names)) == 2  # the forward ran on the worker thread
    with pytest.raises(ZeroDivisionError):
        run(lambda: 1 // 0, lambda: 2)
    with pytest.raises(KeyError):
        run(lambda: 1, lambda: {}["x"])


def test_all_reduce_list_single_rank():
    import torch
    from mitsuba_hip import distributed as D
    ts = [torch.ones(3), torch.arange(4.0)]
    out = D.all_reduce_list_(ts)  # no process group: unchanged
    assert all(torch.equal(a, b) for a, b in zip(out, ts))
