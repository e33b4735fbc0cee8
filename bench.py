#!/usr/bin/env python3
"""bench.py — Msamples/s (pixels x spp / s), `path` forward + `prb` gradient,
cornell_box 512x512 @ 256 spp per GPU (BASELINE.json configs[1] + [2]).

One step = one forward `path` render (max_depth 8) of the rank's 256-spp
sample slab + the RCCL reduce of its RGBW film onto rank 0 + develop, then one PRB
render_backward (max_depth 8) w.r.t. 'white.reflectance.value' with
grad_in = d mean(image) = 1/(H*W*3): the rank's W-image slab is all-reduced,
its gradient slab computed and all-reduced.

Weak scaling: rank r renders samples [256 r, 256 r + 256) of every pixel of a
512x512 @ 256*N spp render (sample-slab sharding); value = N*512*512*256 /
max-over-ranks step time.  Inputs (the scene) are resident in HBM before the
timed region; the timed region ends with the image and gradients on the
device.

Per step two collectives (packed): the film and the W image (which depends
only on the gradient seed's jitters) are summed in ONE all-reduce, the
gradients in another (mitsuba_hip.distributed.fwd_grad_step).  Inside each
call the library runs the fused wavefront's chunks on two streams (mh_api.hip
fork_stream), so the kernel rooflines come from 2 steps with one stream
(MH_WF_STREAMS=1) right after the timed region -- a timed launch shares the
chip with the other chunk's (`roofline_timed`).  --overlap runs the forward
and the gradient pass of a step concurrently instead (two scene handles,
streams and host threads; valid here because grad_in = d mean(image) does
not depend on the image).

--config 5 is BASELINE.json configs[4]: cornell_box 2048x2048 @ 1024 spp
TOTAL (strong scaling: rank r takes samples [1024 r / N, 1024 (r + 1) / N) of
every pixel; the forward runs 2 passes of 512 spp, integrator.cpp:281-295, the
gradient one AD wavefront of 2^32 samples), max_depth 8, same JSON line.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|5]
       torchrun --nproc-per-node N bench.py --gpus N ...   (the driver)
       torchrun --nproc-per-node 8 bench.py --gpus 8 --config 5

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment is
a launcher: before any GPU call it starts `python -m torch.distributed.run
--nproc-per-node N ... bench.py <the same arguments>` as a child process
(rendezvous on 127.0.0.1), lets the ranks' output through (rank 0 prints the
line) and exits with the child's code.  Under a launcher every rank checks
that the process group's size equals --gpus; the line's `n_gpus` is the
process group's size.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd"), os.path.join(ROOT, "tests")]

# MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s (spec)
HBM_PEAK_GBS = 8000.0


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU; default: WORLD_SIZE, else 1). N > 1 without WORLD_SIZE launches "
                        "N ranks through torch.distributed.run")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--res", type=int, default=512)
    p.add_argument("--spp", type=int, default=256, help="samples per pixel per GPU")
    p.add_argument("--max-depth", type=int, default=8)
    p.add_argument("--cpu-seconds", type=float, default=24.0, help="budget of the CPU baseline (thread curve: 1, 4, all threads)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline (profiling runs)")
    p.add_argument("--fwd-only", action="store_true")
    p.add_argument("--local-weights", action="store_true",
                   help="every rank computes the whole W image (no W all-reduce; N x the W splat work)")
    p.add_argument("--film-all-reduce", action="store_true",
                   help="all-reduce the film to every rank instead of reducing it onto rank 0")
    p.add_argument("--config", type=int, default=2, choices=(1, 2, 3, 4, 5),
                   help="BASELINE.json configs[i-1]: 2 (default, the headline): 512^2 @ 256 spp per GPU fwd + PRB "
                        "grad, weak scaling; 5: 2048^2 @ 1024 spp total split over the ranks (strong scaling); "
                        "1: path 256^2 @ 16 (CPU leg: the scalar_rgb restatement); 3: prb gradient wrt a 64^2x3 "
                        "albedo bitmap, 512^2 @ 64; 4: volpath, 256^3 fBm medium + HG, 256^2 @ 64")
    p.add_argument("--unpacked", action="store_true",
                   help="serial step, separate film and W collectives (3 per step) instead of one packed film + W "
                        "all-reduce")
    p.add_argument("--overlap", action="store_true",
                   help="run the forward and the gradient pass of a step concurrently (two scene handles and "
                        "streams; W all-reduce first, film + gradient in one all-reduce after) instead of one after "
                        "the other")
    p.add_argument("--serial", action="store_true", help="(the default) forward, then gradient pass")
    p.add_argument("--backend", default="nccl",
                   help="torch.distributed backend for N > 1 ('nccl' = RCCL over xGMI; 'gloo' to rehearse "
                        "several ranks on one GPU)")
    return p.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(argv, gpus, env=None):
    """The child command that runs `gpus` ranks of this script (one process
    per GPU, torch.distributed.run on 127.0.0.1), or None when this process
    is itself a rank (WORLD_SIZE set) or a single-GPU run.  Makes no GPU call."""
    env = os.environ if env is None else env
    if gpus is None or gpus <= 1 or "WORLD_SIZE" in env:
        return None
    port = env.get("MASTER_PORT") or str(_free_port())
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def world_from(args, env=None):
    """(world, rank, local rank) of this process; a rank under a launcher
    must agree with --gpus."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE is {world}")
    return world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))


def cpu_info():
    """(model name, nproc, affinity) of the host this runs on."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    return model, os.cpu_count() or 1, aff


def cpu_threads():
    """Every core this process may run on, capped by OMP_NUM_THREADS where
    the host sets it (the GPU box: 16, its CPU share of a larger machine)."""
    _, _, aff = cpu_info()
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff
    return max(1, min(aff, cap))


def cpu_baseline(scene, fwd, prb, key, spp_gpu, budget_s, fwd_only):
    """CPU baseline: the oracle -- the
    CPU restatement of llvm_ad_rgb (scalar C, no SIMD), kind 'port' -- on the
    host's cores, on a bounded sample of the same workload: the same scene and
    integrators at a reduced spp.  A thread curve (1, 4 and all the threads
    this job may use): per point one warm-up run (the spp calibration), then
    the min of 2 timed runs sized to ~budget_s / 8 each.  `value` is the
    all-threads point; `per_core` and the linear extrapolation to every core
    of the host are derived from it and labelled as such."""
    import numpy as np
    import oracle_py as O
    threads = cpu_threads()
    model, nproc, aff = cpu_info()
    H, W = scene.height, scene.width
    gi = np.full((H, W, 3), 1.0 / (H * W * 3), np.float32)
    tex = [scene.params[key][1]]

    def run(spp, t):
        t0 = time.perf_counter()
        O.render(scene, fwd, seed=0, spp=spp, threads=t)
        if not fwd_only:
            O.render_backward(scene, prb, 1, spp, gi, tex, [(3,)], threads=t)
        return time.perf_counter() - t0

    curve = []
    for t in sorted({1, min(4, threads), threads}):
        t1 = run(1, t)  # warm-up + calibration
        spp = int(max(1, min(spp_gpu, budget_s / 8 / max(t1, 1e-3))))
        spp = 1 << max(0, spp.bit_length() - 1)
        best = min(run(spp, t) for _ in range(2)) if spp > 1 or t1 < budget_s / 8 else t1
        curve.append({"threads": t, "spp": spp, "seconds": round(best, 3),
                      "value": round(H * W * spp / best / 1e6, 4),
                      "per_core": round(H * W * spp / best / 1e6 / t, 4)})
    top = curve[-1]
    return {"value": top["value"], "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"cornell_box {W}x{H} @ {top['spp']} spp, path fwd" + ("" if fwd_only else " + prb grad")
                      + f" on {threads} threads; min of 2 runs after 1 warm-up, {top['seconds']:.2f} s each",
            "label": "CPU restatement of llvm_ad_rgb (oracle/libmh_oracle.so: scalar C, no SIMD)",
            "thread_curve": curve, "per_core": top["per_core"],
            "extrapolated_all_cores": {"value": round(top["per_core"] * nproc, 2), "cores": nproc,
                                       "label": "linear extrapolation of per_core to every host core "
                                                "(not measured: this job's CPU share is `cores`)"},
            "cpu_model": model, "nproc": nproc, "affinity": aff, "threads": threads}


def pmc_applies(args):
    """The committed PMC passes (tools/profile_r2.sh) profiled the default
    workload: config 2, 512^2 @ 256 spp per rank, max_depth 8.  Their per-launch
    counters describe launches of that workload only."""
    return args.config == 2 and args.res == 512 and args.spp == 256 and args.max_depth == 8


def _roof(kname, achieved_bytes, us, **extra):
    """A roofline object: algorithmic bytes of one launch over its average
    duration (HIP events over the timed region), against the HBM peak."""
    gbs = achieved_bytes / (us / 1e6) / 1e9 if us > 0 else 0.0
    r = {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kname, "kernel_avg_us": round(us, 1),
         "algorithmic_bytes_per_launch": round(achieved_bytes)}
    r.update(extra)
    return r


def splat_roof(st, n_px):
    """k_splat_tile of mh_render: 20 B per sample read (L 12 + position 8) and
    the RGBW film (16 B per pixel) written once per launch."""
    launches = max(1, st.n_aux_launches)
    us = st.ms_aux / launches * 1e3
    b = (20.0 * st.aux_items + 16.0 * n_px * launches) / launches
    return _roof("k_splat_tile<0>", b, us, launches_per_step=int(st.n_aux_launches), samples=int(st.aux_items),
                 bytes_formula="(20 samples + 16 pixels launches) / launches",
                 note="RGBW film L2/MALL-resident; the W image (PRB) rides in the same kernel family")


def bitmap_rooflines(st, n_samples, n_floats):
    """Config 3(b): the PRB bounce family with a bitmap parameter, and the
    texel scatter (k_wf_bitmap_scatter).  Bounce: per survivor the 100-B path
    state (pd 4, ray 28, beta 12, prev_p 12, prev_pdf 4, PCG32 state 8, TEA
    word 4, dL 12, running L 12, record mask 4) read and written; per sample
    the first bounce's grad/W texel (16 B) and the end record (L_total + mask,
    dL: 32 B); per bitmap vertex a 48-B record.  Scatter: per sample the end
    record (32 B, an upper bound: dL is read only for paths with records), per
    vertex record 48 B, and the texel gradients (4 B per float) once."""
    launches = max(1, st.n_trace_launches)
    R, N, V = float(st.rays_closest), float(n_samples), float(st.aux_items)
    b = (2.0 * 100 * (R - N) + (16.0 + 32.0) * N + 48.0 * V) / launches
    bounce = _roof("k_wf_bounce_prb", b, st.ms_trace / launches * 1e3, launches_per_step=int(st.n_trace_launches),
                   rays_closest=int(R), samples=int(N), bitmap_records=int(V), state_bytes=100, first_bytes=16,
                   end_bytes=32, record_bytes=48,
                   bytes_formula="(2 state (R - N) + (first + end) N + record V) / launches",
                   note="includes the Bm instance's vertex-record writes; ms from the bounce span (scatter excluded)")
    sl = max(1, st.n_aux_launches)
    sb = (32.0 * N + 48.0 * V) / sl + 4.0 * n_floats
    scat = _roof("k_wf_bitmap_scatter", sb, st.ms_aux / sl * 1e3, launches_per_step=int(st.n_aux_launches),
                 samples=int(N), bitmap_records=int(V), texel_floats=int(n_floats),
                 bytes_formula="(32 N + 48 V) / launches + 4 texel_floats",
                 note="accumulates in LDS (double); one global add per non-zero texel per workgroup")
    return bounce, scat


def volsched_roofline(st, n_samples, alpha=False):
    """Config 4: k_vol_sched.  Per device-counted density-grid lookup its 8
    float taps (32 B: GridVolume::eval's trilinear stencil), per sample the R G
    B (+ A) W record written (20 B; 24 with alpha).  The medium (64 MiB) is
    L2/MALL-resident in part, so counter traffic exceeds this figure: see
    profiles/ for the PMC passes."""
    launches = max(1, st.n_trace_launches)
    rec = 24.0 if alpha else 20.0
    b = (32.0 * st.grid_lookups + rec * n_samples) / launches
    return _roof("k_vol_sched<VolMachine>", b, st.ms_trace / launches * 1e3, launches_per_step=int(st.n_trace_launches),
                 grid_lookups=int(st.grid_lookups), lookups_per_sample=round(st.grid_lookups / max(1, n_samples), 3),
                 samples=int(n_samples), lookup_bytes=32, sample_bytes=int(rec),
                 bytes_formula="(32 lookups + 20 samples) / launches",
                 limiter="VALU issue and divergence of the phase machine (DESIGN.md section 3), not HBM")


def overlapped_roofline(timed, serial_roofs, ms_step, measured="the timed region: each launch shares the chip"):
    """`roofline_timed` of a bench line: the dominant kernel's figures from
    the timed steps (`timed`, a roofline dict of the same kernel, each launch
    sharing the chip with the other chunk's or pass's), and chip_*: both
    bounce families' algorithmic bytes per step (launches x bytes per launch
    of the one-stream rooflines) over the step time, one rank's bytes over its
    own step."""
    chip = sum(r["algorithmic_bytes_per_launch"] * r["launches_per_step"] for r in serial_roofs if r)
    gbs = chip / (ms_step / 1e3) / 1e9
    out = {k: timed[k] for k in ("kernel", "achieved", "frac", "kernel_avg_us", "launches_per_step",
                                 "algorithmic_bytes_per_launch")}
    out.update(measured=measured,
               chip_bounce_bytes_per_step=round(chip), chip_achieved=round(gbs, 1),
               chip_frac=round(gbs / HBM_PEAK_GBS, 4))
    return out


def build_step(res, spp, max_depth, rank, world, dev, fwd_passes=1):
    """The bench's hot-path wiring (also driven by tests/test_gpu_multirank.py):
    cornell_box res^2, `path` forward + `prb` backward wrt white's rgb
    reflectance, the rank's sample slab of a spp * world render, through the
    HIP C-ABI wrappers of mitsuba_hip.  fwd_passes: the forward's passes
    (integrator.cpp:281-295; its slab counts lanes of one pass).  One device
    buffer holds the film and the W image (StepOps.packed).  The forward
    renders through its own handle of the scene (scene_fwd: the same scene
    description, its own device copy, scratch and stream), so that the
    overlapped step (StepOps.concurrent) can run it alongside the gradient
    pass."""
    import torch
    import mitsuba_hip as mi
    from mitsuba_hip import _abi as A
    from mitsuba_hip import distributed as D
    mi.set_variant("hip_ad_rgb")
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = res
    d["sensor"]["film"]["height"] = res
    scene = mi.load_dict(d)
    scene_fwd = mi.load_dict(d)
    fwd = mi.load_dict({"type": "path", "max_depth": max_depth})
    prb = mi.load_dict({"type": "prb", "max_depth": max_depth})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    grad_in = torch.full((res, res, 3), 1.0 / (res * res * 3), dtype=torch.float32, device=dev)
    st_f, st_b = A.Stats(), A.Stats()
    film = torch.empty((res, res, 4), dtype=torch.float32, device=dev)
    packed = torch.empty(res * res * 5, dtype=torch.float32, device=dev)  # film (RGBW) | W image
    views = (packed, packed[:res * res * 4].view(res, res, 4), packed[res * res * 4:].view(res, res))
    ops = D.StepOps(
        render_film=lambda seed, spp_, b, e, out=None, shared=False: mi.render_film(
            scene_fwd, fwd, seed=seed, spp=spp_, spp_begin=b, spp_end=e, film=film if out is None else out,
            stats=st_f, shared=shared),
        develop=lambda f: mi.develop(scene, f),
        prb_weights=lambda seed, spp_, b, e, out=None: mi.prb_weights(scene, seed, spp_, b, e, out=out),
        render_backward=lambda seed, spp_, b, e, w, shared=False: mi.render_backward(
            scene, params, grad_in, [key], prb, seed=seed, spp=spp_, spp_begin=b, spp_end=e, weights=w,
            stats=st_b, shared=shared),
        seed_grad=lambda seed: mi.sample_tea_32(seed, 1)[0],
        packed=lambda: views,
        concurrent=D.PairRunner((torch.cuda.Stream(dev), torch.cuda.Stream(dev)), dev), shared_hint=True)
    slab = D.sample_slab(rank, world, spp)
    fs = D.sample_slab(rank, world, spp // fwd_passes)
    fwd_slab = D.Slab(slab.spp_total, fs.begin, fs.end)
    return {"scene": scene, "fwd": fwd, "prb": prb, "key": key, "ops": ops,
            "slab": slab, "fwd_slab": fwd_slab, "st_f": st_f, "st_b": st_b}


def single_op(args, rank, world, dev):
    """BASELINE configs 1, 3 and 4 as one-op steps on the rank's sample slab
    (weak scaling; the film or gradient summed over the ranks): 1 = `path`
    256^2 @ 16 (its CPU leg the scalar_rgb restatement, oracle_render_scalar),
    3 = `prb` render_backward wrt a 64^2 x 3 albedo bitmap, 512^2 @ 64,
    4 = `volpath` on the 256^3 fBm medium + HG, 256^2 @ 64."""
    import torch
    import mitsuba_hip as mi
    from mitsuba_hip import _abi as A
    from mitsuba_hip import distributed as D
    mi.set_variant("hip_ad_rgb")
    st = A.Stats()
    c = args.config
    if c == 1:
        res, spp = 256, 16
        d = mi.cornell_box()
        d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = res
        scene = mi.load_dict(d)
        integ = mi.load_dict({"type": "path", "max_depth": args.max_depth})
        work = f"config 1: cornell_box {res}x{res} @ {spp} spp/GPU, path fwd (max_depth {args.max_depth})"
    elif c == 3:
        res, spp = 512, 64
        scene = mi.load_dict(mi.cornell_box_bitmap(64, res, res, spp))
        integ = mi.load_dict({"type": "prb", "max_depth": args.max_depth})
        params = mi.traverse(scene)
        key = "white.reflectance.data"
        grad_in = torch.full((res, res, 3), 1.0 / (res * res * 3), dtype=torch.float32, device=dev)
        work = (f"config 3: cornell_box {res}x{res} @ {spp} spp/GPU, prb render_backward (max_depth "
                f"{args.max_depth}) wrt '{key}' (64x64x3 bitmap)")
    else:
        res, spp = 256, 64
        scene = mi.load_dict(mi.volume_cube(res, res, spp, grid=mi.fbm_grid(256)))
        integ = scene.integrator()
        work = f"config 4: volpath, 256^3 fBm heterogeneous medium + HG, {res}x{res} @ {spp} spp/GPU"
    slab = D.sample_slab(rank, world, spp)

    def step(i):
        if c == 3:
            (g,) = mi.render_backward(scene, params, grad_in, [key], integ, seed=i, spp=slab.spp_total,
                                      spp_begin=slab.begin, spp_end=slab.end, stats=st)
            return D.all_reduce_(g)
        return D.all_reduce_(mi.render_film(scene, integ, seed=i, spp=slab.spp_total, spp_begin=slab.begin,
                                            spp_end=slab.end, stats=st))

    return scene, integ, res, spp, work, step, st


def cpu_single_op(args, scene, integ, res, spp):
    """The CPU leg of configs 1 / 3 / 4 (rank 0, N = 1): the oracle on all the
    job's threads at a bounded spp (config 1: the scalar_rgb restatement)."""
    import numpy as np
    import oracle_py as O
    threads = cpu_threads()
    model, nproc, aff = cpu_info()
    c = args.config
    params = None

    def run(s):
        t0 = time.perf_counter()
        if c == 1:
            O.render_scalar(scene, integ, seed=0, spp=s, threads=threads)
        elif c == 3:
            gi = np.full((res, res, 3), 1.0 / (res * res * 3), np.float32)
            O.render_backward(scene, integ, 1, s, gi, [scene.params["white.reflectance.data"][1]],
                              [(64, 64, 3)], threads=threads)
        else:
            O.render(scene, integ, seed=0, spp=s, threads=threads)
        return time.perf_counter() - t0

    t1 = run(1)
    s = int(max(1, min(spp, args.cpu_seconds / 4 / max(t1, 1e-3))))
    s = 1 << max(0, s.bit_length() - 1)
    best = min(run(s) for _ in range(2)) if s > 1 else t1
    kind = "scalar_rgb restatement (oracle_render_scalar)" if c == 1 else "CPU restatement of llvm_ad_rgb"
    return {"value": round(res * res * s / best / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{res}x{res} @ {s} spp on {threads} threads; min of 2 runs after 1 warm-up, {best:.2f} s each",
            "label": f"{kind} (oracle/libmh_oracle.so: scalar C, no SIMD)", "cpu_model": model, "nproc": nproc,
            "affinity": aff, "threads": threads}


def main():
    args = parse()
    cmd = launch_command(sys.argv[1:], args.gpus)
    if cmd is not None:  # the launcher: no GPU call in this process, the ranks are its child
        import subprocess
        raise SystemExit(subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1")))
    world, rank, local = world_from(args)
    import torch
    import torch.distributed as dist
    dist_on = world > 1
    # one process per GPU; with fewer GPUs than ranks (gloo rehearsal) ranks share devices
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(args.backend)
        world = dist.get_world_size()  # n_gpus comes from the process group, not from a flag
        if args.gpus is not None and world != args.gpus:
            raise SystemExit(f"bench.py: process group has {world} ranks, --gpus {args.gpus}")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    from mitsuba_hip import _abi as A
    from mitsuba_hip import distributed as D
    if args.config in (1, 3, 4):
        return main_single_op(args, rank, world, dev, dist_on)
    if args.config == 5:  # BASELINE.json configs[4]: 2048^2 @ 1024 spp in total, strong scaling
        if 512 % world:
            raise SystemExit("--config 5 needs a rank count that divides 512")
        args.res, args.spp, fwd_passes = 2048, 1024 // world, 2
    else:
        fwd_passes = 1
    w = build_step(args.res, args.spp, args.max_depth, rank, world, dev, fwd_passes)
    scene, fwd, prb, key, ops, slab, fwd_slab, st_f, st_b = (
        w[k] for k in ("scene", "fwd", "prb", "key", "ops", "slab", "fwd_slab", "st_f", "st_b"))
    H = W = args.res
    spp_total = args.spp * world
    overlap = args.overlap and not (args.unpacked or args.fwd_only)
    packed = not (overlap or args.unpacked or args.local_weights or args.fwd_only)

    def step(i):
        return D.fwd_grad_step(ops, slab, i, with_grad=not args.fwd_only, local_weights=args.local_weights,
                               film_to_root=not args.film_all_reduce, packed=packed, fwd_slab=fwd_slab,
                               overlap=overlap)

    for i in range(args.warmup):
        step(1000 + i)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    # N > 1: the collectives are timed (HIP events around each) so that a
    # scaling result splits into collective time, rank imbalance and the rest
    timer = D.CollTimer() if dist_on else None
    D.set_collective_timer(timer)
    fwd_ms, bwd_ms = [], []
    t0 = time.perf_counter()
    for i in range(args.steps):
        img, g = step(i)
        fwd_ms.append(st_f.ms_kernel)
        bwd_ms.append(st_b.ms_kernel)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed_local = time.perf_counter() - t0
    D.set_collective_timer(None)
    elapsed = D.max_over_ranks(elapsed_local, dev)
    ms_step = elapsed / args.steps * 1e3
    multi = None
    if dist_on:
        # the barrier-bracketed time above is the same on every rank; a rank's
        # own work is its step time without the final barrier wait, so the
        # spread comes from its kernel time (fwd + bwd, HIP events) + collectives
        colls = timer.summary(args.steps)
        cms = {k: c["ms_per_step"] for k, c in colls.items()}
        if overlap:  # W and its all-reduce, then the forward alongside the backward
            own = (cms.get("W", 0.0) + max(sum(fwd_ms) / args.steps, sum(bwd_ms) / args.steps) +
                   cms.get("film+gradient", 0.0))
        else:
            own = (sum(fwd_ms) + sum(bwd_ms)) / args.steps + sum(cms.values())
        coll_max = {k: round(D.max_over_ranks(v["ms_per_step"], dev), 3) for k, v in sorted(colls.items())}
        multi = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                 "rank_kernel_plus_collective_ms_min": round(D.min_over_ranks(own, dev), 3),
                 "rank_kernel_plus_collective_ms_max": round(D.max_over_ranks(own, dev), 3),
                 "collective_ms_per_step_max_over_ranks": coll_max,
                 "collective_bytes": {k: v["bytes"] for k, v in sorted(colls.items())},
                 "collective_calls_per_step": {k: round(v["calls_per_step"], 2) for k, v in sorted(colls.items())}}
    samples_step = world * H * W * args.spp
    value = samples_step / (ms_step / 1e3) / 1e6
    # in the timed steps a bounce launch shares the chip with the other
    # chunk's launches (the library's two chunk streams) or with the other
    # pass's (--overlap) for most of its duration: its HIP-event time there is
    # not the kernel's own.  The kernel rooflines come from a roofline pass of
    # 2 serial steps with one stream (MH_WF_STREAMS=1) right after the timed
    # region (same workload, each launch alone on the chip; the timed region's
    # figures are reported beside them as roofline_timed)
    st_f_timed, st_b_timed = A.Stats.from_buffer_copy(st_f), A.Stats.from_buffer_copy(st_b)
    fs_ms, bs_ms = [], []
    old_streams = os.environ.get("MH_WF_STREAMS")
    os.environ["MH_WF_STREAMS"] = "1"
    try:
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for i in range(2):
            D.fwd_grad_step(ops, slab, 2000 + i, with_grad=not args.fwd_only, local_weights=args.local_weights,
                            film_to_root=not args.film_all_reduce, packed=not (args.local_weights or args.fwd_only),
                            fwd_slab=fwd_slab)
            fs_ms.append(st_f.ms_kernel)
            bs_ms.append(st_b.ms_kernel)
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        s_ms = D.max_over_ranks(time.perf_counter() - t1, dev) / 2 * 1e3
    finally:
        if old_streams is None:
            os.environ.pop("MH_WF_STREAMS", None)
        else:
            os.environ["MH_WF_STREAMS"] = old_streams
    fwd_ms_serial, bwd_ms_serial = sum(fs_ms) / 2, sum(bs_ms) / 2
    serial = {"ms_per_step": round(s_ms, 3), "value": round(samples_step / (s_ms / 1e3) / 1e6, 2), "steps": 2,
              "note": "the roofline pass: the same work as a serial step with one stream per call "
                      "(MH_WF_STREAMS=1: no chunk pipelining, no forward || gradient overlap)"}

    if rank == 0:
        # ---- rooflines of the two bounce-kernel families, the dominant one as
        # `roofline`.  One launch = one bounce of every live path
        # of a 2^25-path chunk (closest trace + shading + NEE visibility).
        # mh_render / mh_render_backward time the bounce launches with HIP
        # events on the scene's stream (stats.ms_trace / n_trace_launches).
        # Algorithmic bytes: the path state streamed per path-bounce (the BVH,
        # pair records and shading tables are LDS / scalar-cache resident):
        #   k_wf_bounce      84 B state (pd 4, ray 28, throughput 12, prev_p 12,
        #                    prev_pdf 4, PCG32 state 8 + TEA word 4, L 12) read by every non-first
        #                    bounce and written by every survivor; a finished
        #                    path writes L (12 B); the first bounce writes the
        #                    film position (8 B) of every sample
        #   k_wf_bounce_prb  108 B (the same without L, + dL 12 + A_s 12) read and
        #                    written alike; the first bounce reads the sample's
        #                    grad / W texel (16 B)
        # with R = rays (sum of queue lengths), N = samples: survivors R - N.
        # traffic / VALU issue from the PMC passes of the latest profiles/rN_pmc.json
        # (tools/profile_r2.sh: FETCH/WRITE corrected by the calib_fetch factors
        # for the kernel's access width; VALU issue = SQ_INSTS_VALU x 2 cycles /
        # (1024 SIMDs x launch time x measured clock)).
        avg_f = sum(fwd_ms) / len(fwd_ms)
        avg_b = (sum(bwd_ms) / len(bwd_ms)) if not args.fwd_only else 0.0
        n_local = H * W * args.spp
        pmc = {}
        # tools/profile_r2.sh of the latest round's build.  These counters are
        # NOT measured in this run: the line names the file and the build they
        # come from (traffic_source)
        ppath = next((q for q in (os.path.join(ROOT, "profiles", f"r{r}_pmc.json") for r in (6, 5, 4, 3, 2))
                      if os.path.exists(q)), "")
        traffic_source = None
        if os.path.exists(ppath):
            try:
                pj = json.load(open(ppath))
                pmc = pj.get("kernels", {})
                traffic_source = (os.path.relpath(ppath, ROOT) + " @ " +
                                  pj.get("source", "the build committed with that file") +
                                  " (PMC passes of tools/profile_r2.sh; traffic, valu_issue_frac and clock_ghz are not measured in this run)")
            except Exception:
                pmc = {}

        # the PMC passes profiled the default workload (config 2: 512^2 @ 256 spp
        # per rank, max_depth 8); a launch of another workload (config 5's
        # chunks, another res / spp / depth) does different work per launch, so
        # its counters are not this launch's: omitted, with a note
        applies = pmc_applies(args)
        pmc_note = (None if applies else
                    "traffic / valu_issue_frac omitted: the committed PMC passes profiled config 2's launches "
                    "(512^2 @ 256 spp, max_depth 8), not this workload's")

        def family(kname):
            if not applies:
                return None, None, None
            fam = [v for k, v in pmc.items() if k.startswith(kname + "<") and
                   not (kname == "k_wf_bounce" and k.startswith("k_wf_bounce_prb"))]
            calls = sum(v["calls"] for v in fam)
            if not calls:
                return None, None, None
            mean = lambda f: sum(v["calls"] * v[f] for v in fam if v.get(f) is not None) / calls
            return round(mean("hbm_bytes_per_call")), mean("valu_insts_per_call"), mean("clock_ghz")

        def roof(kname, st, state_b, per_death, per_sample):
            launches = max(1, st.n_trace_launches)
            us = st.ms_trace / launches * 1e3
            R, N = float(st.rays_closest), float(n_local)
            bytes_launch = (2.0 * state_b * (R - N) + per_death * N + per_sample * N) / launches
            achieved = bytes_launch / (us / 1e6) / 1e9
            traffic, valu, clk = family(kname)
            r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                 "traffic_source": traffic_source if traffic is not None else None, "kernel": kname,
                 "kernel_avg_us": round(us, 1), "algorithmic_bytes_per_launch": round(bytes_launch),
                 # everything the bytes come from, so the line alone reproduces them:
                 # bytes = (2 S (R - N) + b_end N + b_first N) / launches
                 "launches_per_step": launches, "rays_closest": int(R), "samples": int(N),
                 "state_bytes": state_b, "end_bytes": per_death, "first_bytes": per_sample}
            if pmc_note:
                r["traffic_note"] = pmc_note
            if valu and clk:
                r["valu_issue_frac"] = round(valu * 2.0 / (1024 * us * 1e-6 * clk * 1e9), 4)
                r["valu_insts_per_launch"] = round(valu)
                r["clock_ghz"] = round(clk, 3)
                r["limiter"] = ("VALU issue + latency of the packet primitive tests, not HBM: "
                                f"valu_issue_frac {r['valu_issue_frac']} vs hbm frac {r['frac']}")
            return r

        roofs = []
        if st_f.mode == 2:
            roofs.append((st_f.ms_trace, roof("k_wf_bounce", st_f, 84.0, 12.0, 8.0)))
        if not args.fwd_only and st_b.mode == 1 and st_b.n_trace_launches:
            roofs.append((st_b.ms_trace, roof("k_wf_bounce_prb", st_b, 108.0, 0.0, 16.0)))
        roofs.sort(key=lambda x: -x[0])
        roofline = roofs[0][1] if roofs else None
        roofline_other = roofs[1][1] if len(roofs) > 1 else None
        roofline_timed = None
        if roofline is not None:
            for r in (roofline, roofline_other):
                if r:
                    r["measured"] = ("roofline pass: 2 serial steps with one stream per call (MH_WF_STREAMS=1) "
                                     "right after the timed region, each launch alone on the chip; HIP events on "
                                     "the kernel's stream")
            # the timed steps: the same kind of launches sharing the chip with
            # the other chunk's (two chunk streams) or pass's (--overlap).
            # chip_*: both bounce families' algorithmic bytes of a step / the
            # step time (what the chip moved for them)
            sts = {"k_wf_bounce": (st_f_timed, 84.0, 12.0, 8.0), "k_wf_bounce_prb": (st_b_timed, 108.0, 0.0, 16.0)}
            roofline_timed = overlapped_roofline(
                roof(roofline["kernel"], *sts[roofline["kernel"]]), (roofline, roofline_other), ms_step,
                "the timed region: " + ("forward || gradient pass" if overlap else "each call's chunks on two streams")
                + ", each launch sharing the chip")
        # the forward's film splat (k_splat_tile): per sample its L (12 B) and
        # film position (8 B) read, per launch the RGBW film (16 B per pixel)
        # added once; timed by HIP events after the bounce span of each chunk
        roofline_splat = splat_roof(st_f, H * W) if st_f.n_aux_launches else None
        cpu = None
        if not args.no_cpu and world == 1:  # the CPU leg: rank 0 at N = 1 only
            cscene = scene
            if args.res > 512:  # a bounded sample: the same scene at 512^2 (per-sample work is resolution-free)
                import mitsuba_hip as mi
                d = mi.cornell_box()
                d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 512
                cscene = mi.load_dict(d)
            cpu = cpu_baseline(cscene, fwd, prb, key, args.spp, args.cpu_seconds, args.fwd_only)
        coll = ("RCCL" if args.backend == "nccl" else args.backend)
        if overlap:
            par = (f"sample-slab x{world}; forward || gradient pass (two scene handles, two HIP streams); {coll}" +
                   (" local W" if args.local_weights else " all-reduce (W)") +
                   " + all-reduce (film + gradient, one buffer)")
        elif packed:
            par = f"sample-slab x{world} + {coll} all-reduce (film + W, one packed buffer) + all-reduce (gradient)"
        else:
            par = (f"sample-slab x{world} + {coll}" +
                   (" all-reduce (film)" if args.film_all_reduce else " reduce to rank 0 (film)") +
                   (", local W" if args.local_weights else ", all-reduce (W)") + ", all-reduce (gradient)")
        cfg5 = args.config == 5
        line = {
            "metric": "Msamples/s (pixels×spp/s) fwd + PRB grad, cornell_box 512²; 1/2/4/8 GPU",
            "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong" if cfg5 else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (cornell_box scene, seeded PCG32)",
            "config": {"workload": (f"config 5: cornell_box {W}x{H} @ {spp_total} spp total ({args.spp}/GPU; "
                                    f"forward in 2 passes): path fwd (max_depth {args.max_depth})" if cfg5 else
                                    f"cornell_box {W}x{H} @ {args.spp} spp/GPU: path fwd (max_depth {args.max_depth})")
                                   + ("" if args.fwd_only else f" + prb backward wrt '{key}'"),
                       "film": f"{W}x{H}", "spp_per_gpu": args.spp, "spp_total": spp_total,
                       "parallelism": par,
                       "step": ("overlapped: forward || gradient pass" if overlap else
                                "serial: forward, then gradient pass; each call's fused-wavefront chunks on two "
                                "streams (mh_api.hip fork_stream)"),
                       "collectives_per_step": ((1 if args.local_weights else 2) if overlap else
                                                2 if packed else (1 if args.fwd_only else (2 if args.local_weights else 3))),
                       "collective_bytes": (dict(({} if args.local_weights else {"W": H * W * 4}),
                                                 **{"film+gradient": H * W * 16 + 12}) if overlap else
                                            {"film+W": H * W * 20, "gradient": 12} if packed else
                                            {"film": H * W * 16, "W": 0 if args.local_weights else H * W * 4,
                                             "gradient": 12})},
            "fwd_kernel_ms": round(avg_f, 3), "bwd_kernel_ms": round(avg_b, 3),
            "fwd_kernel_ms_one_stream": round(fwd_ms_serial, 3),
            "bwd_kernel_ms_one_stream": round(bwd_ms_serial, 3) if not args.fwd_only else None,
            "rays_closest_per_sample": round(st_f.rays_closest / max(1, n_local), 4),
            "rays_shadow_per_sample": round(st_f.rays_shadow / max(1, n_local), 4),
            "rays_closest_per_sample_prb": (round(st_b.rays_closest / max(1, n_local), 4)
                                            if not args.fwd_only else None),
            "rays_shadow_per_sample_prb": (round(st_b.rays_shadow / max(1, n_local), 4)
                                           if not args.fwd_only else None),
            "roofline": roofline, "roofline_other": roofline_other, "roofline_splat": roofline_splat,
            "roofline_timed": roofline_timed, "one_stream_step": serial,
            "cpu_baseline": cpu,
        }
        if multi is not None:
            line["multi_gpu"] = multi
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


def main_single_op(args, rank, world, dev, dist_on):
    import torch
    import torch.distributed as dist
    from mitsuba_hip import _abi as A
    from mitsuba_hip import distributed as D
    scene, integ, res, spp, work, step, st = single_op(args, rank, world, dev)
    for i in range(args.warmup):
        step(1000 + i)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
        kms.append(st.ms_kernel)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = D.max_over_ranks(time.perf_counter() - t0, dev)
    ms_step = elapsed / args.steps * 1e3
    value = world * res * res * spp / (ms_step / 1e3) / 1e6
    # configs 1 / 3: the fused wavefront runs the call's two chunks on two
    # streams (mh_api.hip fork_stream), so a timed launch shares the chip with
    # the other chunk's; the rooflines come from 2 one-stream steps
    # (MH_WF_STREAMS=1) right after the timed region, the timed figures sit
    # beside them (roofline_two_streams)
    st_timed = A.Stats.from_buffer_copy(st)
    if args.config in (1, 3):
        old = os.environ.get("MH_WF_STREAMS")
        os.environ["MH_WF_STREAMS"] = "1"
        try:
            for i in range(2):
                step(3000 + i)
            torch.cuda.synchronize()
        finally:
            if old is None:
                os.environ.pop("MH_WF_STREAMS", None)
            else:
                os.environ["MH_WF_STREAMS"] = old
    if rank == 0:
        n_local = res * res * spp
        roof = roof_other = two = None
        if args.config == 3 and st.n_aux_launches:
            roof, roof_other = bitmap_rooflines(st, n_local, 64 * 64 * 3)  # config 3(b): a 64^2 x 3 bitmap
            note = "one-stream pass: 2 steps with MH_WF_STREAMS=1 right after the timed region"
            roof["measured"] = roof_other["measured"] = note
            if st_timed.n_aux_launches > st.n_aux_launches:  # the timed steps ran the two-stream pipeline
                tb, ts = bitmap_rooflines(st_timed, n_local, 64 * 64 * 3)
                two = {"measured": "the timed region: the two chunks on two streams, each launch sharing the chip",
                       "kernels": [{k: r[k] for k in ("kernel", "achieved", "frac", "kernel_avg_us",
                                                      "launches_per_step")} for r in (tb, ts)]}
        elif args.config == 4 and st.mode == 3 and st.n_trace_launches:
            roof = volsched_roofline(st, n_local)
            # config 4's own PMC passes (tools/profile_volsched.sh): traffic and
            # VALU issue of the same launch shape (one k_vol_sched per render)
            pc = os.path.join(ROOT, "profiles", "r6_pmc_config4.json")
            if os.path.exists(pc):
                pj = json.load(open(pc))
                k = next((v for n_, v in pj.get("kernels", {}).items() if n_.startswith("k_vol_sched<VolMachine")), None)
                if k:
                    roof["traffic"] = round(k["hbm_bytes_per_call"])
                    roof["valu_issue_frac"] = round(k["valu_issue_frac"], 4)
                    roof["traffic_source"] = ("profiles/r6_pmc_config4.json @ " + pj.get("source", "") +
                                              " (not measured in this run)")
        elif args.config == 1 and st.mode == 2:
            def c1_roofs(s):
                launches = max(1, s.n_trace_launches)
                R, N = float(s.rays_closest), float(n_local)
                return (_roof("k_wf_bounce", (2.0 * 84 * (R - N) + 20.0 * N) / launches, s.ms_trace / launches * 1e3,
                              launches_per_step=int(s.n_trace_launches), rays_closest=int(R), samples=int(N),
                              state_bytes=84, end_bytes=12, first_bytes=8,
                              bytes_formula="(2 state (R - N) + (end + first) N) / launches"),
                        splat_roof(s, res * res))
            roof, roof_other = c1_roofs(st)
            note = "one-stream pass: 2 steps with MH_WF_STREAMS=1 right after the timed region"
            roof["measured"] = roof_other["measured"] = note
            if st_timed.n_aux_launches > st.n_aux_launches:  # the timed steps ran the two-stream pipeline
                tb, ts = c1_roofs(st_timed)
                two = {"measured": "the timed region: the two chunks on two streams, each launch sharing the chip",
                       "kernels": [{k: r[k] for k in ("kernel", "achieved", "frac", "kernel_avg_us",
                                                      "launches_per_step")} for r in (tb, ts)]}
        cpu = None if (args.no_cpu or world > 1) else cpu_single_op(args, scene, integ, res, spp)
        names = {1: "path fwd", 3: "PRB grad (bitmap albedo)", 4: "volpath fwd"}
        line = {
            "metric": f"Msamples/s (pixels×spp/s) {names[args.config]}, BASELINE config {args.config}",
            "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded PCG32; procedural fBm grid for config 4)",
            "config": {"workload": work, "film": f"{res}x{res}", "spp_per_gpu": spp, "spp_total": spp * world,
                       "parallelism": f"sample-slab x{world}" + (" + all-reduce" if world > 1 else "")},
            "kernel_ms": round(sum(kms) / len(kms), 3),
            "rays_closest_per_sample": round(st.rays_closest / max(1, res * res * spp), 4),
            "rays_shadow_per_sample": round(st.rays_shadow / max(1, res * res * spp), 4),
            "roofline": roof, "roofline_other": roof_other,
            "cpu_baseline": cpu,
        }
        if two:
            line["roofline_two_streams"] = two
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
