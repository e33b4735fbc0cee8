#!/usr/bin/env python3
"""Host-side cost of one bench step (config 2): wall time of each StepOps call
with the device synchronised around it, against the call's own kernel time
(the HIP-event stats), and a cProfile of the Python layer over 5 steps.
Diagnostic only (not the bench line)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mitsuba3-nasa_amd")]


def main():
    import torch
    import bench
    from mitsuba_hip import distributed as D
    dev = torch.device("cuda:0")
    w = bench.build_step(512, 256, 8, 0, 1, dev)
    ops, slab = w["ops"], w["slab"]
    for s in range(3):
        D.fwd_grad_step(ops, slab, s, packed=True, fwd_slab=w["fwd_slab"])
    torch.cuda.synchronize()
    buf, fv, wv = ops.packed()
    sg = ops.seed_grad(7)

    def timed(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        print(f"{name:16s} {1e3 * (time.perf_counter() - t0):8.3f} ms wall", flush=True)
        return r
    for _ in range(2):
        timed("render_film", lambda: ops.render_film(7, 256, slab.begin, slab.end, out=fv))
        print(f"{'':16s} {w['st_f'].ms_kernel:8.3f} ms kernels (stats)")
        timed("prb_weights", lambda: ops.prb_weights(sg, 256, slab.begin, slab.end, out=wv))
        timed("develop", lambda: ops.develop(fv))
        timed("render_backward", lambda: ops.render_backward(sg, 256, slab.begin, slab.end, wv))
        print(f"{'':16s} {w['st_b'].ms_kernel:8.3f} ms kernels (stats)")
    pr = cProfile.Profile()
    pr.enable()
    for s in range(5):
        D.fwd_grad_step(ops, slab, s, packed=True, fwd_slab=w["fwd_slab"])
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(15)


if __name__ == "__main__":
    main()
