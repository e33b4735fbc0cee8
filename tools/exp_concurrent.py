#!/usr/bin/env python3
"""Experiment (round 6): the bench step's forward render and PRB backward are
independent (different seeds; the backward needs only the W image), so they
can run concurrently on two scene handles, two streams and two host threads
(the C-ABI calls release the GIL; concurrent handles on distinct scenes are
allowed, include/mitsuba_hip.h).  Prints the step time of cornell_box
512^2 @ 256 spp fwd + PRB grad (one MI355X): sequential; concurrent on two
streams; and four-way (each pass split into two sample slabs on four handles
and streams).  DESIGN.md §9 round 6 records the results (stream priorities
were measured with an earlier version of this script)."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd")]


def main():
    import torch
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    res, spp, steps = 512, 256, int(sys.argv[1]) if len(sys.argv) > 1 else 8
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = res
    sa, sb = mi.load_dict(d), mi.load_dict(d)
    fwd = mi.load_dict({"type": "path", "max_depth": 8})
    prb = mi.load_dict({"type": "prb", "max_depth": 8})
    key = "white.reflectance.value"
    pa, pb = mi.traverse(sa), mi.traverse(sb)
    gi = torch.full((res, res, 3), 1.0 / (res * res * 3), device="cuda")
    hi = torch.cuda.Stream.priority_range()[1]  # the highest priority
    pairs = {"": (torch.cuda.Stream(), torch.cuda.Stream()),
             "_bwd_hi": (torch.cuda.Stream(), torch.cuda.Stream(priority=hi)),
             "_fwd_hi": (torch.cuda.Stream(priority=hi), torch.cuda.Stream())}
    st_a, st_b = pairs[""]

    def fwd_call(scene, seed, stream):
        with torch.cuda.stream(stream):
            mi.render_film(scene, fwd, seed=seed, spp=spp)

    def bwd_call(scene, params, seed, w, stream):
        with torch.cuda.stream(stream):
            mi.render_backward(scene, params, gi, [key], prb, seed=seed, spp=spp, weights=w)

    def step_seq(i):
        sg = mi.sample_tea_32(i, 1)[0]
        fwd_call(sa, i, st_a)
        with torch.cuda.stream(st_a):
            w = mi.prb_weights(sa, sg, spp)
        bwd_call(sa, pa, sg, w, st_a)

    def step_conc(i, st_a=None, st_b=None):
        st_a, st_b = st_a or pairs[""][0], st_b or pairs[""][1]
        sg = mi.sample_tea_32(i, 1)[0]
        with torch.cuda.stream(st_b):
            w = mi.prb_weights(sb, sg, spp)
        t1 = threading.Thread(target=fwd_call, args=(sa, i, st_a))
        t2 = threading.Thread(target=bwd_call, args=(sb, pb, sg, w, st_b))
        t1.start(); t2.start(); t1.join(); t2.join()

    # 4-way: the forward and the gradient pass each split into two sample
    # slabs (the multi-GPU slab decomposition) on four handles and streams
    s4 = [mi.load_dict(d) for _ in range(4)]
    p4 = [mi.traverse(x) for x in s4]
    st4 = [torch.cuda.Stream() for _ in range(4)]
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(3)

    def step_4way(i):
        sg = mi.sample_tea_32(i, 1)[0]
        with torch.cuda.stream(st4[2]):
            w = mi.prb_weights(s4[2], sg, spp)
        torch.cuda.current_stream().synchronize()
        h = spp // 2

        def f(k):
            torch.cuda.set_device(0)
            with torch.cuda.stream(st4[k]):
                if k < 2:
                    mi.render_film(s4[k], fwd, seed=i, spp=spp, spp_begin=k * h, spp_end=(k + 1) * h)
                else:
                    b = (k - 2) * h
                    mi.render_backward(s4[k], p4[k], gi, [key], prb, seed=sg, spp=spp, spp_begin=b, spp_end=b + h,
                                       weights=w)
        futs = [pool.submit(f, k) for k in range(3)]
        f(3)
        for x in futs:
            x.result()

    out = {}
    runs = [("sequential", step_seq)]
    for r in range(2):
        runs.append((f"concurrent_{r}", step_conc))
        runs.append((f"four_way_{r}", step_4way))
    for name, fn in runs:
        for i in range(2):
            fn(1000 + i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            fn(i)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        out[name] = {"ms_per_step": round(ms, 3), "msamples_s": round(res * res * spp / ms / 1e3, 1)}
    # the gradients of both modes agree (same seeds; float atomics: order only)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
