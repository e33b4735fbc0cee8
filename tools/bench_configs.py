#!/usr/bin/env python3
"""Per-configuration timings on one MI355X: config 2
forward (path 512^2 @ 256), config 3(a) PRB gradient wrt white's rgb
reflectance and 3(b) wrt a 64^2 bitmap (512^2 @ 64 spp), each as
Msamples/s of the timed call.  One JSON line per config."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd")]


def timeit(fn, steps=3):
    import torch
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    import torch
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 512
    scene = mi.load_dict(d)
    path = mi.load_dict({"type": "path", "max_depth": 8})
    prb = mi.load_dict({"type": "prb", "max_depth": 8})
    film = torch.empty((512, 512, 4), dtype=torch.float32, device="cuda")
    n = 512 * 512 * 256
    dt = timeit(lambda: mi.render_film(scene, path, seed=0, spp=256, film=film))
    print(json.dumps({"config": "2: path fwd 512^2 @ 256", "Msamples_s": round(n / dt / 1e6, 1),
                      "ms": round(dt * 1e3, 2)}), flush=True)
    gi = torch.full((512, 512, 3), 1.0 / (512 * 512 * 3), dtype=torch.float32, device="cuda")
    params = mi.traverse(scene)
    n = 512 * 512 * 64
    sg = mi.sample_tea_32(0, 1)[0]
    for mode in ("auto", "replay"):
        dt = timeit(lambda: mi.render_backward(scene, params, gi, ["white.reflectance.value"], prb, seed=sg,
                                               spp=64, mode=mode))
        print(json.dumps({"config": f"3(a): prb grad wrt white rgb, 512^2 @ 64 ({mode})",
                          "Msamples_s": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 2)}), flush=True)
    sb = mi.load_dict(mi.cornell_box_bitmap(64, 512, 512, 64))
    pb = mi.traverse(sb)
    for mode in ("auto", "replay"):
        dt = timeit(lambda: mi.render_backward(sb, pb, gi, ["white.reflectance.data"], prb, seed=sg, spp=64,
                                               mode=mode))
        print(json.dumps({"config": f"3(b): prb grad wrt white 64^2 bitmap, 512^2 @ 64 ({mode})",
                          "Msamples_s": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 2)}), flush=True)
    # render_forward (common.py:696-826): forward-mode gradient images
    tw = {"white.reflectance.value": torch.tensor([1.0, 0.5, 0.25], device="cuda")}
    dt = timeit(lambda: mi.render_forward(scene, params, tw, prb, seed=sg, spp=64))
    print(json.dumps({"config": "render_forward: prb wrt white rgb, 512^2 @ 64",
                      "Msamples_s": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 2)}), flush=True)
    tb = {"white.reflectance.data": torch.ones(tuple(pb["white.reflectance.data"].shape), device="cuda")}
    dt = timeit(lambda: mi.render_forward(sb, pb, tb, prb, seed=sg, spp=64))
    print(json.dumps({"config": "render_forward: prb wrt white 64^2 bitmap, 512^2 @ 64",
                      "Msamples_s": round(n / dt / 1e6, 1), "ms": round(dt * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
