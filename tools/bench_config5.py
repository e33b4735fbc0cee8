#!/usr/bin/env python3
"""Config 5 on one GPU's share: cornell_box 2048x2048 @ 1024 spp, forward +
PRB gradient, rank 0 of N (--ranks, default 8) sample slabs.

  forward  `path` (SamplingIntegrator::render): 2 passes of 512 spp
           (integrator.cpp:281-295); the rank renders lanes [0, 512/N) of
           every pass-pixel on the multi-pass wavefront
  gradient `prb` render_backward wrt white.reflectance.value: ONE AD wavefront
           of exactly 2^32 samples (common.py:571-578); the rank computes its
           W slab (all-reduced across ranks in bench.py's step) and the
           gradient of samples [0, 1024/N) of every pixel

Prints one JSON line per leg plus the fwd + grad total per rank.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-nasa_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--mega", action="store_true", help="also time the forward megakernel")
    a = ap.parse_args()
    import torch
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 2048
    scene = mi.load_dict(d)
    fwd = mi.load_dict({"type": "path", "max_depth": 8})
    prb = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    key = "white.reflectance.value"
    spp, passes = 1024, 2
    lanes = (spp // passes) // a.ranks  # lanes of each forward pass per rank
    slab = spp // a.ranks               # samples of the AD wavefront per pixel per rank
    n_rank = 2048 * 2048 * slab         # samples per rank (forward and gradient)
    gi = torch.full((2048, 2048, 3), 1.0 / (2048 * 2048 * 3), dtype=torch.float32, device="cuda")

    def timed(fn):
        best = 1e9
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    modes = ("wavefront", "mega") if a.mega else ("wavefront",)
    t_fwd = None
    for mode in modes:
        t = timed(lambda: mi.render_film(scene, fwd, seed=0, spp=spp, spp_begin=0, spp_end=lanes, mode=mode))
        t_fwd = t if t_fwd is None else t_fwd
        print(json.dumps({"config": f"5: path fwd 2048^2 @ 1024 (2 passes), one of {a.ranks} sample slabs",
                          "mode": mode, "Msamples_s": round(n_rank / t / 1e6, 1), "ms": round(t * 1e3, 1)}),
              flush=True)
    sg = mi.sample_tea_32(0, 1)[0]
    t_w = timed(lambda: mi.prb_weights(scene, sg, spp, 0, slab))
    w = mi.prb_weights(scene, sg, spp)
    t_g = timed(lambda: mi.render_backward(scene, params, gi, [key], prb, seed=sg, spp=spp, spp_begin=0,
                                           spp_end=slab, weights=w))
    print(json.dumps({"config": f"5: prb grad 2048^2 @ 1024 (one 2^32 AD wavefront), one of {a.ranks} slabs",
                      "ms_weights": round(t_w * 1e3, 1), "ms_backward": round(t_g * 1e3, 1),
                      "Msamples_s": round(n_rank / (t_w + t_g) / 1e6, 1)}), flush=True)
    tot = t_fwd + t_w + t_g
    print(json.dumps({"config": "5: fwd + grad per rank", "ms": round(tot * 1e3, 1),
                      "Msamples_s_per_rank": round(n_rank / tot / 1e6, 1),
                      "Msamples_s_8_ranks_ideal": round(a.ranks * n_rank / tot / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
