#!/usr/bin/env python3
"""Config 3(b) alone: prb gradient wrt a 64^2 x 3 bitmap (512^2 @ 64 spp),
`--reps` timed calls after one warm-up (profiling target)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-nasa_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--tex-res", type=int, default=64, help="bitmap resolution (> 73: the global-atomic scatter)")
    a = ap.parse_args()
    import torch
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    sb = mi.load_dict(mi.cornell_box_bitmap(a.tex_res, 512, 512, 64))
    pb = mi.traverse(sb)
    prb = mi.load_dict({"type": "prb", "max_depth": 8})
    gi = torch.full((512, 512, 3), 1.0 / (512 * 512 * 3), dtype=torch.float32, device="cuda")
    sg = mi.sample_tea_32(0, 1)[0]
    f = lambda: mi.render_backward(sb, pb, gi, ["white.reflectance.data"], prb, seed=sg, spp=64, mode=a.mode)
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    print(json.dumps({"config": f"3(b) ({a.mode}, {a.tex_res}^2 x 3 bitmap)", "ms": round(dt * 1e3, 2),
                      "Msamples_s": round(512 * 512 * 64 / dt / 1e6, 1)}))


if __name__ == "__main__":
    main()
