#!/usr/bin/env python3
"""Large-mesh traversal roofline from tools/profile_mesh.sh output dirs
(pmc.json of tools/make_pmc.py + bench.txt): per stream-engine kernel the
launches, average duration, rays per launch, Grays/s, the algorithmic HBM
rate (48 B per closest ray = 28-B ray in + 20-B hit out,
32 B per shadow ray = 28-B ray + 4-B id) as a fraction of the 8 TB/s peak,
the counter bytes per ray (FETCH_SIZE x2 + WRITE_SIZE, calibrated), L2 hit
rate, wait_any and VALU issue.  usage: mesh_roofline.py <dir> [<dir> ...]"""
import json
import os
import sys

PEAK = 8000.0
ALG = {"k_wf_trace": 48.0, "k_wf_shadow": 32.0}


def main():
    for d in sys.argv[1:]:
        pmc = json.load(open(os.path.join(d, "pmc.json")))["kernels"]
        b = [json.loads(l) for l in open(os.path.join(d, "bench.txt")) if l.startswith("{")][-1]
        print(f"{b['triangles']:,} triangles, BVH {b['bvh_mb']} MB: {b['msamples_s']} Msamples/s, "
              f"{b['ms_per_render']} ms per render (path 512^2 @ 64, max_depth 8)")
        for k, rec in sorted(pmc.items()):
            fam = next((f for f in ALG if k.startswith(f + "<")), None)
            if not fam:
                continue
            rays = b["rays_closest"] if fam == "k_wf_trace" else b["rays_shadow"]
            per = rays / rec["calls"]
            us = rec["avg_us"]
            alg = ALG[fam] * per / (us * 1e-6) / 1e9
            hb = rec.get("hbm_bytes_per_call")
            print(f"  {k:28s} launches {rec['calls']:2d}  avg {us:8.1f} us  rays/launch {per / 1e6:5.2f} M  "
                  f"{per / us / 1e3:5.2f} Grays/s  alg {alg:6.1f} GB/s = {alg / PEAK:.4f}  "
                  f"counter {hb / per if hb else 0:5.0f} B/ray  {hb / (us * 1e-6) / 1e9 if hb else 0:6.1f} GB/s = "
                  f"{(hb / (us * 1e-6) / 1e9 / PEAK) if hb else 0:.3f}  L2 hit {rec.get('l2_hit') or 0:.2f}  "
                  f"wait_any {rec.get('wait_any') or 0:.2f}  VALU issue {rec.get('valu_issue_frac') or 0:.3f}")


if __name__ == "__main__":
    main()
