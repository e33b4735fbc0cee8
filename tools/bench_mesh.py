#!/usr/bin/env python3
"""Large-mesh measurement (meshes make the BVH
HBM/L2-resident).  A procedural displaced sphere of ~N triangles (written to
and loaded from a binary PLY, i.e. the ply plugin path) sits in the cornell
box; `path` renders it on one MI355X.  Prints one JSON line per N: scene
load / BVH build time, BVH size, forward Msamples/s and closest + shadow
Grays/s.  Not the driver's bench line (bench.py measures BASELINE.json's)."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd")]


def sphere_mesh(n_tri: int):
    """UV sphere with a bumpy radius; ~n_tri triangles."""
    m = max(8, int(np.sqrt(n_tri / 4)))
    th = np.linspace(0, np.pi, m + 1)
    ph = np.linspace(0, 2 * np.pi, 2 * m + 1)
    T, P = np.meshgrid(th, ph, indexing="ij")
    r = 1.0 + 0.08 * np.sin(7 * T) * np.cos(9 * P) + 0.03 * np.sin(23 * P + 3 * T)
    V = np.stack([r * np.sin(T) * np.cos(P), r * np.cos(T), r * np.sin(T) * np.sin(P)], -1).reshape(-1, 3)
    a = (np.arange(m)[:, None] * (2 * m + 1) + np.arange(2 * m)[None, :]).reshape(-1)
    F = np.concatenate([np.stack([a, a + 2 * m + 1, a + 1], 1), np.stack([a + 1, a + 2 * m + 1, a + 2 * m + 2], 1)])
    return V.astype(np.float32), F.astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=str, default="100000,1000000,4000000")
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    import torch
    import mitsuba_hip as mi
    from mitsuba_hip import _abi as A
    mi.set_variant("hip_ad_rgb")
    T = mi.Transform4f
    tmp = tempfile.mkdtemp()
    for n in [int(x) for x in a.tris.split(",")]:
        V, F = sphere_mesh(n)
        p = os.path.join(tmp, f"s{n}.ply")
        mi.meshio.write_ply(p, V, F)
        d = mi.cornell_box()
        d["sensor"]["film"].update(width=a.res, height=a.res)
        d.pop("small-box")
        d.pop("large-box")
        d["blob"] = {"type": "ply", "filename": p, "to_world": T.translate([0, -0.45, 0]) @ T.scale(0.45),
                     "bsdf": {"type": "ref", "id": "white"}}
        t0 = time.time()
        scene = mi.load_dict(d)
        t_host = time.time() - t0
        t0 = time.time()
        h = scene.handle(0)
        t_dev = time.time() - t0
        import ctypes as C
        nn, npr, dep = C.c_uint32(), C.c_uint32(), C.c_uint32()
        A.lib().mh_scene_bvh_info(h, C.byref(nn), C.byref(npr), C.byref(dep))
        st = A.Stats()
        film = torch.empty((a.res, a.res, 4), device="cuda")
        for i in range(a.warmup):
            mi.render_film(scene, seed=100 + i, spp=a.spp, film=film, stats=st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ks, ts = [], []
        for i in range(a.steps):
            mi.render_film(scene, seed=i, spp=a.spp, film=film, stats=st)
            ks.append(st.ms_kernel)
            ts.append(st.ms_trace)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        ns = a.res * a.res * a.spp
        print(json.dumps({
            "triangles": int(len(F)), "bvh_nodes": nn.value, "bvh_depth": dep.value,
            "bvh_mb": round((nn.value * 64 + npr.value * 64) / 2**20, 1),
            "load_host_s": round(t_host, 2), "scene_create_s": round(t_dev, 2),
            "msamples_s": round(ns / dt / 1e6, 1), "ms_per_render": round(dt * 1e3, 2),
            "kernel_ms": round(sum(ks) / len(ks), 2), "mode": st.mode,
            "grays_s_closest": round(st.rays_closest / (dt * 1e9), 2),
            "grays_s_shadow": round(st.rays_shadow / (dt * 1e9), 2),
            # k_wf_trace (closest hits) timed by HIP events on the scene's stream:
            # algorithmic bytes 48 per closest ray (28-B ray in, 20-B hit out)
            "rays_closest": int(st.rays_closest), "rays_shadow": int(st.rays_shadow),
            "trace_ms": round(sum(ts) / len(ts), 3), "trace_launches": int(st.n_trace_launches),
            "trace_grays_s": round(st.rays_closest / (sum(ts) / len(ts) * 1e6), 2) if sum(ts) else None,
            "trace_alg_gbs": round(48 * st.rays_closest / (sum(ts) / len(ts) * 1e6), 1) if sum(ts) else None,
            "config": f"cornell box + {len(F)}-triangle PLY blob, {a.res}^2 @ {a.spp} spp, path max_depth 8"}),
            flush=True)
        scene.release()


if __name__ == "__main__":
    main()
