"""First-contact GPU script (not a pytest file): exercises every kernel once
and prints parity diagnostics.  Run: python tests/test_gpu_smoke_quick.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def main():
    import mitsuba_hip as mi
    print("available:", mi.is_available(), flush=True)
    scene = T.cbox(mi, 32, 32, 16)
    rays = T.random_rays(scene, 1 << 16)
    t, u, v, prim, shape, occ = T.gpu_trace(mi, scene, rays)
    rt, ru, rv, rprim, rshape = O.trace_closest(scene, rays)
    rocc = O.trace_shadow(scene, rays)
    same = (shape == rshape) & ((t == rt) | (np.isinf(t) & np.isinf(rt)))
    print("trace closest agree", same.mean(), "shadow agree", (occ == rocc).mean(), flush=True)
    for it in ["path", "prb"]:
        integ = mi.load_dict({"type": it, "max_depth": 8})
        L, pos = T._gpu_samples(mi, scene, integ, 3, 4)
        rL, rpos, _ = O.sample_range(scene, integ, 3, 4, 0, L.shape[0])
        print(it, "pos equal", np.array_equal(pos, rpos), "L exact", np.all(L == rL, 1).mean(),
              "max abs", np.abs(L - rL).max(), flush=True)
    integ = scene.integrator()
    film = mi.render_film(scene, integ, seed=5, spp=16).cpu().numpy()
    ref = O.render(scene, integ, seed=5, spp=16)
    print("film close", T._film_close(film, ref), "max rel",
          (np.abs(film - ref) / np.maximum(1, np.abs(ref))).max(), flush=True)
    import torch
    pr = mi.load_dict({"type": "prb", "max_depth": 8})
    params = mi.traverse(scene)
    gi = np.full((32, 32, 3), 1 / (32 * 32 * 3), np.float32)
    g = mi.render_backward(scene, params, torch.from_numpy(gi).cuda(), ["white.reflectance.value"], pr, 11, 16)
    rg = O.render_backward(scene, pr, 11, 16, gi, [params.texture_of("white.reflectance.value")], [(3,)])
    print("grad gpu", g[0].cpu().numpy(), "oracle", rg[0], flush=True)
    # timing of the config-2 forward
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = 512
    d["sensor"]["film"]["height"] = 512
    big = mi.load_dict(d)
    from mitsuba_hip import _abi as A
    st = A.Stats()
    for mode in ["mega", "wavefront"]:
        for i in range(3):
            torch.cuda.synchronize()
            t0 = time.time()
            mi.render_film(big, big.integrator(), seed=0, spp=256, stats=st, mode=mode)
            torch.cuda.synchronize()
            dt = time.time() - t0
            print(f"{mode}: 512^2 x 256spp path: {dt*1e3:.1f} ms  {512*512*256/dt/1e6:.1f} Msamples/s  "
                  f"kernel {st.ms_kernel:.1f} ms trace {st.ms_trace:.1f} ms ({st.n_trace_launches} launches) "
                  f"rays {st.rays_closest} shadow {st.rays_shadow}", flush=True)
    f1 = mi.render_film(big, big.integrator(), seed=0, spp=64, mode="mega").cpu().numpy()
    f2 = mi.render_film(big, big.integrator(), seed=0, spp=64, mode="wavefront").cpu().numpy()
    print("mega vs wavefront film max rel", (np.abs(f1 - f2) / np.maximum(1, np.abs(f1))).max(), flush=True)


if __name__ == "__main__":
    main()
