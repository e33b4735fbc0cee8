#!/usr/bin/env python3
"""Time config-2 forward (cornell 512^2 @ 256 spp, path) in each execution mode
and wavefront chunk size; prints one line per variant."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd"), os.path.join(ROOT, "tests")]


def main():
    import torch
    import mitsuba_hip as mi
    from mitsuba_hip import _abi as A
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 512
    scene = mi.load_dict(d)
    integ = scene.integrator()
    st = A.Stats()
    variants = [("mega", None)] + [("wavefront", c) for c in (sys.argv[1:] or ["1048576", "2097152", "4194304", "8388608"])]
    for mode, chunk in variants:
        if chunk:
            os.environ["MH_WF_CHUNK"] = chunk
        best = 1e9
        for i in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mi.render_film(scene, integ, seed=0, spp=256, stats=st, mode=mode)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(f"{mode:9s} chunk={chunk or '-':>8s}: {best*1e3:7.1f} ms {512*512*256/best/1e6:8.1f} Msamples/s "
              f"kernel {st.ms_kernel:6.1f} ms trace {st.ms_trace:6.1f} ms ({st.n_trace_launches} launches, "
              f"{st.rays_closest/max(st.ms_trace,1e-9)/1e6:.2f} Grays/s)", flush=True)


if __name__ == "__main__":
    main()
