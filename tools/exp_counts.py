"""Packet-engine event counts of one forward render (diagnostic build only).

usage: tools/build_variant.sh cnt -DMH_EXP_COUNT
       MH_LIB=gpurun_exp/lib_cnt.so python tools/exp_counts.py [spp]
Counts are per wave (one per 64-lane batch step), closest / shadow rays."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba3-nasa_amd"))

import torch  # noqa: E402

import mitsuba_hip as mi  # noqa: E402
from mitsuba_hip import _abi  # noqa: E402

NAMES = ["rect_pair", "rect_pair_pass", "tri_pair", "tri_pair_pass", "rect_one(+pass)", "tri_one(+pass)",
         "node_visits", "batches"]


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    mi.set_variant("hip_ad_rgb")
    torch.cuda.set_device(0)
    scene = mi.load_dict(mi.cornell_box())
    integ = scene.integrator()
    L = _abi.lib()
    fn = L.mh_exp_counters
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 16)()
    mi.render_film(scene, integ, seed=0, spp=spp)
    torch.cuda.synchronize()
    fn(buf, 1)
    mi.render_film(scene, integ, seed=1, spp=spp)
    torch.cuda.synchronize()
    fn(buf, 1)
    for k, name in enumerate(NAMES):
        b = max(buf[7], 1), max(buf[15], 1)
        print(f"{name:18s} closest {buf[k]:14d} ({buf[k] / b[0]:7.2f}/batch)   shadow {buf[8 + k]:14d} "
              f"({buf[8 + k] / b[1]:7.2f}/batch)")


if __name__ == "__main__":
    main()
