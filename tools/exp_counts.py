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
    buf = (C.c_ulonglong * 32)()
    nb = C.c_uint32(); npr = C.c_uint32(); dep = C.c_uint32()
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
    # live lanes per pair test (of 64) and accepted primitives per ray-batch
    for k, name, den in ((0, "rect_pair live lanes/call", 0), (1, "tri_pair live lanes/call", 2),
                         (2, "rect accepts/batch", 7), (3, "tri accepts/batch", 7)):
        print(f"{name:26s} closest {buf[16 + k] / max(buf[den], 1):7.2f}   shadow {buf[24 + k] / max(buf[8 + den], 1):7.2f}")
    L.mh_scene_bvh_info(scene.handle(0), C.byref(nb), C.byref(npr), C.byref(dep))
    print("bvh nodes", nb.value, "prims", npr.value, "depth", dep.value)


if __name__ == "__main__":
    main()
