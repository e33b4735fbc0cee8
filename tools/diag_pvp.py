"""Per-sample prbvolpath / volpath radiance of the test scene (tests/test_gpu_parity.py
_pvp_scene) to an npz, for diffing two library builds (MH_LIB)."""
import os
import sys
import ctypes as C
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd"), os.path.join(ROOT, "tests")]
import mitsuba_hip as mi
from mitsuba_hip import _abi as A
import oracle_py as O
mi.set_variant("hip_ad_rgb")
d = mi.volume_cube(24, 20, 8, grid=mi.fbm_grid(16), scale=4.0)
d["integrator"] = {"type": sys.argv[2], "max_depth": 6, "rr_depth": 5}
T = mi.Transform4f
d["floor"] = {"type": "rectangle", "to_world": T.translate([0, -1.2, 0]) @ T.rotate([1, 0, 0], -90) @ T.scale([3, 3, 3]),
              "bsdf": {"type": "diffuse", "reflectance": {"type": "rgb", "value": [0.6, 0.5, 0.4]}}}
scene = mi.load_dict(d)
integ = scene.integrator()
n = 24 * 20 * 8
out = np.zeros(5 * n, np.float32)
ic = integ.c()
A.check(A.lib().mh_render_samples(scene.handle(0), C.byref(ic), 3, 8, 0, 0, out.ctypes.data_as(C.c_void_p), 0))
rL, rpos, _ = O.sample_range(scene, integ, 3, 8, 0, n)
np.savez(sys.argv[1], L=out[:3 * n].reshape(3, n).T, ref=rL)
