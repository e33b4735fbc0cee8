"""Diagnostic (not collected): GPU trace vs the golden fixture, printing mismatches."""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "mitsuba3-nasa_amd"), HERE]
import torch  # noqa
import mitsuba_hip as mi
from test_gpu_parity import gpu_trace
REG = np.load(os.path.join(HERE, "golden", "oracle_regression.npz"))
d = mi.cornell_box(); d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 32
scene = mi.load_dict(d)
t, u, v, prim, shape, occ = gpu_trace(mi, scene, REG["trace_rays"])
bad = np.where(~((t == REG["trace_t"]) & (prim == REG["trace_prim"]) & (shape == REG["trace_shape"])))[0]
print("mismatches", len(bad))
for i in bad[:20]:
    print(i, REG["trace_rays"][:, i], "gpu", t[i], prim[i], shape[i], "ref", REG["trace_t"][i], REG["trace_prim"][i], REG["trace_shape"][i])
