#!/usr/bin/env python3
"""Generates the committed fixtures under tests/golden/.

1. known_answers.json — known-answer vectors of the reference's own tests,
   extracted (as data) from the reference test files when /root/reference is
   present, plus the published pcg-basic demo stream.  Each entry records its
   provenance (file:line).  The tests read only this JSON (the reference does
   not exist on the GPU box).
2. oracle_regression.npz — outputs of the CPU restatement (oracle/) on small
   seeded inputs: PCG32 sampler floats, camera rays,
   cornell hit records, a 32x32 @ 16 spp film and a PRB gradient.  They pin
   the oracle against silent drift and give the GPU tests a fixed target.

usage: python tests/golden/make_golden.py [--check]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [os.path.join(ROOT, "mitsuba3-nasa_amd"), os.path.join(ROOT, "tests")]


def _lines(path):
    with open(os.path.join(REF, path)) as f:
        return f.read().split("\n")


def tea_table():
    path = "src/core/tests/test_random.py"
    out = {"float32": [], "float64": []}
    pat = re.compile(r"mi\.sample_tea_float(32|64)\((\d+), (\d+), (\d+)\) == ([0-9.e-]+)")
    for i, ln in enumerate(_lines(path), 1):
        m = pat.search(ln)
        if m:
            out["float" + m.group(1)].append(
                {"v0": int(m.group(2)), "v1": int(m.group(3)), "rounds": int(m.group(4)),
                 "value": float(m.group(5)), "source": f"{path}:{i}"})
    return out


def gaussian():
    path = "src/rfilters/tests/test_rfilter.py"
    L = _lines(path)
    out = []
    for i, ln in enumerate(L, 1):
        m = re.search(r"dr\.allclose\(f\.eval\(([0-9.]+)\), ([0-9.]+), atol=([0-9.e-]+)\)", ln)
        if m and "gaussian" in "".join(L[max(0, i - 4):i]):
            out.append({"x": float(m.group(1)), "value": float(m.group(2)), "atol": float(m.group(3)),
                        "source": f"{path}:{i}"})
        m = re.search(r"assert f\.eval\(([0-9.]+)\) == 0", ln)
        if m and "gaussian" in "".join(L[max(0, i - 5):i]):
            out.append({"x": float(m.group(1)), "value": 0.0, "atol": 0.0, "source": f"{path}:{i}"})
    return out


def rectangle():
    path = "src/shapes/tests/test_rectangle.py"
    L = _lines(path)
    src = "\n".join(L)
    assert "mi.Transform4f.scale((2.0, 0.5, 1.0))" in src and "valid_count == 7" in src
    line = next(i for i, ln in enumerate(L, 1) if "valid_count == 7" in ln)
    return {"scale": [2.0, 0.5, 1.0], "n": 15, "origin_z": 5.0, "dir": [0, 0, -1],
            "hit_rule": "abs(a) <= 0.5", "valid_count": 7, "source": f"{path}:34-60 (assert at :{line})"}


def cube():
    path = "src/shapes/tests/test_cube.py"
    src = "\n".join(_lines(path))
    assert "[-1.5, -0.9, -0.5, 0, 0.5, 0.9, 1.5]" in src
    faces = [[[0, 0, -8], [0, 0, 1], [0, 0, -1]], [[0, 0, 8], [0, 0, -1], [0, 0, 1]],
             [[-8, 0, 0], [1, 0, 0], [-1, 0, 0]], [[8, 0, 0], [-1, 0, 0], [1, 0, 0]],
             [[0, -8, 0], [0, 1, 0], [0, -1, 0]], [[0, 8, 0], [0, -1, 0], [0, 1, 0]]]
    return {"scales": [[1, 1, 1], [2, 1, 1], [1, 2, 1]], "coords": [-1.5, -0.9, -0.5, 0, 0.5, 0.9, 1.5],
            "origin_z": -8.0, "dir": [0, 0, 1], "hit_rule": "abs(x) <= sx and abs(y) <= sy",
            "faces": faces, "source": f"{path}:26-90 (test03_ray_intersect), :91-120 (test05_check_normals)"}


def diffuse():
    path = "src/bsdfs/tests/test_diffuse.py"
    src = "\n".join(_lines(path))
    assert "assert dr.allclose(v_eval, 0.5 * wo[2] / dr.pi)" in src
    return {"n": 20, "reflectance": 0.5, "wi": [0, 0, 1], "theta": "i / 19 * pi / 2",
            "pdf": "cos(theta) / pi", "eval": "0.5 * cos(theta) / pi", "source": f"{path}:13-35"}


def known_answers():
    return {
        "tea": tea_table(),
        "gaussian": gaussian(),
        "rectangle": rectangle(),
        "cube": cube(),
        "diffuse": diffuse(),
        "pcg32_demo": {"initstate": 42, "initseq": 54,
                       "values": [0xa15c02b7, 0x7b47f409, 0xba1d3330, 0x83d2f293, 0xbfa4784b, 0xcbed606e],
                       "source": "pcg-basic pcg32-demo, pcg32_srandom(42u, 54u) (drjit PCG32 seeds identically: "
                                 "sampler.cpp:128-132 -> drjit/random.h)"},
        "linearity": {"source": "src/render/tests/test_ad.py:6-92",
                      "note": "loss(rho + lr) == loss(rho) + lr * dloss/drho for a one-bounce scene"},
    }


def oracle_regression():
    import numpy as np
    import mitsuba_hip as mi
    import oracle_py as O
    import ctypes as C
    L = O.lib()
    out = {}
    sf = np.zeros((64, 8), np.float32)
    for lane in range(64):
        L.oracle_sampler_floats(0, lane * 16, 8, sf[lane].ctypes.data_as(C.c_void_p))
    out["sampler_floats_seed0"] = sf
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = 32
    d["sensor"]["film"]["height"] = 32
    scene = mi.load_dict(d)
    rng = np.random.default_rng(7)
    pos = rng.random((64, 2), dtype=np.float32)
    cam = np.zeros((64, 7), np.float32)
    for i in range(64):
        o = np.zeros(3, np.float32); dd = np.zeros(3, np.float32); mt = C.c_float()
        O.check(L.oracle_camera_ray(C.byref(scene.desc), pos[i].ctypes.data_as(C.c_void_p),
                                    o.ctypes.data_as(C.c_void_p), dd.ctypes.data_as(C.c_void_p), C.byref(mt)))
        cam[i, :3], cam[i, 3:6], cam[i, 6] = o, dd, mt.value
    out["camera_pos"], out["camera_rays"] = pos, cam
    n = 4096
    o = rng.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    v = rng.normal(size=(n, 3)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    rays = np.concatenate([o.T, v.T, np.full((1, n), np.finfo(np.float32).max, np.float32)]).astype(np.float32)
    t, u, vv, prim, shape = O.trace_closest(scene, rays)
    out["trace_rays"] = rays
    out["trace_t"], out["trace_u"], out["trace_v"], out["trace_prim"], out["trace_shape"] = t, u, vv, prim, shape
    integ = mi.load_dict({"type": "path", "max_depth": 8})
    out["film_32_spp16_seed1"] = O.render(scene, integ, seed=1, spp=16, threads=4)
    prb = mi.load_dict({"type": "prb", "max_depth": 8})
    gi = np.full((32, 32, 3), 1.0 / (32 * 32 * 3), np.float32)
    key = "white.reflectance.value"
    out["prb_grad_white_32_spp16_seed5"] = O.render_backward(scene, prb, 5, 16, gi, [scene.params[key][1]],
                                                             [(3,)], threads=4)[0]
    return out


def main():
    import numpy as np
    check = "--check" in sys.argv
    if os.path.isdir(REF):
        ka = known_answers()
        path = os.path.join(HERE, "known_answers.json")
        if check:
            assert json.load(open(path)) == json.loads(json.dumps(ka)), "known_answers.json is stale"
        else:
            json.dump(ka, open(path, "w"), indent=1)
    reg = oracle_regression()
    path = os.path.join(HERE, "oracle_regression.npz")
    if check:
        old = np.load(path)
        for k, v in reg.items():
            assert np.array_equal(old[k], v), k
    else:
        np.savez_compressed(path, **reg)
    print("ok")


if __name__ == "__main__":
    main()
