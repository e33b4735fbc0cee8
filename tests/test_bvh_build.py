"""Host BVH builder (mitsuba3-nasa_amd/csrc/mh_bvh.cpp, the OptiX GAS build
slot of scene_optix.inl:449-514): binned SAH with the O(n) passes of large
ranges split over threads and subtrees built by workers.  tools/bvh_check.cpp
builds a clustered synthetic soup and checks every primitive sits in exactly
one leaf whose box (and every ancestor's) contains it; the node / primitive
arrays must not depend on the thread count.  The quantised BVH4 of the
stream engine (build_qbvh4) is checked the same way on its float-decoded
child boxes."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bvh_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("bvh") / "bvh_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                    os.path.join(ROOT, "tools", "bvh_check.cpp"),
                    os.path.join(ROOT, "mitsuba3-nasa_amd", "csrc", "mh_bvh.cpp"), "-o", exe, "-lpthread"],
                   check=True, capture_output=True)
    return exe


def run(exe, n, threads):
    r = subprocess.run([exe, str(n)], env=dict(os.environ, MH_BVH_THREADS=str(threads)), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("n", [1, 2, 5, 1000, 200000])
def test_bvh_valid_and_thread_independent(bvh_check, n):
    a = run(bvh_check, n, 1)
    b = run(bvh_check, n, 4)
    assert a["bad"] == 0 and b["bad"] == 0
    assert a["qbad"] == 0 and b["qbad"] == 0   # the quantised BVH4 is conservative and complete
    assert a["hash"] == b["hash"], (a, b)
    assert a["leaves"] == a["nodes"] + 1 and a["depth"] < 48
