"""CPU: the drop-in boundary.  libmitsuba_hip.so loads (gfx950 code objects
inside; no GPU needed to load), exports every function include/mitsuba_hip.h
declares, and the ctypes mirrors in mitsuba_hip/_abi.py match the C struct
layouts byte for byte (checked against gcc's view of the header).  No
compute call is made here."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mitsuba_hip.h")
LIBSO = os.path.join(ROOT, "mitsuba3-nasa_amd", "mitsuba_hip", "libmitsuba_hip.so")

STRUCTS = {"mh_shape": "Shape", "mh_texture": "Texture", "mh_bsdf": "Bsdf", "mh_emitter": "Emitter",
           "mh_medium": "Medium", "mh_sensor": "Sensor", "mh_scene_desc": "SceneDesc",
           "mh_integrator": "Integrator", "mh_stats": "Stats"}


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(mh_\w+)\s*\(", src, flags=re.M)))


def test_header_and_exports_list_agree():
    from mitsuba_hip import _abi as A
    assert header_functions() == sorted(A.EXPORTS)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIBSO):
        pytest.skip("libmitsuba_hip.so not built (run __graft_entry__.build())")
    from mitsuba_hip import _abi as A
    return A.lib()


def test_library_exports_every_symbol(lib):
    raw = C.CDLL(LIBSO)
    for name in header_functions():
        assert hasattr(raw, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", LIBSO], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in nm.splitlines() if " T " in ln}
    assert set(header_functions()) <= exported


def test_abi_version(lib):
    from mitsuba_hip import _abi as A
    assert lib.mh_abi_version() == A.ABI_VERSION
    m = re.search(r"#define MH_ABI_VERSION (\d+)u", open(HEADER).read())
    assert int(m.group(1)) == A.ABI_VERSION


def test_library_contains_gfx950_code():
    if not os.path.exists(LIBSO):
        pytest.skip("not built")
    blob = open(LIBSO, "rb").read()
    assert b"gfx950" in blob


def test_struct_layouts_match_header():
    from mitsuba_hip import _abi as A
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cs, py in STRUCTS.items():
        T = getattr(A, py)
        lines.append(f'printf("{py} sizeof %zu\\n", sizeof({cs}));')
        for f in T._fields_:
            lines.append(f'printf("{py} {f[0]} %zu\\n", offsetof({cs}, {f[0]}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "layout.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(d, "layout")
        subprocess.run(["gcc", "-std=c11", "-o", exe, c], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    for ln in out.splitlines():
        py, field, val = ln.split()
        T = getattr(A, py)
        got = C.sizeof(T) if field == "sizeof" else getattr(T, field).offset
        assert got == int(val), (py, field, got, val)


def test_flags_match_header():
    from mitsuba_hip import _abi as A
    src = open(HEADER).read()
    for name in ("DEVICE_POINTERS", "ACCUMULATE", "NO_SYNC", "MEGAKERNEL", "WAVEFRONT", "PRB_REPLAY", "DETERMINISTIC", "REDUCE",
                 "REDUCE_ROOT", "LOCAL_WEIGHTS", "SHARED_DEVICE"):
        m = re.search(rf"MH_FLAG_{name}\s*=\s*1u << (\d+)", src)
        assert m, name
        assert getattr(A, "FLAG_" + name) == 1 << int(m.group(1))


def test_product_path_has_no_cpu_fallback():
    """Without a HIP device the product entry points raise; they never route
    through the oracle (the package must not import it)."""
    import mitsuba_hip as mi
    import torch
    pkg = os.path.join(ROOT, "mitsuba3-nasa_amd", "mitsuba_hip")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert not re.search(r"oracle_py|libmh_oracle|import\s+oracle", src), f
    if not torch.cuda.is_available():
        scene = mi.load_dict({"type": "scene", "r": {"type": "rectangle"}})
        with pytest.raises(Exception):
            mi.render_film(scene, spp=1)


def test_comm_entry_points_without_a_device(lib):
    """The multi-GPU C ABI loads RCCL lazily: a unique id can be made on any
    host (RCCL's bootstrap handle), and creating a rank without a device
    fails with MH_ERR_NO_DEVICE and a message -- no CPU fallback."""
    from mitsuba_hip import _abi as A
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present (covered by tests/test_gpu_comm.py)")
    uid = C.create_string_buffer(A.COMM_ID_BYTES)
    rc = lib.mh_comm_unique_id(uid)
    if rc == A.MH_ERR_UNSUPPORTED:  # RCCL not installed on this host
        assert b"RCCL" in lib.mh_last_error()
        return
    assert rc == A.MH_OK and any(uid.raw)
    h = C.c_void_p()
    assert lib.mh_comm_create(uid, 1, 0, 0, C.byref(h)) == A.MH_ERR_NO_DEVICE
    assert b"no HIP device" in lib.mh_last_error()
    assert lib.mh_comm_create(uid, 2, 2, 0, C.byref(h)) == A.MH_ERR_INVALID_ARGUMENT
    assert lib.mh_scene_set_comm(None, None) == A.MH_ERR_INVALID_ARGUMENT
    assert lib.mh_comm_reduce(None, 0, None, 0, None, -1) == A.MH_ERR_INVALID_ARGUMENT
    assert lib.mh_render_sharded(None, 0, None, 0, 1, None, 0, None) == A.MH_ERR_INVALID_ARGUMENT
    assert lib.mh_comm_destroy(None) == A.MH_OK
