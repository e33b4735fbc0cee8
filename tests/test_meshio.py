"""CPU: OBJ / PLY loaders and vertex-normal recomputation (SURVEY.md §8(f)
rank 2; src/shapes/obj.cpp, src/shapes/ply.cpp, src/render/mesh.cpp:321-409).

The reference's mesh fixtures (resources/data/tests/{ply,obj}/...) are not
vendored; the files are re-created here from the values its tests assert
(src/render/tests/test_mesh.py test02-test06)."""
import numpy as np
import pytest

import oracle_py as O


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


TRI_PLY = """ply
format ascii 1.0
element vertex 3
property float x
property float y
property float z
element face 1
property list uchar int vertex_indices
end_header
0 0 0
0 0 1
0 1 0
3 0 1 2
"""


def test_ply_triangle_and_computed_normals(tmp_path):
    """test_mesh.py test02 / test03."""
    from mitsuba_hip import meshio
    p = tmp_path / "triangle.ply"
    p.write_text(TRI_PLY)
    m = meshio.read_ply(str(p), face_normals=True)
    assert m["normals"] is None and not m["recompute_normals"]
    np.testing.assert_array_equal(m["positions"], [[0, 0, 0], [0, 0, 1], [0, 1, 0]])
    np.testing.assert_array_equal(m["faces"], [[0, 1, 2]])
    m = meshio.read_ply(str(p))
    assert m["recompute_normals"]
    n = meshio.recompute_vertex_normals(m["positions"], m["faces"])
    np.testing.assert_allclose(n, [[-1, 0, 0]] * 3, atol=1e-6)


def test_normal_weighting_scheme():
    """test_mesh.py test04: angle-weighted vertex normals."""
    from mitsuba_hip import meshio
    a, b = 1.0, 0.5
    V = np.array([0, 0, 0, -a, 1, 0, a, 1, 0, -b, 0, 1, b, 0, 1], np.float32).reshape(-1, 3)
    F = np.array([0, 1, 2, 0, 3, 4], np.uint32).reshape(-1, 3)
    n0, n1 = np.array([0.0, 0.0, -1.0]), np.array([0.0, 1.0, 0.0])
    n2 = n0 * (np.pi / 2) + n1 * np.arccos(3.0 / 5.0)
    n2 /= np.linalg.norm(n2)
    ref = np.vstack([n2, n0, n0, n1, n1])
    np.testing.assert_allclose(meshio.recompute_vertex_normals(V, F), ref, atol=5e-4)


RECT_V = np.array([[-2.85, 0.0, -7.6], [-2.85, 0.0, 0.599999], [2.85, 0.0, 0.599999], [2.85, 0.0, -7.6]], np.float32)
RECT_UV = np.array([[0.950589, 0.988416], [0.025105, 0.988416], [0.025105, 0.689127], [0.950589, 0.689127]],
                   np.float32)
RECT_F = np.array([[0, 1, 2], [0, 2, 3]], np.uint32)


@pytest.mark.parametrize("fmt", ["obj", "ply", "ply_ascii"])
@pytest.mark.parametrize("features", ["normals", "uv", "normals_uv"])
@pytest.mark.parametrize("face_normals", [True, False])
def test_load_various_features(tmp_path, fmt, features, face_normals):
    """test_mesh.py test06: OBJ flips uv.y by default, PLY does not."""
    from mitsuba_hip import meshio
    N = np.tile([0.0, 1.0, 0.0], (4, 1)).astype(np.float32) if "normals" in features else None
    UV = RECT_UV if "uv" in features else None
    p = str(tmp_path / f"rect.{fmt[:3]}")
    if fmt == "obj":
        # the reference fixture stores vt as 1 - uv (written by an exporter with flipped v)
        meshio.write_obj(p, RECT_V, RECT_F, N, None if UV is None else np.stack([UV[:, 0], 1 - UV[:, 1]], 1))
        m = meshio.read_obj(p, face_normals=face_normals)
    else:
        meshio.write_ply(p, RECT_V, RECT_F, N, UV, binary=fmt == "ply")
        m = meshio.read_ply(p, face_normals=face_normals)
    np.testing.assert_allclose(m["positions"][[0, 2, 3]], RECT_V[[0, 2, 3]], atol=1e-3)
    assert (m["normals"] is not None) == (not face_normals and N is not None)
    if UV is not None:
        want = np.stack([UV[:, 0], 1 - UV[:, 1]], 1) if fmt == "obj" else UV
        np.testing.assert_allclose(m["texcoords"][[0, 2, 3]], want[[0, 2, 3]], atol=1e-3)
    if m["normals"] is not None:
        np.testing.assert_allclose(m["normals"], np.tile([0, 1, 0], (4, 1)))


def test_obj_corner_dedup_and_fan_triangulation(tmp_path):
    from mitsuba_hip import meshio
    p = tmp_path / "quad.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\n"
                 "f 1/1 2/2 3/3 4/4\nf 1/1 3/3 4/2\n")
    m = meshio.read_obj(str(p))
    np.testing.assert_array_equal(m["faces"], [[0, 1, 2], [0, 2, 3], [0, 2, 4]])
    assert m["positions"].shape == (5, 3)               # (4, vt 2) is a new corner
    np.testing.assert_array_equal(m["positions"][4], [0, 1, 0])
    np.testing.assert_allclose(m["texcoords"][4], [1, 1])   # vt 2 = (1, 0), flipped


def test_ply_binary_endianness_and_errors(tmp_path):
    from mitsuba_hip import meshio
    rng = np.random.default_rng(0)
    V = rng.random((10, 3)).astype(np.float32)
    F = rng.integers(0, 10, (7, 3)).astype(np.uint32)
    a = tmp_path / "a.ply"
    meshio.write_ply(str(a), V, F)
    # re-encode big-endian by hand
    hdr, body = a.read_bytes().split(b"end_header\n", 1)
    vb = np.frombuffer(body[:10 * 12], "<f4").astype(">f4").tobytes()
    fa = np.frombuffer(body[10 * 12:], np.dtype([("n", "u1"), ("i", "<i4", (3,))]))
    fb = np.empty(len(fa), np.dtype([("n", "u1"), ("i", ">i4", (3,))]))
    fb["n"], fb["i"] = fa["n"], fa["i"]
    b = tmp_path / "b.ply"
    b.write_bytes(hdr.replace(b"binary_little_endian", b"binary_big_endian") + b"end_header\n" + vb + fb.tobytes())
    for path in (a, b):
        m = meshio.read_ply(str(path))
        np.testing.assert_array_equal(m["positions"], V)
        np.testing.assert_array_equal(m["faces"], F)
    q = tmp_path / "quad.ply"
    q.write_text(TRI_PLY.replace("element vertex 3", "element vertex 4").replace("0 1 0\n3 0 1 2", "0 1 0\n1 1 0\n4 0 1 2 3"))
    with pytest.raises(RuntimeError, match="triangle mesh"):
        meshio.read_ply(str(q))
    with pytest.raises(RuntimeError, match="file not found"):
        meshio.read_ply(str(tmp_path / "missing.ply"))


def _bumpy_mesh(n=12):
    """A small height-field mesh with uvs (positions, faces, uv)."""
    x, y = np.meshgrid(np.linspace(-0.8, 0.8, n), np.linspace(-0.8, 0.8, n))
    z = 0.15 * np.sin(3 * x) * np.cos(2 * y)
    V = np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)
    UV = np.stack([(x + 0.8) / 1.6, (y + 0.8) / 1.6], -1).reshape(-1, 2).astype(np.float32)
    i = np.arange(n - 1)
    a = (i[:, None] * n + i[None, :]).reshape(-1)
    F = np.concatenate([np.stack([a, a + 1, a + n + 1], 1), np.stack([a, a + n + 1, a + n], 1)]).astype(np.uint32)
    return V, F, UV


@pytest.mark.parametrize("fmt", ["obj", "ply"])
def test_file_mesh_renders_like_the_in_memory_mesh(tmp_path, fmt):
    """A mesh loaded from a file (normals recomputed as the reference does)
    is the same scene as the in-memory mesh carrying those normals."""
    mi = _mi()
    from mitsuba_hip import meshio
    V, F, UV = _bumpy_mesh()
    T = mi.Transform4f
    to_world = T.translate([0, 0.1, 0]) @ T.rotate([1, 0, 0], -70)
    p = str(tmp_path / f"bumpy.{fmt}")
    if fmt == "obj":
        meshio.write_obj(p, V, F, texcoords=UV)
    else:
        meshio.write_ply(p, V, F, texcoords=UV)

    def scene(shape):
        d = mi.cornell_box()
        d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 24
        d.pop("small-box")
        d.pop("large-box")
        d["bumpy"] = shape
        return mi.load_dict(d)

    a = scene({"type": fmt, "filename": p, "to_world": to_world, "bsdf": {"type": "ref", "id": "white"}})
    Vw = (V.astype(np.float64) @ to_world.matrix[:3, :3].T + to_world.matrix[:3, 3]).astype(np.float32)
    N = meshio.recompute_vertex_normals(Vw, F)
    b = scene({"type": "mesh", "vertex_positions": Vw, "faces": F, "vertex_normals": N, "vertex_texcoords": UV,
               "bsdf": {"type": "ref", "id": "white"}})
    fa = O.render(a, seed=1, spp=4)
    fb = O.render(b, seed=1, spp=4)
    assert fa[..., :3].max() > 0
    np.testing.assert_array_equal(fa, fb)
