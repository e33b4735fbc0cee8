"""Mesh file formats of the hot path's scenes.

Host-side loaders with the reference's semantics:
  * OBJ  (src/shapes/obj.cpp:148-411): v / vn / vt / f records; face corners
    are de-duplicated by their (v, vt, vn) index triple in first-use order;
    polygons are fan-triangulated; vt.y is flipped unless
    flip_tex_coords=False; 1-based indices only.
  * PLY  (src/shapes/ply.cpp:165-450): ascii / binary_little_endian /
    binary_big_endian; vertex x y z [nx ny nz] [u v | texture_u texture_v |
    s t]; face 'vertex_indices' or 'vertex_index' lists of exactly three
    entries; other elements are skipped; flip_tex_coords defaults to False.
  * recompute_vertex_normals (src/render/mesh.cpp:321-409, the JIT branch):
    angle-weighted face normals, normalised.
Loaders return object-space float32 arrays; the scene builder applies
`to_world` (positions affine, normals by the inverse transpose, normalised).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1",
    "short": "i2", "int16": "i2", "ushort": "u2", "uint16": "u2",
    "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


def _fail(kind: str, path, descr: str):
    raise RuntimeError(f'Error while loading {kind} file "{os.path.basename(str(path))}": {descr}')


# ---------------------------------------------------------------------------
# OBJ
# ---------------------------------------------------------------------------
def read_obj(path, flip_tex_coords: bool = True, face_normals: bool = False) -> Dict[str, Optional[np.ndarray]]:
    if not os.path.exists(path):
        _fail("OBJ", path, "file not found")
    v, vn, vt = [], [], []
    corner_id: Dict[tuple, int] = {}
    keys = []
    tris = []
    with open(path, "r", errors="replace") as f:
        for line in f:
            s = line.strip()
            if not s or s[0] == "#":
                continue
            tok = s.split()
            head = tok[0]
            try:
                if head == "v":
                    v.append([float(x) for x in tok[1:4]])
                elif head == "vn":
                    if not face_normals:
                        vn.append([float(x) for x in tok[1:4]])
                elif head == "vt":
                    uv = [float(x) for x in tok[1:3]]
                    if flip_tex_coords:
                        uv[1] = 1.0 - uv[1]
                    vt.append(uv)
                elif head == "f":
                    ids = []
                    for c in tok[1:]:
                        parts = c.split("/")
                        key = [0, 0, 0]
                        for i, p in enumerate(parts[:3]):
                            if p:
                                key[i] = int(p)
                        if key[0] < 1 or key[0] > len(v):
                            _fail("OBJ", path, f"reference to invalid vertex {key[0]}!")
                        key = tuple(key)
                        cid = corner_id.get(key)
                        if cid is None:
                            cid = corner_id[key] = len(keys)
                            keys.append(key)
                        ids.append(cid)
                    for k in range(2, len(ids)):          # fan: (0, k-1, k)
                        tris.append((ids[0], ids[k - 1], ids[k]))
            except ValueError:
                _fail("OBJ", path, f'could not parse line "{s}"')
    V = np.asarray(v, np.float32).reshape(-1, 3)
    if V.size and not np.all(np.isfinite(V)):
        _fail("OBJ", path, "mesh contains invalid vertex position data")
    K = np.asarray(keys, np.int64).reshape(-1, 3)
    out_v = V[K[:, 0] - 1] if len(K) else np.zeros((0, 3), np.float32)
    out_uv = None
    if vt:
        T = np.asarray(vt, np.float32).reshape(-1, 2)
        if np.any(K[:, 1] > len(T)):
            _fail("OBJ", path, f"reference to invalid texture coordinate {int(K[:, 1].max())}!")
        out_uv = np.where(K[:, 1:2] > 0, T[np.maximum(K[:, 1] - 1, 0)], 0.0).astype(np.float32)
    out_n = None
    if not face_normals and vn:
        N = np.asarray(vn, np.float32).reshape(-1, 3)
        if np.any(K[:, 2] > len(N)):
            _fail("OBJ", path, f"reference to invalid normal {int(K[:, 2].max())}!")
        out_n = np.where(K[:, 2:3] > 0, N[np.maximum(K[:, 2] - 1, 0)], 0.0).astype(np.float32)
    return {"positions": out_v, "normals": out_n, "texcoords": out_uv,
            "faces": np.asarray(tris, np.uint32).reshape(-1, 3),
            "recompute_normals": not face_normals and not vn}


def write_obj(path, positions, faces, normals=None, texcoords=None):
    """Writes v/vt/vn/f with one index per vertex (vt stored un-flipped, so
    read_obj's default flip restores the given texcoords)."""
    P = np.asarray(positions, np.float32).reshape(-1, 3)
    F = np.asarray(faces, np.int64).reshape(-1, 3) + 1
    with open(path, "w") as f:
        for p in P:
            f.write("v %.9g %.9g %.9g\n" % tuple(p))
        if texcoords is not None:
            for t in np.asarray(texcoords, np.float32).reshape(-1, 2):
                f.write("vt %.9g %.9g\n" % (t[0], 1.0 - np.float64(t[1])))
        if normals is not None:
            for n in np.asarray(normals, np.float32).reshape(-1, 3):
                f.write("vn %.9g %.9g %.9g\n" % tuple(n))
        ht, hn = texcoords is not None, normals is not None
        for tri in F:
            if ht and hn:
                f.write("f " + " ".join(f"{i}/{i}/{i}" for i in tri) + "\n")
            elif ht:
                f.write("f " + " ".join(f"{i}/{i}" for i in tri) + "\n")
            elif hn:
                f.write("f " + " ".join(f"{i}//{i}" for i in tri) + "\n")
            else:
                f.write("f %d %d %d\n" % tuple(tri))


# ---------------------------------------------------------------------------
# PLY
# ---------------------------------------------------------------------------
def _ply_header(fh, path):
    line = fh.readline().strip()
    if line != b"ply":
        _fail("PLY", path, 'invalid PLY header: missing "ply" tag')
    fmt, elements = None, []
    while True:
        raw = fh.readline()
        if not raw:
            _fail("PLY", path, "invalid PLY header: missing end_header")
        tok = raw.decode("ascii", "replace").split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            if len(tok) < 3 or tok[2] != "1.0":
                _fail("PLY", path, "invalid PLY header: unknown version number")
            fmt = tok[1]
            if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
                _fail("PLY", path, f'invalid PLY header: invalid token after "format"')
        elif tok[0] == "element":
            elements.append({"name": tok[1], "count": int(tok[2]), "props": []})
        elif tok[0] == "property":
            if not elements:
                _fail("PLY", path, 'invalid PLY header: encountered "property" before "element"')
            if tok[1] == "list":
                if tok[2] not in _PLY_TYPES or tok[3] not in _PLY_TYPES:
                    _fail("PLY", path, f'invalid PLY header: unknown format type "{tok[2]}"')
                elements[-1]["props"].append((tok[4], "list", _PLY_TYPES[tok[2]], _PLY_TYPES[tok[3]]))
            else:
                if tok[1] not in _PLY_TYPES:
                    _fail("PLY", path, f'invalid PLY header: unknown format type "{tok[1]}"')
                elements[-1]["props"].append((tok[2], "scalar", _PLY_TYPES[tok[1]], None))
        elif tok[0] == "end_header":
            break
    if fmt is None:
        _fail("PLY", path, 'invalid PLY header: missing "format"')
    return fmt, elements


def read_ply(path, flip_tex_coords: bool = False, face_normals: bool = False) -> Dict[str, Optional[np.ndarray]]:
    if not os.path.exists(path):
        _fail("PLY", path, "file not found")
    with open(path, "rb") as fh:
        fmt, elements = _ply_header(fh, path)
        body = fh.read()
    ascii_ = fmt == "ascii"
    end = "<" if fmt == "binary_little_endian" else ">"
    toks = body.split() if ascii_ else None
    tpos = 0
    off = 0
    data = {}
    for el in elements:
        props, n = el["props"], el["count"]
        has_list = any(p[1] == "list" for p in props)
        if ascii_:
            if not has_list:
                k = len(props)
                arr = np.array(toks[tpos:tpos + k * n], dtype=np.float64).reshape(n, k)
                tpos += k * n
                data[el["name"]] = {p[0]: arr[:, i] for i, p in enumerate(props)}
            else:
                cols = {p[0]: [] for p in props}
                for _ in range(n):
                    for p in props:
                        if p[1] == "list":
                            c = int(toks[tpos]); tpos += 1
                            cols[p[0]].append([float(x) for x in toks[tpos:tpos + c]]); tpos += c
                        else:
                            cols[p[0]].append(float(toks[tpos])); tpos += 1
                data[el["name"]] = cols
            continue
        if not has_list:
            dt = np.dtype([(p[0], end + p[2]) for p in props])
            arr = np.frombuffer(body, dtype=dt, count=n, offset=off)
            off += dt.itemsize * n
            data[el["name"]] = {p[0]: arr[p[0]].astype(np.float64) for p in props}
            continue
        # list element: fast path when every list holds three entries (triangle meshes)
        fields = []
        for p in props:
            if p[1] == "list":
                fields += [(p[0] + ".count", end + p[2]), (p[0], end + p[3], (3,))]
            else:
                fields.append((p[0], end + p[2]))
        dt = np.dtype(fields)
        ok = n == 0 or off + dt.itemsize * n <= len(body)
        arr = np.frombuffer(body, dtype=dt, count=n, offset=off) if ok and n else None
        lists = [p for p in props if p[1] == "list"]
        if arr is None or any(np.any(arr[p[0] + ".count"] != 3) for p in lists):
            if el["name"] == "face":
                _fail("PLY", path, "incompatible contents -- is this a triangle mesh?")
            # skip a non-face list element generically
            for _ in range(n):
                for p in props:
                    if p[1] == "list":
                        c = int(np.frombuffer(body, end + p[2], 1, off)[0])
                        off += np.dtype(p[2]).itemsize + c * np.dtype(p[3]).itemsize
                    else:
                        off += np.dtype(p[2]).itemsize
            continue
        off += dt.itemsize * n
        data[el["name"]] = {p[0]: arr[p[0]] for p in props}
    if not ascii_ and off != len(body):
        _fail("PLY", path, "invalid file -- trailing content")

    vx = data.get("vertex")
    if vx is None or not all(k in vx for k in ("x", "y", "z")):
        _fail("PLY", path, "vertex element with x, y, z properties not found")
    P = np.stack([np.asarray(vx[k], np.float32) for k in ("x", "y", "z")], 1)
    if P.size and not np.all(np.isfinite(P)):
        _fail("PLY", path, "mesh contains invalid vertex position data")
    N = None
    if not face_normals and all(k in vx for k in ("nx", "ny", "nz")):
        N = np.stack([np.asarray(vx[k], np.float32) for k in ("nx", "ny", "nz")], 1)
    UV = None
    for a, b in (("u", "v"), ("texture_u", "texture_v"), ("s", "t")):
        if a in vx and b in vx:
            UV = np.stack([np.asarray(vx[a], np.float32), np.asarray(vx[b], np.float32)], 1)
            if flip_tex_coords:
                UV[:, 1] = np.float32(1.0) - UV[:, 1]
            break
    fc = data.get("face")
    F = np.zeros((0, 3), np.uint32)
    if fc is not None:
        key = "vertex_index" if "vertex_index" in fc else ("vertex_indices" if "vertex_indices" in fc else None)
        if key is None:
            _fail("PLY", path, "vertex_index/vertex_indices property not found")
        lst = fc[key]
        if isinstance(lst, list):
            if any(len(t) != 3 for t in lst):
                _fail("PLY", path, "incompatible contents -- is this a triangle mesh?")
        F = np.asarray(lst, np.int64).reshape(-1, 3).astype(np.uint32)
    return {"positions": P, "normals": N, "texcoords": UV, "faces": F,
            "recompute_normals": not face_normals and N is None}


def write_ply(path, positions, faces, normals=None, texcoords=None, binary: bool = True):
    P = np.asarray(positions, np.float32).reshape(-1, 3)
    F = np.asarray(faces, np.uint32).reshape(-1, 3)
    cols = [("x", P[:, 0]), ("y", P[:, 1]), ("z", P[:, 2])]
    if normals is not None:
        Nn = np.asarray(normals, np.float32).reshape(-1, 3)
        cols += [("nx", Nn[:, 0]), ("ny", Nn[:, 1]), ("nz", Nn[:, 2])]
    if texcoords is not None:
        T = np.asarray(texcoords, np.float32).reshape(-1, 2)
        cols += [("u", T[:, 0]), ("v", T[:, 1])]
    hdr = ["ply", "format %s 1.0" % ("binary_little_endian" if binary else "ascii"),
           f"element vertex {len(P)}"] + [f"property float {c[0]}" for c in cols] + \
          [f"element face {len(F)}", "property list uchar int vertex_indices", "end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(hdr) + "\n").encode("ascii"))
        if binary:
            vdt = np.dtype([(c[0], "<f4") for c in cols])
            va = np.empty(len(P), vdt)
            for c in cols:
                va[c[0]] = c[1]
            f.write(va.tobytes())
            fdt = np.dtype([("n", "u1"), ("i", "<i4", (3,))])
            fa = np.empty(len(F), fdt)
            fa["n"] = 3
            fa["i"] = F.astype(np.int32)
            f.write(fa.tobytes())
        else:
            for i in range(len(P)):
                f.write((" ".join("%.9g" % c[1][i] for c in cols) + "\n").encode())
            for t in F:
                f.write(("3 %d %d %d\n" % tuple(t)).encode())


# ---------------------------------------------------------------------------
# Mesh::recompute_vertex_normals (mesh.cpp:377-409, the JIT branch)
# ---------------------------------------------------------------------------
def recompute_vertex_normals(positions, faces) -> np.ndarray:
    V = np.asarray(positions, np.float32).reshape(-1, 3)
    F = np.asarray(faces, np.int64).reshape(-1, 3)
    v = [V[F[:, i]] for i in range(3)]

    def normalize(x):
        with np.errstate(invalid="ignore", divide="ignore"):
            return (x / np.sqrt((x * x).sum(1, dtype=np.float32))[:, None]).astype(np.float32)

    n = normalize(np.cross(v[1] - v[0], v[2] - v[0]).astype(np.float32))
    acc = np.zeros_like(V)
    for i in range(3):
        d0 = normalize(v[(i + 1) % 3] - v[i])
        d1 = normalize(v[(i + 2) % 3] - v[i])
        ang = np.arccos(np.clip((d0 * d1).sum(1, dtype=np.float32), -1.0, 1.0)).astype(np.float32)
        np.add.at(acc, F[:, i], n * ang[:, None])
    return normalize(acc)
