"""CPU: film output formats: OpenEXR / PFM / PNG
writers and readers, and hdrfilm's luminance / xyz develop
(hdrfilm.cpp:313-401, spectrum.h:396-434)."""
import struct

import numpy as np
import pytest

import oracle_py as O


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


@pytest.mark.parametrize("compression", ["none", "zips", "zip"])
@pytest.mark.parametrize("half", [False, True])
def test_exr_roundtrip(tmp_path, compression, half):
    from mitsuba_hip import imageio
    rng = np.random.default_rng(0)
    img = (rng.random((37, 29, 3)) * 10).astype(np.float32)
    img[0, 0] = [0.0, 1e-3, 65000.0]
    p = tmp_path / "a.exr"
    imageio.write_exr(p, img, half=half, compression=compression)
    b = p.read_bytes()
    assert struct.unpack("<ii", b[:8]) == (20000630, 2)
    for attr in (b"channels\0chlist\0", b"compression\0compression\0", b"dataWindow\0box2i\0",
                 b"displayWindow\0box2i\0", b"lineOrder\0lineOrder\0", b"pixelAspectRatio\0float\0",
                 b"screenWindowCenter\0v2f\0", b"screenWindowWidth\0float\0"):
        assert attr in b
    out, names = imageio.read_exr(p)
    assert names == ["B", "G", "R"]               # alphabetical, as the format stores them
    rgb = out[..., [2, 1, 0]]
    want = img.astype(np.float16).astype(np.float32) if half else img
    np.testing.assert_array_equal(rgb, want)
    if compression != "none":   # smooth images compress (random mantissas do not)
        sm = np.broadcast_to(np.linspace(0, 1, 64, dtype=np.float32)[None, :, None], (48, 64, 3)).copy()
        imageio.write_exr(tmp_path / "s.exr", sm, half=half, compression=compression)
        assert (tmp_path / "s.exr").stat().st_size < sm.nbytes // (4 if half else 2)
        np.testing.assert_array_equal(imageio.read_exr(tmp_path / "s.exr")[0][..., [2, 1, 0]],
                                      sm.astype(np.float16).astype(np.float32) if half else sm)


def test_pfm_and_png(tmp_path):
    from mitsuba_hip import imageio
    from PIL import Image
    rng = np.random.default_rng(1)
    img = rng.random((9, 13, 3)).astype(np.float32)
    imageio.write_pfm(tmp_path / "a.pfm", img)
    np.testing.assert_array_equal(imageio.read_pfm(tmp_path / "a.pfm"), img)
    y = img[..., :1]
    imageio.write_pfm(tmp_path / "y.pfm", y)
    np.testing.assert_array_equal(imageio.read_pfm(tmp_path / "y.pfm"), y)
    imageio.write_png(tmp_path / "a.png", img)
    q = np.asarray(Image.open(tmp_path / "a.png"))
    assert q.shape == (9, 13, 3) and q.dtype == np.uint8
    np.testing.assert_array_equal(q, np.clip(np.round(imageio.linear_to_srgb(img) * 255), 0, 255))
    back = imageio.read_bitmap(tmp_path / "a.png")
    np.testing.assert_allclose(back, img, atol=0.01)


@pytest.mark.parametrize("pf", ["luminance", "xyz"])
def test_develop_pixel_formats(pf):
    mi = _mi()
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 16
    d["sensor"]["film"]["pixel_format"] = pf
    sc = mi.load_dict(d)
    film = O.render(sc, seed=0, spp=4)
    rgb = O.develop(film, 0).astype(np.float64)
    out = O.develop(film, sc.desc.sensor.pixel_format)
    M = np.array([[0.412453, 0.357580, 0.180423], [0.212671, 0.715160, 0.072169],
                  [0.019334, 0.119193, 0.950227]])
    want = rgb @ M.T
    if pf == "luminance":
        assert out.shape == (16, 16, 1)
        want = want[..., 1:2]
    np.testing.assert_allclose(out, want, rtol=1e-5, atol=1e-7)
    with pytest.raises(RuntimeError, match="pixel_format"):
        d["sensor"]["film"]["pixel_format"] = "rgbe"
        mi.load_dict(d)


def test_bitmap_texture_from_file(tmp_path):
    """bitmap 'filename' (EXR) loads the same texels as the in-memory tensor."""
    mi = _mi()
    from mitsuba_hip import imageio
    tex = np.random.default_rng(2).random((8, 8, 3)).astype(np.float32)
    imageio.write_exr(tmp_path / "t.exr", tex)
    a = mi.load_dict(mi.cornell_box_bitmap(tex_res=8, width=16, height=16, spp=4))
    d = mi.cornell_box_bitmap(tex_res=8, width=16, height=16, spp=4)
    spec = d["white"]["reflectance"]
    spec.pop("data")
    spec["filename"] = str(tmp_path / "t.exr")
    b = mi.load_dict(d)
    assert b.texture_data(mi.traverse(b).texture_of("white.reflectance.data")).shape == (8 * 8 * 3,)
    np.testing.assert_array_equal(b.texture_data(mi.traverse(b).texture_of("white.reflectance.data")),
                                  tex.reshape(-1))
