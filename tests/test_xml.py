"""CPU: mi.load_file / load_string (src/core/xml.cpp)
for the hot path's plugins: the XML form of a scene loads to the same scene
as its dictionary form."""
import numpy as np
import pytest

import oracle_py as O


def _mi():
    import mitsuba_hip as mi
    mi.set_variant("hip_ad_rgb")
    return mi


CBOX_XML = """<scene version="3.0.0">
    <default name="spp" value="64"/>
    <default name="res" value="256"/>
    <integrator type="path">
        <integer name="max_depth" value="8"/>
    </integrator>
    <sensor type="perspective">
        <string name="fov_axis" value="smaller"/>
        <float name="near_clip" value="0.001"/>
        <float name="far_clip" value="100.0"/>
        <float name="fov" value="39.3077"/>
        <transform name="to_world">
            <lookat origin="0, 0, 3.90" target="0, 0, 0" up="0, 1, 0"/>
        </transform>
        <sampler type="independent">
            <integer name="sample_count" value="$spp"/>
        </sampler>
        <film type="hdrfilm">
            <integer name="width" value="$res"/>
            <integer name="height" value="$res"/>
            <rfilter type="gaussian"/>
        </film>
    </sensor>
    <bsdf type="diffuse" id="white"><rgb name="reflectance" value="0.885809, 0.698859, 0.666422"/></bsdf>
    <bsdf type="diffuse" id="green"><rgb name="reflectance" value="0.105421, 0.37798, 0.076425"/></bsdf>
    <bsdf type="diffuse" id="red"><rgb name="reflectance" value="0.570068, 0.0430135, 0.0443706"/></bsdf>
    <shape type="rectangle" id="light">
        <transform name="to_world">
            <scale x="0.23" y="0.19" z="0.19"/>
            <rotate x="1" angle="90"/>
            <translate x="0" y="0.99" z="0.01"/>
        </transform>
        <ref id="white"/>
        <emitter type="area"><rgb name="radiance" value="18.387, 13.9873, 6.75357"/></emitter>
    </shape>
    <shape type="rectangle" id="floor">
        <transform name="to_world"><rotate x="1" angle="-90"/><translate y="-1"/></transform>
        <ref id="white"/>
    </shape>
    <shape type="rectangle" id="ceiling">
        <transform name="to_world"><rotate x="1" angle="90"/><translate y="1"/></transform>
        <ref id="white"/>
    </shape>
    <shape type="rectangle" id="back">
        <transform name="to_world"><translate z="-1"/></transform>
        <ref id="white"/>
    </shape>
    <shape type="rectangle" id="green-wall">
        <transform name="to_world"><rotate y="1" angle="-90"/><translate x="1"/></transform>
        <ref id="green"/>
    </shape>
    <shape type="rectangle" id="red-wall">
        <transform name="to_world"><rotate y="1" angle="90"/><translate x="-1"/></transform>
        <ref id="red"/>
    </shape>
    <shape type="cube" id="small-box">
        <transform name="to_world"><scale value="0.3"/><rotate y="1" angle="-17"/><translate x="0.335" y="-0.7" z="0.38"/></transform>
        <ref id="white"/>
    </shape>
    <shape type="cube" id="large-box">
        <transform name="to_world"><scale x="0.3" y="0.61" z="0.3"/><rotate y="1" angle="18.25"/><translate x="-0.33" y="-0.4" z="-0.28"/></transform>
        <ref id="white"/>
    </shape>
</scene>
"""


def test_cornell_box_xml_equals_dict(tmp_path):
    mi = _mi()
    p = tmp_path / "cbox.xml"
    p.write_text(CBOX_XML)
    a = mi.load_file(str(p), spp=16, res=32)
    d = mi.cornell_box()
    d["sensor"]["film"]["width"] = d["sensor"]["film"]["height"] = 32
    d["sensor"]["sampler"]["sample_count"] = 16
    b = mi.load_dict(d)
    assert (a.width, a.height, a.sample_count()) == (32, 32, 16)
    assert a.integrator().max_depth == 8
    assert sorted(mi.traverse(a).keys()) == sorted(mi.traverse(b).keys())
    fa, fb = O.render(a, seed=3, spp=16), O.render(b, seed=3, spp=16)
    assert fa[..., :3].mean() > 0.05
    # the same scene up to float64 transform-product association (ulps)
    np.testing.assert_allclose(fa, fb, rtol=1e-4, atol=1e-5)


def test_volume_scene_xml(tmp_path):
    """prbvolpath + heterogeneous .vol medium + obj emitter + $parameters."""
    mi = _mi()
    from mitsuba_hip import meshio
    g = mi.fbm_grid(8)
    mi.VolumeGrid(g, (-1, -1, -1), (1, 1, 1)).write(tmp_path / "smoke.vol")
    V = np.array([[-1, 0, -1], [1, 0, -1], [1, 0, 1], [-1, 0, 1]], np.float32)
    meshio.write_obj(str(tmp_path / "lamp.obj"), V, np.array([[0, 2, 1], [0, 3, 2]], np.uint32))
    xml = """<scene version="3.0.0">
        <default name="g" value="0.5"/>
        <integrator type="prbvolpath"><integer name="max_depth" value="6"/></integrator>
        <sensor type="perspective">
            <float name="fov" value="39.3077"/>
            <transform name="to_world"><lookat origin="0, 0, 4" target="0, 0, 0" up="0, 1, 0"/></transform>
            <sampler type="independent"><integer name="sample_count" value="4"/></sampler>
            <film type="hdrfilm"><integer name="width" value="16"/><integer name="height" value="16"/></film>
        </sensor>
        <medium type="heterogeneous" id="smoke">
            <volume type="gridvolume" name="sigma_t">
                <string name="filename" value="smoke.vol"/>
                <boolean name="use_grid_bbox" value="true"/>
            </volume>
            <float name="scale" value="4"/>
            <rgb name="albedo" value="0.8"/>
            <phase type="hg"><float name="g" value="$g"/></phase>
        </medium>
        <shape type="cube">
            <bsdf type="null"/>
            <ref name="interior" id="smoke"/>
        </shape>
        <shape type="obj" id="lamp">
            <string name="filename" value="lamp.obj"/>
            <boolean name="face_normals" value="true"/>
            <transform name="to_world"><scale value="0.5"/><rotate x="1" angle="180"/><translate y="1.5"/></transform>
            <emitter type="area"><rgb name="radiance" value="8"/></emitter>
        </shape>
        <emitter type="constant"><rgb name="radiance" value="0.1"/></emitter>
    </scene>"""
    p = tmp_path / "vol.xml"
    p.write_text(xml)
    sc = mi.load_file(str(p), g=0.3)
    assert sc.integrator().type == "prbvolpath"
    keys = set(mi.traverse(sc).keys())
    assert {"smoke.sigma_t.data", "smoke.albedo.value"} <= keys
    assert sc.medium(0).g == pytest.approx(0.3)
    film = O.render(sc, seed=1, spp=4)
    assert np.isfinite(film).all() and film[..., :3].max() > 0


def test_xml_errors():
    mi = _mi()
    with pytest.raises(RuntimeError, match="undefined parameter"):
        mi.load_string('<scene version="3.0.0"><integrator type="path"><integer name="max_depth" value="$d"/>'
                       '</integrator></scene>')
    with pytest.raises(RuntimeError, match="not available"):
        mi.load_string('<scene version="3.0.0"><shape type="sphere"/></scene>')
