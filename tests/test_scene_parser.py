"""YAML scene front-end: rtamd.SceneParser, the C++
restatement of scene-parser/src/lib.rs.

CPU: the reference's own tests (lib.rs:538-576) on its example files (copied
as data fixtures into tests/golden/scenes), YAML-subset and error-path cases,
and an independent Python restatement of the element semantics (PyYAML for
the syntax, this file's `restate()` for define / extend / transform order)
whose shapes must be byte-identical to the C++ parser's. GPU: parsed scenes
render like the oracle, and the render_scene CLI writes the same PPM.
"""
import math
import os
import subprocess

import numpy as np
import pytest
import yaml as pyyaml

from conftest import PKG

HERE = os.path.dirname(os.path.abspath(__file__))
SCENES = os.path.join(HERE, "golden", "scenes")
TOL = 1e-5


def _parse(rt, name):
    p = rt.SceneParser()
    p.load_file(os.path.join(SCENES, name))
    return p


# ---------------------------------------------------------------- reference tests
def test_load_file(rt):  # lib.rs:541-554
    p = _parse(rt, "reflect-refract.yml")
    assert p.camera is not None
    assert len(p.lights) == 1
    assert len(p.shapes) == 13
    assert len(p.materials) == 1


def test_load_other_file(rt):  # lib.rs:556-563
    p = _parse(rt, "cover.yml")
    assert p.camera is not None and p.camera.hsize == 4000
    assert len(p.lights) == 2 and len(p.shapes) == 19


def test_is_add_and_define_element(rt):  # lib.rs:565-576
    p = rt.SceneParser()
    p.load_str("- add: light\n  at: [1, 2, 3]\n  intensity: [1, 1, 1]\n- define: m\n  value:\n    ambient: 0.5\n")
    assert len(p.lights) == 1 and list(p.materials) == ["m"]


# ---------------------------------------------------- independent restatement
def restate(rt, text):
    """The scene semantics of scene-parser/src/lib.rs over PyYAML's parse."""
    doc = pyyaml.safe_load(text)
    mats, tfs, shapes, lights, cam = {}, {}, [], [], None

    def f64(v):
        assert isinstance(v, (int, float)) and not isinstance(v, bool)
        return float(v)

    def tf(items):
        m = rt.Matrix.identity(4, 4)
        for it in items:
            if isinstance(it, str):
                x = tfs[it]
            else:
                k, a = it[0], [f64(v) for v in it[1:]]
                x = {"scale": lambda: rt.scaling(*a[:3]), "translate": lambda: rt.translation(*a[:3]),
                     "rotate-x": lambda: rt.rotation_x(a[0]), "rotate-y": lambda: rt.rotation_y(a[0]),
                     "rotate-z": lambda: rt.rotation_z(a[0])}[k]()
            m = x * m
        return m

    def color(v):
        return rt.Color(*[f64(x) for x in v])

    def material(base, d):
        m = base
        if "color" in d:
            m.color = color(d["color"])
        if "pattern" in d:
            p = d["pattern"]
            cs = [color(c) for c in p["colors"]]
            pat = {"stripes": lambda: rt.stripe_pattern(cs[0], cs[1]),
                   "checkers": lambda: rt.checkers_pattern(cs[0], cs[1])}.get(p["type"], rt.test_pattern)()
            m.set_pattern(pat)  # the pattern's `transform` key is ignored (lib.rs:450-486)
        for key, attr in (("ambient", "ambient"), ("diffuse", "diffuse"), ("specular", "specular"),
                          ("shininess", "shininess"), ("reflective", "reflective"),
                          ("transparency", "transparency"), ("refractive-index", "refractive_index")):
            if key in d:
                setattr(m, attr, f64(d[key]))
        return m

    for el in doc:
        if isinstance(el, dict) and "define" in el:
            v = el["value"]
            if isinstance(v, list):
                tfs[el["define"]] = tf(v)
            else:
                base = mats[el["extend"]].copy() if "extend" in el else rt.Material()
                mats[el["define"]] = material(base, v)
    for el in doc:
        if not (isinstance(el, dict) and "add" in el):
            continue
        k = el["add"]
        if k == "camera":
            cam = (el["width"], el["height"], el["field-of-view"], el["from"], el["to"], el["up"])
        elif k == "light":
            lights.append((el["at"], el["intensity"]))
        elif k in ("sphere", "plane", "cube"):
            s = {"sphere": rt.Sphere, "plane": rt.Plane, "cube": rt.Cube}[k]()
            if "transform" in el:
                s.set_transform(tf(el["transform"]))
            if "material" in el:
                m = el["material"]
                s.material = mats[m].copy() if isinstance(m, str) else material(rt.Material(), m)
            shapes.append(s)
    return cam, lights, shapes


@pytest.mark.parametrize("name", ["reflect-refract.yml", "cover.yml"])
def test_parser_matches_independent_restatement(rt, name):
    text = open(os.path.join(SCENES, name)).read()
    p = rt.SceneParser()
    p.load_str(text)
    cam, lights, shapes = restate(rt, text)
    assert [s.desc_bytes() for s in p.shapes] == [s.desc_bytes() for s in shapes]
    assert len(p.lights) == len(lights)
    for got, (at, inten) in zip(p.lights, lights):
        assert got.position.tuple() == tuple(float(x) for x in at)
        assert (got.intensity.red, got.intensity.green, got.intensity.blue) == tuple(float(x) for x in inten)
    w, h, fov, frm, to, up = cam
    c = rt.Camera(w, h, fov)
    c.set_transform(rt.view_transform(rt.Point(*map(float, frm)), rt.Point(*map(float, to)),
                                      rt.Vector(*map(float, up))))
    assert p.camera.desc_bytes() == c.desc_bytes()


# ------------------------------------------------------------- YAML subset
def test_yaml_subset_and_scalar_resolution(rt):
    text = """
# comment line
- define: base   # trailing comment
  value: {ambient: 0.25, diffuse: 1}
- define: t
  value:
  - [translate, 1, 0x2, +3]
  - ['rotate-y', 1e-1]
- add: "sphere"
  material: base
  transform:
    - t
    - [scale, .5, 2., 1]
---
- add: plane
"""
    p = rt.SceneParser()
    p.load_str(text)
    assert len(p.shapes) == 1  # first document only
    m = p.shapes[0].material
    assert (m.ambient, m.diffuse) == (0.25, 1.0)
    want = rt.scaling(0.5, 2.0, 1.0) * (rt.rotation_y(0.1) * rt.translation(1, 2, 3))
    s = rt.Sphere()
    s.set_transform(want)
    assert p.shapes[0].desc_bytes()[:8 + 256] == s.desc_bytes()[:8 + 256]


@pytest.mark.parametrize("text,err", [
    ("- add: camera\n  width: 10\n  height: 10\n  field-of-view: 1\n  from: [0,0,0]\n  to: [0,0,1]\n  up: [0,1,0]\n",
     "failed to parse `field-of-view` as f64"),  # yaml-rust as_f64: Integer is not a Real
    ("- add: camera\n  width: 10\n  height: 10\n  field-of-view: 1.0\n  to: [0,0,1]\n  up: [0,1,0]\n",
     "missing required key `from`"),
    ("- add: sphere\n  material: nope\n", "failed to parse material"),
    ("- add: sphere\n  transform:\n    - [shear, 1, 2, 3]\n", "failed to parse transform"),
    ("- define: x\n  extend: missing\n  value: {ambient: 1}\n", "invalid define element found"),
    ("- add: [1, 2]\n", "invalid add element found"),
    ("add: sphere\n", "invalid input file"),
])
def test_parser_errors(rt, text, err):
    p = rt.SceneParser()
    with pytest.raises(rt.SceneParserError, match=err.replace("`", ".").replace("(", ".").replace(")", ".")):
        p.load_str(text)


def test_unhandled_kinds_are_skipped(rt):  # lib.rs:134
    p = rt.SceneParser()
    p.load_str("- add: cylinder\n  min: 0\n- add: group\n- add: cube\n")
    assert len(p.shapes) == 1 and p.messages == ["unhandled element: cylinder", "unhandled element: group"]


def test_pattern_kinds(rt):
    p = rt.SceneParser()
    p.load_str("- add: sphere\n  material:\n    pattern:\n      type: rings\n      colors: [[1,0,0],[0,1,0]]\n"
               "- add: cube\n  material:\n    pattern: {type: stripes, colors: [[1,0,0],[0,1,0]], "
               "transform: [[scale, 2, 2, 2]]}\n")
    assert p.shapes[0].material.pattern.kind == 0   # Pattern::default() = test pattern
    pat = p.shapes[1].material.pattern
    assert pat.kind == 1 and pat.transform.to_list() == rt.Matrix.identity(4, 4).to_list()


def test_render_scene_cli_usage():
    exe = os.path.join(PKG, "bin", "render_scene")
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "usage: render_scene" in r.stdout


# --------------------------------------------------------------------- GPU
def _small_camera(rt, p, w, h):
    c = rt.Camera(w, h, p.camera.field_of_view)
    c.set_transform(p.camera.transform)
    return c


@pytest.mark.gpu
@pytest.mark.parametrize("name,w,h", [("reflect-refract.yml", 256, 144), ("cover.yml", 160, 160)])
def test_parsed_scene_renders_like_oracle(rt, oracle, name, w, h):
    p = _parse(rt, name)
    world = p.build_world()
    cam = _small_camera(rt, p, w, h)
    canvas, st = cam.render(world, 5)
    g = canvas.to_numpy()
    ref, rst = oracle.OracleWorld.from_world(world).render(cam.desc_bytes(), 5, nthreads=16)
    assert np.abs(g - ref).max() <= TOL
    assert rt.canvas_to_ppm(g) == oracle.canvas_to_ppm(ref)
    for k in rst:
        assert st[k] == rst[k], k


@pytest.mark.gpu
def test_render_scene_cli_writes_the_ppm(rt, oracle, tmp_path):
    text = open(os.path.join(SCENES, "reflect-refract.yml")).read().replace("width: 2560", "width: 96") \
        .replace("height: 1440", "height: 54")
    src = tmp_path / "scene.yml"
    src.write_text(text)
    out = tmp_path / "scene.ppm"
    exe = os.path.join(PKG, "bin", "render_scene")
    r = subprocess.run([exe, str(src), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    p = rt.SceneParser()
    p.load_str(text)
    ref, _ = oracle.OracleWorld.from_world(p.build_world()).render(p.camera.desc_bytes(), 5, nthreads=16)
    assert out.read_bytes() == oracle.canvas_to_ppm(ref)
