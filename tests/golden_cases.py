"""Scene factories of the golden fixtures (shared by tests/golden/make_golden.py
and tests/test_golden.py)."""
import math


def scene(rt, kind, kw):
    """(world, camera, depth) for a golden case; `rt` is the rtamd module."""
    if kind == "kat11":  # camera.rs:327-337
        w = rt.World.default()
        c = rt.Camera(11, 11, math.pi / 2.0)
        c.set_transform(rt.view_transform(rt.Point(0, 0, -5), rt.Point(0, 0, 0), rt.Vector(0, 1, 0)))
        return w, c, 5
    if kind == "yaml":  # scene-parser front-end, camera resized to (width, height)
        import os
        p = rt.SceneParser()
        p.load_file(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scenes", kw["file"]))
        c = rt.Camera(kw["width"], kw["height"], p.camera.field_of_view)
        c.set_transform(p.camera.transform)
        return p.build_world(), c, 5
    from rtamd import scenes
    return scenes.CONFIGS[kind](**kw)
