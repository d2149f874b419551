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
    from rtamd import scenes
    return scenes.CONFIGS[kind](**kw)
