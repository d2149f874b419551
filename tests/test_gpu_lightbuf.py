"""Light buffer (DESIGN.md "Light buffer"): shadow rays answered from the
per-light cube-map cell lists must reproduce the exhaustive `is_shadowed`
(world.rs:95-105) bit for bit.

Every comparison renders the same world three ways: the fast path with the
light buffer (default), the fast path with the per-lane BVH shadow traversal
(`shadow_lb` off), and the counted launch (exhaustive loops, whose counters
equal the oracle's). The cases aim at the builder's and the query's edges:
cell resolutions from 1 to 512, lights inside and on spheres (records listed
in every cell), far origins beyond the validity radius (exhaustive fallback),
several lights, shadowless spheres, and a light far away.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
PI = math.pi


def _three(rt, make, lb_res=256):
    rt._rtamd._tuning_set("lb_res", lb_res)
    try:
        w, cam, depth = make(rt)
        prof_world = w
        fast, _ = cam.render(w, depth, want_stats=False)
        w.tune("shadow_lb", 0)
        try:
            bvh, _ = cam.render(w, depth, want_stats=False)
        finally:
            w.tune("shadow_lb", 1)
        exact, _ = cam.render(w, depth, want_stats=True)
        p = rt._rtamd._wf_profile(prof_world, -1, True)
    finally:
        rt._rtamd._tuning_set("lb_res", -1)  # (the default: by scene size)
    return fast.to_numpy(), bvh.to_numpy(), exact.to_numpy(), p


def _cluster(rt, light, n=300, seed=7, cam_from=(0, 2, -9), cam_to=(0, 1, 2), shadowless_every=0, lights=None,
             size=(96, 64)):
    rng = np.random.default_rng(seed)
    w = rt.World()
    floor = rt.Plane()
    floor.material.reflective = 0.3
    w.add_object(floor)
    for i in range(n):
        s = rt.glass_sphere() if i % 3 else rt.Sphere()
        r = rng.uniform(0.2, 0.9)
        c = rng.uniform([-3, r, -3], [3, 3, 3])
        s.set_transform(rt.translation(*c) * rt.scaling(r, r, r))
        s.material.reflective = rng.uniform(0, 0.9)
        s.material.color = rt.Color(*rng.uniform(0, 1, 3))
        if shadowless_every and i % shadowless_every == 0:
            s.no_shadow()
        w.add_object(s)
    for p in (lights or [light]):
        w.add_light(rt.PointLight(rt.Point(*p), rt.Color(1, 1, 1)))
    cam = rt.Camera(size[0], size[1], PI / 2.5)
    cam.set_transform(rt.view_transform(rt.Point(*cam_from), rt.Point(*cam_to), rt.Vector(0, 1, 0)))
    return w, cam, 5


@pytest.mark.parametrize("lb_res", [1, 3, 16, 128, 256, 512])
def test_lightbuf_c3_any_resolution(rt, lb_res):
    from rtamd import scenes
    fast, bvh, exact, p = _three(rt, lambda rt: scenes.c3(192, 108), lb_res)
    assert p["lb_res"] == lb_res and p["lb_items"] > 0
    assert fast.tobytes() == exact.tobytes()
    assert bvh.tobytes() == exact.tobytes()


@pytest.mark.parametrize("light", [(0.0, 1.5, 0.0), (0.3, 0.9, -0.2), (10, 10, -10), (-10, 10, -10)])
def test_lightbuf_light_inside_and_outside_cluster(rt, light):
    """A light among (and inside) overlapping spheres: records that contain
    or nearly touch the light are listed in every cell."""
    fast, bvh, exact, _ = _three(rt, lambda rt: _cluster(rt, light))
    assert fast.tobytes() == exact.tobytes()


def test_lightbuf_light_on_sphere_surface(rt):
    w_light = (1.0, 1.0, 0.0)

    def make(rt):
        w, cam, depth = _cluster(rt, w_light, n=120, seed=2)
        s = rt.Sphere()  # unit sphere at (0,1,0): the light sits on its surface
        s.set_transform(rt.translation(0, 1, 0))
        w.add_object(s)
        return w, cam, depth

    fast, _, exact, _ = _three(rt, make)
    assert fast.tobytes() == exact.tobytes()


def test_lightbuf_far_origins_take_exhaustive_path(rt):
    """Shadow-ray origins beyond the light's validity radius (2^24 x the
    nearest shadow-casting box's distance) test every sphere: a huge
    shadowless sphere 1e9 away fills the view behind the cluster, and its
    shadow rays cross the cluster on their way to the light."""

    def make(rt):
        w, _, depth = _cluster(rt, (0.0, 8.0, 0.0), n=150, seed=4)
        s = rt.Sphere()
        s.set_transform(rt.translation(0.0, 1.0, 1e9) * rt.scaling(3e8, 3e8, 3e8))
        s.no_shadow()
        w.add_object(s)
        cam = rt.Camera(128, 64, PI / 2.0)
        cam.set_transform(rt.view_transform(rt.Point(0, 2, -9), rt.Point(0, 1, 10), rt.Vector(0, 1, 0)))
        return w, cam, depth

    fast, _, exact, _ = _three(rt, make)
    assert fast.tobytes() == exact.tobytes()


def test_lightbuf_several_lights_and_shadowless(rt):
    lights = [(-10, 10, -10), (0.0, 1.2, 0.5), (5, 30, 5)]
    fast, _, exact, _ = _three(rt, lambda rt: _cluster(rt, None, n=250, seed=9, lights=lights, shadowless_every=4))
    assert fast.tobytes() == exact.tobytes()


def test_lightbuf_distant_light(rt):
    fast, _, exact, _ = _three(rt, lambda rt: _cluster(rt, (3e5, 4e5, -2e5), n=200, seed=12))
    assert fast.tobytes() == exact.tobytes()


def test_lightbuf_c5_slice(rt):
    """Four planes, 2 lights, 10 000 spheres (records stay in global memory)."""
    from rtamd import scenes
    fast, _, exact, p = _three(rt, lambda rt: scenes.c5(96, 96))
    assert p["lb_items"] > 0
    assert fast.tobytes() == exact.tobytes()


def test_lightbuf_color_at_batch_random_rays(rt):
    """Rays from everywhere (inside spheres, grazing, behind the light)."""
    rng = np.random.default_rng(1)
    o = rng.uniform([-4, -0.5, -4], [4, 4, 4], size=(20000, 3))
    d = rng.normal(size=(20000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.hstack([o, d])
    rt._rtamd._tuning_set("lb_res", 64)
    try:
        w, _, _ = _cluster(rt, (0.5, 2.0, 0.5), n=400, seed=5)
        for depth in (0, 1, 4):
            fast, _ = w.color_at_batch(rays, depth, want_stats=False)
            exact, _ = w.color_at_batch(rays, depth, want_stats=True)
            assert fast.tobytes() == exact.tobytes(), depth
        assert rt._rtamd._wf_profile(w, -1, True)["lb_res"] == 64
    finally:
        rt._rtamd._tuning_set("lb_res", -1)  # (the default: by scene size)


@pytest.mark.parametrize("own", [0, 1, 2])
def test_own_sphere_rules(rt, own):
    """The shadow rays of a hit on a sphere record (WfTuning::own_sphere,
    rt_trace.hpp shadow_trace): from inside (glass) that sphere is tested
    first; from outside, towards a light in front of the surface, it is left
    out. Ellipsoids; patterned spheres, whose shadow rays are traced with the
    light behind the surface (there the own sphere blocks: the rule keeps it,
    though lighting() then ignores the answer, so no frame can show it);
    lights level with the cluster, so many hits lie on a terminator
    (light . normal ~ 0); a sphere too large for the rule (semi-axis 5e3) and
    one too far (centre 2e6): the fast frame equals the exhaustive one."""

    def make(rt):
        w, cam, depth = _cluster(rt, None, n=160, seed=21, lights=[(40.0, 1.5, 0.3), (0.2, 1.4, -0.1), (-6, 9, -6)],
                                 size=(128, 96))
        rng = np.random.default_rng(3)
        for i in range(90):
            s = rt.Sphere() if i % 2 else rt.glass_sphere()
            c = rng.uniform([-3, 0.6, -3], [3, 3, 3])
            s.set_transform(rt.translation(*c) * rt.scaling(*rng.uniform(0.1, 0.6, 3)))
            if i % 3 == 0:
                s.material.set_pattern(rt.checkers_pattern(rt.Color(1, 0, 0), rt.Color(0, 0, 1)))
            w.add_object(s)
        big = rt.Sphere()
        big.set_transform(rt.translation(-5e3 - 4.0, 1.0, 0.0) * rt.scaling(5e3, 5e3, 5e3))
        w.add_object(big)
        far = rt.Sphere()
        far.set_transform(rt.translation(0.0, 1.0, 2e6) * rt.scaling(5e5, 5e5, 5e5))
        w.add_object(far)
        w.tune("own_sphere", own)
        return w, cam, depth

    fast, bvh, exact, _ = _three(rt, make)
    assert fast.tobytes() == exact.tobytes()
    assert bvh.tobytes() == exact.tobytes()
