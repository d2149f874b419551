"""Groups and their bounding boxes (geometry/shape/group.rs, bounding_box.rs).

CPU: the host builder's BoundingBox and Group restate the reference's own unit
tests (bounding_box.rs:187-507, group.rs:215-391, cylinder/cone/plane boxes),
and the flattened hierarchy the device receives (groups_bytes / shape_groups)
has the reference's shape: parents before children, every member gated by its
innermost group. GPU: frames of grouped scenes (the hexagon demo, the feature
scene `groups`, a divided lattice) match the oracle within 1e-5 with the same
PPM bytes and exact counters, the uncounted fast path equals the counted one
bit for bit, and row-block shards reassemble exactly.
"""
import math

import numpy as np
import pytest

SQRT_2 = math.sqrt(2.0)
INF = math.inf


def _p(rt, *xyz):
    return rt.Point(*[float(v) for v in xyz])


def _box(rt, lo, hi):
    return rt.BoundingBox(_p(rt, *lo), _p(rt, *hi))


def _xyz(p):
    return (p.x, p.y, p.z)


# --- bounding_box.rs ---------------------------------------------------------

def test_default_box_is_empty(rt):  # :187-197
    bb = rt.BoundingBox()
    assert _xyz(bb.min) == (INF, INF, INF)
    assert _xyz(bb.max) == (-INF, -INF, -INF)


def test_add_points_and_boxes(rt):  # :206-228
    bb = rt.BoundingBox()
    bb.add_point(_p(rt, -5, 2, 0))
    bb.add_point(_p(rt, 7, 0, -3))
    assert _xyz(bb.min) == (-5, 0, -3) and _xyz(bb.max) == (7, 2, 0)
    b1 = _box(rt, (-5, -2, 0), (7, 4, 4))
    b1.add_bounding_box(_box(rt, (8, -7, -2), (14, 2, 8)))
    assert _xyz(b1.min) == (-5, -7, -2) and _xyz(b1.max) == (14, 4, 8)


def test_contains(rt):  # :230-264
    bb = _box(rt, (5, -2, 0), (11, 4, 7))
    for p, want in [((5, -2, 0), True), ((11, 4, 7), True), ((8, 1, 3), True), ((3, 0, 3), False),
                    ((8, -4, 3), False), ((8, 1, -1), False), ((13, 1, 3), False), ((8, 5, 3), False),
                    ((8, 1, 8), False)]:
        assert bb.contains_point(_p(rt, *p)) == want, p
    for lo, hi, want in [((5, -2, 0), (11, 4, 7), True), ((6, -1, 1), (10, 3, 6), True),
                         ((4, -3, -1), (10, 3, 6), False), ((6, -1, 1), (12, 5, 8), False)]:
        assert bb.contains_bounding_box(_box(rt, lo, hi)) == want
    assert not bb.contains_point(_p(rt, math.nan, 0, 3))  # RangeInclusive::contains(NaN)


def test_transform_box(rt):  # :266-274
    bb = _box(rt, (-1, -1, -1), (1, 1, 1)).transform(rt.rotation_x(math.pi / 4) * rt.rotation_y(math.pi / 4))
    assert bb.min == rt.Point(-SQRT_2, -1.70711, -1.70711)
    assert bb.max == rt.Point(SQRT_2, 1.70711, 1.70711)


def test_parent_space_bounds(rt):  # :276-284
    s = rt.Sphere()
    s.set_transform(rt.translation(1, -3, 5) * rt.scaling(0.5, 2.0, 4.0))
    bb = s.parent_space_bounds()
    assert bb.min == rt.Point(0.5, -5.0, 1.0) and bb.max == rt.Point(1.5, -1.0, 9.0)


@pytest.mark.parametrize("lo,hi,cases", [
    ((-1, -1, -1), (1, 1, 1), [  # :286-327
        ((5, 0.5, 0), (-1, 0, 0), True), ((-5, 0.5, 0), (1, 0, 0), True), ((0.5, 5, 0), (0, -1, 0), True),
        ((0.5, -5, 0), (0, 1, 0), True), ((0.5, 0, 5), (0, 0, -1), True), ((0.5, 0, -5), (0, 0, 1), True),
        ((0, 0.5, 0), (0, 0, 1), True), ((-2, 0, 0), (2, 4, 6), False), ((0, -2, 0), (6, 2, 4), False),
        ((0, 0, -2), (4, 6, 2), False), ((2, 0, 2), (0, 0, -1), False), ((0, 2, 2), (0, -1, 0), False),
        ((2, 2, 0), (-1, 0, 0), False)]),
    ((5, -2, 0), (11, 4, 7), [  # :329-370
        ((15, 1, 2), (-1, 0, 0), True), ((-5, -1, 4), (1, 0, 0), True), ((7, 6, 5), (0, -1, 0), True),
        ((9, -5, 6), (0, 1, 0), True), ((8, 2, 12), (0, 0, -1), True), ((6, 0, -5), (0, 0, 1), True),
        ((8, 1, 3.5), (0, 0, 1), True), ((9, -1, -8), (2, 4, 6), False), ((8, 3, -4), (6, 2, 4), False),
        ((9, -1, -2), (4, 6, 2), False), ((4, 0, 9), (0, 0, -1), False), ((8, 6, -1), (0, -1, 0), False),
        ((12, 5, 4), (-1, 0, 0), False)]),
])
def test_ray_box_intersects(rt, lo, hi, cases):
    bb = _box(rt, lo, hi)
    for o, d, want in cases:
        r = rt.Ray(_p(rt, *o), rt.Vector(*[float(v) for v in d]).normalize())
        assert bb.intersects(r) == want, (o, d)


@pytest.mark.parametrize("lo,hi,left_hi,right_lo", [  # :455-501
    ((-1, -4, -5), (9, 6, 5), (4, 6, 5), (4, -4, -5)),
    ((-1, -2, -3), (9, 5.5, 3), (4, 5.5, 3), (4, -2, -3)),
    ((-1, -2, -3), (5, 8, 3), (5, 3, 3), (-1, 3, -3)),
    ((-1, -2, -3), (5, 3, 7), (5, 3, 2), (-1, -2, 2)),
])
def test_split(rt, lo, hi, left_hi, right_lo):
    left, right = _box(rt, lo, hi).split()
    assert _xyz(left.min) == lo and _xyz(left.max) == left_hi
    assert _xyz(right.min) == right_lo and _xyz(right.max) == hi


def test_primitive_boxes(rt):
    """Per-kind boxes: sphere/cube unit box, plane infinite in x and z
    (plane.rs), cylinder (cylinder.rs:30-33), cone's limit (cone.rs:29-31)."""
    assert (_xyz(rt.Sphere().get_bounds().min), _xyz(rt.Cube().get_bounds().max)) == ((-1, -1, -1), (1, 1, 1))
    pb = rt.Plane().get_bounds()
    assert _xyz(pb.min) == (-INF, 0, -INF) and _xyz(pb.max) == (INF, 0, INF)
    cb = rt.Cylinder(-2.0, 3.0, True).get_bounds()
    assert _xyz(cb.min) == (-1, -2, -1) and _xyz(cb.max) == (1, 3, 1)
    kb = rt.Cone(-5.0, 3.0, False).get_bounds()
    assert _xyz(kb.min) == (-5, -5, -5) and _xyz(kb.max) == (5, 3, 5)
    ib = rt.Cylinder().get_bounds()
    assert _xyz(ib.min) == (-1, -INF, -1) and _xyz(ib.max) == (1, INF, 1)


def test_plane_box_under_transform_is_empty(rt):
    """A plane's box through set_transform multiplies 0 by its infinite corners:
    every corner has a NaN coordinate, which add_point never takes, so the box
    comes out empty (the reference's quirk that makes a group holding a plane
    see it only through its other children's boxes)."""
    for m in (rt.translation(0, 1, 0), rt.rotation_z(0.5)):
        p = rt.Plane()
        p.set_transform(m)
        b = p.get_bounds()
        assert _xyz(b.min) == (INF, INF, INF) and _xyz(b.max) == (-INF, -INF, -INF)


# --- group.rs ------------------------------------------------------------------

def test_create_group_and_add_child(rt):  # :215-229
    g = rt.Group()
    assert g.n_children() == 0 and g.transform == rt.Matrix.identity(4, 4)
    g.add_child(rt.Sphere())
    assert g.n_children() == 1


def test_group_box_contains_children(rt):  # :280-297
    s = rt.Sphere()
    s.set_transform(rt.translation(2, 5, -3) * rt.scaling(2, 2, 2))
    c = rt.Cylinder(-2.0, 2.0, False)
    c.set_transform(rt.translation(-4, -1, 4) * rt.scaling(0.5, 1.0, 0.5))
    g = rt.Group()
    g.add_child(s)
    g.add_child(c)
    bb = g.get_bounds()
    assert bb.min == rt.Point(-4.5, -3.0, -5.0) and bb.max == rt.Point(4.0, 7.0, 4.5)


def test_transform_is_baked_into_children(rt):  # group.rs:71-94,128-133
    g = rt.Group()
    g.set_transform(rt.scaling(2, 2, 2))
    s = rt.Sphere()
    s.set_transform(rt.translation(5, 0, 0))
    g.add_child(s)
    assert g.child(0).transform == rt.scaling(2, 2, 2) * rt.translation(5, 0, 0)
    g.set_transform(rt.translation(0, 1, 0))  # undo the scaling, apply the translation
    assert g.child(0).transform == rt.translation(0, 1, 0) * rt.translation(5, 0, 0)


def test_groups_own_their_children(rt):
    """add_child takes the group (Box<dyn Shape>, group.rs:128-133): a group added
    to another, then transformed through its parent, leaves the caller's object
    as it was; child(i) hands out a copy."""
    inner = rt.Group()
    s = rt.Sphere()
    s.set_transform(rt.translation(1, 0, 0))
    inner.add_child(s)
    outer = rt.Group()
    outer.add_child(inner)
    outer.set_transform(rt.scaling(2, 2, 2))
    assert inner.child(0).transform == rt.translation(1, 0, 0)
    assert outer.child(0).child(0).transform == rt.scaling(2, 2, 2) * rt.translation(1, 0, 0)
    c = outer.child(0)
    c.set_transform(rt.translation(0, 5, 0))
    assert outer.child(0).child(0).transform == rt.scaling(2, 2, 2) * rt.translation(1, 0, 0)


def test_set_material_recurses(rt):  # group.rs:96-102
    inner = rt.Group()
    inner.add_child(rt.Sphere())
    outer = rt.Group()
    outer.add_child(inner)
    outer.add_child(rt.Cube())
    m = rt.Material()
    m.reflective = 0.75
    outer.set_material(m)
    assert outer.child(0).child(0).material.reflective == 0.75
    assert outer.child(1).material.reflective == 0.75


def test_subdividing_partitions_children(rt):  # group.rs:348-391
    s1, s2, s3 = rt.Sphere(), rt.Sphere(), rt.Sphere()
    s1.set_transform(rt.translation(-2, -2, 0))
    s2.set_transform(rt.translation(-2, 2, 0))
    s3.set_transform(rt.scaling(4, 4, 4))
    g = rt.Group()
    for s in (s1, s2, s3):
        g.add_child(s)
    g.divide(1)
    assert g.n_children() == 2
    assert g.child(0).transform == rt.scaling(4, 4, 4)
    sub = g.child(1)
    assert isinstance(sub, rt.Group) and sub.n_children() == 2
    assert sub.child(0).child(0).transform == rt.translation(-2, -2, 0)
    assert sub.child(1).child(0).transform == rt.translation(-2, 2, 0)


def test_divide_below_threshold_is_a_no_op(rt):  # group.rs:108-122
    g = rt.Group()
    for x in (-2, 2):
        s = rt.Sphere()
        s.set_transform(rt.translation(x, 0, 0))
        g.add_child(s)
    g.divide(3)
    assert g.n_children() == 2 and all(isinstance(g.child(i), rt.Shape) for i in range(2))
    g.divide(2)  # partition_children (group.rs:299-327): one per half
    assert g.n_children() == 2 and all(isinstance(g.child(i), rt.Group) for i in range(2))


def test_flattened_hierarchy(rt):
    """World.groups_bytes / shape_groups: groups in DFS order, parents first
    (rt_group_desc.parent < own index, -1 for a root), each shape tagged with its
    innermost group (-1 for an ungrouped one); the boxes are the host's."""
    from rtamd import scenes
    w, _, _ = scenes.divided(16, 9)
    gb = w.groups_bytes()
    assert len(gb) % 56 == 0
    n = len(gb) // 56
    boxes = np.frombuffer(gb, dtype=np.float64).reshape(n, 7)[:, :6]
    par = np.frombuffer(gb, dtype=np.int32).reshape(n, 14)[:, 12]
    assert par[0] == -1 and all(-1 <= p < i for i, p in enumerate(par))
    sg = w.shape_groups()
    assert sg[0] == -1 and all(0 <= g < n for g in sg[1:])
    for i, p in enumerate(par):  # a child group's box lies inside its parent's
        if p >= 0:
            assert (boxes[i, :3] >= boxes[p, :3] - 1e-9).all() and (boxes[i, 3:] <= boxes[p, 3:] + 1e-9).all()


def _normal_on_child_world(rt):
    """geometry/mod.rs:126-150: a sphere translated by (5, 0, 0) inside a group
    scaled by (1, 2, 3) inside a group rotated by pi/2 about y."""
    g1 = rt.Group()
    g1.set_transform(rt.rotation_y(math.pi / 2.0))
    g2 = rt.Group()
    g2.set_transform(rt.scaling(1, 2, 3))
    s = rt.Sphere()
    s.set_transform(rt.translation(5, 0, 0))
    g2.add_child(s)
    g1.add_child(g2)
    w = rt.World()
    w.add_object(g1)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    return w


NORMAL_KAT = ((1.7321, 1.1547, -5.5774), (0.2857, 0.42854, -0.85716))  # geometry/mod.rs:148-153


def test_normal_on_child_object_oracle(rt, oracle):
    """The transforms baked into a nested group's member give the reference's
    normal (geometry/mod.rs:126-153): a ray cast at the KAT's point along the
    KAT's normal hits there and prepare_computations returns that normal."""
    w = _normal_on_child_world(rt)
    p, n = (np.array(v) for v in NORMAL_KAT)
    h = oracle.OracleWorld.from_world(w).hit(p + 2.0 * n, -n)
    assert h[0] == 0
    assert np.abs(h[2:5] - p).max() < 1e-3 and np.abs(h[14:17] - n).max() < 1e-3


@pytest.mark.gpu
def test_gpu_group_hits_bitwise_vs_oracle(rt, oracle):
    """World::intersect + hit + prepare_computations through group gates: the
    KAT's nested-group normal, and random rays through the groups scene, bitwise
    equal to the oracle (geometry exact; schlick within 1e-12)."""
    w = _normal_on_child_world(rt)
    p, n = (np.array(v) for v in NORMAL_KAT)
    ray = np.array([list(p + 2.0 * n) + list(-n)])
    g = w.hit_batch(ray)
    ref = oracle.OracleWorld.from_world(w).hit(ray[0, :3], ray[0, 3:])
    assert np.array_equal(g[0, :23], ref[:23])
    from rtamd import scenes
    rng = np.random.default_rng(5)
    for make in (lambda: scenes.groups(32, 24), lambda: scenes.divided(32, 18), lambda: scenes.hexagon(32, 18)):
        w, _, _ = make()
        ow = oracle.OracleWorld.from_world(w)
        k = 3000
        o = rng.uniform([-3, 0.05, -6], [3, 3, 3], size=(k, 3))
        d = rng.normal(size=(k, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays = np.hstack([o, d])
        g = w.hit_batch(rays)
        ref = np.array([ow.hit(r[:3], r[3:]) for r in rays])
        hits = ref[:, 0] >= 0
        assert hits.sum() > 50
        assert np.array_equal(g[:, 0], ref[:, 0])
        assert np.array_equal(g[hits, 1:23], ref[hits, 1:23])
        assert np.abs(g[hits, 23] - ref[hits, 23]).max() <= 1e-12


# --- GPU -------------------------------------------------------------------------

TOL = 1e-5
GROUP_SCENES = [("hexagon", {"width": 160, "height": 90}), ("groups", {"width": 120, "height": 90}),
                ("divided", {"width": 128, "height": 72})]


def _gpu_vs_oracle(rt, oracle, w, cam, depth, rows=None, aa=1):
    if aa == 1:
        canvas, st = cam.render(w, depth)
    else:
        cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
        canvas, st = cam.render_multithreaded(w, depth)
    g = canvas.to_numpy()
    rows = list(range(cam.vsize)) if rows is None else rows
    ref, rst = oracle.OracleWorld.from_world(w).render_rows(cam.desc_bytes(), depth, rows, 8, aa_samples=aa)
    assert np.isfinite(g).all()
    assert np.abs(g[rows] - ref).max() <= TOL
    assert rt.canvas_to_ppm(g[rows]) == oracle.canvas_to_ppm(ref)
    if len(rows) == cam.vsize:
        for k in ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow",
                  "sphere_tests", "plane_tests", "sphere_disc_ge0", "other_tests"):
            assert st[k] == rst[k], (k, st[k], rst[k])
    return g


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kw", GROUP_SCENES)
def test_gpu_group_scene_vs_oracle(rt, oracle, kind, kw):
    from rtamd import scenes
    w, cam, depth = scenes.CONFIGS[kind](**kw)
    _gpu_vs_oracle(rt, oracle, w, cam, depth)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kw", GROUP_SCENES)
def test_gpu_group_fast_equals_counted(rt, kind, kw):
    from rtamd import scenes
    w, cam, depth = scenes.CONFIGS[kind](**kw)
    fast, _ = cam.render(w, depth, want_stats=False)
    exact, _ = cam.render(w, depth, want_stats=True)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()


@pytest.mark.gpu
def test_gpu_hexagon_full_size_sampled_rows(rt, oracle):
    """The demo at its own size (bin/hexagon.rs: 2560x1440), oracle on a spread of rows."""
    from rtamd import scenes
    w, cam, depth = scenes.hexagon()
    _gpu_vs_oracle(rt, oracle, w, cam, depth, rows=[0, 500, 640, 720, 811, 900, 1439])


@pytest.mark.gpu
def test_gpu_groups_aa(rt, oracle):
    from rtamd import scenes
    w, cam, depth = scenes.groups(48, 36)
    _gpu_vs_oracle(rt, oracle, w, cam, depth, aa=4)


@pytest.mark.gpu
def test_gpu_group_shards_reassemble(rt):
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.divided(160, 90)
    full = cam.render(w, depth)[0].to_numpy()
    n_shards, block = 3, 8
    out = np.zeros_like(full)
    for s in range(n_shards):
        rows = rt.shard_rows(cam.vsize, block, s, n_shards)
        buf = torch.empty((rows, cam.hsize, 3), dtype=torch.float64, device="cuda")
        cam.render_shard_device(w, depth, block, s, n_shards, buf.data_ptr(),
                                torch.cuda.current_stream().cuda_stream, False)
        torch.cuda.synchronize()
        ys = [y for y in range(cam.vsize) if (y // block) % n_shards == s]
        out[ys] = buf.cpu().numpy()
    assert out.tobytes() == full.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kw", GROUP_SCENES)
def test_gpu_group_counted_fast_path_counters(rt, kind, kw):
    """Grouped shapes sit in the fast path's hierarchies with their group gate
    tested at the leaf; a counted fast-path render still reports the
    reference's ray and shape-test counts (the gates each ray met, counted
    over every grouped record), equal to the exhaustive loop's."""
    from rtamd import scenes
    w, cam, depth = scenes.CONFIGS[kind](**kw)
    exact, se = cam.render(w, depth, want_stats=True)
    fast, sf = cam.render(w, depth, want_stats=True, exhaustive=False)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()
    for k in ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "plane_tests",
              "other_tests"):
        if sf.get(k) is not None:
            assert sf[k] == se[k], k


@pytest.mark.gpu
def test_gpu_divided_group_is_culled(rt):
    """A Group::divide'd lattice of 12 x 12 x 2 shapes (group.rs:108-197): its
    shapes are culled by the fast path's hierarchies (group gates at the
    leaves), frames bitwise equal to the exhaustive loop."""
    from rtamd import scenes
    w, cam, depth = scenes.divided(96, 54, n=12, threshold=4)
    exact, se = cam.render(w, depth, want_stats=True)
    fast, _ = cam.render(w, depth, want_stats=False)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()
    cam.render(w, depth, want_stats=True, exhaustive=False)
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["fused"] and p["n_other_culled"] >= 190
