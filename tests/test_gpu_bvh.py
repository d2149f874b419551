"""Exact culling: the BVH traversal must reproduce the
exhaustive `World::intersect` bit for bit.

The counted launches (want_stats=True) run the exhaustive loops, whose
counters equal the oracle's; the fast path (want_stats=False, what bench.py
and the C++ drop-in run) traverses the sphere BVH. Every comparison here is
bitwise between the two, plus the oracle on a few frames.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
PI = math.pi


def _both(rt, w, cam, depth, aa=1):
    if aa == 1:
        fast, _ = cam.render(w, depth, want_stats=False)
        exact, st = cam.render(w, depth, want_stats=True)
    else:
        cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
        fast, _ = cam.render_multithreaded(w, depth, want_stats=False)
        exact, st = cam.render_multithreaded(w, depth, want_stats=True)
    prof = rt._rtamd._wf_profile(w, -1, True)
    return fast.to_numpy(), exact.to_numpy(), st


def _glass_cluster(rt, n=300, seed=7, inside=True, neg_zero=False):
    """Overlapping glass and mirror spheres (containers several deep), and a
    camera that may sit inside one of them."""
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
        s.material.refractive_index = 1.0 + rng.uniform(0, 1.5)
        s.material.reflective = rng.uniform(0, 0.9)
        s.material.color = rt.Color(*rng.uniform(0, 1, 3))
        if neg_zero and i % 2:
            s.material.color = rt.Color(-0.0, 0.5, -0.0)
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    cam = rt.Camera(96, 64, PI / 2.5)
    frm = (0.2, 1.1, -0.4) if inside else (0, 2, -9)
    cam.set_transform(rt.view_transform(rt.Point(*frm), rt.Point(0, 1, 2), rt.Vector(0, 1, 0)))
    return w, cam, 6


SCENES = {
    "c3_192x108": lambda rt: __import__("rtamd.scenes", fromlist=["c3"]).c3(192, 108),
    "c3_3000": lambda rt: __import__("rtamd.scenes", fromlist=["c3"]).c3(160, 90, n_spheres=3000, seed=99),
    "zoo": lambda rt: __import__("rtamd.scenes", fromlist=["zoo"]).zoo(120, 90),
    "solids": lambda rt: __import__("rtamd.scenes", fromlist=["solids"]).solids(120, 90),
    "first_scene": lambda rt: __import__("rtamd.scenes", fromlist=["first_scene"]).first_scene(160, 90),
    "glass_inside": lambda rt: _glass_cluster(rt, inside=True),
    "glass_outside": lambda rt: _glass_cluster(rt, n=500, seed=3, inside=False),
}


@pytest.mark.parametrize("name", sorted(SCENES))
def test_bvh_frames_bitwise_equal_exhaustive(rt, name):
    w, cam, depth = SCENES[name](rt)
    fast, exact, _ = _both(rt, w, cam, depth)
    assert rt._rtamd._wf_profile(w, -1, True)["n_bvh_nodes"] > 0
    assert fast.tobytes() == exact.tobytes()


def test_bvh_is_the_fast_path(rt):
    from rtamd import scenes
    w, cam, depth = scenes.c3(64, 36, n_spheres=200)
    cam.render(w, depth, want_stats=False)
    assert rt._rtamd._wf_profile(w, -1, True)["bvh"]
    cam.render(w, depth, want_stats=True, exhaustive=False)  # the fast path, counting its work
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["bvh"] and 0 < p["tests"]["primary"] < p["rays"]["primary"] * 200
    cam.render(w, depth, want_stats=True)
    assert not rt._rtamd._wf_profile(w, -1, True)["bvh"]


@pytest.mark.parametrize("stream", ["default", "torch"])
def test_profile_counts_the_generations(rt, stream):
    """The fast path's generations size themselves on the device; the profile
    (bench.py's roofline) takes their ray counts from the workspace's record,
    also for a frame rendered on the null stream: the secondary rays equal the
    counted frame's reflected + refracted rays."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(64, 36, n_spheres=200)
    b = torch.empty((36, 64, 3), dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream() if stream == "torch" else None
    torch.cuda.synchronize()
    st = cam.render_shard_device(w, depth, 8, 0, 1, b.data_ptr(), s.cuda_stream if s else 0, True, exhaustive=False)
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["fused"] and p["rays"]["primary"] == 64 * 36
    assert p["rays"]["closest"] == st["rays_reflect"] + st["rays_refract"] > 0


def test_bvh_vs_oracle_c3(rt, oracle):
    from rtamd import scenes
    w, cam, depth = scenes.c3(128, 72)
    fast, _ = cam.render(w, depth, want_stats=False)
    ref, _ = oracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=16)
    g = fast.to_numpy()
    assert np.abs(g - ref).max() <= 1e-5
    assert rt.canvas_to_ppm(g) == oracle.canvas_to_ppm(ref)


@pytest.mark.parametrize("aa", [4, 16])
def test_bvh_aa_bitwise(rt, aa):
    w, cam, depth = _glass_cluster(rt, n=120, seed=11, inside=False)
    fast, exact, _ = _both(rt, w, cam, depth, aa=aa)
    assert fast.tobytes() == exact.tobytes()


def test_bvh_color_at_batch_random_rays(rt):
    """Rays from everywhere (inside spheres, grazing, behind) at several depths."""
    w, _, _ = _glass_cluster(rt, n=400, seed=5)
    rng = np.random.default_rng(1)
    o = rng.uniform([-4, -0.5, -4], [4, 4, 4], size=(20000, 3))
    d = rng.normal(size=(20000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.hstack([o, d])
    for depth in (0, 1, 4):
        fast, _ = w.color_at_batch(rays, depth, want_stats=False)
        exact, _ = w.color_at_batch(rays, depth, want_stats=True)
        assert fast.tobytes() == exact.tobytes(), depth


@pytest.mark.parametrize("offset,image,lds_wide", [(0.0, 0, 0), (1e5, 0, 0), (-3e7, 0, 0), (0.0, 3, 0), (1e5, 3, 0),
                                                   (-3e7, 3, 0), (1e5, 0, 1), (-3e7, 0, 1)])
def test_bvh_binary32_slabs_far_and_axis_rays(rt, offset, image, lds_wide):
    """The per-lane traversal's binary32 slab test (DESIGN.md §5.2 error
    bound): a cluster far from the origin, rays from just outside it with
    direction components exactly 0, grazing rays tangent to spheres, and
    origins on box faces, all bitwise equal to the exhaustive loop; for the
    pair image (image 0), the four-wide walk over global memory (image 3) and
    the four-wide image in LDS (lds_wide), whose empty slots' inverted boxes
    must cull themselves for axis-parallel rays too."""
    rng = np.random.default_rng(int(abs(offset)) % 997 + 3)
    w = rt.World()
    centres, radii = [], []
    for i in range(300):
        r = float(rng.uniform(0.05, 0.6))
        c = rng.uniform(-4, 4, 3) + offset
        s = rt.glass_sphere() if i % 4 == 0 else rt.Sphere()
        s.set_transform(rt.translation(*c) * rt.scaling(r, r, r))
        s.material.reflective = 0.5
        w.add_object(s)
        centres.append(c)
        radii.append(r)
    w.add_light(rt.PointLight(rt.Point(offset - 10, offset + 10, offset - 10), rt.Color(1, 1, 1)))
    rays = []
    for c, r in zip(centres[:200], radii[:200]):
        for ax in range(3):
            o = np.array(c, dtype=np.float64)
            o[ax] -= 6.0
            d = np.zeros(3)
            d[ax] = 1.0
            rays.append(np.hstack([o, d]))                          # axis ray through the centre
            o2 = o.copy()
            o2[(ax + 1) % 3] += r                                     # tangent (grazing) axis ray
            rays.append(np.hstack([o2, d]))
            o3 = o.copy()
            o3[(ax + 1) % 3] += r * (1 + 1e-12)                     # just outside the tangent
            rays.append(np.hstack([o3, d]))
    o = np.array(centres)[rng.integers(0, 300, 4000)] + rng.normal(scale=1.0, size=(4000, 3))
    d = rng.normal(size=(4000, 3))
    d[::3, 0] = 0.0                                                  # zero components
    d[1::3, 1:] = 0.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.vstack([np.array(rays), np.hstack([o, d])])
    w.tune("image", image)
    w.tune("lds_wide", lds_wide)
    try:
        for depth in (0, 3):
            fast, _ = w.color_at_batch(rays, depth, want_stats=False)
            exact, _ = w.color_at_batch(rays, depth, want_stats=True)
            assert fast.tobytes() == exact.tobytes(), depth
    finally:
        w.tune("image", 0)
        w.tune("lds_wide", 1)
    assert rt._rtamd._wf_profile(w, -1, True)["n_bvh_nodes"] > 0


def test_bvh_shard_device_bitwise(rt):
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(200, 120, n_spheres=700)
    full, _ = cam.render(w, depth, want_stats=True)
    full = full.to_numpy()
    out = np.zeros_like(full)
    for s in range(3):
        rows = rt.shard_rows(cam.vsize, 8, s, 3)
        buf = torch.empty((rows, cam.hsize, 3), dtype=torch.float64, device="cuda")
        cam.render_shard_device(w, depth, 8, s, 3, buf.data_ptr(), torch.cuda.current_stream().cuda_stream, False)
        torch.cuda.synchronize()
        out[[y for y in range(cam.vsize) if (y // 8) % 3 == s]] = buf.cpu().numpy()
    assert out.tobytes() == full.tobytes()


def test_accel_knob_off_matches(rt):
    from rtamd import scenes
    w, cam, depth = scenes.zoo(80, 60)
    a, _ = cam.render(w, depth, want_stats=False)
    w.tune("accel", 0)
    try:
        b, _ = cam.render(w, depth, want_stats=False)
        assert not rt._rtamd._wf_profile(w, -1, True)["bvh"]
    finally:
        w.tune("accel", 1)
    assert a.to_numpy().tobytes() == b.to_numpy().tobytes()


@pytest.mark.parametrize("neg_zero", [False, True])
def test_skipped_shadow_rays_bitwise(rt, neg_zero):
    """The fast path leaves out shadow rays whose answer cannot change the
    colour (light behind the surface, DESIGN.md "Skipped shadow rays"). The
    frame must stay bitwise equal to the exhaustive one, also with -0.0 colour
    components (where ambient and ambient + 0 + 0 differ, so nothing may be
    skipped), and fewer shadow rays must actually be traced."""
    w, cam, depth = _glass_cluster(rt, n=200, seed=31, inside=False, neg_zero=neg_zero)
    exact, st = cam.render(w, depth, want_stats=True)
    fast, _ = cam.render(w, depth, want_stats=False)
    counted, sf = cam.render(w, depth, want_stats=True, exhaustive=False)  # the fast path, counting
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()
    assert counted.to_numpy().tobytes() == exact.to_numpy().tobytes()
    assert 0 < sf["rays_shadow_traced"] < st["rays_shadow"]
    w.tune("skip_shadow", 0)
    try:
        full, _ = cam.render(w, depth, want_stats=False)
        _, sa = cam.render(w, depth, want_stats=True, exhaustive=False)
        assert sa["rays_shadow_traced"] == st["rays_shadow"]
    finally:
        w.tune("skip_shadow", 1)
    assert full.to_numpy().tobytes() == exact.to_numpy().tobytes()


@pytest.mark.parametrize("image,shadow_lb,wide,lds_wide", [
    (0, 1, 1, 0), (0, 0, 1, 0), (0, 1, 1, 1), (0, 0, 1, 1),
    (3, 1, 1, 0), (3, 0, 1, 0), (3, 1, 0, 0), (3, 0, 0, 0), (1, 1, 1, 0), (1, 0, 1, 0)])
def test_fused_images_bitwise(rt, image, shadow_lb, wide, lds_wide):
    """Every scene image of the fast-path kernels (pair layout in LDS, the
    four-wide hierarchy in LDS (the default), nodes and records in global
    memory: the four-wide hierarchy (wide) or the binary one with an LDS stack /
    with a scratch stack), with shadow rays through the light buffer or through
    the BVH, gives the exhaustive frame. The scenes above that do not fit in LDS
    (3000 spheres) run a global image on their own."""
    w, cam, depth = _glass_cluster(rt, n=250, seed=21, inside=False)
    exact, _ = cam.render(w, depth, want_stats=True)
    w.tune("image", image)
    w.tune("shadow_lb", shadow_lb)
    w.tune("wide", wide)
    w.tune("lds_wide", lds_wide)
    try:
        fast, _ = cam.render(w, depth, want_stats=False)
        p = rt._rtamd._wf_profile(w, -1, True)
        assert p["fused"]
        assert p["n_bvh_wide"] > 0 and p["wide_stack"] > 0
    finally:
        w.tune("image", 0)
        w.tune("shadow_lb", 1)
        w.tune("wide", 1)
        w.tune("lds_wide", 1)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()


@pytest.mark.parametrize("leaf", [1, 2, 6])
def test_wide_hierarchy_bitwise(rt, leaf):
    """The four-wide hierarchy over the global-memory image (LANE 4): binary
    leaves of one or several records (opened into one record per leaf),
    frames, color_at rays from inside glass and shadows through the hierarchy
    all equal the exhaustive answers and the binary walk's; the two walks count
    different box tests (each ran)."""
    import numpy as np
    rt._rtamd._tuning_set("bvh_leaf", leaf)
    try:
        w, cam, depth = _glass_cluster(rt, n=700, seed=5, inside=True)
        exact, _ = cam.render(w, depth, want_stats=True)
    finally:
        rt._rtamd._tuning_set("bvh_leaf", 0)
    rng = np.random.default_rng(leaf)
    rays = np.concatenate([rng.uniform(-3, 3, (3000, 3)), rng.normal(size=(3000, 3))], 1)
    rays[:, 3:] /= np.linalg.norm(rays[:, 3:], axis=1, keepdims=True)
    col_exact, _ = w.color_at_batch(rays, depth, True, True)
    boxes = {}
    try:
        for image, wide, lds_wide in ((3, 1, 0), (0, 1, 1), (3, 0, 0)):
            w.tune("image", image)
            w.tune("wide", wide)
            w.tune("lds_wide", lds_wide)
            for lb in (1, 0):
                w.tune("shadow_lb", lb)
                fast, _ = cam.render(w, depth, want_stats=False)
                assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes(), (wide, lb)
                col, _ = w.color_at_batch(rays, depth, False)
                assert col.tobytes() == col_exact.tobytes(), (wide, lb)
            _, st = cam.render(w, depth, want_stats=True, exhaustive=False)
            boxes[(image, wide)] = st["box_tests_executed"]
    finally:
        w.tune("image", 0)
        w.tune("wide", 1)
        w.tune("lds_wide", 1)
        w.tune("shadow_lb", 1)
    assert boxes[(3, 1)] != boxes[(3, 0)] and boxes[(3, 1)] > 0 and boxes[(0, 1)] > 0


@pytest.mark.parametrize("n_streams,kind", [(2, "torch"), (18, "torch"), (4, "plain"), (4, "dedicated")])
def test_frames_in_flight_bitwise(rt, n_streams, kind):
    """Frames rendered concurrently on several streams (one workspace per
    stream; with 18 streams, more than the pool's 16 workspaces, so workspaces
    change hands in stream order) all equal the exhaustive frame, for the
    whole frame and for an 8-way shard, on torch streams and on the
    library's render streams (rtamd.render_stream, plain and CU-masked)."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(240, 136, n_spheres=600)
    full, _ = cam.render(w, depth, want_stats=True)
    full = full.to_numpy()
    rows8 = [y for y in range(cam.vsize) if (y // 8) % 8 == 5]
    if kind == "torch":
        streams = [torch.cuda.Stream() for _ in range(n_streams)]
    else:  # rtamd.render_stream: library-made plain or CU-masked (own hardware queue) streams
        streams = [rt.render_stream(kind == "dedicated") for _ in range(n_streams)]
    frames = 3 * n_streams
    bufs = [torch.full((cam.vsize, cam.hsize, 3), -1.0, dtype=torch.float64, device="cuda") for _ in range(frames)]
    sh = [torch.full((len(rows8), cam.hsize, 3), -1.0, dtype=torch.float64, device="cuda") for _ in range(frames)]
    torch.cuda.synchronize()
    for f in range(frames):
        st = streams[f % n_streams].cuda_stream
        cam.render_shard_device(w, depth, 8, 0, 1, bufs[f].data_ptr(), st, False)
        cam.render_shard_device(w, depth, 8, 5, 8, sh[f].data_ptr(), st, False)
    torch.cuda.synchronize()
    for f in range(frames):
        assert bufs[f].cpu().numpy().tobytes() == full.tobytes(), f
        assert sh[f].cpu().numpy().tobytes() == full[rows8].tobytes(), f


def _general_field(rt, n=360, seed=17):
    """Every shape kind under general transforms (rotated, sheared, scaled):
    spheres, cubes and closed bounded cylinders (culled by the other records'
    hierarchy), open bounded cylinders and cones (the line hierarchy), an
    infinite cylinder (exhaustive), a few diagonal spheres, glass and mirrors
    nested in each other."""
    rng = np.random.default_rng(seed)
    w = rt.World()
    floor = rt.Plane()
    floor.material.reflective = 0.25
    w.add_object(floor)
    pole = rt.Cylinder()  # infinite: stays exhaustive
    pole.set_transform(rt.translation(4.5, 0, 4.5) * rt.scaling(0.2, 1.0, 0.2))
    w.add_object(pole)
    for i in range(n):
        k = i % 6
        if k in (0, 1):
            s = rt.glass_sphere() if i % 4 == 0 else rt.Sphere()
        elif k == 2:
            s = rt.Cube()
        elif k == 3:
            lo = float(rng.uniform(-1.0, 0.0))
            s = rt.Cylinder(lo, lo + float(rng.uniform(0.2, 1.5)), bool(i % 2))
        elif k == 4:
            s = rt.Cone(float(rng.uniform(-1.0, -0.2)), float(rng.uniform(0.0, 0.8)), True)
        else:
            s = rt.Sphere()
        r = float(rng.uniform(0.15, 0.5))
        c = rng.uniform([-4, r, -4], [4, 3, 4])
        if k == 5:  # diagonal (translation . scaling): the sphere hierarchy
            tf = rt.translation(*c) * rt.scaling(r, r * 0.8, r * 1.2)
        else:
            tf = (rt.translation(*c) * rt.rotation_y(float(rng.uniform(0, 6.3)))
                  * rt.rotation_x(float(rng.uniform(0, 6.3)))
                  * rt.shearing(*[float(x) for x in rng.uniform(-0.3, 0.3, 6)]) * rt.scaling(r, r * 0.7, r * 1.1))
        s.set_transform(tf)
        s.material.color = rt.Color(*rng.uniform(0, 1, 3))
        if i % 3 == 1:
            s.material.transparency = 0.8
            s.material.refractive_index = float(1.0 + rng.uniform(0, 1.2))
            s.material.reflective = 0.5
        elif i % 3 == 2:
            s.material.reflective = float(rng.uniform(0.2, 0.9))
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    return w


@pytest.mark.parametrize("frm", [(0, 2.5, -9), (0.0, 1.2, 0.0), (-2.0, 1.5, -1.0)])
def test_other_records_hierarchy_bitwise(rt, frm):
    """General-transform spheres, cubes and bounded cylinders are culled by a
    hierarchy of their own (Group::divide's role, group.rs:108-188, over
    padded world boxes of the transformed shapes); the frames stay bitwise
    equal to the exhaustive loop, from outside and from inside the field."""
    w = _general_field(rt)
    cam = rt.Camera(128, 96, PI / 2.5)
    cam.set_transform(rt.view_transform(rt.Point(*frm), rt.Point(0, 1, 2), rt.Vector(0, 1, 0)))
    fast, exact, st = _both(rt, w, cam, 6)
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["n_other_culled"] > 200 and p["n_obvh_nodes"] > 0
    assert fast.tobytes() == exact.tobytes()


def test_other_records_hierarchy_random_rays(rt):
    """color_at from random origins (inside solids too) and directions, with
    axis-aligned and grazing directions, at several depths."""
    w = _general_field(rt, n=240, seed=5)
    rng = np.random.default_rng(9)
    o = rng.uniform([-4.5, -0.5, -4.5], [4.5, 3.5, 4.5], size=(16000, 3))
    d = rng.normal(size=(16000, 3))
    d[::5, 1:] = 0.0
    d[1::5, ::2] = 0.0
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.hstack([o, d])
    for depth in (0, 2, 5):
        fast, _ = w.color_at_batch(rays, depth, want_stats=False)
        exact, _ = w.color_at_batch(rays, depth, want_stats=True)
        assert fast.tobytes() == exact.tobytes(), depth


def test_open_glass_tubes_stay_containers(rt):
    """Open finite glass tubes (refractive index 1.5, so n1/n2 sees them):
    a ray whose origin lies outside a tube's box can have its backward line
    cross exactly one wall inside [min, max] and leave through the open end,
    which makes the tube a `containers` entry (intersection.rs:63-90) for a
    ray whose [0, t_hi] never meets the box. The line hierarchy tests such
    tubes' boxes over the whole backward line; fast == exhaustive bitwise on
    crafted and random rays."""
    rng = np.random.default_rng(13)
    w = rt.World()
    w.add_object(rt.Plane())
    tubes = []
    for i in range(40):
        t = rt.Cylinder(0.0, 1.0, False)
        c = rng.uniform([-5, 0, -5], [5, 2, 5])
        t.set_transform(rt.translation(*c) * rt.rotation_z(float(rng.uniform(-0.4, 0.4))) * rt.scaling(0.5, 1.2, 0.5))
        t.material.transparency = 0.9
        t.material.reflective = 0.3
        t.material.refractive_index = 1.5
        w.add_object(t)
        tubes.append(c)
    for i in range(60):  # glass spheres ahead of the rays: their n1 shows a wrong container
        s = rt.glass_sphere()
        r = float(rng.uniform(0.2, 0.5))
        s.set_transform(rt.translation(*rng.uniform([-6, r, -6], [6, 3, 6])) * rt.scaling(r, r, r))
        s.material.refractive_index = 2.0
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    rays = []
    for c in tubes:  # origin beside the tube, above its top; backward line: one wall, then out the open end
        for k in range(8):
            o = np.array(c) + np.array([1.5 + 0.3 * k, 2.2 + 0.2 * k, 0.05 * k])
            d = np.array([0.6, 0.5 + 0.05 * k, 0.1 * (k - 4)])
            rays.append(np.hstack([o, d / np.linalg.norm(d)]))
    o = rng.uniform([-6, -0.5, -6], [6, 3.5, 6], size=(12000, 3))
    d = rng.normal(size=(12000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.vstack([np.array(rays), np.hstack([o, d])])
    for depth in (0, 1, 4):
        fast, _ = w.color_at_batch(rays, depth, want_stats=False)
        exact, _ = w.color_at_batch(rays, depth, want_stats=True)
        assert fast.tobytes() == exact.tobytes(), depth
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["n_other_culled"] == 0 and p["n_line_culled"] == 40  # open tubes: the line hierarchy


def _cone_field(rt, n=240, seed=23, upright_share=0.5):
    """Cones (closed and open, finite bounds, some spanning y = 0: two nappes)
    and open tubes, half of the cones upright with one scale (their gates
    close tightly), the rest under random rotations and shears; glass and
    mirrors among them, a floor and diagonal spheres."""
    rng = np.random.default_rng(seed)
    w = rt.World()
    floor = rt.Plane()
    floor.material.reflective = 0.3
    w.add_object(floor)
    for i in range(n):
        c = rng.uniform([-5, 0.5, -5], [5, 3, 5])
        if i % 4 == 3:
            s = rt.Cylinder(float(rng.uniform(-1.0, 0.0)), float(rng.uniform(0.2, 1.0)), False)
            tf = rt.translation(*c) * rt.rotation_z(float(rng.uniform(-1, 1))) * rt.scaling(0.3, 0.5, 0.3)
        elif i % 4 == 2 and i % 8 != 2:
            s = rt.Sphere()
            tf = rt.translation(*c) * rt.scaling(0.3, 0.3, 0.3)
        else:
            lo = float(rng.uniform(-1.0, 0.3))
            s = rt.Cone(lo, lo + float(rng.uniform(0.3, 1.2)), bool(i % 3))
            if rng.uniform() < upright_share:
                tf = rt.translation(*c) * rt.scaling(0.4, 0.4, 0.4)
            else:
                tf = (rt.translation(*c) * rt.rotation_y(float(rng.uniform(0, 6.3)))
                      * rt.rotation_x(float(rng.uniform(0, 6.3)))
                      * rt.shearing(*[float(x) for x in rng.uniform(-0.2, 0.2, 6)]) * rt.scaling(0.4, 0.5, 0.3))
        s.set_transform(tf)
        s.material.color = rt.Color(*rng.uniform(0, 1, 3))
        if i % 5 == 1:
            s.material.transparency = 0.8
            s.material.refractive_index = float(1.0 + rng.uniform(0, 1.0))
            s.material.reflective = 0.4
        elif i % 5 == 2:
            s.material.reflective = float(rng.uniform(0.2, 0.9))
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    return w


@pytest.mark.parametrize("frm,upright", [((0, 2.5, -11), 0.5), ((0.0, 1.5, 0.0), 0.5), ((3.0, 4.0, -6.0), 1.0),
                                         ((-1.0, 1.0, -2.0), 0.0)])
def test_line_hierarchy_cones_bitwise(rt, frm, upright):
    """Cones and open tubes culled by the line hierarchy (their boxes over the
    whole line up to the hit, each cone behind its a ~ 0 gate, cone.rs:94-134,
    cylinder.rs:88-119): frames bitwise equal to the exhaustive loop, from
    outside and inside the field, with every cone upright, none, or half."""
    w = _cone_field(rt, upright_share=upright)
    cam = rt.Camera(128, 96, PI / 2.5)
    cam.set_transform(rt.view_transform(rt.Point(*frm), rt.Point(0, 1, 1), rt.Vector(0, 1, 0)))
    fast, exact, st = _both(rt, w, cam, 6)
    assert fast.tobytes() == exact.tobytes()
    counted, _ = cam.render(w, 6, want_stats=True, exhaustive=False)  # the fast path, counting its work
    assert counted.to_numpy().tobytes() == exact.tobytes()
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["n_line_culled"] > 150 and p["n_lbvh_nodes"] > 0 and p["fused"]


def test_cone_a_zero_branch_rays(rt):
    """Rays along a cone's generators take the reference's a ~ 0 branch
    (cone.rs:102-110), whose root t = -c / 2.0 * b lies anywhere on the line,
    far outside the cone's box: the gates must send these rays to the cone
    whatever its box says. Upright cones of one scale, directions with
    dx^2 + dz^2 = dy^2 exactly and perturbed around it (|a| just below and
    above EPSILON), origins far from every box; then random rays."""
    rng = np.random.default_rng(31)
    w = rt.World()
    centres = []
    for i in range(60):
        s = rt.Cone(-1.0, 1.0, bool(i % 2))
        c = rng.uniform([-6, 1, -6], [6, 3, 6])
        s.set_transform(rt.translation(*c) * rt.scaling(0.5, 0.5, 0.5))
        s.material.color = rt.Color(*rng.uniform(0, 1, 3))
        if i % 3 == 0:
            s.material.transparency = 0.7
            s.material.refractive_index = 1.4
        w.add_object(s)
        centres.append(c)
    for i in range(30):  # spheres to hit behind the quirk roots
        s = rt.Sphere()
        s.set_transform(rt.translation(*rng.uniform([-8, 0, -8], [8, 4, 8])) * rt.scaling(0.4, 0.4, 0.4))
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    dirs = []
    for ex, ez in ((1, 0), (0, 1), (0.6, 0.8), (-0.8, 0.6), (0.28, -0.96)):
        for sy in (1, -1):
            for eps in (0.0, 2e-6, -2e-6, 4e-6, 1e-5, -1e-5, 3e-5):
                d = np.array([ex, sy * (1.0 + eps), ez])
                dirs.append(d / np.linalg.norm(d))
    rays = []
    for k in range(4000):
        d = dirs[k % len(dirs)]
        o = rng.uniform([-30, -10, -30], [30, 14, 30])
        rays.append(np.hstack([o, d]))
    # the crafted rays do take the branch: (ray, cone) pairs with |a| < EPSILON, |b| >= EPSILON
    # and a root t = -c / 2.0 * b >= 0 (object space: 2 (o - centre), 2 d)
    cr = np.array(rays)
    quirk = 0
    for c in centres:
        lo_, ld = 2.0 * (cr[:, :3] - c), 2.0 * cr[:, 3:]
        a = ld[:, 0] * ld[:, 0] - ld[:, 1] * ld[:, 1] + ld[:, 2] * ld[:, 2]
        b = 2.0 * lo_[:, 0] * ld[:, 0] - 2.0 * lo_[:, 1] * ld[:, 1] + 2.0 * lo_[:, 2] * ld[:, 2]
        cc = lo_[:, 0] * lo_[:, 0] - lo_[:, 1] * lo_[:, 1] + lo_[:, 2] * lo_[:, 2]
        quirk += int(np.sum((np.abs(a) < 1e-5) & (np.abs(b) >= 1e-5) & (-cc / 2.0 * b >= 0.0)))
    assert quirk > 1000
    o = rng.uniform([-7, -0.5, -7], [7, 4.5, 7], size=(8000, 3))
    d = rng.normal(size=(8000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.vstack([cr, np.hstack([o, d])])
    for depth in (0, 1, 4):
        fast, _ = w.color_at_batch(rays, depth, want_stats=False)
        exact, _ = w.color_at_batch(rays, depth, want_stats=True)
        assert fast.tobytes() == exact.tobytes(), depth
    assert rt._rtamd._wf_profile(w, -1, True)["n_line_culled"] == 60


def test_other_records_only_scene_takes_fast_path(rt):
    """A scene without diagonal spheres (only general solids) still takes the
    fast path through the other records' hierarchy, and culls: it executes
    far fewer record tests than the reference's loop."""
    rng = np.random.default_rng(4)
    w = rt.World()
    w.add_object(rt.Plane())
    for i in range(300):
        s = rt.Cube() if i % 2 else rt.Sphere()
        c = rng.uniform([-6, 0.3, -6], [6, 3, 6])
        s.set_transform(rt.translation(*c) * rt.rotation_y(float(rng.uniform(0, 3))) * rt.scaling(0.3, 0.2, 0.25))
        s.material.reflective = 0.4
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    cam = rt.Camera(96, 64, PI / 3)
    cam.set_transform(rt.view_transform(rt.Point(0, 4, -12), rt.Point(0, 1, 0), rt.Vector(0, 1, 0)))
    exact, st = cam.render(w, 5, want_stats=True)
    fast, fst = cam.render(w, 5, want_stats=True, exhaustive=False)  # the fast path, counting its work
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["bvh"] and p["fused"]
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()
    # executed record tests (closest-hit + shadow) against the reference's every-shape loop
    executed = sum(p["tests"].values())
    reference = (st["rays_primary"] + st["rays_reflect"] + st["rays_refract"] + st["rays_shadow"]) * 300
    assert executed < reference / 10


def test_line_hierarchy_small_a_near_tangent(rt):
    """The line hierarchy's padding where the roots are least accurate (advisor
    r05): open tubes and cones with |a| between EPSILON and 10 EPSILON for the
    ray (directions within a hair of a tube's axis or of a cone's generators)
    and near-tangent rays (discriminant ~ 0), with small spheres placed just
    past rays' roots on the shapes, so that a root found on the wrong side of a
    box's t_hi would change the hit. Fast path == every-shape loop, bitwise."""
    rng = np.random.default_rng(47)
    w = rt.World()
    shapes = []
    for i in range(48):
        c = rng.uniform([-8, 1, -8], [8, 3, 8])
        if i % 2:
            s = rt.Cylinder(-1.0, 1.0, False)
            sc = np.array([0.5, 1.0, 0.5])
        else:
            s = rt.Cone(-1.0, 1.0, False)
            sc = np.array([0.5, 0.5, 0.5])
        s.set_transform(rt.translation(*c) * rt.scaling(*sc))
        s.material.color = rt.Color(*rng.uniform(0, 1, 3))
        w.add_object(s)
        shapes.append((i % 2, c, sc))
    rays, blockers = [], []
    for k in range(3000):
        tube, c, sc = shapes[k % len(shapes)]
        a = float(rng.uniform(1.05e-5, 1e-4)) * (1 if rng.uniform() < 0.8 else -1)
        phi = float(rng.uniform(0, 2 * np.pi))
        side = np.array([-np.sin(phi), 0.0, np.cos(phi)])
        if tube:  # object direction (ex, 1, ez) with ex^2 + ez^2 = |a|; the line ~1 from the axis
            r = np.sqrt(abs(a))
            ld = np.array([r * np.cos(phi), 1.0, r * np.sin(phi)])
            lo = side * (1.0 + float(rng.uniform(-1e-7, 1e-7))) + np.array([0.0, float(rng.uniform(-3, -1.5)), 0.0])
            qa, qb = ld[0] ** 2 + ld[2] ** 2, 2 * (lo[0] * ld[0] + lo[2] * ld[2])
            qc = lo[0] ** 2 + lo[2] ** 2 - 1.0
        else:  # cone: ex^2 - 1 + ez^2 = a; the line just beside a generator
            r = np.sqrt(1.0 + a)
            ld = np.array([r * np.cos(phi), 1.0, r * np.sin(phi)])
            lo = side * float(rng.uniform(1e-6, 1e-3)) + np.array([0.0, float(rng.uniform(-3, -1.5)), 0.0])
            qa = ld[0] ** 2 - ld[1] ** 2 + ld[2] ** 2
            qb = 2 * (lo[0] * ld[0] - lo[1] * ld[1] + lo[2] * ld[2])
            qc = lo[0] ** 2 - lo[1] ** 2 + lo[2] ** 2
        d = ld * sc
        o = lo * sc + c
        dn = d / np.linalg.norm(d)
        rays.append(np.hstack([o, dn]))
        disc = qb * qb - 4 * qa * qc
        if k % 5 == 0 and disc >= 0 and len(blockers) < 80:
            for t in sorted(((-qb - np.sqrt(disc)) / (2 * qa), (-qb + np.sqrt(disc)) / (2 * qa))):
                if t > 0:  # just past the first root ahead (world distance t |d|)
                    blockers.append(o + dn * (t * np.linalg.norm(d) + float(rng.uniform(1e-3, 5e-2))))
                    break
    for b in blockers:
        s = rt.Sphere()
        s.set_transform(rt.translation(*b) * rt.scaling(0.03, 0.03, 0.03))  # (det >= EPSILON: invertible)
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    assert len(blockers) > 40
    rays = np.array(rays)
    for depth in (0, 1, 3):
        fast, _ = w.color_at_batch(rays, depth, want_stats=False)
        exact, _ = w.color_at_batch(rays, depth, want_stats=True)
        assert fast.tobytes() == exact.tobytes(), depth
    assert rt._rtamd._wf_profile(w, -1, True)["n_line_culled"] == 48
