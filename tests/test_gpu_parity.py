"""GPU parity: the HIP render path vs the CPU oracle on identical scenes.

Bar (north star): every colour channel within 1e-5 abs of the oracle, the
quantised PPM bytes identical, and the exact work counters (rays by kind, shape
tests) identical. Geometry (hit object, t, points, normals, n1/n2) must be
bit-identical: it uses only IEEE-exact +,-,*,/,sqrt in the reference's order.
Colours may differ in the last bits only through `pow` (OCML vs glibc).
"""
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-5  # north star: within 1e-5 abs per colour channel
NTHREADS = max(1, min(16, os.cpu_count() or 1))
PI = math.pi


def _oracle_world(oracle, w):
    return oracle.OracleWorld.from_world(w)


def _compare_frame(rt, oracle, w, cam, depth, rows=None, aa=1):
    if aa == 1:
        canvas, st = cam.render(w, depth)
    else:
        cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
        canvas, st = cam.render_multithreaded(w, depth)
    gpu = canvas.to_numpy()
    ow = _oracle_world(oracle, w)
    rows = list(range(cam.vsize)) if rows is None else rows
    ref, rst = ow.render_rows(cam.desc_bytes(), depth, rows, NTHREADS, aa_samples=aa)
    g = gpu[rows]
    diff = np.abs(g - ref)
    assert np.isfinite(g).all()
    assert diff.max() <= TOL, f"max |delta| {diff.max()}"
    assert rt.canvas_to_ppm(g) == oracle.canvas_to_ppm(ref)
    if len(rows) == cam.vsize:
        for k in ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow",
                  "sphere_tests", "plane_tests", "sphere_disc_ge0", "other_tests"):
            assert st[k] == rst[k], (k, st[k], rst[k])
    return gpu, ref, st


def test_render_world_with_camera(rt):
    # camera.rs:327-337
    w = rt.World.default()
    c = rt.Camera(11, 11, PI / 2.0)
    c.set_transform(rt.view_transform(rt.Point(0, 0, -5), rt.Point(0, 0, 0), rt.Vector(0, 1, 0)))
    canvas, st = c.render(w)
    assert canvas.get_pixel(5, 5) == rt.Color(0.38066, 0.47583, 0.2855)
    assert st["rays_primary"] == 121


def test_world_color_at_kats(rt):
    # world.rs:220-234
    w = rt.World.default()
    assert w.color_at(rt.Ray(rt.Point(0, 0, -5), rt.Vector(0, 1, 0)), 5) == rt.Color(0, 0, 0)
    assert w.color_at(rt.Ray(rt.Point(0, 0, -5), rt.Vector(0, 0, 1)), 5) == rt.Color(0.38066, 0.47583, 0.2855)


def test_is_shadowed_kats(rt):
    # world.rs:248-274
    w = rt.World.default()
    assert not w.is_shadowed(rt.Point(0, 10, 0), 0)
    assert w.is_shadowed(rt.Point(10, -10, 10), 0)
    assert not w.is_shadowed(rt.Point(-20, 20, -20), 0)
    assert not w.is_shadowed(rt.Point(-2, 2, -2), 0)


def test_reflection_refraction_kats(rt):
    s2 = math.sqrt(2.0) / 2.0
    # world.rs:330-347 shade_hit_with_reflective_surface, via color_at on the same ray
    w = rt.World.default()
    p = rt.Plane()
    p.material.reflective = 0.5
    p.set_transform(rt.translation(0, -1, 0))
    w.add_object(p)
    c = w.color_at(rt.Ray(rt.Point(0, 0, -3), rt.Vector(0.0, -s2, s2)), 5)
    assert c == rt.Color(0.87676, 0.92435, 0.82918)
    # world.rs:493-520 shade_hit_with_reflective_transparent_material
    w = rt.World.default()
    floor = rt.Plane()
    floor.set_transform(rt.translation(0, -1, 0))
    floor.material.reflective = 0.5
    floor.material.transparency = 0.5
    floor.material.refractive_index = 1.5
    w.add_object(floor)
    ball = rt.Sphere()
    ball.material.color = rt.Color(1.0, 0.0, 0.0)
    ball.material.ambient = 0.5
    ball.set_transform(rt.translation(0.0, -3.5, -0.5))
    w.add_object(ball)
    c = w.color_at(rt.Ray(rt.Point(0, 0, -3), rt.Vector(0.0, -s2, s2)), 5)
    assert c == rt.Color(0.93391, 0.69643, 0.69243)
    # world.rs:349-366 mutually reflective planes terminate (depth bound)
    w = rt.World()
    w.add_light(rt.PointLight(rt.Point(0, 0, 0), rt.Color(1, 1, 1)))
    for y in (-1, 1):
        pl = rt.Plane()
        pl.material.reflective = 1.0
        pl.set_transform(rt.translation(0, y, 0))
        w.add_object(pl)
    rays = np.array([[0, 0, 0, 0, 1, 0]], dtype=np.float64)
    out, st = w.color_at_batch(rays, 5)
    assert st["rays_primary"] + st["rays_reflect"] == 6 and np.isfinite(out).all()


def test_hit_batch_bitwise_vs_oracle(rt, oracle):
    """World::intersect + hit + prepare_computations (+ n1/n2, schlick) per ray."""
    from rtamd import scenes
    rng = np.random.default_rng(11)
    for make in (scenes.zoo, lambda: scenes.c3(64, 36, n_spheres=200), scenes.solids, scenes.first_scene):
        w, cam, _ = make()
        ow = _oracle_world(oracle, w)
        n = 3000
        o = rng.uniform([-3, 0.05, -6], [3, 3, 4], size=(n, 3))
        d = rng.normal(size=(n, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays = np.hstack([o, d])
        g = w.hit_batch(rays)
        ref = np.array([ow.hit(r[:3], r[3:]) for r in rays])
        hits = ref[:, 0] >= 0
        assert hits.sum() > 100
        assert np.array_equal(g[:, 0], ref[:, 0])
        # geometry is exact: bitwise on t, point, over/under, eyev, normal, inside, reflectv, n1, n2
        assert np.array_equal(g[hits, 1:23], ref[hits, 1:23]), np.abs(g[hits, 1:23] - ref[hits, 1:23]).max()
        assert np.abs(g[hits, 23] - ref[hits, 23]).max() <= 1e-12  # schlick


def test_is_shadowed_batch_vs_oracle(rt, oracle):
    from rtamd import scenes
    w, _, _ = scenes.zoo()
    ow = _oracle_world(oracle, w)
    rng = np.random.default_rng(5)
    pts = rng.uniform([-3, -0.5, -4], [3, 3, 3], size=(4000, 3))
    for light in range(w.n_lights()):
        g = w.is_shadowed_batch(pts, light)
        ref = np.array([ow.is_shadowed(p, light) for p in pts])
        assert np.array_equal(g.astype(bool), ref)
        assert 0 < ref.sum() < len(ref)


def test_color_at_batch_vs_oracle_depths(rt, oracle):
    from rtamd import scenes
    w, cam, _ = scenes.zoo()
    ow = _oracle_world(oracle, w)
    rng = np.random.default_rng(3)
    o = np.tile([0.0, 1.5, -5.0], (600, 1))
    d = rng.normal([0, -0.1, 1], [0.35, 0.25, 0.05], size=(600, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.hstack([o, d])
    for depth in (0, 1, 2, 5, 9):
        g, st = w.color_at_batch(rays, depth)
        ref, rst = ow.color_at_batch(rays, depth)
        assert np.abs(g - ref).max() <= TOL
        for k in rst:
            assert st[k] == rst[k], (depth, k)


def test_c1_full_frame(rt, oracle):
    from rtamd import scenes
    w, cam, depth = scenes.c1()
    _compare_frame(rt, oracle, w, cam, depth)


def test_c2_full_frame(rt, oracle):
    from rtamd import scenes
    w, cam, depth = scenes.c2()
    _compare_frame(rt, oracle, w, cam, depth)


def test_zoo_full_frame(rt, oracle):
    from rtamd import scenes
    w, cam, depth = scenes.zoo(200, 150)
    gpu, ref, st = _compare_frame(rt, oracle, w, cam, depth)
    assert st["rays_refract"] > 0 and st["rays_reflect"] > 0


def test_c3_downscaled_full_frame(rt, oracle):
    """The headline scene (1000 spheres, depth 5) at 192x108."""
    from rtamd import scenes
    w, cam, depth = scenes.c3(192, 108)
    gpu, ref, st = _compare_frame(rt, oracle, w, cam, depth)
    assert st["rays_refract"] > 0


def test_c3_full_size_sampled_rows(rt, oracle):
    """Full 1920x1080 C3 frame on the GPU; oracle on a spread of rows."""
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    rows = [0, 137, 301, 540, 541, 777, 1079]
    _compare_frame(rt, oracle, w, cam, depth, rows=rows)


def test_c5_sampled_rows(rt, oracle):
    """C5 (4 planes + 9996 spheres, 2 lights, depth 8) at 384x384 on the GPU;
    oracle on a few rows (10k-object intersection lists on the CPU)."""
    from rtamd import scenes
    w, cam, depth = scenes.c5(384, 384)
    _compare_frame(rt, oracle, w, cam, depth, rows=[0, 150, 191, 300])


def test_c5_fast_path_bitwise(rt):
    from rtamd import scenes
    w, cam, depth = scenes.c5(256, 256)
    fast, _ = cam.render(w, depth, want_stats=False)
    exact, _ = cam.render(w, depth, want_stats=True)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()


def test_shards_reassemble_bitwise(rt):
    """Interleaved row-block shards (the multi-GPU partition) rendered one at a
    time into device buffers reassemble into the single-launch frame exactly."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(320, 181, n_spheres=300)
    full, _ = cam.render(w, depth)
    full = full.to_numpy()
    for n_shards, block in [(2, 8), (3, 16), (4, 1), (8, 8)]:
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


def test_deterministic_and_counters_full_c3(rt):
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    a, sa = cam.render(w, depth)
    b, sb = cam.render(w, depth)
    assert a.to_numpy().tobytes() == b.to_numpy().tobytes()
    assert sa["rays_primary"] == 1920 * 1080
    for k in ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "sphere_disc_ge0"):
        assert sa[k] == sb[k]
    n_rays = sa["rays_primary"] + sa["rays_reflect"] + sa["rays_refract"] + sa["rays_shadow"]
    assert sa["sphere_tests"] == n_rays * 1000 and sa["plane_tests"] == n_rays


def test_edge_cases(rt, oracle):
    # empty world -> black; no lights -> surface is (0,0,0); 1x1 canvas; portrait camera
    w = rt.World()
    c = rt.Camera(3, 2, PI / 2.0)
    canvas, st = c.render(w)
    assert not canvas.to_numpy().any() and st["rays_primary"] == 6
    w = rt.World()
    s = rt.Sphere()
    s.material.reflective = 0.5
    w.add_object(s)
    c = rt.Camera(1, 1, PI / 3.0)
    c.set_transform(rt.view_transform(rt.Point(0, 0, -5), rt.Point(0, 0, 0), rt.Vector(0, 1, 0)))
    canvas, _ = c.render(w)
    assert canvas.get_pixel(0, 0) == rt.Color(0, 0, 0)
    from rtamd import scenes
    w, cam, depth = scenes.zoo(37, 61)  # portrait, odd sizes
    _compare_frame(rt, oracle, w, cam, depth)


def test_deep_recursion_limit(rt, oracle):
    """A hall of mirrors at depths past the default 5 (up to the supported 64)."""
    w = rt.World()
    w.add_light(rt.PointLight(rt.Point(0, 0.5, 0), rt.Color(1, 1, 1)))
    for y, col in ((-1, (0.9, 0.2, 0.2)), (1, (0.2, 0.2, 0.9))):
        pl = rt.Plane()
        pl.material.reflective = 0.9
        pl.material.color = rt.Color(*col)
        pl.set_transform(rt.translation(0, y, 0))
        w.add_object(pl)
    ow = _oracle_world(oracle, w)
    d = np.array([0.1, 0.9, 0.3])
    d /= np.linalg.norm(d)
    rays = np.array([[0, 0, 0, *d]])
    for depth in (5, 8, 16, 40, 64):
        g, st = w.color_at_batch(rays, depth)
        ref, rst = ow.color_at_batch(rays, depth)
        assert np.abs(g - ref).max() <= TOL and st["rays_reflect"] == rst["rays_reflect"] == depth
    with pytest.raises(rt.RtError):
        w.color_at_batch(rays, 65)


# ------------------------------------------------- SURVEY §8f rows 1-2
def test_solids_full_frame(rt, oracle):
    """Cube / Cylinder / Cone (cube.rs, cylinder.rs, cone.rs): glass solids
    nested in each other (containers with up to 4 intersections per object)."""
    from rtamd import scenes
    w, cam, depth = scenes.solids(200, 150)
    gpu, ref, st = _compare_frame(rt, oracle, w, cam, depth)
    assert st["other_tests"] > 0 and st["rays_refract"] > 0


def test_first_scene_demo(rt, oracle):
    """The reference's bin/first_scene.rs (cube + cylinder + cone + 2 lights)."""
    from rtamd import scenes
    w, cam, depth = scenes.first_scene(256, 144)
    _compare_frame(rt, oracle, w, cam, depth)


@pytest.mark.parametrize("aa", [1, 2, 4, 8, 16])
def test_render_multithreaded_aa(rt, oracle, aa):
    """render_multithreaded: rays_for_pixel offsets + Color::average."""
    from rtamd import scenes
    w, cam, depth = scenes.first_scene(64, 36)
    gpu, ref, st = _compare_frame(rt, oracle, w, cam, depth, aa=aa)
    assert st["rays_primary"] == 64 * 36 * aa


def test_aa_shards_reassemble_bitwise(rt):
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.solids(96, 70)
    cam.render_opts.aa_samples(rt.AASamples.X4)
    full, _ = cam.render_multithreaded(w, depth)
    full = full.to_numpy()
    for n_shards, block in [(2, 8), (3, 5)]:
        out = np.zeros_like(full)
        for s in range(n_shards):
            rows = rt.shard_rows(cam.vsize, block, s, n_shards)
            buf = torch.empty((rows, cam.hsize, 3), dtype=torch.float64, device="cuda")
            cam.render_shard_device(w, depth, block, s, n_shards, buf.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream, False, aa_samples=4)
            torch.cuda.synchronize()
            ys = [y for y in range(cam.vsize) if (y // block) % n_shards == s]
            out[ys] = buf.cpu().numpy()
        assert out.tobytes() == full.tobytes()


def test_solid_shadows_and_color_at(rt, oracle):
    from rtamd import scenes
    w, cam, _ = scenes.solids()
    ow = _oracle_world(oracle, w)
    rng = np.random.default_rng(17)
    pts = rng.uniform([-3, -0.2, -3], [3, 2.5, 3], size=(3000, 3))
    for light in range(w.n_lights()):
        g = w.is_shadowed_batch(pts, light)
        ref = np.array([ow.is_shadowed(p, light) for p in pts])
        assert np.array_equal(g.astype(bool), ref)
    o = np.tile([0.0, 2.0, -5.5], (500, 1))
    d = rng.normal([0, -0.2, 1], [0.3, 0.2, 0.05], size=(500, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.hstack([o, d])
    for depth in (0, 3, 8):
        g, st = w.color_at_batch(rays, depth)
        r, rst = ow.color_at_batch(rays, depth)
        assert np.abs(g - r).max() <= TOL
        for k in rst:
            assert st[k] == rst[k], (depth, k)


def test_bad_aa_rejected(rt):
    w = rt.World.default()
    c = rt.Camera(4, 4, 1.0)
    import torch
    buf = torch.empty((4, 4, 3), dtype=torch.float64, device="cuda")
    with pytest.raises(rt.RtError, match="aa_samples"):
        c.render_shard_device(w, 5, 8, 0, 1, buf.data_ptr(), 0, False, aa_samples=3)


def test_rccl_stream_gather_hooks(rt):
    """The library's per-stream RCCL hooks (bench.py's N-GPU assembler):
    a one-rank communicator gathers a buffer on a render stream."""
    import torch
    comm = rt._rtamd._nccl_comm_init(1, rt._rtamd._nccl_unique_id(), 0, 0)
    try:
        st = rt.render_stream(False)
        send = torch.arange(3000, dtype=torch.float64, device="cuda")
        recv = torch.full_like(send, -1.0)
        torch.cuda.synchronize()
        rt._rtamd._nccl_gather_f64(send.data_ptr(), recv.data_ptr(), send.numel(), 0, comm, st.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(send, recv)
    finally:
        rt._rtamd._nccl_comm_destroy(comm)
