"""GPU parity sweep over seeded random scenes (rtamd.scenes.fuzz): planes,
spheres with non-uniform scales, rotations and shears, nested glass of assorted
indices, cubes, open and closed cylinders and cones, groups (divided or not),
every pattern kind, shadowless objects, one to three lights, random cameras and
depths 1-6 — geometry the culling hierarchies and the light buffer were not
tuned on.

Per seed (96 seeds), the whole 96x72 frame three ways:
- the fast path (what bench.py and the C++ drop-in run),
- the exhaustive counted render (the reference's every-shape loop on the GPU),
- the CPU oracle (oracle/rt_oracle.c, the reference's algorithm restated).
Bar: fast == exhaustive bit for bit; every channel within 1e-5 of the oracle
(the north star) and the PPM bytes identical; the exact work counters equal the
oracle's. The colours are also expected bit-identical to the oracle (the
specular `pow` is glibc's own algorithm, rt_pow.hpp): that is asserted too.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-5
NTHREADS = max(1, min(16, os.cpu_count() or 1))
COUNTERS = ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "plane_tests",
            "sphere_disc_ge0", "other_tests")


@pytest.mark.parametrize("seed", range(96))
def test_fuzz_scene_vs_oracle(rt, oracle, seed):
    from rtamd import scenes
    w, cam, depth = scenes.fuzz(seed, 96, 72)
    fast, _ = cam.render(w, depth, want_stats=False)
    exh, st = cam.render(w, depth)
    f, e = fast.to_numpy(), exh.to_numpy()
    assert f.tobytes() == e.tobytes(), f"seed {seed}: fast path differs from the exhaustive frame"
    ref, rst = oracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=NTHREADS)
    assert np.isfinite(e).all()
    diff = np.abs(e - ref)
    assert diff.max() <= TOL, f"seed {seed}: max |delta| {diff.max()}"
    assert rt.canvas_to_ppm(e) == oracle.canvas_to_ppm(ref)
    for k in COUNTERS:
        assert st[k] == rst[k], (seed, k, st[k], rst[k])
    n_diff = int((e != ref).sum())
    assert n_diff == 0, f"seed {seed}: {n_diff} channels differ from the oracle in the last bits"
    w.check()


@pytest.mark.parametrize("seed,aa", [(3, 4), (7, 2), (11, 16)])
def test_fuzz_scene_aa_vs_oracle(rt, oracle, seed, aa):
    """render_multithreaded with AA (camera.rs:150-217): the fast path's
    averaged samples against the oracle's."""
    from rtamd import scenes
    w, cam, depth = scenes.fuzz(seed, 48, 36)
    cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
    canvas, _ = cam.render_multithreaded(w, depth)
    g = canvas.to_numpy()
    ref, _ = oracle.OracleWorld.from_world(w).render_rows(cam.desc_bytes(), depth, list(range(cam.vsize)), NTHREADS,
                                                          aa_samples=aa)
    assert np.abs(g - ref).max() <= TOL
    assert rt.canvas_to_ppm(g) == oracle.canvas_to_ppm(ref)
    assert int((g != ref).sum()) == 0


@pytest.mark.parametrize("seed,spheres", [(100, 900), (101, 2500), (102, 6000)])
def test_fuzz_dense_scene_vs_oracle(rt, oracle, seed, spheres):
    """Thousands of random spheres in the same volume (overlapping, nested,
    glass among them): the sphere records and the deeper hierarchy leave LDS
    for the global-memory images; the whole 64x48 frame against the oracle and
    the fast path against the exhaustive frame."""
    from rtamd import scenes
    w, cam, depth = scenes.fuzz(seed, 64, 48, n_spheres=spheres)
    fast, _ = cam.render(w, depth, want_stats=False)
    exh, st = cam.render(w, depth)
    e = exh.to_numpy()
    assert fast.to_numpy().tobytes() == e.tobytes()
    ref, rst = oracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=NTHREADS)
    assert np.abs(e - ref).max() <= TOL
    assert rt.canvas_to_ppm(e) == oracle.canvas_to_ppm(ref)
    for k in COUNTERS:
        assert st[k] == rst[k], (seed, k)
    assert int((e != ref).sum()) == 0


@pytest.mark.parametrize("seed", [200, 201, 202, 203])
def test_fuzz_scene_large_frame_fast_equals_exhaustive(rt, seed):
    """The fast path against the exhaustive GPU frame on 640x480 frames of the
    random scenes (no oracle: 307 200 pixels), bit for bit."""
    from rtamd import scenes
    w, cam, depth = scenes.fuzz(seed, 640, 480)
    fast, _ = cam.render(w, depth, want_stats=False)
    exh, _ = cam.render(w, depth)
    assert fast.to_numpy().tobytes() == exh.to_numpy().tobytes()


@pytest.mark.parametrize("seed", range(300, 316))
def test_fuzz_ray_batches_vs_oracle(rt, oracle, seed):
    """World::intersect + hit + prepare_computations, World::is_shadowed and
    World::color_at for random rays whose origins fill the random scene's volume
    (many inside spheres and solids): geometry bitwise, shadows equal, colours
    bit-identical and counters equal."""
    from rtamd import scenes
    w, _, depth = scenes.fuzz(seed)
    ow = oracle.OracleWorld.from_world(w)
    rng = np.random.default_rng(seed)
    n = 1500
    o = rng.uniform([-4.5, -0.2, -2.5], [4.5, 3.5, 6.5], size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.hstack([o, d])
    g = w.hit_batch(rays)
    ref = np.array([ow.hit(r[:3], r[3:]) for r in rays])
    hits = ref[:, 0] >= 0
    assert np.array_equal(g[:, 0], ref[:, 0])
    assert np.array_equal(g[hits, 1:23], ref[hits, 1:23])
    assert np.abs(g[hits, 23] - ref[hits, 23]).max(initial=0.0) <= 1e-12  # schlick
    for light in range(w.n_lights()):
        gs = w.is_shadowed_batch(o, light)
        rs = np.array([ow.is_shadowed(p, light) for p in o])
        assert np.array_equal(gs.astype(bool), rs)
    gc, st = w.color_at_batch(rays, depth)
    rc, rst = ow.color_at_batch(rays, depth)
    assert np.abs(gc - rc).max() <= TOL
    assert int((gc != rc).sum()) == 0
    for k in rst:
        assert st[k] == rst[k], (seed, k)
