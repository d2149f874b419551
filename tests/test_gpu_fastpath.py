"""The benchmarked fast path at full size, the fast path's counters, the
boundary's multi-device entry point and the device-side queue check.

bench.py times the fast path (exact-culling BVH, light buffer, shadow rays
that cannot change a colour left out) on the full 1920x1080 C3 frame and the
4096x4096 C5 frame. These tests require those frames to equal the
reference's every-shape loop (RT_RENDER_EXHAUSTIVE) bit for bit, and the fast
frame to match the oracle (camera.rs:133-148) on sampled rows and scattered
pixels of the full-size frames: 60 whole rows and 4096 pixels of C3, 2048
pixels of C5, each within the north-star tolerance and with identical PPM
bytes.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TOL = 1e-5
NTHREADS = max(1, min(16, os.cpu_count() or 1))
RAY_KEYS = ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "plane_tests",
            "other_tests")


def _device_frame(cam, w, depth, exhaustive, stream=None):
    import torch
    buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
    st = cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(),
                                 (stream or torch.cuda.current_stream()).cuda_stream, True, exhaustive=exhaustive)
    torch.cuda.synchronize()
    return buf, st


def test_c3_full_frame_fast_equals_exhaustive(rt, oracle):
    """C3 at 1920x1080 (the headline frame): fast == exhaustive bitwise, the
    fast frame vs the oracle on sampled rows, and the fast path's counters."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    exact, se = _device_frame(cam, w, depth, True)
    fast, sf = _device_frame(cam, w, depth, False)
    assert torch.equal(fast, exact)
    assert se["exhaustive"] and not sf["exhaustive"]
    for k in RAY_KEYS:  # the reference's work, exact on both paths
        assert sf[k] == se[k], k
    assert sf["sphere_disc_ge0"] is None and se["sphere_disc_ge0"] > 0
    assert se["rays_shadow_traced"] == se["rays_shadow"]
    assert 0 < sf["rays_shadow_traced"] < sf["rays_shadow"]
    assert sf["sphere_tests_executed"] < se["sphere_tests_executed"] / 50
    assert sf["box_tests_executed"] > 0 and se["box_tests_executed"] == 0
    rows = list(range(3, 1080, 18))  # 60 rows, every part of the frame
    ow = oracle.OracleWorld.from_world(w)
    ref, _ = ow.render_rows(cam.desc_bytes(), depth, rows, NTHREADS)
    got = fast.cpu().numpy()[rows]
    assert np.abs(got - ref).max() <= TOL
    # bit for bit: the specular pow is glibc's own algorithm (rt_pow.hpp)
    assert got.tobytes() == ref.tobytes(), int((got != ref).sum())
    assert rt.canvas_to_ppm(got) == oracle.canvas_to_ppm(ref)
    _check_pixels(rt, oracle, ow, cam, depth, fast, 4096, seed=3)


def _check_pixels(rt, oracle, ow, cam, depth, frame, n, seed):
    """n scattered pixels of a full-size device frame against the oracle:
    bit for bit (so within TOL), and the same PPM bytes (one row of n pixels)."""
    rng = np.random.default_rng(seed)
    xy = np.stack([rng.integers(0, cam.hsize, n), rng.integers(0, cam.vsize, n)], 1)
    ref, st = ow.render_pixels(cam.desc_bytes(), depth, xy, NTHREADS)
    got = frame[xy[:, 1], xy[:, 0]].cpu().numpy()
    assert st["rays_primary"] == n
    assert np.abs(got - ref).max() <= TOL
    # bit for bit (round 5 counted 3 of 12288 C3 and 5 of 6144 C5 channels 1-2 ulps apart with
    # OCML's pow; the specular pow is now glibc's own algorithm, rt_pow.hpp)
    assert got.tobytes() == ref.tobytes(), int((got != ref).sum())
    assert rt.canvas_to_ppm(got[None]) == oracle.canvas_to_ppm(ref[None])


def test_c3_full_frame_frames_in_flight_equal(rt):
    """bench.py's timed configuration: 4 frames in flight on 4 render streams
    (each its own workspace, device-sized generations), every frame bitwise
    equal to the exhaustive frame."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    exact, _ = _device_frame(cam, w, depth, True)
    streams = [rt.render_stream(False) for _ in range(4)]
    bufs = [torch.empty_like(exact) for _ in streams]
    for f in range(12):
        k = f % 4
        bufs[k].fill_(-1.0)
        torch.cuda.current_stream().synchronize()
        cam.render_shard_device(w, depth, 8, 0, 1, bufs[k].data_ptr(), streams[k].cuda_stream, False)
    torch.cuda.synchronize()
    for b in bufs:
        assert torch.equal(b, exact)


def test_c3_full_frame_aa_and_zoo_fast_equal_exhaustive(rt):
    """render_multithreaded X4 (camera.rs:150-253) at the full 1920x1080 of C3,
    and the feature zoo (every pattern, rotated / sheared solids, nested glass,
    a shadowless object, two lights) at 1920x1080: fast == exhaustive bitwise."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    for flags in (True, False):
        buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
        cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), torch.cuda.current_stream().cuda_stream, True,
                                exhaustive=flags, aa_samples=4)
        torch.cuda.synchronize()
        if flags:
            exact = buf
        else:
            assert torch.equal(buf, exact)
    del exact, buf
    w, cam, depth = scenes.zoo(1920, 1080)
    exact, _ = _device_frame(cam, w, depth, True)
    fast, _ = _device_frame(cam, w, depth, False)
    assert torch.equal(fast, exact)


def test_c5_full_frame_fast_equals_exhaustive(rt, oracle):
    """C5 at its full 4096x4096 (4 planes + 9996 spheres, 2 lights, depth 8):
    fast == exhaustive bitwise, and 2048 scattered pixels of the fast frame vs
    the oracle."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c5()
    exact, se = _device_frame(cam, w, depth, True)
    fast, sf = _device_frame(cam, w, depth, False)
    assert torch.equal(fast, exact)
    for k in RAY_KEYS:
        assert sf[k] == se[k], k
    del exact
    _check_pixels(rt, oracle, oracle.OracleWorld.from_world(w), cam, depth, fast, 2048, seed=5)
    del fast
    torch.cuda.empty_cache()


def test_host_render_stats_from_fast_path(rt, oracle):
    """rt_render with stats runs the fast path (asking for counters never
    changes the algorithm); the reference ray counts still equal the oracle's."""
    from rtamd import scenes
    w, cam, depth = scenes.c3(160, 90, n_spheres=300)
    fast, sf = cam.render(w, depth, want_stats=True, exhaustive=False)
    exact, se = cam.render(w, depth, want_stats=True)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()
    _, rst = oracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=NTHREADS)
    for k in RAY_KEYS:
        assert sf[k] == rst[k] == se[k], k
    assert se["sphere_disc_ge0"] == rst["sphere_disc_ge0"] and sf["sphere_disc_ge0"] is None


def test_render_multi_one_device_equals_render(rt):
    """rt_render_multi (render_multithreaded across devices, camera.rs:150) with
    n_devices = 1: bitwise equal to rt_render / rt_render_aa, on repeated calls
    (cached buffers), for AA and odd row blocks."""
    from rtamd import scenes
    w, cam, depth = scenes.c3(200, 113, n_spheres=300)
    ref, _ = cam.render(w, depth, want_stats=False)
    for row_block in (8, 3, 113):
        got, st = cam.render_multi([w], depth, row_block)
        assert got.to_numpy().tobytes() == ref.to_numpy().tobytes()
        assert st["rays_primary"] == 200 * 113 and st["sphere_disc_ge0"] is None
    _, se = cam.render(w, depth)
    for k in RAY_KEYS:
        assert st[k] == se[k], k
    cam.render_opts.aa_samples(rt.AASamples.X4)
    ref4, _ = cam.render_multithreaded(w, depth, want_stats=False)
    got4, st4 = cam.render_multi([w], depth, 8, 4)
    assert got4.to_numpy().tobytes() == ref4.to_numpy().tobytes()
    assert st4["rays_primary"] == 4 * 200 * 113


def test_arena_overflow_sync_rerenders_async_reports(rt):
    """Device-sized generations: the queue arenas are sized from a
    hint, and a generation that does not fit spawns no children and raises the
    workspace's overflow record. Forced here by shrinking the arenas to 2 % of
    the hint (test hook arena_pct):
    - a synchronous render (rt_render to a host canvas) notices it, grows the
      arenas and renders again: its frame is complete;
    - an asynchronous render (rt_render_shard_device) cannot finish the frame:
      its canvas is filled with NaN on the device (never a partial frame that
      looks valid, camera.rs:133-148), and rt_scene_check (or the next call)
      reports it; the arenas have grown, so the next frame is complete."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(96, 54, n_spheres=200)
    exact, _ = _device_frame(cam, w, depth, True)
    w.tune("arena_pct", 2)
    try:
        host, _ = cam.render(w, depth, want_stats=False)
    finally:
        w.tune("arena_pct", 100)
    assert host.to_numpy().tobytes() == exact.cpu().numpy().tobytes()
    st = rt.render_stream(False)
    buf = torch.empty_like(exact)
    w.tune("arena_pct", 2)
    try:
        cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), st.cuda_stream, False)
        torch.cuda.synchronize()
    finally:
        w.tune("arena_pct", 100)
    assert _valid_or_poisoned(buf, exact) == "poisoned"
    with pytest.raises(rt.RtError, match="overflow"):
        w.check()
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), st.cuda_stream, False)
    torch.cuda.synchronize()
    w.check()
    assert torch.equal(buf, exact)


def test_first_seen_cameras_async_bitwise(rt):
    """A fresh scene, 8 distinct cameras per batch on 4 streams, no render
    before: every call is asynchronous from its first frame (no calibration,
    device-sized generations) and every frame equals its exhaustive frame."""
    import math
    import torch
    from rtamd import scenes
    w, cam0, depth = scenes.c3(320, 180, n_spheres=600)
    cams = []
    for k in range(32):
        c = rt.Camera(320, 180, math.pi / 3.0)
        a = 2 * math.pi * k / 32
        c.set_transform(rt.view_transform(rt.Point(14 * math.sin(a), 2.5 + 0.1 * k, -14 * math.cos(a)),
                                          rt.Point(0, 1, 0), rt.Vector(0, 1, 0)))
        cams.append(c)
    streams = [rt.render_stream(False) for _ in range(4)]
    bufs = [torch.full((180, 320, 3), -1.0, dtype=torch.float64, device="cuda") for _ in cams]
    torch.cuda.synchronize()
    for b in range(4):
        rt.render_frames_device(w, cams[8 * b:8 * b + 8], depth, 8, 0, 1, [x.data_ptr() for x in bufs[8 * b:8 * b + 8]],
                                streams[b].cuda_stream)
    torch.cuda.synchronize()
    w.check()
    for k, c in enumerate(cams):
        exact, _ = _device_frame(c, w, depth, True)
        assert torch.equal(bufs[k], exact), k


@pytest.mark.parametrize("glass", [False, True])
def test_ray_classes_single_class_generations(rt, glass):
    """Ray classes (shard_append): between two mirror planes every generation
    is all plane reflections (the back ends of the reflected half's regions fill
    alone); with glass spheres between them, refractions entering and leaving
    join. Deep recursion, fast == exhaustive bitwise, counters equal."""
    import math
    w = rt.World()
    floor = rt.Plane()
    floor.material.reflective = 1.0
    floor.material.color = rt.Color(0.2, 0.3, 0.4)
    w.add_object(floor)
    ceil = rt.Plane()
    ceil.set_transform(rt.translation(0, 4, 0))
    ceil.material.reflective = 0.9
    w.add_object(ceil)
    rng = np.random.default_rng(3)
    for k in range(40 if glass else 0):
        s = rt.glass_sphere()
        r = rng.uniform(0.2, 0.6)
        s.set_transform(rt.translation(*rng.uniform([-6, r, -2], [6, 4 - r, 12])) * rt.scaling(r, r, r))
        s.material.refractive_index = 1.2 + 0.01 * k
        s.material.reflective = 0.5
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-5, 3.5, -5), rt.Color(1, 1, 1)))
    cam = rt.Camera(160, 120, math.pi / 2.5)
    cam.set_transform(rt.view_transform(rt.Point(0, 2, -6), rt.Point(0, 1.2, 4), rt.Vector(0, 1, 0)))
    exact, se = _device_frame(cam, w, 12, True)
    fast, sf = _device_frame(cam, w, 12, False)
    import torch
    assert torch.equal(fast, exact)
    for k in RAY_KEYS:
        assert sf[k] == se[k], k
    assert sf["rays_reflect"] > 10 * sf["rays_primary"]  # the mirrors keep every ray alive


@pytest.mark.parametrize("knob,value,image", [("prim_lane", 1, 0), ("prim_lane", 1, 3), ("prim_lane", 0, 0),
                                              ("prim_lane", 2, 3)])
def test_fast_path_variants_bitwise(rt, knob, value, image):
    """The fast path's measured variants: primary rays by the
    per-lane pair traversal over the LDS image (image 0) or by the per-lane
    four-wide walk of the global-memory image (image 3) instead of the wave
    traversal. Each frame equals the exhaustive frame bit for bit, alone and
    in a batch of 3 cameras (root rays not a multiple of 64: padded chunks)."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(333, 187)
    exact, _ = _device_frame(cam, w, depth, True)
    w.tune("image", image)
    w.tune(knob, value)
    try:
        fast, _ = _device_frame(cam, w, depth, False)
        assert torch.equal(fast, exact)
        bufs = [torch.full_like(exact, -1.0) for _ in range(3)]
        rt.render_frames_device(w, [cam] * 3, depth, 8, 0, 1, [b.data_ptr() for b in bufs],
                                torch.cuda.current_stream().cuda_stream, False, 1)
        torch.cuda.synchronize()
        w.check()
        for b in bufs:
            assert torch.equal(b, exact)
    finally:
        w.tune(knob, 1)  # (the default: the per-lane walk for primary rays over any image)
        w.tune("image", 0)


def _valid_or_poisoned(buf, exact):
    """An asynchronous frame is either complete (bitwise the exhaustive frame)
    or entirely NaN (it outgrew its queue arenas); anything else fails."""
    import torch
    if torch.equal(buf, exact):
        return "complete"
    assert bool(torch.isnan(buf).all()), "an incomplete frame that is not poisoned"
    return "poisoned"


@pytest.mark.parametrize("aa", [1, 4])
def test_arena_overflow_batch_poisoned(rt, aa):
    """rt_render_frames_device (batches) with forced overflows (arena_pct): every
    frame of an overflowing pass is all NaN, never a partial canvas, for plain
    and AA frames (wf_average); the overflow is reported once; after it the
    arenas fit and the same batch renders every frame bitwise. With arenas at
    60 % of the hint a pass may or may not fit: each frame is still either
    complete or poisoned."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(128, 72, n_spheres=300)
    exact = torch.empty((72, 128, 3), dtype=torch.float64, device="cuda")
    cam.render_shard_device(w, depth, 8, 0, 1, exact.data_ptr(), torch.cuda.current_stream().cuda_stream, True,
                            exhaustive=True, aa_samples=aa)
    torch.cuda.synchronize()
    st = rt.render_stream(False)
    bufs = [torch.full_like(exact, -1.0) for _ in range(5)]

    def batch():
        rt.render_frames_device(w, [cam] * len(bufs), depth, 8, 0, 1, [b.data_ptr() for b in bufs], st.cuda_stream,
                                False, aa)
        torch.cuda.synchronize()
    batch()  # learn the scene's sizes
    w.check()
    for pct, want in ((2, "poisoned"), (60, None)):
        w.tune("arena_pct", pct)
        try:
            for b in bufs:
                b.fill_(-1.0)
            batch()
        finally:
            w.tune("arena_pct", 100)
        kinds = {_valid_or_poisoned(b, exact) for b in bufs}
        assert len(kinds) == 1  # one pass: all its frames complete, or all poisoned
        if want:
            assert kinds == {want}
        if kinds == {"poisoned"}:
            with pytest.raises(rt.RtError, match="overflow"):
                w.check()
        w.check()  # reported once
        batch()
        w.check()
        for b in bufs:
            assert torch.equal(b, exact)


@pytest.mark.parametrize("aa", [2, 4])
def test_host_render_banded_aa_bitwise(rt, aa):
    """render_multithreaded with AA (camera.rs:150-253) into a host canvas of
    the full C3 frame goes through the row bands too (n_pix * aa >= 2^20): each
    band averages its own pixels' samples; bitwise the exhaustive device frame,
    and identical to the unbanded host render."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), torch.cuda.current_stream().cuda_stream, True,
                            exhaustive=True, aa_samples=aa)
    torch.cuda.synchronize()
    ref = buf.cpu().numpy().tobytes()
    cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
    banded, _ = cam.render_multithreaded(w, depth, want_stats=False)
    assert banded.to_numpy().tobytes() == ref
    w.tune("bands", 1)
    try:
        whole, _ = cam.render_multithreaded(w, depth, want_stats=False)
    finally:
        w.tune("bands", 4)
    assert whole.to_numpy().tobytes() == ref


@pytest.mark.parametrize("bands,pct,gen,ratio", [(4, 35, 1, 100), (2, 55, -1, 100), (3, 40, -1, 100),
                                                 (4, 25, -1, 100), (1, 55, -1, 100), (2, 60, 1, 100),
                                                 (3, 45, 0, 70), (4, 45, 2, 60)])
def test_host_render_banded_bitwise(rt, bands, pct, gen, ratio):
    """rt_render into a host canvas (Camera::render -> Canvas, camera.rs:133-148)
    of the full 1920x1080 C3 frame in row bands, each band's device-to-host copy
    behind its render: bitwise the exhaustive frame, into a
    pageable and into a pinned canvas; with arenas forced to overflow, every band
    is still complete (re-rendered before the call returns). `gen` >= 0: each
    band starts once the previous band's generation `gen` has been launched
    (band_gen), so consecutive bands' renders overlap."""
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    exact, _ = _device_frame(cam, w, depth, True)
    ref = exact.cpu().numpy().tobytes()
    w.tune("bands", bands)
    w.tune("band_pct", pct)
    w.tune("band_gen", gen)
    w.tune("band_ratio", ratio)
    try:
        for _ in range(2):
            host, _ = cam.render(w, depth, want_stats=False)
            assert host.to_numpy().tobytes() == ref
        w.tune("arena_pct", 30)
        host, _ = cam.render(w, depth, want_stats=False)
        assert host.to_numpy().tobytes() == ref
    finally:
        w.tune("arena_pct", 100)
        w.tune("bands", 4)
        w.tune("band_pct", 35)
        w.tune("band_gen", 1)
        w.tune("band_ratio", 100)
    w.check()
