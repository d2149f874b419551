"""The persistent frame kernel (rt_persist.hip, DESIGN.md §5.1 "Persistent
frames"): one launch renders every recursion depth, with shade_hit's combine
folded into the children's delivery (an atomic countdown per parent record).
It is an opt-in fast path (WfTuning::persist) for max_depth <= 8; every frame
here must equal the exhaustive frame (the reference's every-shape loop, itself
checked against the oracle) bit for bit, and its counters must equal the
reference's."""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
PI = math.pi


def _glass(rt, n=200, seed=7, inside=False):
    rng = np.random.default_rng(seed)
    w = rt.World()
    floor = rt.Plane()
    floor.material.reflective = 0.3
    w.add_object(floor)
    for i in range(n):
        s = rt.glass_sphere() if i % 3 else rt.Sphere()
        r = rng.uniform(0.2, 0.9)
        s.set_transform(rt.translation(*rng.uniform([-3, r, -3], [3, 3, 3])) * rt.scaling(r, r, r))
        s.material.refractive_index = 1.0 + rng.uniform(0, 1.5)
        s.material.reflective = rng.uniform(0, 0.9)
        s.material.color = rt.Color(*rng.uniform(0, 1, 3))
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    w.tune("persist", 1)
    cam = rt.Camera(80, 56, PI / 2.5)
    frm = (0.2, 1.1, -0.4) if inside else (0, 2, -9)
    cam.set_transform(rt.view_transform(rt.Point(*frm), rt.Point(0, 1, 2), rt.Vector(0, 1, 0)))
    return w, cam


@pytest.mark.parametrize("depth", [0, 1, 2, 5, 8, 9])
@pytest.mark.parametrize("inside", [False, True])
def test_persist_frames_bitwise(rt, depth, inside):
    w, cam = _glass(rt, inside=inside)
    fast, _ = cam.render(w, depth, want_stats=False)
    p = rt._rtamd._wf_profile(w, -1, True)
    assert p["persist"] == (depth <= 8)  # deeper recursion takes the generation pipeline
    exact, _ = cam.render(w, depth, want_stats=True)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()


@pytest.mark.parametrize("name", ["c3", "zoo", "solids", "first_scene"])
def test_persist_scenes_bitwise(rt, name):
    from rtamd import scenes
    w, cam, depth = {"c3": lambda: scenes.c3(192, 108), "zoo": lambda: scenes.zoo(120, 90),
                     "solids": lambda: scenes.solids(120, 90),
                     "first_scene": lambda: scenes.first_scene(160, 90)}[name]()
    w.tune("persist", 1)
    fast, _ = cam.render(w, depth, want_stats=False)
    assert rt._rtamd._wf_profile(w, -1, True)["persist"]
    exact, _ = cam.render(w, depth, want_stats=True)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()


def test_persist_counters_equal_reference(rt):
    """A counted persistent frame (stats, fast path) counts exactly the
    reference's rays: its per-depth tallies replace the generation queues."""
    w, cam = _glass(rt, n=150, seed=3)
    _, ex = cam.render(w, 6, want_stats=True)
    _, fs = cam.render(w, 6, want_stats=True, exhaustive=False)
    assert rt._rtamd._wf_profile(w, -1, True)["persist"]
    for k in ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "plane_tests"):
        assert fs[k] == ex[k], k
    assert 0 < fs["rays_shadow_traced"] <= ex["rays_shadow"]
    assert not fs["exhaustive"] and fs["sphere_disc_ge0"] is None


@pytest.mark.parametrize("aa", [2, 16])
def test_persist_aa_bitwise(rt, aa):
    w, cam = _glass(rt, n=100, seed=11)
    cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
    fast, _ = cam.render_multithreaded(w, 5, want_stats=False)
    assert rt._rtamd._wf_profile(w, -1, True)["persist"]
    exact, _ = cam.render_multithreaded(w, 5, want_stats=True)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()


def test_persist_color_at_batch(rt):
    w, _ = _glass(rt, n=300, seed=5, inside=True)
    rng = np.random.default_rng(2)
    o = rng.uniform([-4, -0.5, -4], [4, 4, 4], size=(30001, 3))
    d = rng.normal(size=(30001, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.hstack([o, d])
    for depth in (0, 3, 8):
        fast, _ = w.color_at_batch(rays, depth, want_stats=False)
        assert rt._rtamd._wf_profile(w, -1, True)["persist"]
        exact, _ = w.color_at_batch(rays, depth, want_stats=True)
        assert fast.tobytes() == exact.tobytes(), depth


@pytest.mark.parametrize("hw", [(1, 1), (3, 2), (9, 7), (65, 1)])
def test_persist_tiny_frames(rt, hw):
    """Fewer root rays than one chunk, one workgroup, ragged last chunk."""
    w, _ = _glass(rt, n=60, seed=9)
    cam = rt.Camera(hw[0], hw[1], PI / 3)
    cam.set_transform(rt.view_transform(rt.Point(0, 2, -9), rt.Point(0, 1, 2), rt.Vector(0, 1, 0)))
    fast, _ = cam.render(w, 5, want_stats=False)
    exact, _ = cam.render(w, 5, want_stats=True)
    assert fast.to_numpy().tobytes() == exact.to_numpy().tobytes()


def test_persist_back_to_back_and_shards(rt):
    """Frame after frame on one workspace (the last workgroup of each launch
    zeroes the next launch's counters) and 8-way shards on several streams,
    all equal to the exhaustive frame."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(240, 136, n_spheres=600)
    w.tune("persist", 1)
    full, _ = cam.render(w, depth, want_stats=True)
    full = torch.from_numpy(full.to_numpy()).cuda()
    st = torch.cuda.current_stream().cuda_stream
    bufs = [torch.full_like(full, -1.0) for _ in range(12)]
    for b in bufs:
        cam.render_shard_device(w, depth, 8, 0, 1, b.data_ptr(), st, False)
    streams = [rt.render_stream() for _ in range(4)]
    shards = [torch.full((rt.shard_rows(cam.vsize, 8, s, 8), cam.hsize, 3), -1.0, dtype=torch.float64, device="cuda")
              for s in range(8)]
    torch.cuda.synchronize()  # the fills (current stream) before the renders (other streams)
    for s in range(8):
        cam.render_shard_device(w, depth, 8, s, 8, shards[s].data_ptr(), streams[s % 4].cuda_stream, False)
    torch.cuda.synchronize()
    w.check()
    for b in bufs:
        assert torch.equal(b, full)
    for s, buf in enumerate(shards):
        rows = [y for y in range(cam.vsize) if (y // 8) % 8 == s]
        assert torch.equal(buf, full[rows])


def test_persist_off_matches(rt):
    """The generation pipeline (persist off, the default) renders the same frame."""
    w, cam = _glass(rt, n=200, seed=17)
    a, _ = cam.render(w, 6, want_stats=False)
    w.tune("persist", 0)
    try:
        b, _ = cam.render(w, 6, want_stats=False)
        p = rt._rtamd._wf_profile(w, -1, True)
        assert p["fused"] and not p["persist"]
    finally:
        w.tune("persist", 1)
    assert a.to_numpy().tobytes() == b.to_numpy().tobytes()
