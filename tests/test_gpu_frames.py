"""Batches of frames (rt_render_frames_device, DESIGN.md §5.8 "Frame
batches"): up to 16 cameras share each launch of the generation pipeline.
Every frame of a batch must equal the same camera's rt_render_shard_device
frame bit for bit (itself checked against the exhaustive frame and the
oracle elsewhere), for whole frames and shards, with and without AA, ragged
frame sizes (root rays not a multiple of 64), more frames than one pass
holds, and scenes the batch cannot take (rendered frame by frame)."""
import math

import pytest

pytestmark = pytest.mark.gpu
PI = math.pi


def _cameras(rt, n, w, h):
    cams = []
    for k in range(n):
        c = rt.Camera(w, h, PI / 3.0)
        a = 2 * PI * k / max(n, 1)
        c.set_transform(rt.view_transform(rt.Point(12 * math.sin(a), 3 + 0.3 * k, -12 * math.cos(a)),
                                          rt.Point(0, 1, 5), rt.Vector(0, 1, 0)))
        cams.append(c)
    return cams


def _check(rt, w, cams, depth, row_block, shard, n_shards, aa=1):
    import torch
    rows = rt.shard_rows(cams[0].vsize, row_block, shard, n_shards)
    bat = [torch.full((rows, cams[0].hsize, 3), -1.0, dtype=torch.float64, device="cuda") for _ in cams]
    one = [torch.full_like(b, -2.0) for b in bat]
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    rt.render_frames_device(w, cams, depth, row_block, shard, n_shards, [b.data_ptr() for b in bat], st, False, aa)
    for c, b in zip(cams, one):
        c.render_shard_device(w, depth, row_block, shard, n_shards, b.data_ptr(), st, False, aa)
    torch.cuda.synchronize()
    w.check()
    for k, (b, o) in enumerate(zip(bat, one)):
        assert torch.equal(b, o), k
    # the same cameras again, into fresh buffers, take the
    # asynchronous path the bench times (sizes from the scene's learned sizing,
    # the device queue check afterwards): bitwise the same frames.
    again = [torch.full_like(b, -3.0) for b in bat]
    torch.cuda.synchronize()
    rt.render_frames_device(w, cams, depth, row_block, shard, n_shards, [b.data_ptr() for b in again], st, False, aa)
    torch.cuda.synchronize()
    w.check()
    for k, (b, o) in enumerate(zip(again, one)):
        assert torch.equal(b, o), ("again", k)


@pytest.mark.parametrize("n", [2, 16, 19])
def test_frames_whole_bitwise(rt, n):
    from rtamd import scenes
    w, _, depth = scenes.c3(96, 54, n_spheres=400)
    _check(rt, w, _cameras(rt, n, 96, 54), depth, 8, 0, 1)


@pytest.mark.parametrize("shard", [0, 3, 7])
def test_frames_shards_bitwise(rt, shard):
    from rtamd import scenes
    w, _, depth = scenes.c3(200, 113, n_spheres=600)
    _check(rt, w, _cameras(rt, 5, 200, 113), depth, 8, shard, 8)


@pytest.mark.parametrize("aa", [2, 4])
def test_frames_aa_bitwise(rt, aa):
    from rtamd import scenes
    w, _, depth = scenes.c3(37, 23, n_spheres=300)  # ragged: 37*23*aa root rays per frame
    _check(rt, w, _cameras(rt, 6, 37, 23), depth, 8, 1, 2, aa)


@pytest.mark.parametrize("hw", [(1, 1), (7, 3), (65, 1)])
def test_frames_tiny(rt, hw):
    from rtamd import scenes
    w, _, depth = scenes.c3(8, 8, n_spheres=100)
    _check(rt, w, _cameras(rt, 3, *hw), depth, 8, 0, 1)


def test_frames_zoo_and_deep(rt):
    """Every shape kind and pattern (the other-shape hierarchy) and deep recursion."""
    from rtamd import scenes
    w, cam, _ = scenes.zoo(64, 48)
    cams = _cameras(rt, 4, 64, 48)
    _check(rt, w, cams, 5, 8, 0, 1)
    _check(rt, w, cams, 12, 8, 0, 1)


def test_frames_unbatchable_scene(rt):
    """A scene without the fast path's hierarchies (planes only) is rendered
    frame by frame by the same call."""
    w = rt.World()
    fl = rt.Plane()
    fl.material.reflective = 0.5
    w.add_object(fl)
    wall = rt.Plane()
    wall.set_transform(rt.translation(0, 0, 10) * rt.rotation_x(PI / 2))
    w.add_object(wall)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1, 1, 1)))
    _check(rt, w, _cameras(rt, 3, 40, 30), 5, 8, 0, 1)


def test_frames_stats_sum(rt):
    """With stats the frames are counted one by one and the counters summed."""
    import torch
    from rtamd import scenes
    w, _, depth = scenes.c3(64, 36, n_spheres=200)
    cams = _cameras(rt, 3, 64, 36)
    bufs = [torch.empty((36, 64, 3), dtype=torch.float64, device="cuda") for _ in cams]
    st = rt.render_frames_device(w, cams, depth, 8, 0, 1, [b.data_ptr() for b in bufs], 0, True)
    tot = {}
    for c in cams:
        _, s = c.render(w, depth, want_stats=True, exhaustive=False)
        for k in ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "plane_tests"):
            tot[k] = tot.get(k, 0) + s[k]
    for k, v in tot.items():
        assert st[k] == v, k


def test_bindings_keep_the_uploaded_scene(rt):
    """tune / check / render_frames_device / render must reuse
    the scene a rank uploaded to its own device and never re-upload it to
    device 0. The scene is relabelled as if it lived on GPU 5 (one-GPU box);
    any path that asked for device 0 would drop and recreate it."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(32, 18, n_spheres=50)
    w.upload(0)
    h = w._scene_handle()
    w._debug_relabel_device(5)
    w.tune("skip_shadow", 1)
    w.check()
    b = torch.empty((18, 32, 3), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    rt.render_frames_device(w, [cam, cam], depth, 8, 0, 1, [b.data_ptr(), b.data_ptr()],
                            torch.cuda.current_stream().cuda_stream)
    cam.render_shard_device(w, depth, 8, 0, 1, b.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    w.check()
    cam.render(w, depth, want_stats=False)
    assert w._scene_handle() == h and w.scene_device == 5
    w._debug_relabel_device(0)


def test_frames_errors(rt):
    import torch
    from rtamd import scenes
    w, _, depth = scenes.c3(16, 16, n_spheres=10)
    b = torch.empty((16, 16, 3), dtype=torch.float64, device="cuda")
    with pytest.raises(rt.RtError):  # sizes differ
        rt.render_frames_device(w, [rt.Camera(16, 16, 1.0), rt.Camera(16, 8, 1.0)], depth, 8, 0, 1,
                                [b.data_ptr(), b.data_ptr()])
    with pytest.raises(rt.RtError):
        rt.render_frames_device(w, [rt.Camera(16, 16, 1.0)], depth, 8, 1, 1, [b.data_ptr()])
    with pytest.raises(rt.RtError):
        rt.render_frames_device(w, [rt.Camera(16, 16, 1.0)], depth, 8, 0, 1, [b.data_ptr()], 0, False, 3)
    rt.render_frames_device(w, [], depth, 8, 0, 1, [])  # nothing to render


def test_frames_pass_cap(rt):
    """A pass holds at most 2^25 root rays: 1024x1024 frames at AA 16 (2^24 root
    rays each) go two per pass, so 3 frames make a pass of 2 and a pass of 1."""
    from rtamd import scenes
    w, _, depth = scenes.c3(1024, 1024, n_spheres=200)
    _check(rt, w, _cameras(rt, 3, 1024, 1024), depth, 8, 0, 1, aa=16)


@pytest.mark.parametrize("n_ranks,share,aa", [(8, 0.75, 1), (4, 0.9, 1), (3, 0.8, 4), (8, 1.0, 1), (2, 0.5, 2)])
def test_block_pattern_frames_bitwise(rt, n_ranks, share, aa):
    """rt_render_block_pattern_device (ABI 6): every rank's rows of a block
    pattern (rtamd.distributed.block_patterns, rank 0 at `share` of an equal
    share), for a batch of cameras and one camera, equal the same rows of the
    whole exhaustive frame bit for bit; the ranks' rows cover the frame once.
    The plain pattern (share 1) equals rt_render_frames_device's shards."""
    import torch
    from rtamd import scenes
    from rtamd.distributed import block_patterns, pattern_row_ids
    w, _, depth = scenes.c3(120, 77, n_spheres=300)
    cams = _cameras(rt, 3, 120, 77)
    st = torch.cuda.current_stream().cuda_stream
    whole = []
    for c in cams:
        b = torch.empty((77, 120, 3), dtype=torch.float64, device="cuda")
        c.render_shard_device(w, depth, 8, 0, 1, b.data_ptr(), st, True, aa, exhaustive=True)
        whole.append(b)
    period, masks = block_patterns(n_ranks, share)
    covered = []
    for r, m in enumerate(masks):
        rows = pattern_row_ids(77, 8, period, m)
        assert len(rows) == rt.pattern_rows(77, 8, period, m)
        covered += rows
        bufs = [torch.full((len(rows), 120, 3), -1.0, dtype=torch.float64, device="cuda") for _ in cams]
        rt.render_block_pattern_device(w, cams, depth, 8, period, m, [b.data_ptr() for b in bufs], st, False, aa)
        one = torch.full_like(bufs[0], -2.0)
        rt.render_block_pattern_device(w, cams[:1], depth, 8, period, m, [one.data_ptr()], st, False, aa)
        torch.cuda.synchronize()
        w.check()
        idx = torch.tensor(rows, device="cuda")
        for k, b in enumerate(bufs):
            assert torch.equal(b, whole[k].index_select(0, idx)), (r, k)
        assert torch.equal(one, bufs[0])
        if share == 1.0:  # the plain interleave: mask 1 << r is shard r of n
            sh = torch.full_like(one, -3.0)
            cams[0].render_shard_device(w, depth, 8, r, n_ranks, sh.data_ptr(), st, False, aa)
            torch.cuda.synchronize()
            assert torch.equal(sh, one)
    assert sorted(covered) == list(range(77))
    with pytest.raises(rt.RtError, match="block pattern"):
        rt.render_block_pattern_device(w, cams[:1], depth, 8, 8, 1 << 9, [whole[0].data_ptr()], st)
    counted = rt.render_block_pattern_device(w, cams[:1], depth, 8, period, masks[0], [whole[0].data_ptr()], st,
                                             True, aa, True)
    assert counted["exhaustive"] and counted["rays_primary"] == aa * 120 * len(pattern_row_ids(77, 8, period,
                                                                                               masks[0]))
