"""Split generations (WfTuning::split): each generation of the fast path as a
walk launch (wf_walk: closest hits only, a lane takes the generation's next ray
as soon as its walk is done) and a shading launch that reads the hits
(wf_trace_fused<..., SPLIT>). Every frame must equal the fused pipeline's, and
so the exhaustive (every-shape) frame, bit for bit: the walk visits, tests
and keeps exactly what lane_trace_wide does for each ray (world.rs:31-38,
intersection.rs:108-120)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(cam, w, depth, exhaustive=False, aa=1):
    import torch
    buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), torch.cuda.current_stream().cuda_stream, False,
                            aa_samples=aa, exhaustive=exhaustive)
    torch.cuda.synchronize()
    return buf


def _scenes():
    from rtamd import scenes
    return [("c3_small", scenes.c3(320, 180, n_spheres=400)), ("zoo", scenes.zoo()), ("solids", scenes.solids()),
            ("first_scene", scenes.first_scene(320, 180)), ("groups", scenes.groups())]


@pytest.mark.parametrize("refill", [1, 16, 64])
def test_split_equals_fused_and_exhaustive(rt, refill):
    """Small scenes (spheres only, planes, solids and patterns, groups): the
    split frame equals the fused frame and the exhaustive frame, for refill
    thresholds 1, 16 and 64 (64: a wave refills only when all its lanes are
    idle), with and without AA."""
    import torch
    for name, (w, cam, depth) in _scenes():
        fused = _frame(cam, w, depth)
        exact = _frame(cam, w, depth, exhaustive=True)
        w.tune("split", 1)
        w.tune("refill", refill)
        try:
            split = _frame(cam, w, depth)
            split4 = _frame(cam, w, depth, aa=4)
        finally:
            w.tune("split", 0)
            w.tune("refill", 16)
        fused4 = _frame(cam, w, depth, aa=4)
        assert torch.equal(split, fused), name
        assert torch.equal(split, exact), name
        assert torch.equal(split4, fused4), name
        w.check()


def test_split_full_size_c3_batches(rt):
    """C3 at 1920x1080 in batches of 8 frames (the benched launches, every
    generation split): each frame equals the exhaustive frame, and so does
    rt_render's banded host canvas rendered split."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    exact = _frame(cam, w, depth, exhaustive=True)
    w.tune("split", 1)
    try:
        bufs = [torch.empty_like(exact) for _ in range(8)]
        rt.render_frames_device(w, [cam] * 8, depth, 8, 0, 1, [b.data_ptr() for b in bufs],
                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        w.check()
        for b in bufs:
            assert torch.equal(b, exact)
        host, _ = cam.render(w, depth, want_stats=False)  # rt_render's banded host path, split
        assert np.array_equal(host.to_numpy(), exact.cpu().numpy())
    finally:
        w.tune("split", 0)
