"""`render_multithreaded` across devices (camera.rs:150-217): rt_render_multi.

The multi-device entry point returns a host canvas, like the reference's owned
`Canvas`. Each device renders its interleaved row blocks (the reference's
row-block partition, camera.rs:157-172) and copies them straight into the
canvas rows it owns over its own link; the RCCL form (every shard gathered
into device 0 by one grouped `ncclGather`) stays behind the scene knob
`multi_gather`.

One GPU runs every part of both forms here:
- the RCCL form through a single-rank communicator (`ncclCommInitAll` over one
  device, then the same grouped gather an 8-device call issues), including a
  forced arena overflow that renders and gathers the frame again;
- the direct form's per-device work (`_render_shard_host`: one shard rendered
  and copied into its rows of a full-size canvas, a 2-D copy for its row
  blocks) for 2, 3, 4 and 8 shards, sequentially and from concurrent host
  threads, as rt_render_multi's workers run it.
Every canvas must equal rt_render's bit for bit.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
RAY_KEYS = ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "plane_tests",
            "other_tests")


def _small():
    from rtamd import scenes
    return scenes.c3(200, 113, n_spheres=300)


def test_multi_rccl_gather_single_rank_bitwise(rt):
    """rt_render_multi's RCCL form on one device (ncclCommInitAll + grouped
    ncclGather through a single-rank communicator): bitwise rt_render, for
    odd row blocks, AA X4 and repeated calls (cached communicator)."""
    w, cam, depth = _small()
    ref, _ = cam.render(w, depth, want_stats=False)
    w.tune("multi_gather", 1)
    try:
        for row_block in (8, 3, 113, 8):
            got, st = cam.render_multi([w], depth, row_block)
            assert got.to_numpy().tobytes() == ref.to_numpy().tobytes(), row_block
            assert st["rays_primary"] == 200 * 113
        _, se = cam.render(w, depth)
        for k in RAY_KEYS:
            assert st[k] == se[k], k
        cam.render_opts.aa_samples(rt.AASamples.X4)
        ref4, _ = cam.render_multithreaded(w, depth, want_stats=False)
        got4, st4 = cam.render_multi([w], depth, 8, 4)
        assert got4.to_numpy().tobytes() == ref4.to_numpy().tobytes()
        assert st4["rays_primary"] == 4 * 200 * 113
    finally:
        w.tune("multi_gather", 0)


def test_multi_rccl_gather_forced_overflow(rt):
    """The RCCL form with the queue arenas shrunk to 5 % of their hint (test
    hook arena_pct): the shard overflows, the call grows the arenas, renders
    and gathers the frame again, and returns the complete frame."""
    w, cam, depth = _small()
    ref, _ = cam.render(w, depth, want_stats=False)
    w.tune("multi_gather", 1)
    w.tune("arena_pct", 5)
    try:
        for _ in range(2):
            got, _ = cam.render_multi([w], depth, 8)
            assert got.to_numpy().tobytes() == ref.to_numpy().tobytes()
        w.check()
    finally:
        w.tune("arena_pct", 100)
        w.tune("multi_gather", 0)


def test_multi_direct_one_device_full_size(rt):
    """The direct form at C3's full 1920x1080 on one device (the banded path:
    each band's copy behind the next band's render): bitwise rt_render, also
    with a forced overflow."""
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    ref, _ = cam.render(w, depth, want_stats=False)
    got, _ = cam.render_multi([w], depth, 8)
    assert got.to_numpy().tobytes() == ref.to_numpy().tobytes()
    w.tune("arena_pct", 5)
    try:
        got, _ = cam.render_multi([w], depth, 8)
        assert got.to_numpy().tobytes() == ref.to_numpy().tobytes()
    finally:
        w.tune("arena_pct", 100)
    w.check()


@pytest.mark.parametrize("n,row_block", [(2, 8), (3, 5), (4, 8), (8, 8), (8, 17)])
def test_shard_parts_assemble_bitwise(rt, n, row_block):
    """Every device's part of the direct form, run on one device: shard i of n
    renders and 2-D-copies its row blocks into a full-size pageable canvas
    (registered for the call); the assembled canvas equals rt_render, and the
    parts' counters sum to the whole frame's."""
    w, cam, depth = _small()
    ref, se = cam.render(w, depth)
    canvas = np.full((cam.vsize, cam.hsize, 3), np.nan)
    tot = dict.fromkeys(RAY_KEYS, 0)
    for i in range(n):
        st = rt._rtamd._render_shard_host(w, cam, depth, row_block, i, n, canvas, 1, True)
        for k in RAY_KEYS:
            tot[k] += st[k]
    assert canvas.tobytes() == ref.to_numpy().tobytes()
    for k in RAY_KEYS:
        assert tot[k] == se[k], k


@pytest.mark.parametrize("pinned", [True, False])
def test_shard_parts_concurrent_threads_full_size(rt, pinned):
    """rt_render_multi's workers as it runs them, on one device: 8 host threads,
    each rendering and copying its shard of C3's full frame at once into one
    canvas (a pinned pool block, or pageable memory that the concurrent parts
    register once between them); bitwise rt_render."""
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    ref, _ = cam.render(w, depth, want_stats=False)
    H, W = cam.vsize, cam.hsize
    if pinned:
        canvas = rt._rtamd.host_buffer(H * W * 3 * 8).view(np.float64).reshape(H, W, 3)
    else:
        canvas = np.full((H, W, 3), np.nan)
    errors = []

    def part(i):
        try:
            rt._rtamd._render_shard_host(w, cam, depth, 8, i, 8, canvas, 1, False)
        except Exception as e:  # reported below
            errors.append(e)
    for _ in range(2):
        canvas[:] = np.nan
        th = [threading.Thread(target=part, args=(i,)) for i in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        assert canvas.tobytes() == ref.to_numpy().tobytes()
    w.check()
