"""The boundary's threading and device contract (include/rt_render.h,
"Threads and devices"; SURVEY.md §8b: callable from any host thread).

- Every entry point restores the caller's current HIP device before it
  returns, whether it succeeds or fails (a multi-device caller's own choice of
  device survives the call).
- Host threads may call the synchronous entry points on one scene at once:
  each call leases a context of its own (stream, device buffers) and waits on
  the device without the scene's lock, and every frame is the frame a
  sequential call renders.
"""
import ctypes
import math
import os
import threading

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "raytracer-challenge-rs_amd", "lib", "librtamd.so")


def _hip():
    try:
        return ctypes.CDLL("libamdhip64.so")
    except OSError:
        return ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")


def _current_device(hip):
    d = ctypes.c_int(-7)
    rc = hip.hipGetDevice(ctypes.byref(d))
    return rc, d.value


def test_failing_calls_leave_the_current_device(rt):
    """Calls that fail (bad arguments, no usable device on a CPU host, a bad
    device ordinal) leave hipGetDevice's answer as it was."""
    hip = _hip()
    lib = ctypes.CDLL(LIB)
    before = _current_device(hip)
    out = ctypes.c_void_p()
    shape = (ctypes.c_char * int(lib.rt_sizeof_shape_desc()))()
    assert lib.rt_scene_create(shape, 0, None, 0, 9999, ctypes.byref(out)) != 0  # bad ordinal (or no device)
    assert lib.rt_render(None, None, 5, None, None) != 0
    assert lib.rt_scene_check(None) != 0
    assert _current_device(hip) == before


@pytest.mark.gpu
def test_calls_restore_the_current_device(rt):
    """On the GPU box: successful and failing calls on a scene of device 0 all
    return with the caller's current device unchanged."""
    from rtamd import scenes
    hip = _hip()
    w, cam, depth = scenes.c3(32, 18, n_spheres=20)
    w.upload(0)
    assert hip.hipSetDevice(0) == 0
    before = _current_device(hip)
    cam.render(w, depth, want_stats=False)
    big = rt.Camera(50000, 50000, 1.0)  # a shard of 2.5e9 root rays: refused after the device is selected
    with pytest.raises(rt.RtError):
        big.render_shard_device(w, depth, 8, 0, 1, 8)  # (never written: refused first)
    w.check()
    assert _current_device(hip) == before


@pytest.mark.gpu
def test_concurrent_host_renders_of_one_scene(rt):
    """Six threads render six cameras of one scene at once through rt_render
    (the GIL is released inside), plus rt_render_ppm and rt_color_at_batch
    threads: every result equals the same call made alone."""
    import numpy as np
    from rtamd import scenes
    w, _, depth = scenes.c3(160, 90, n_spheres=300)
    cams = [scenes.c3_orbit(k, 6, 160, 90) for k in range(6)]
    alone = [c.render(w, depth, want_stats=False)[0].to_numpy() for c in cams]
    ppm_alone, _ = cams[0].render_ppm(w, depth)
    rng = np.random.default_rng(3)
    rays = np.concatenate([rng.uniform(-5, 5, (4096, 3)), rng.normal(size=(4096, 3))], 1)
    rays[:, 1] = np.abs(rays[:, 1]) + 0.5
    rays[:, 3:] /= np.linalg.norm(rays[:, 3:], axis=1, keepdims=True)
    col_alone, _ = w.color_at_batch(rays, depth, False)
    got, errors = {}, []

    def run(key, fn):
        try:
            for _ in range(3):
                got[key] = fn()
        except Exception as e:  # pragma: no cover - reported below
            errors.append((key, e))

    threads = [threading.Thread(target=run, args=(k, lambda c=c: c.render(w, depth, want_stats=False)[0].to_numpy()))
               for k, c in enumerate(cams)]
    threads.append(threading.Thread(target=run, args=("ppm", lambda: cams[0].render_ppm(w, depth)[0])))
    threads.append(threading.Thread(target=run, args=("col", lambda: w.color_at_batch(rays, depth, False)[0])))
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
    w.check()
    for k in range(6):
        assert got[k].tobytes() == alone[k].tobytes(), k
    assert bytes(got["ppm"]) == bytes(ppm_alone)
    assert got["col"].tobytes() == col_alone.tobytes()
    assert math.isfinite(float(alone[0].sum()))


def _run_threads(jobs, rounds=3):
    """Run each (key, fn) in its own thread `rounds` times; results of the last round, and errors."""
    got, errors = {}, []

    def run(key, fn):
        try:
            for _ in range(rounds):
                got[key] = fn()
        except Exception as e:  # pragma: no cover - reported by the caller
            errors.append((key, e))

    threads = [threading.Thread(target=run, args=kf) for kf in jobs]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    return got, errors


@pytest.mark.gpu
def test_render_multi_and_render_threads_with_overflows(rt):
    """rt_render_multi and rt_render from two threads on one scene while every
    arena overflows (test hook arena_pct = 2 %): each synchronous call takes
    the overflow flags of the workspaces it used only, re-renders its own frame
    and returns it complete; no call swallows or reports another's overflow,
    so the scene is clean afterwards (advisor, round 4)."""
    from rtamd import scenes
    w, cam, depth = scenes.c3(96, 54, n_spheres=200)
    cam2 = scenes.c3_orbit(3, 8, 96, 54)
    a_ref = cam.render(w, depth, want_stats=False)[0].to_numpy()
    b_ref = cam2.render(w, depth, want_stats=False)[0].to_numpy()
    w.tune("arena_pct", 2)
    try:
        got, errors = _run_threads([("multi", lambda: cam.render_multi([w], depth, 8)[0].to_numpy()),
                                    ("render", lambda: cam2.render(w, depth, want_stats=False)[0].to_numpy())])
    finally:
        w.tune("arena_pct", 100)
    assert not errors, errors
    assert got["multi"].tobytes() == a_ref.tobytes()
    assert got["render"].tobytes() == b_ref.tobytes()
    w.check()


@pytest.mark.gpu
def test_counted_device_renders_share_a_stream(rt):
    """Two threads make synchronous counted calls (rt_render_shard_device_ex
    with stats) on the same caller stream: each gets a workspace of its own,
    so each call returns its own frame and its own counters, equal to the same
    call made alone (advisor, round 4)."""
    import torch
    from rtamd import scenes
    w, cam, depth = scenes.c3(96, 54, n_spheres=200)
    cam2 = scenes.c3_orbit(5, 8, 96, 54)
    s0 = torch.cuda.current_stream().cuda_stream

    def call(c):
        buf = torch.empty((c.vsize, c.hsize, 3), dtype=torch.float64, device="cuda")
        st = c.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s0, True, exhaustive=False)
        torch.cuda.synchronize()
        return buf.cpu().numpy(), {k: st[k] for k in ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow")}

    alone = [call(cam), call(cam2)]
    assert alone[0][1] != alone[1][1]  # different cameras, different counts
    got, errors = _run_threads([(0, lambda: call(cam)), (1, lambda: call(cam2))], rounds=4)
    assert not errors, errors
    for k in (0, 1):
        assert got[k][0].tobytes() == alone[k][0].tobytes(), k
        assert got[k][1] == alone[k][1], k
    w.check()
