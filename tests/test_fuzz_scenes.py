"""The seeded random scenes of tests/test_gpu_fuzz.py (rtamd.scenes.fuzz) on
the CPU: the same seed builds the same scene (the oracle renders it to the same
bytes), different seeds differ, and every seed renders finite colours."""
import numpy as np


def _render(seed):
    from oracle import pyoracle
    from rtamd import scenes
    w, cam, depth = scenes.fuzz(seed, 32, 24)
    ref, st = pyoracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=4)
    return ref, st


def test_fuzz_scenes_deterministic_and_distinct():
    a, sa = _render(5)
    b, sb = _render(5)
    c, _ = _render(6)
    assert a.tobytes() == b.tobytes() and sa == sb
    assert a.tobytes() != c.tobytes()


def test_fuzz_scenes_render_finite():
    for seed in range(24):
        ref, st = _render(seed)
        assert np.isfinite(ref).all(), seed
        assert st["rays_primary"] == 32 * 24
