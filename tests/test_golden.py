"""Whole-frame golden fixtures (tests/golden, made by tests/golden/make_golden.py).

CPU: the oracle and the host-side scene/camera builders reproduce the committed
fixtures bit for bit (catches drift in either). GPU: the HIP render path
matches the fixture canvases within the north-star tolerance, with identical
PPM bytes and identical exact counters.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import golden_cases

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
INDEX = json.load(open(os.path.join(HERE, "index.json")))
TOL = 1e-5  # north star: within 1e-5 abs per colour channel


def _load(name):
    z = np.load(os.path.join(HERE, name + ".npz"))  # allow_pickle=False (default)
    ppm = open(os.path.join(HERE, name + ".ppm"), "rb").read()
    return z["canvas"], z["camera"].tobytes(), ppm


@pytest.mark.parametrize("name", sorted(INDEX))
def test_fixture_integrity(name):
    canvas, _, ppm = _load(name)
    e = INDEX[name]
    assert canvas.shape == (e["height"], e["width"], 3)
    assert hashlib.sha256(ppm).hexdigest() == e["ppm_sha256"]
    assert hashlib.sha256(np.ascontiguousarray(canvas).tobytes()).hexdigest() == e["canvas_sha256"]


@pytest.mark.parametrize("name", sorted(INDEX))
def test_oracle_reproduces_golden(rt, oracle, name):
    e = INDEX[name]
    canvas, cam_bytes, ppm = _load(name)
    w, cam, depth = golden_cases.scene(rt, e["scene"], e["args"])
    assert cam.desc_bytes() == cam_bytes, "host camera builder drifted"
    assert depth == e["depth"]
    ref, st = oracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=4, aa_samples=e["aa"])
    assert np.array_equal(ref, canvas)
    assert oracle.canvas_to_ppm(ref) == ppm
    assert {k: int(st[k]) for k in e["counters"]} == e["counters"]


def test_oracle_pixels_equal_rows(rt, oracle):
    """oracle_render_pixels (scattered samples of a large frame, used by the
    full-size GPU tests) computes each pixel exactly as oracle_render_rows,
    plain and with AA X4; out-of-frame pixels are refused."""
    import numpy as np
    from rtamd import scenes
    w, cam, depth = scenes.c3(96, 54, n_spheres=120)
    ow = oracle.OracleWorld.from_world(w)
    rng = np.random.default_rng(7)
    xy = np.stack([rng.integers(0, 96, 300), rng.integers(0, 54, 300)], 1)
    for aa in (1, 4):
        full, fst = ow.render_rows(cam.desc_bytes(), depth, list(range(54)), 4, aa_samples=aa)
        px, pst = ow.render_pixels(cam.desc_bytes(), depth, xy, 4, aa_samples=aa)
        assert px.tobytes() == full[xy[:, 1], xy[:, 0]].tobytes()
        assert pst["rays_primary"] == 300 * aa
    with pytest.raises(ValueError):
        ow.render_pixels(cam.desc_bytes(), depth, [(96, 0)], 1)


def test_kat11_center_pixel():
    # camera.rs:327-337: pixel (5,5) of the 11x11 default-world render
    canvas, _, _ = _load("kat11")
    assert np.allclose(canvas[5, 5], [0.38066, 0.47583, 0.2855], atol=1e-5, rtol=0)


def test_product_ppm_writer_matches_golden(rt):
    for name in sorted(INDEX):
        canvas, _, ppm = _load(name)
        assert rt.canvas_to_ppm(canvas) == ppm, name


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(INDEX))
def test_gpu_matches_golden(rt, name):
    e = INDEX[name]
    canvas, _, ppm = _load(name)
    w, cam, depth = golden_cases.scene(rt, e["scene"], e["args"])
    if e["aa"] == 1:
        out, st = cam.render(w, depth)
    else:
        cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{e['aa']}"))
        out, st = cam.render_multithreaded(w, depth)
    g = out.to_numpy()
    assert np.isfinite(g).all()
    assert np.abs(g - canvas).max() <= TOL
    assert rt.canvas_to_ppm(g) == ppm
    assert {k: int(st[k]) for k in e["counters"]} == e["counters"]
    # the fast path (the hierarchies, no counters) against the same fixture
    if e["aa"] == 1:
        fast, _ = cam.render(w, depth, want_stats=False)
    else:
        fast, _ = cam.render_multithreaded(w, depth, want_stats=False)
    f = fast.to_numpy()
    assert np.abs(f - canvas).max() <= TOL
    assert rt.canvas_to_ppm(f) == ppm
