"""canvas_to_ppm on the device (image/ppm.rs:24-75) and the one-call
render-to-PPM entry point (camera.rs:133-148 then ppm.rs:24-51).

The device encoder must write exactly the bytes of the reference's writer:
the oracle's `canvas_to_ppm` (a restatement of ppm.rs, pinned by the
reference's PPM tests in test_oracle_kat.py) and the host `rt_canvas_to_ppm`.
Inputs cover the quantisation edges (`(v*255).round() as u8`: halves,
negatives, NaN, infinities, values above 1), every token length, the
70-column breaks at every offset (widths 1..80 and long rows) and the C3/C5
frames the bench renders.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _device_ppm(rt, canvas):
    import torch
    h, w = canvas.shape[0], canvas.shape[1]
    d = torch.from_numpy(np.ascontiguousarray(canvas, dtype=np.float64)).cuda()
    cap = 12 * w * h + h + 32
    out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    n = rt._rtamd.canvas_to_ppm_device(d.data_ptr(), w, h, out.data_ptr(), cap,
                                       torch.cuda.current_stream().cuda_stream)
    assert rt._rtamd.canvas_to_ppm_device(d.data_ptr(), w, h, 0, 0, 0) == n  # length query
    return out[:n].cpu().numpy().tobytes()


def _edge_values(rng, n):
    halves = (np.arange(256) + 0.5) / 255.0
    v = np.concatenate([halves, np.nextafter(halves, 0), np.nextafter(halves, 2), np.arange(256) / 255.0,
                        [0.0, -0.0, -1e-300, -0.5, 1.0, 1.0000001, 2.0, 1e300, np.inf, -np.inf, np.nan],
                        rng.uniform(-0.2, 1.2, n)])
    return v


@pytest.mark.parametrize("width", list(range(1, 81)) + [255, 1000, 1920])
def test_device_ppm_equals_reference_writer(rt, oracle, width):
    rng = np.random.default_rng(width)
    h = 3 if width < 1000 else 2
    vals = _edge_values(rng, 3 * width * h)
    canvas = rng.choice(vals, size=(h, width, 3))
    # rows whose tokens are all 1, 2 or 3 digits (breaks at every line length)
    canvas[0] = rng.choice(np.arange(10) / 255.0, size=(width, 3))
    if h > 2:
        canvas[2] = rng.choice(np.arange(100, 256) / 255.0, size=(width, 3))
    got = _device_ppm(rt, canvas)
    assert got == _as_bytes(oracle.canvas_to_ppm(canvas))
    assert got == _as_bytes(rt.canvas_to_ppm(canvas))


def _as_bytes(x):
    return x.encode() if isinstance(x, str) else bytes(x)


def test_device_ppm_buffer_too_small_and_bad_width(rt):
    import torch
    canvas = torch.full((4, 5, 3), 0.5, dtype=torch.float64, device="cuda")
    n = rt._rtamd.canvas_to_ppm_device(canvas.data_ptr(), 5, 4, 0, 0, 0)
    out = torch.zeros(n, dtype=torch.uint8, device="cuda")
    with pytest.raises(rt.RtError):
        rt._rtamd.canvas_to_ppm_device(canvas.data_ptr(), 5, 4, out.data_ptr(), n - 1, 0)
    assert rt._rtamd.canvas_to_ppm_device(canvas.data_ptr(), 5, 4, out.data_ptr(), n, 0) == n
    assert out.cpu().numpy().tobytes() == _as_bytes(rt.canvas_to_ppm(canvas.cpu().numpy()))
    with pytest.raises(rt.RtError):
        rt._rtamd.canvas_to_ppm_device(canvas.data_ptr(), 20000, 1, 0, 0, 0)


def test_render_ppm_c3_equals_canvas_to_ppm(rt, oracle):
    """The one-call drop-in (render + device PPM) on the headline frame equals
    canvas_to_ppm of the rendered canvas; a slice also vs the oracle."""
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    ppm, _ = cam.render_ppm(w, depth)
    canvas, _ = cam.render(w, depth, want_stats=False)
    assert ppm == _as_bytes(rt.canvas_to_ppm(canvas.to_numpy()))
    w, cam, depth = scenes.c3(96, 54)
    ppm, st = cam.render_ppm(w, depth, want_stats=True)
    ref, rst = oracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=8)
    assert ppm == _as_bytes(oracle.canvas_to_ppm(ref))
    assert st["rays_shadow"] == rst["rays_shadow"] and st["rays_reflect"] == rst["rays_reflect"]


def test_render_ppm_aa_and_c5_slice(rt):
    from rtamd import scenes
    w, cam, depth = scenes.c3(160, 90)
    for aa in (2, 4):
        cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
        canvas, _ = cam.render_multithreaded(w, depth, want_stats=False)
        ppm, _ = cam.render_ppm(w, depth, aa)
        assert ppm == _as_bytes(rt.canvas_to_ppm(canvas.to_numpy()))
    w, cam, depth = scenes.c5(512, 512)
    canvas, _ = cam.render(w, depth, want_stats=False)
    ppm, _ = cam.render_ppm(w, depth)
    assert ppm == _as_bytes(rt.canvas_to_ppm(canvas.to_numpy()))


def test_device_ppm_empty_canvases(rt, oracle):
    """Zero width (every row is "\\n", ppm.rs:47-48) and zero height (the header
    alone), as the host writer and the oracle produce them."""
    import torch
    for h, w in [(3, 0), (0, 4), (0, 0)]:
        img = np.zeros((h, w, 3))
        d = torch.zeros(max(1, h * w * 3), dtype=torch.float64, device="cuda")
        cap = 12 * w * h + h + 32
        out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        n = rt._rtamd.canvas_to_ppm_device(d.data_ptr(), w, h, out.data_ptr(), cap, 0)
        got = out[:n].cpu().numpy().tobytes()
        assert got == _as_bytes(oracle.canvas_to_ppm(img)) == _as_bytes(rt.canvas_to_ppm(img)), (h, w)


def test_render_ppm_buffers_and_overflow(rt):
    """rt_render_ppm on C3's full frame (one pass of the stream for the render,
    the encoder and the text's length, then the copy): the same text through
    the binding (a pooled pinned block, copied into a bytes object by a few
    threads), into a reused pinned block, into a reused pageable buffer, with
    AA X2, and after a forced arena overflow (the frame is rendered again before
    the text is encoded); a buffer one byte short is refused."""
    import numpy as np
    from rtamd import scenes
    w, cam, depth = scenes.c3()
    canvas, _ = cam.render(w, depth, want_stats=False)
    whole = _as_bytes(rt.canvas_to_ppm(canvas.to_numpy()))
    ppm, _ = cam.render_ppm(w, depth)
    assert ppm == whole
    cam.render_opts.aa_samples(rt.AASamples.X2)
    canvas2, _ = cam.render_multithreaded(w, depth, want_stats=False)
    ppm2, _ = cam.render_ppm(w, depth, 2)
    assert ppm2 == _as_bytes(rt.canvas_to_ppm(canvas2.to_numpy()))
    pinned = rt._rtamd.host_buffer(len(whole) + 4096)
    pageable = np.zeros(len(whole) + 4096, dtype=np.uint8)
    for buf in (pinned, pageable, pinned):
        n = cam.render_ppm_into(w, buf, depth)
        assert n == len(whole) and buf[:n].tobytes() == whole
    w.tune("arena_pct", 5)
    try:
        over, _ = cam.render_ppm(w, depth)
    finally:
        w.tune("arena_pct", 100)
    assert over == whole
    short = np.zeros(len(whole) - 1, dtype=np.uint8)
    with pytest.raises(rt.RtError):
        cam.render_ppm_into(w, short, depth)
    w.check()
