"""End-to-end probe of the drop-in entry point (dev tool): `rt_render` into a
fresh host Canvas (Camera::render, camera.rs:133-148) per d2h mode, the host
`rt_canvas_to_ppm`, and `rt_render_ppm`, one frame at a time.
Usage: e2e_probe.py [--frames K]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402,F401

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=5)
a = ap.parse_args()
w, cam, depth = scenes.c3()
w.upload(0)
ref = None
for mode in (1, 0, 1):
    w.tune("d2h", mode)
    cam.render(w, depth, want_stats=False)
    ts = []
    for _ in range(a.frames):
        t0 = time.perf_counter()
        canvas, _ = cam.render(w, depth, want_stats=False)
        ts.append(time.perf_counter() - t0)
    arr = canvas.to_numpy()
    same = ref is None or arr.tobytes() == ref
    ref = arr.tobytes()
    print(json.dumps({"d2h": mode, "ms_render_to_host": [round(t * 1e3, 3) for t in ts], "same": same}), flush=True)
t0 = time.perf_counter()
ppm = rtamd.canvas_to_ppm(arr)
t_ppm = time.perf_counter() - t0
ts = []
for _ in range(a.frames):
    t0 = time.perf_counter()
    dev_ppm, _ = cam.render_ppm(w, depth)
    ts.append(time.perf_counter() - t0)
print(json.dumps({"ms_canvas_to_ppm": round(t_ppm * 1e3, 3), "ms_render_ppm": [round(t * 1e3, 3) for t in ts],
                  "ppm_same": bytes(dev_ppm) == (ppm.encode() if isinstance(ppm, str) else bytes(ppm))}), flush=True)
