"""Where `canvas_to_ppm(&camera.render(&world))` spends its time (dev probe;
VERDICT r05 item 4): rt_render_ppm on the C3 frame through the allocating
binding (fresh std::string + Python bytes per call), into a reused pageable
buffer, into a reused pinned buffer (rt_host_buffer_alloc), beside rt_render to
a host canvas and a device-only frame. One frame at a time, medians of --frames.
Usage: ppm_probe.py [--frames K]"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=10)
a = ap.parse_args()
w, cam, depth = scenes.c3()
w.upload(0)
out = {}


def timed(name, fn):
    for _ in range(3):
        r = fn()
    ts = []
    for _ in range(a.frames):
        t0 = time.perf_counter()
        r = fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    out[name] = {"median_ms": round(statistics.median(ts), 3), "min_ms": round(min(ts), 3)}
    print(json.dumps({name: out[name]}), flush=True)
    return r


buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def dev_frame():
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), st, False)
    torch.cuda.synchronize()


timed("device_frame", dev_frame)
timed("render_to_host_canvas", lambda: cam.render(w, depth, want_stats=False))
ref = timed("render_ppm_binding_alloc", lambda: cam.render_ppm(w, depth)[0])
cap = 32 + 12 * cam.hsize * cam.vsize + cam.vsize
pageable = np.zeros(cap, dtype=np.uint8)
n = timed("render_ppm_into_pageable", lambda: cam.render_ppm_into(w, pageable, depth))
assert pageable[:n].tobytes() == bytes(ref)
pinned = rtamd._rtamd.host_buffer(cap)
n = timed("render_ppm_into_pinned", lambda: cam.render_ppm_into(w, pinned, depth))
assert pinned[:n].tobytes() == bytes(ref)
timed("bytes_of_pinned_text", lambda: bytes(pinned[:n]))
timed("render_ppm_into_pinned_then_bytes", lambda: bytes(pinned[:cam.render_ppm_into(w, pinned, depth)]))
timed("host_buffer_alloc_free", lambda: rtamd._rtamd.host_buffer(cap))

out["ppm_bytes"] = n
print(json.dumps(out), flush=True)
