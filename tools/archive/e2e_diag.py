"""rt_render to a host canvas on C3 (dev tool): per-frame times of a loop that
drops each canvas before the next render and of one that holds the previous
canvas (as bench.py's end_to_end), before and after device-resident batches
on 4 streams (bench.py's timed region); the held loop with an idle gap before
each call, and the device render alone."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402


def loop(cam, w, depth, hold, n=12, gap_ms=0.0):
    ts = []
    keep = None
    for _ in range(n):
        if gap_ms:
            t1 = time.perf_counter()
            while (time.perf_counter() - t1) * 1e3 < gap_ms:
                pass
        t0 = time.perf_counter()
        c, _ = cam.render(w, depth, want_stats=False)
        ts.append(round((time.perf_counter() - t0) * 1e3, 3))
        keep = c if hold else None
        del c
    del keep
    return ts


w, cam, depth = scenes.c3()
w.upload(0)
out = {"drop_1": loop(cam, w, depth, False), "hold_1": loop(cam, w, depth, True)}
streams = [rtamd.render_stream(False) for _ in range(4)]
bufs = [torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda") for _ in range(32)]
for it in range(8):
    for k in range(4):
        rtamd._rtamd.render_frames_device(w, [cam] * 8, depth, 8, 0, 1, [b.data_ptr() for b in bufs[8 * k:8 * k + 8]],
                                          streams[k].cuda_stream)
torch.cuda.synchronize()
out["drop_2"] = loop(cam, w, depth, False)
out["hold_2"] = loop(cam, w, depth, True)
# the same loop with an idle gap before each call (is a call slowed by the one before it?)
for gap in (0.5, 2.0):
    out[f"hold_gap{gap}"] = loop(cam, w, depth, True, gap_ms=gap)
# one call's phases: the render alone into a device buffer, then the whole call again
dev = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
s0 = torch.cuda.current_stream()
ts = []
for _ in range(12):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cam.render_shard_device(w, depth, 8, 0, 1, dev.data_ptr(), s0.cuda_stream, False)
    torch.cuda.synchronize()
    ts.append(round((time.perf_counter() - t0) * 1e3, 3))
out["device_render_only"] = ts
out["hold_3"] = loop(cam, w, depth, True)
print(json.dumps(out))
