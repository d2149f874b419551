"""rt_render_multi's host-canvas path, one device's part at a time (dev probe;
VERDICT r05 item 3): for N = 1, 2, 4, 8, every shard i of N rendered on this
GPU and copied into its rows of a full-size host canvas (_render_shard_host:
what device i's worker does), beside the same shard rendered into HBM only.
Each device has its own link to the host, so the projected N-device frame time
is the slowest shard's (render + its own copy). Also the one-device
rt_render_multi in both forms (direct, RCCL gather) against rt_render.
Usage: multi_probe.py [--frames K]"""
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
ap.add_argument("--row-block", type=int, default=8)
a = ap.parse_args()
w, cam, depth = scenes.c3()
w.upload(0)
H, W, B = cam.vsize, cam.hsize, a.row_block


def med(fn):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(a.frames):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(statistics.median(ts), 4)


ref, _ = cam.render(w, depth, want_stats=False)
refb = ref.to_numpy().tobytes()
res = {"render_to_host_ms": med(lambda: cam.render(w, depth, want_stats=False))}
got, _ = cam.render_multi([w], depth, B)
res["multi_direct_n1_bitwise"] = got.to_numpy().tobytes() == refb
res["multi_direct_n1_ms"] = med(lambda: cam.render_multi([w], depth, B, 1, False))
w.tune("multi_gather", 1)
got, _ = cam.render_multi([w], depth, B)
res["multi_gather_n1_bitwise"] = got.to_numpy().tobytes() == refb
res["multi_gather_n1_ms"] = med(lambda: cam.render_multi([w], depth, B, 1, False))
w.tune("multi_gather", 0)
print(json.dumps(res), flush=True)
pinned = rtamd._rtamd.host_buffer(H * W * 3 * 8).view(np.float64).reshape(H, W, 3)
stream = torch.cuda.current_stream().cuda_stream
for n in (1, 2, 4, 8):
    rows = [rtamd.shard_rows(H, B, i, n) for i in range(n)]
    dev = [torch.empty((max(r, 1), W, 3), dtype=torch.float64, device="cuda") for r in rows]
    shard_dev, shard_host = [], []
    for i in range(n):
        def d(i=i):
            cam.render_shard_device(w, depth, B, i, n, dev[i].data_ptr(), stream, False)
            torch.cuda.synchronize()
        shard_dev.append(med(d))
        shard_host.append(med(lambda i=i: rtamd._rtamd._render_shard_host(w, cam, depth, B, i, n, pinned, 1, False)))
    ok = pinned.tobytes() == refb
    line = {"n": n, "shard_device_ms": shard_dev, "shard_to_host_ms": shard_host,
            "copy_ms": [round(h - d, 4) for h, d in zip(shard_host, shard_dev)],
            "copy_gb_s": [round(r * W * 24 / 1e6 / max(h - d, 1e-6), 2) for r, h, d in zip(rows, shard_host, shard_dev)],
            "projected_frame_ms": max(shard_host), "assembled_bitwise": ok}
    print(json.dumps(line), flush=True)
