"""Line hierarchy timing (dev tool): renders scenes.cones on one GPU, the fast
path, and prints one JSON line with the frame time and the executed record
tests per frame. Run it against two builds (LD_LIBRARY_PATH, tools/archive/exp_time.sh)
to compare the culled cones and open tubes with the exhaustive loop.
Usage: line_time.py [--n N] [--upright F] [--width W --height H] [--frames K]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=600)
ap.add_argument("--upright", type=float, default=0.5)
ap.add_argument("--width", type=int, default=640)
ap.add_argument("--height", type=int, default=480)
ap.add_argument("--frames", type=int, default=5)
ap.add_argument("--tag", default="")
a = ap.parse_args()
w, cam, depth = scenes.cones(a.width, a.height, a.n, a.upright)
w.upload(0)
buf = torch.empty((a.height, a.width, 3), dtype=torch.float64, device="cuda")
s0 = torch.cuda.current_stream().cuda_stream
cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s0, False)  # warm
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.frames):
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s0, False)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.frames * 1e3
cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s0, True, exhaustive=False)  # counted fast path
p = rtamd._rtamd._wf_profile(w, -1, True)
print(json.dumps({"tag": a.tag, "n": a.n, "upright": a.upright, "ms_per_frame": round(ms, 3),
                  "tests": {k: int(v) for k, v in p["tests"].items()}, "n_line_culled": p.get("n_line_culled", 0),
                  "n_quads_exhaustive": p["n_quads"], "fused": p["fused"]}), flush=True)
