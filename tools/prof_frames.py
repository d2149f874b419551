"""Render N frames of the bench workload on the fast path only (no counted
frame), for rocprofv3 kernel-trace / PMC passes (dev tool). Per-frame
figures = totals / N (tools/pmc_summary.py divides by the wf_prim_prep
count, one per frame)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=5)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spheres", type=int, default=1000)
ap.add_argument("--exhaustive", action="store_true")
a = ap.parse_args()
w, cam, depth = scenes.c3(a.width, a.height, a.spheres)
w.upload(0)
if a.exhaustive:
    rtamd._rtamd._tuning_set("accel", 0)
buf = torch.empty((a.height, a.width, 3), dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(a.frames):
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s, False)
torch.cuda.synchronize()
print("frames", a.frames, "checksum", float(buf.sum()))
