"""Render N frames of the bench workload on the fast path only (no counted
frame), for rocprofv3 kernel-trace / PMC passes (dev tool), in batches of
--batch frames per call as bench.py renders them. Per-frame figures =
totals / N (tools/pmc_summary.py: wf_frame_init count x batch)."""
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
ap.add_argument("--config", default="c3", choices=["c3", "c5"])
ap.add_argument("--inflight", type=int, default=1, help="frames in flight (streams); 1 = serialized, as bench.py's roofline pass")
ap.add_argument("--shard", default="0/1", help="render rank r of an n-way row split: r/n (dev)")
ap.add_argument("--knob", action="append", default=[], help="tuning knob k=v (dev)")
ap.add_argument("--batch", type=int, default=1, help="frames per render call (rt_render_frames_device)")
a = ap.parse_args()
for kv in a.knob:
    k, v = kv.split("=")
    rtamd._rtamd._tuning_set(k, int(v))
w, cam, depth = scenes.c3(a.width, a.height, a.spheres) if a.config == "c3" else scenes.c5(a.width, a.height, a.spheres)
w.upload(0)
if a.exhaustive:
    w.tune("accel", 0)
r, n = (int(x) for x in a.shard.split("/"))
rows = rtamd.shard_rows(a.height, 8, r, n)
F = max(1, a.inflight)
w.tune("shadow_stream", 0)  # as bench.py (its serialized roofline pass: one stream)
NB = max(1, a.batch)
bufs = [torch.empty((rows, a.width, 3), dtype=torch.float64, device="cuda") for _ in range(F * NB)]
streams = [torch.cuda.Stream() for _ in range(F)] if F > 1 else [torch.cuda.current_stream()]
torch.cuda.synchronize()
for c in range(a.frames // NB):
    k = c % F
    if NB == 1:
        cam.render_shard_device(w, depth, 8, r, n, bufs[k].data_ptr(), streams[k].cuda_stream, False)
    else:
        rtamd.render_frames_device(w, [cam] * NB, depth, 8, r, n, [b.data_ptr() for b in bufs[k * NB:(k + 1) * NB]],
                                   streams[k].cuda_stream)
buf = bufs[0]
torch.cuda.synchronize()
print("frames", a.frames, "checksum", float(buf.sum()))
