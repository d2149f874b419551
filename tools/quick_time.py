"""Quick timing probe of the fast path (dev tool): renders the bench workload
on one GPU with F frames in flight and prints one JSON line with the frame
time, Mrays/s (reference rays from a counted fast-path frame) and the
per-class kernel times of a serialized pass. No exhaustive frame, no parity
check (bench.py does those). Knobs that act at scene creation (lb_res,
bvh_leaf, bvh_ct) are applied before the upload.
Usage: quick_time.py [--config c3|c5] [--frames K] [--inflight F] [--knob k=v ...]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:  # as bench.py
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3", choices=["c3", "c5"])
ap.add_argument("--width", type=int, default=None)
ap.add_argument("--height", type=int, default=None)
ap.add_argument("--spheres", type=int, default=None)
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--inflight", type=int, default=None)
ap.add_argument("--shard", default="0/1", help="r/n: render rank r's rows of an n-way split")
ap.add_argument("--knob", action="append", default=[])
ap.add_argument("--tag", default="")
a = ap.parse_args()
for kv in a.knob:
    k, v = kv.split("=")
    rtamd._rtamd._tuning_set(k, int(v))
dflt = {"c3": (1920, 1080, 1000), "c5": (4096, 4096, 9996)}[a.config]
W, H, S = a.width or dflt[0], a.height or dflt[1], a.spheres or dflt[2]
w, cam, depth = getattr(scenes, a.config)(W, H, S)
t0 = time.perf_counter()
w.upload(0)
t_up = time.perf_counter() - t0
F = a.inflight or (4 if a.config == "c3" else 1)
r, n = (int(x) for x in a.shard.split("/"))
rows = rtamd.shard_rows(H, 8, r, n)
w.tune("shadow_stream", 0)
streams = [rtamd.render_stream(False) for _ in range(F)] if F > 1 else [torch.cuda.current_stream()]
bufs = [torch.empty((rows, W, 3), dtype=torch.float64, device="cuda") for _ in range(F)]
s0 = torch.cuda.current_stream().cuda_stream
st = cam.render_shard_device(w, depth, 8, r, n, bufs[0].data_ptr(), s0, True, exhaustive=False)
ref_rays = st["rays_primary"] + st["rays_reflect"] + st["rays_refract"] + st["rays_shadow"]
for f in range(2 * F):
    cam.render_shard_device(w, depth, 8, r, n, bufs[f % F].data_ptr(), streams[f % F].cuda_stream, False)
torch.cuda.synchronize()
t0 = time.perf_counter()
for f in range(a.frames):
    cam.render_shard_device(w, depth, 8, r, n, bufs[f % F].data_ptr(), streams[f % F].cuda_stream, False)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.frames * 1e3
rtamd._rtamd._wf_profile(w, 1, False)
for f in range(min(a.frames, 5)):
    cam.render_shard_device(w, depth, 8, r, n, bufs[0].data_ptr(), s0, False)
torch.cuda.synchronize()
rtamd._rtamd._wf_profile(w, 0, False)
cam.render_shard_device(w, depth, 8, r, n, bufs[0].data_ptr(), s0, True, exhaustive=False)  # counted: the work tallies
p = rtamd._rtamd._wf_profile(w, -1, True)
print(json.dumps({"tag": a.tag, "config": a.config, "shard": a.shard, "knobs": a.knob, "inflight": F,
                  "ms_per_frame": round(ms, 4), "mrays_per_s": round(ref_rays / ms / 1e3, 1),
                  "ref_rays": ref_rays, "traced_shadow": st["rays_shadow_traced"], "upload_s": round(t_up, 2),
                  "class_ms": {k: round(v, 4) for k, v in p["ms"].items()},
                  "tests": {k: int(v) for k, v in p["tests"].items()}, "boxes": {k: int(v) for k, v in p["boxes"].items()},
                  "n_bvh_nodes": p["n_bvh_nodes"], "bvh_depth": p["bvh_depth"]}), flush=True)
