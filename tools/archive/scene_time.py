"""Frame time of any rtamd.scenes config on one GPU (dev tool): the fast path
into a device buffer, K frames after a warm one; prints one JSON line.
Run it against two builds (LD_LIBRARY_PATH) to compare them.
Usage: scene_time.py --config hexagon [--kw '{"width": 2560, "height": 1440}'] [--frames K] [--tag T]"""
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
ap.add_argument("--config", required=True)
ap.add_argument("--kw", default="{}")
ap.add_argument("--frames", type=int, default=5)
ap.add_argument("--tag", default="")
a = ap.parse_args()
w, cam, depth = scenes.CONFIGS[a.config](**json.loads(a.kw))
w.upload(0)
buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
s0 = torch.cuda.current_stream().cuda_stream
cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s0, False)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.frames):
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s0, False)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.frames * 1e3
p = rtamd._rtamd._wf_profile(w, -1, True)
print(json.dumps({"tag": a.tag, "config": a.config, "kw": json.loads(a.kw), "ms_per_frame": round(ms, 3),
                  "fused": p["fused"], "n_other_culled": p["n_other_culled"], "n_line_culled": p.get("n_line_culled", 0)}),
      flush=True)
