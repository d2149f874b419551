"""Rays per generation of one fast-path frame (dev tool): C3 and C5 at full
size, from the workspace's host-mapped record (rtamd_wf_gen_counts).
Usage: gen_probe.py [--config c3|c5 ...]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", action="append", default=[])
a = ap.parse_args()
for cfg in a.config or ["c3", "c5"]:
    w, cam, depth = getattr(scenes, cfg)()
    w.upload(0)
    out = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    st = cam.render_shard_device(w, depth, 8, 0, 1, out.data_ptr(), s, True, exhaustive=False)
    torch.cuda.synchronize()
    counts = rtamd._rtamd._wf_gen_counts(w)
    print(json.dumps({"config": cfg, "gen_rays": counts, "total": sum(counts),
                      "rays_reflect": st["rays_reflect"], "rays_refract": st["rays_refract"],
                      "rays_shadow": st["rays_shadow"]}), flush=True)
