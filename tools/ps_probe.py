"""Persistent-kernel probe (dev tool): for each knob setting, the C3 frame
time with F frames in flight and one at a time, and a counted frame's work
items (lane use of the chunks) and where the waves' time goes.
Usage: ps_probe.py [--config c3|c5] [--shard r/n] [--frames K] [set ...]
  a set is comma-separated k=v render-time knobs, e.g. ps_policy=1,ps_trees=16"""
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
ap.add_argument("--shard", default="0/1")
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--inflight", type=int, default=4)
ap.add_argument("sets", nargs="*", default=[""])
a = ap.parse_args()
w, cam, depth = scenes.c3() if a.config == "c3" else scenes.c5()
w.upload(0)
w.tune("shadow_stream", 0)
r, n = (int(x) for x in a.shard.split("/"))
rows = rtamd.shard_rows(cam.vsize, 8, r, n)
F = max(1, a.inflight)
bufs = [torch.empty((rows, cam.hsize, 3), dtype=torch.float64, device="cuda") for _ in range(F)]
streams = [rtamd.render_stream() for _ in range(F)]
cur = torch.cuda.current_stream()
ref = torch.empty_like(bufs[0])
cam.render_shard_device(w, depth, 8, r, n, ref.data_ptr(), cur.cuda_stream, True, exhaustive=True)
torch.cuda.synchronize()


def run(frames, inflight):
    sts = streams[:inflight] if inflight > 1 else [cur]
    for f in range(2 * inflight):
        cam.render_shard_device(w, depth, 8, r, n, bufs[f % F].data_ptr(), sts[f % len(sts)].cuda_stream, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(frames):
        cam.render_shard_device(w, depth, 8, r, n, bufs[f % F].data_ptr(), sts[f % len(sts)].cuda_stream, False)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / frames * 1e3


for st in a.sets:
    knobs = dict(kv.split("=") for kv in st.split(",") if kv)
    for k, v in knobs.items():
        w.tune(k, int(v))
    ms_f = run(a.frames, F)
    ms_1 = run(a.frames, 1)
    ok = bool(torch.equal(bufs[0], ref))
    cam.render_shard_device(w, depth, 8, r, n, bufs[0].data_ptr(), cur.cuda_stream, True, exhaustive=False)
    p = rtamd._rtamd._wf_profile(w, -1, True)
    ps = p["ps"]
    cyc = sum(v for k, v in ps.items() if k.startswith("cycles_")) or 1.0
    out = {"knobs": knobs, "ms_inflight": round(ms_f, 4), "ms_serial": round(ms_1, 4), "bitwise": ok,
           "persist": p["persist"],
           "lane_use_roots": round(ps["lanes_roots"] / max(1.0, 64 * ps["items_roots"]), 3),
           "lane_use_queued": round(ps["lanes_queued"] / max(1.0, 64 * ps["items_queued"]), 3),
           "items": [int(ps["items_roots"]), int(ps["items_queued"])],
           "time_split": {k[7:]: round(ps[k] / cyc, 3) for k in ps if k.startswith("cycles_")}}
    print(json.dumps(out), flush=True)
    for k in knobs:  # back to the defaults (rt_wavefront.hpp WfTuning)
        w.tune(k, 1 if k in ("persist", "accel", "skip_shadow", "shadow_lb", "treelet", "shadow_stream") else 0)
    w.tune("shadow_stream", 0)
