"""The CPU baseline on the full C3 frame against bench.py's row sample (dev
probe): the C oracle (oracle/rt_oracle.c, the reference
algorithm) renders every row of the 1920x1080 frame on this host's cores in
contiguous row blocks (camera.rs:157-172), then bench.py's sample (every third
row); both as reference rays per second. Host only: no GPU call.
Usage: cpu_full_frame.py [--threads N]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]

from bench import cpu_baseline, host_cores  # noqa: E402
from oracle import pyoracle  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=None)
a = ap.parse_args()
w, cam, depth = scenes.c3()
n = a.threads or host_cores()
ow = pyoracle.OracleWorld.from_world(w)
t0 = time.perf_counter()
_, st = ow.render_rows(cam.desc_bytes(), depth, list(range(cam.vsize)), n)
dt = time.perf_counter() - t0
rays = st["rays_primary"] + st["rays_reflect"] + st["rays_refract"] + st["rays_shadow"]
full = {"value": rays / dt / 1e6, "rays": rays, "seconds": round(dt, 2), "threads": n}
print(json.dumps({"full_frame": full}), flush=True)
sample = cpu_baseline(w, cam, depth, 15.0)
print(json.dumps({"full_frame": full, "bench_sample": {"value": sample["value"], "sample": sample["sample"]},
                  "sample_over_full": round(sample["value"] / full["value"], 4)}), flush=True)
