"""A/B tuning variants of the wavefront pipeline in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24). Dev tool.
Knob: wf_waves (trace-kernel occupancy, 4 or 8 waves/SIMD)."""
import os, sys, statistics, argparse
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa
import rtamd
from rtamd import scenes
ap = argparse.ArgumentParser()
ap.add_argument("--waves", default="8,4")
ap.add_argument("--knob", default="wf_waves")
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--scene", default="c3")
a = ap.parse_args()
w, cam, depth = scenes.CONFIGS[a.scene]() if a.scene != "c5" else scenes.c5(2048, 2048)
w.upload()
res = {v: [] for v in a.waves.split(",")}
ref = None
for r in range(a.rounds):
    for v in res:
        rtamd._rtamd._tuning_set(a.knob, int(v))
        canvas, st = cam.render(w, depth)
        img = canvas.to_numpy()
        if ref is None:
            ref = img
        assert img.tobytes() == ref.tobytes(), f"variant {v} changed the image"
        res[v].append(st["ms_kernel"])
n = st["rays_primary"] + st["rays_reflect"] + st["rays_refract"] + st["rays_shadow"]
for v, ms in res.items():
    print(f"{a.knob}={v}: median {statistics.median(ms):.3f} ms  min {min(ms):.3f}  -> {n/min(ms)/1e3:.1f} Mrays/s  all={['%.2f'%x for x in ms]}", flush=True)
