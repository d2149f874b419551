"""Dev diagnostic: bench.py's headline batches, then the orbit of first-seen
cameras (bench.py distinct_cameras) three times, with phase markers on stderr
(a debug build prints its arena regrowths there)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

w, cam, depth = scenes.c3()
w.upload(0)
w.tune("shadow_stream", 0)
rs = [rtamd.render_stream(False) for _ in range(4)]
H, W = cam.vsize, cam.hsize
bufs = [[torch.empty((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(8)] for _ in range(4)]


def batches(cams_for, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(n):
        rtamd.render_frames_device(w, cams_for(b), depth, 8, 0, 1, [x.data_ptr() for x in bufs[b % 4]], rs[b % 4].cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (n * 8) * 1e3


print("PHASE headline", file=sys.stderr, flush=True)
print("headline warm", batches(lambda b: [cam] * 8, 8), flush=True)
print("headline", batches(lambda b: [cam] * 8, 16), flush=True)
for rep in range(3):
    cams = [scenes.c3_orbit(k, 64) for k in range(64)]
    print(f"PHASE distinct {rep}", file=sys.stderr, flush=True)
    print("distinct", rep, batches(lambda b: cams[b * 8:(b + 1) * 8], 8), flush=True)
print("PHASE e2e", file=sys.stderr, flush=True)
for _ in range(5):
    cam.render(w, depth, want_stats=False)
for rep in range(3):
    cams = [scenes.c3_orbit(k, 64) for k in range(64)]
    print(f"PHASE distinct-after-e2e {rep}", file=sys.stderr, flush=True)
    print("distinct-after-e2e", rep, batches(lambda b: cams[b * 8:(b + 1) * 8], 8), flush=True)
w.check()
