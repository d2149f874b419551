"""Where a small random-scene frame's time goes (dev tool, GPU box): for seeds
of rtamd.scenes.fuzz at 320x240, the host-canvas frame time (median of 20),
the object kinds, the fast path's executed work (a counted fast-path frame)
and the frame time under library knob variants.
Usage: python tools/small_frame_probe.py SEED [SEED ...]"""
import collections
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
from rtamd import scenes  # noqa: E402

VARIANTS = [{}, {"spread": 1}, {"lds_wide": 0}, {"shadow_lb": 0}, {"image": 3}, {"image": 3, "spread": 1}]


def frame_ms(w, cam, depth, n=20):
    for _ in range(3):
        cam.render(w, depth, want_stats=False)
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        cam.render(w, depth, want_stats=False)
        ts.append((time.perf_counter() - t) * 1e3)
    return statistics.median(ts)


for seed in [int(x) for x in sys.argv[1:]] or [130]:
    w, cam, depth = scenes.fuzz(seed, 320, 240)
    kinds = collections.Counter()
    for i in range(w.n_objects()):
        try:
            kinds[w.object(i).kind] += 1
        except ValueError:  # a Group
            kinds["group"] += 1
    _, st = cam.render(w, depth, want_stats=True, exhaustive=False)
    keys = [k for k in st if k.endswith("_executed") or k.startswith("rays_")]
    print(f"seed {seed} depth {depth} lights {w.n_lights()} kinds {dict(kinds)}")
    print("  fast-path counters: " + ", ".join(f"{k}={st[k]}" for k in keys))
    for v in VARIANTS:
        for k, x in v.items():
            w.tune(k, x)
        ms = frame_ms(w, cam, depth)
        print(f"  {str(v) or 'default':24s} {ms:7.3f} ms", flush=True)
        for k in v:
            w.tune(k, {"lds_wide": 1, "shadow_lb": 1, "prim_lane": 1, "own_sphere": 2, "image": 0, "spread": 0}[k])
