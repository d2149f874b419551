"""rt_render into a host canvas (Camera::render -> Canvas) under library knob
variants, alternating, on the C3 frame: per variant the median and mean of
single-frame calls, every frame checked bitwise against the first variant's.
Dev tool (GPU box): python tools/host_render_probe.py [--frames 20] [--rounds 3]
  [--variant "bands=4"] [--variant "bands=3,band_pct=40,band_gen=0"] ...
"""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-challenge-rs_amd"))

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

DEFAULTS = {"bands": 4, "band_pct": 35, "band_ratio": 100, "band_gen": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variant", action="append", default=[])
    a = ap.parse_args()
    variants = a.variant or ["bands=4", "bands=3,band_pct=40,band_gen=0"]
    w, cam, depth = scenes.c3()
    ref = None
    res = {v: [] for v in variants}
    for r in range(a.rounds):
        for v in variants:
            knobs = dict(DEFAULTS)
            for kv in filter(None, v.split(",")):
                k, x = kv.split("=")
                knobs[k] = int(x)
            for k, x in knobs.items():
                w.tune(k, x)
            for _ in range(3):
                c, _ = cam.render(w, depth, want_stats=False)
            got = c.to_numpy().tobytes()
            if ref is None:
                ref = got
            if got != ref:
                raise SystemExit(f"variant {v}: frame differs")
            ts = []
            for _ in range(a.frames):
                t0 = time.perf_counter()
                c, _ = cam.render(w, depth, want_stats=False)
                ts.append((time.perf_counter() - t0) * 1e3)
            if c.to_numpy().tobytes() != ref:
                raise SystemExit(f"variant {v}: timed frame differs")
            res[v] += ts
            print(f"round {r} {v:40s} median {statistics.median(ts):.3f} mean {statistics.mean(ts):.3f} ms", flush=True)
    w.check()
    print("# all rounds (frames bitwise equal across variants)")
    for v, ts in res.items():
        print(f"{v:40s} median {statistics.median(ts):.3f} mean {statistics.mean(ts):.3f} min {min(ts):.3f} ms")


if __name__ == "__main__":
    main()
