"""Soak run of the random-scene parity sweep (dev tool, GPU box): seeds
[--start, --start + --seeds) of rtamd.scenes.fuzz at --width x --height, each
rendered by the fast path and the exhaustive counted render on the GPU and by
the oracle on the host; prints one line per failing seed and a JSON summary
(seeds, bitwise-equal frames, max |delta|, total rays, wall time).
Every 50 seeds a progress line (gpurun's hang watchdog)."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import rtamd as rt  # noqa: E402
from oracle import pyoracle  # noqa: E402
from rtamd import scenes  # noqa: E402

COUNTERS = ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow", "sphere_tests", "plane_tests",
            "sphere_disc_ge0", "other_tests")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=1000)
    ap.add_argument("--seeds", type=int, default=500)
    ap.add_argument("--width", type=int, default=96)
    ap.add_argument("--height", type=int, default=72)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dense", action="store_true", help="500-8000 random spheres per scene (global-memory images)")
    a = ap.parse_args()
    t0 = time.time()
    bad, bitwise, maxd, rays = [], 0, 0.0, 0
    for i, seed in enumerate(range(a.start, a.start + a.seeds)):
        w, cam, depth = scenes.fuzz(seed, a.width, a.height,
                                    n_spheres=(500 + seed * 7919 % 7500) if a.dense else None)
        fast, _ = cam.render(w, depth, want_stats=False)
        exh, st = cam.render(w, depth)
        f, e = fast.to_numpy(), exh.to_numpy()
        ref, rst = pyoracle.OracleWorld.from_world(w).render(cam.desc_bytes(), depth, nthreads=a.threads)
        d = float(np.abs(e - ref).max())
        maxd = max(maxd, d)
        rays += sum(int(st[k]) for k in COUNTERS[:4])
        why = []
        if f.tobytes() != e.tobytes():
            why.append("fast != exhaustive")
        if not d <= 1e-5:
            why.append(f"max|delta| {d}")
        if rt.canvas_to_ppm(e) != pyoracle.canvas_to_ppm(ref):
            why.append("PPM bytes differ")
        why += [f"{k} {st[k]} != {rst[k]}" for k in COUNTERS if st[k] != rst[k]]
        if e.tobytes() == ref.tobytes():
            bitwise += 1
        else:
            why.append(f"{int((e != ref).sum())} channels not bit-identical")
        if why:
            bad.append(seed)
            print(f"seed {seed}: " + "; ".join(why), flush=True)
        if (i + 1) % (10 if a.dense else 50) == 0:
            print(f"... {i + 1} seeds, {len(bad)} failing, {time.time() - t0:.0f}s", flush=True)
    w.check()
    print(json.dumps({"seeds": a.seeds, "start": a.start, "size": [a.width, a.height], "dense": a.dense,
                      "failing": bad,
                      "bit_identical_frames": bitwise, "max_abs_delta": maxd, "rays": rays,
                      "wall_s": round(time.time() - t0, 1)}))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
