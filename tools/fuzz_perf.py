"""Fast path against the exhaustive loop on random scenes (dev tool, GPU box):
per seed of rtamd.scenes.fuzz at --width x --height, the median of 3 fast-path
frame times and one exhaustive frame time (synchronous rt_render calls into a
host canvas; both include the copy), printed worst ratio first, so that a scene
on which the culling does not pay shows up. Progress lines every 25 seeds."""
import argparse
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
from rtamd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=0)
    ap.add_argument("--seeds", type=int, default=200)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--height", type=int, default=240)
    a = ap.parse_args()
    res = []
    t0 = time.time()
    for i, seed in enumerate(range(a.start, a.start + a.seeds)):
        w, cam, depth = scenes.fuzz(seed, a.width, a.height)
        cam.render(w, depth, want_stats=False)  # warm: upload, workspace, arenas
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            cam.render(w, depth, want_stats=False)
            ts.append(time.perf_counter() - t)
        t = time.perf_counter()
        _, st = cam.render(w, depth)  # counted: the exhaustive loop
        tex = time.perf_counter() - t
        tf = statistics.median(ts)
        res.append((tex / tf, seed, tf * 1e3, tex * 1e3, depth, int(st["sphere_tests"]), int(st["other_tests"])))
        if (i + 1) % 25 == 0:
            print(f"... {i + 1} seeds, {time.time() - t0:.0f}s", flush=True)
    res.sort()
    print("speedup(exh/fast) seed fast_ms exh_ms depth sphere_tests other_tests  (worst first)")
    for r in res[:15]:
        print(f"{r[0]:8.2f} {r[1]:6d} {r[2]:8.3f} {r[3]:8.3f} {r[4]:2d} {r[5]:10d} {r[6]:10d}")
    sp = [r[0] for r in res]
    print(f"median speedup {statistics.median(sp):.2f}, min {min(sp):.2f}, max {max(sp):.2f} over {len(sp)} seeds")


if __name__ == "__main__":
    main()
