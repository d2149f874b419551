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


def check_aa(w, cam, depth, seed, a):
    aa = (2, 4, 8)[seed % 3]
    cam.render_opts.aa_samples(getattr(rt.AASamples, f"X{aa}"))
    g = cam.render_multithreaded(w, depth)[0].to_numpy()
    ref, _ = pyoracle.OracleWorld.from_world(w).render_rows(cam.desc_bytes(), depth, list(range(cam.vsize)),
                                                            a.threads, aa_samples=aa)
    if g.tobytes() != ref.tobytes():
        return f"AA {aa}: {int((g != ref).sum())} channels not bit-identical, max|delta| {float(np.abs(g - ref).max())}"
    return None


def check_batch(w, cam, depth, seed, a):
    import torch
    rng = np.random.default_rng(seed)
    cams = [cam]
    for _ in range(4):
        c = rt.Camera(cam.hsize, cam.vsize, float(rng.uniform(0.6, 1.6)))
        c.set_transform(rt.view_transform(rt.Point(*rng.uniform([-6, 0.5, -10], [6, 5, -4])),
                                          rt.Point(*rng.uniform([-1, 0.3, 0], [1, 1.5, 3])), rt.Vector(0, 1, 0)))
        cams.append(c)
    n = int(rng.integers(1, 5))
    shard = int(rng.integers(0, n))
    rows = rt.shard_rows(cam.vsize, 8, shard, n)
    bat = [torch.full((rows, cam.hsize, 3), -1.0, dtype=torch.float64, device="cuda") for _ in cams]
    one = [torch.full_like(b, -2.0) for b in bat]
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    rt.render_frames_device(w, cams, depth, 8, shard, n, [b.data_ptr() for b in bat], st, False, 1)
    for c, b in zip(cams, one):
        c.render_shard_device(w, depth, 8, shard, n, b.data_ptr(), st, False, 1, exhaustive=True)
    torch.cuda.synchronize()
    w.check()
    diff = [k for k, (b, o) in enumerate(zip(bat, one)) if not torch.equal(b, o)]
    return f"batch frames {diff} of shard {shard}/{n} differ from the exhaustive shards" if diff else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=1000)
    ap.add_argument("--seeds", type=int, default=500)
    ap.add_argument("--width", type=int, default=96)
    ap.add_argument("--height", type=int, default=72)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dense", action="store_true", help="500-8000 random spheres per scene (global-memory images)")
    ap.add_argument("--mode", default="frame", choices=["frame", "aa", "batch"],
                    help="frame: the checks above; aa: render_multithreaded with AA 2/4/8 vs the oracle; batch: 5 "
                         "cameras in one rt_render_frames_device call over a random 1-4-way shard vs exhaustive "
                         "single-frame shards, bit for bit (no oracle)")
    a = ap.parse_args()
    t0 = time.time()
    bad, bitwise, maxd, rays = [], 0, 0.0, 0
    for i, seed in enumerate(range(a.start, a.start + a.seeds)):
        w, cam, depth = scenes.fuzz(seed, a.width, a.height,
                                    n_spheres=(500 + seed * 7919 % 7500) if a.dense else None)
        if a.mode != "frame":
            why = (check_aa if a.mode == "aa" else check_batch)(w, cam, depth, seed, a)
            if why:
                bad.append(seed)
                print(f"seed {seed}: {why}", flush=True)
            else:
                bitwise += 1
            if (i + 1) % 50 == 0:
                print(f"... {i + 1} seeds, {len(bad)} failing, {time.time() - t0:.0f}s", flush=True)
            continue
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
