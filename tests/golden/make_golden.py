#!/usr/bin/env python3
"""Generate the committed whole-frame golden fixtures (TEST INFRASTRUCTURE).

The reference holds no golden images (`renders/` is
git-ignored and the Rust crate cannot be built here), so whole-frame goldens
come from the C oracle (oracle/rt_oracle.c), which is itself pinned by the
reference's 67 known-answer tests (tests/test_oracle_kat.py). The fixtures
freeze the oracle's output so that (1) a change to the oracle is caught on CPU
and (2) the GPU path is checked against files, not only against a live oracle.

Per case <name> (aa > 1: `render_multithreaded` with that many AA samples):
  <name>.ppm        P3 bytes of the frame (canvas.rs:43-48 / ppm.rs:24-75)
  <name>.npz        f64 canvas (H, W, 3) `canvas` + the camera descriptor bytes
  index.json        per case: scene, size, depth, the exact counters, sha256
                    of the PPM and of the canvas bytes

Run from the repo root:  python tests/golden/make_golden.py [case ...]
(with case names, only those are regenerated and merged into index.json)
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd"), os.path.join(REPO, "tests")]

import rtamd  # noqa: E402  (host-side scene builder; no GPU needed)
from oracle import pyoracle  # noqa: E402
from golden_cases import scene  # noqa: E402

# (name, scene factory, kwargs): small enough for the oracle to finish in seconds
CASES = [
    ("kat11", "kat11", {}),
    ("c1", "c1", {"width": 200, "height": 100}),
    ("c2_80x60", "c2", {"width": 80, "height": 60}),
    ("c3_96x54", "c3", {"width": 96, "height": 54}),
    ("c3_64x36_s200", "c3", {"width": 64, "height": 36, "n_spheres": 200}),
    ("zoo_64x48", "zoo", {"width": 64, "height": 48}),
    ("first_scene_96x54", "first_scene", {"width": 96, "height": 54}),
    ("solids_64x48", "solids", {"width": 64, "height": 48}),
    # YAML scenes through rtamd.SceneParser (scene-parser/examples, camera resized)
    ("yaml_reflect_refract_128x72", "yaml", {"file": "reflect-refract.yml", "width": 128, "height": 72}),
    ("yaml_cover_80x80", "yaml", {"file": "cover.yml", "width": 80, "height": 80}),
    # render_multithreaded with AA (camera.rs:150-214)
    ("first_scene_48x27_aa4", "first_scene", {"width": 48, "height": 27}, 4),
    ("solids_40x30_aa16", "solids", {"width": 40, "height": 30}, 16),
    ("c3_48x27_s100_aa2", "c3", {"width": 48, "height": 27, "n_spheres": 100}, 2),
    ("zoo_32x24_aa8", "zoo", {"width": 32, "height": 24}, 8),
    # Group bounding-box gates (group.rs:60-75, bounding_box.rs:95-136)
    ("hexagon_64x36", "hexagon", {"width": 64, "height": 36}),
    ("groups_80x60", "groups", {"width": 80, "height": 60}),
    ("groups_40x30_aa4", "groups", {"width": 40, "height": 30}, 4),
    ("divided_96x54", "divided", {"width": 96, "height": 54}),
    # cones and open tubes (the line hierarchy: cone.rs, cylinder.rs)
    ("cones_64x48", "cones", {"width": 64, "height": 48, "n": 120}),
]
COUNTERS = ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow",
            "sphere_tests", "plane_tests", "sphere_disc_ge0", "other_tests")


def main(only=()):
    index = {}
    if only:
        with open(os.path.join(HERE, "index.json")) as f:
            index = json.load(f)
    for case in CASES:
        name, kind, kw = case[:3]
        if only and name not in only:
            continue
        aa = case[3] if len(case) > 3 else 1
        w, cam, depth = scene(rtamd, kind, kw)
        ow = pyoracle.OracleWorld.from_world(w)
        canvas, st = ow.render(cam.desc_bytes(), depth, nthreads=8, aa_samples=aa)
        ppm = pyoracle.canvas_to_ppm(canvas)
        with open(os.path.join(HERE, name + ".ppm"), "wb") as f:
            f.write(ppm)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), canvas=canvas,
                            camera=np.frombuffer(cam.desc_bytes(), dtype=np.uint8))
        index[name] = {
            "scene": kind, "args": kw, "width": cam.hsize, "height": cam.vsize, "depth": depth, "aa": aa,
            "counters": {k: int(st[k]) for k in COUNTERS},
            "ppm_sha256": hashlib.sha256(ppm).hexdigest(),
            "canvas_sha256": hashlib.sha256(np.ascontiguousarray(canvas).tobytes()).hexdigest(),
        }
        print(name, cam.hsize, cam.vsize, index[name]["counters"])
    with open(os.path.join(HERE, "index.json"), "w") as f:
        json.dump(index, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
