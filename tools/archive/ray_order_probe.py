"""Does ray order matter to the per-lane closest-hit traversal? (dev probe)
2 M rays with origins inside the C3 sphere field and random directions,
traced at depth 0 through color_at_batch in four orders; prints the
closest-hit class time of each (launch-carried events)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import numpy as np
import torch  # noqa
import rtamd  # noqa
from rtamd import scenes  # noqa
w, cam, depth = scenes.c3()
rng = np.random.default_rng(3)
n = 2_000_000
o = rng.uniform([-10, 0.2, -2], [10, 3.0, 20], size=(n, 3))
d = rng.normal(size=(n, 3))
d /= np.linalg.norm(d, axis=1, keepdims=True)
octant = (d[:, 0] > 0) * 1 + (d[:, 1] > 0) * 2 + (d[:, 2] > 0) * 4
cell = np.floor((o - [-10, 0.2, -2]) / ([20, 2.8, 22]) * 8).clip(0, 7).astype(int)
morton = np.zeros(n, dtype=np.int64)
for b in range(3):
    for ax in range(3):
        morton |= ((cell[:, ax] >> b) & 1) << (3 * b + ax)
orders = {
    "random": np.arange(n),
    "octant": np.argsort(octant, kind="stable"),
    "cell": np.argsort(morton, kind="stable"),
    "octant+cell": np.lexsort((morton, octant)),
    "cell+octant": np.lexsort((octant, morton)),
}
rays = np.hstack([o, d])
for rep in range(2):
    for name, idx in orders.items():
        r = np.ascontiguousarray(rays[idx])
        w.color_at_batch(r, 0, False)
        rtamd._rtamd._wf_profile(w, 1, False)
        for _ in range(3):
            w.color_at_batch(r, 0, False)
        p = rtamd._rtamd._wf_profile(w, 0, True)
        print(f"{name:12s} closest {p['ms']['closest']:.3f} ms  shadow {p['ms']['shadow']:.3f} ms  "
              f"tests {p['tests']['closest'] / n:.2f}/ray boxes {p['boxes']['closest'] / n:.1f}/ray", flush=True)
