"""rt_render to a host canvas on C3 in a held loop (dev tool, for a kernel and
copy trace of the banded render: rocprofv3 --kernel-trace --memory-copy-trace
-- python tools/archive/e2e_loop.py); prints the per-frame wall times."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402,F401

import rtamd  # noqa: E402,F401
from rtamd import scenes  # noqa: E402

w, cam, depth = scenes.c3()
w.upload(0)
ts, keep = [], None
for _ in range(14):
    t0 = time.perf_counter()
    c, _ = cam.render(w, depth, want_stats=False)
    ts.append(round((time.perf_counter() - t0) * 1e3, 3))
    keep = c
print(json.dumps({"ms": ts}))
