"""Phase cycles of the closest-hit trace kernels (dev tool; needs the
RTAMD_PHASE build: make -C raytracer-challenge-rs_amd LIB=lib_phase
OBJ=lib_phase/obj EXTRA=-DRTAMD_PHASE lib_phase/librtamd.so, run with
LD_LIBRARY_PATH=raytracer-challenge-rs_amd/lib_phase). Prints, per class and
frame, the shader cycles summed over waves of LDS staging, traversal and
shading + spawn, and the same divided by the wave count (rays / 64, rounded
up per launch is not known here: an estimate). Usage: phase_time.py r/n [c3|c5]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

r, n = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0/1").split("/"))
w, cam, depth = getattr(scenes, sys.argv[2] if len(sys.argv) > 2 else "c3")()
w.upload(0)
rows = rtamd.shard_rows(cam.vsize, 8, r, n)
buf = torch.empty((rows, cam.hsize, 3), dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    cam.render_shard_device(w, depth, 8, r, n, buf.data_ptr(), s, False)
torch.cuda.synchronize()
rtamd._rtamd._wf_profile(w, 1, False)
cam.render_shard_device(w, depth, 8, r, n, buf.data_ptr(), s, False)
torch.cuda.synchronize()
p = rtamd._rtamd._wf_profile(w, 0, True)
print("keys", list(p.keys()))
for c in ("primary", "closest"):
    rays = p["rays"][c]
    waves = max(rays / 64.0, 1.0)
    st, tr, pr = p["disc"][c], p["tests"][c], p["boxes"][c]
    print(f"{c}: rays {rays:.0f} ms {p['ms'][c]:.3f}  cycles/frame stage {st:.3g} trav {tr:.3g} prep {pr:.3g}"
          f"  per 64 rays: stage {st / waves:.0f} trav {tr / waves:.0f} prep {pr / waves:.0f}")
# shading sub-phases of the closest class (fused kernels; lane 0 of each wave)
sub = {"prepare": p["disc"]["shadow"], "append": p["tests"]["shadow"], "spawn": p["boxes"]["shadow"],
       "lights": p["shadow_tests_in"]["primary"], "writes": p["shadow_rays_in"]["primary"]}
tot = sum(sub.values()) or 1.0
print("closest shading sub-phases (share of lane 0's shading cycles):",
      {k: round(v / tot, 3) for k, v in sub.items()})
