"""Wall time per frame with and without the per-kernel HIP-event profiling (dev tool)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa
import rtamd
from rtamd import scenes
w, cam, depth = scenes.c3()
w.upload(0)
buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s, True)
for _ in range(5):
    cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s, False)
torch.cuda.synchronize()
for rnd in range(3):
    for prof in (0, 1, 5):
        rtamd._rtamd._wf_profile(w, prof, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s, False)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 50 * 1e3
        p = rtamd._rtamd._wf_profile(w, 0, True)
        print(f"profiling={prof}: {dt:.4f} ms/frame  kernel sum {sum(p['ms'].values()) if prof else 0:.4f}", flush=True)
