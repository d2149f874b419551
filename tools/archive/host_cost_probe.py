"""Host-side cost of enqueueing one frame (dev probe): times N calls of
render_shard_device without synchronising (host enqueue rate) and with the
final synchronise (device rate), for the whole frame and an 8-way shard, and
the cost of torch's wait_stream between two streams."""
import os, sys, time
os.environ["GPU_MAX_HW_QUEUES"] = "8"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa
import rtamd  # noqa
from rtamd import scenes  # noqa
rtamd._rtamd._tuning_set("shadow_stream", 0)
w, cam, depth = scenes.c3()
w.upload(0)
F = 4
sts = [rtamd.render_stream(False) for _ in range(F)]
for sh in ((0, 1), (0, 8), (0, 64)):
    rows = rtamd.shard_rows(cam.vsize, 8, sh[0], sh[1])
    bufs = [torch.empty((rows, cam.hsize, 3), dtype=torch.float64, device="cuda") for _ in range(F)]
    for f in range(3 * F):
        cam.render_shard_device(w, depth, 8, sh[0], sh[1], bufs[f % F].data_ptr(), sts[f % F].cuda_stream, False)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for f in range(n):
        cam.render_shard_device(w, depth, 8, sh[0], sh[1], bufs[f % F].data_ptr(), sts[f % F].cuda_stream, False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"shard {sh}: host enqueue {(t1 - t0) / n * 1e6:.1f} us/frame, device {(t2 - t0) / n * 1e6:.1f} us/frame", flush=True)
a, b = sts[0], sts[1]
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(1000):
    b.wait_stream(a)
t1 = time.perf_counter()
print(f"torch wait_stream: {(t1 - t0) / 1000 * 1e6:.1f} us host each", flush=True)
