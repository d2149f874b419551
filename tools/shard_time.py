"""Per-GPU frame time of one shard of the bench workload at N = 1, 2, 4, 8
(dev tool): renders rank r's interleaved row blocks of an N-way split on the
one local GPU, so the render part of the multi-GPU scaling curve can be read
without N GPUs (the RCCL gather is not included). Prints, per N, the mean
frame time over the ranks and the worst rank, and the per-class breakdown of
rank 0. --batch B renders B frames per call (rt_render_frames_device; the
frame count stays K). Usage: shard_time.py [--frames K] [--batch B] [--knob k=v ...]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:  # as bench.py
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--row-block", type=int, default=8)
ap.add_argument("--knob", action="append", default=[])
ap.add_argument("--ns", default="1,2,4,8")
ap.add_argument("--inflight", type=int, default=4)
ap.add_argument("--streams", default="raw", choices=["torch", "once", "raw", "cumask"],
                help="torch: new torch streams per rank; once: torch streams made once; raw / cumask: library-made streams (cumask: hipExtStreamCreateWithCUMask), made once")
ap.add_argument("--reverse", action="store_true", help="measure the ranks last to first")
ap.add_argument("--ranks", action="store_true", help="print every rank's time")
ap.add_argument("--batch", type=int, default=1)
a = ap.parse_args()
for kv in a.knob:
    k, v = kv.split("=")
    rtamd._rtamd._tuning_set(k, int(v))
w, cam, depth = scenes.c3()
w.upload(0)
H, W, B = cam.vsize, cam.hsize, a.row_block
s = torch.cuda.current_stream().cuda_stream
base = None
_F = max(1, a.inflight)
if a.streams == "once":
    _made = [torch.cuda.Stream() for _ in range(_F)]
elif a.streams in ("raw", "cumask"):
    _made = [torch.cuda.ExternalStream(rtamd._rtamd._stream_create(a.streams == "cumask")) for _ in range(_F)]
else:
    _made = None
for n in [int(x) for x in a.ns.split(",")]:

    order = list(range(n))[::-1] if a.reverse else list(range(n))
    times = [0.0] * n
    for r in order:
        rows = rtamd.shard_rows(H, B, r, n)
        F = max(1, a.inflight)
        if F > 1:
            w.tune("shadow_stream", 0)  # as bench.py
        NB = max(1, a.batch)
        bufs = [torch.empty((rows, W, 3), dtype=torch.float64, device="cuda") for _ in range(F * NB)]
        sts = _made or ([torch.cuda.Stream() for _ in range(F)] if F > 1 else [torch.cuda.current_stream()])

        def one(f):
            if NB == 1:
                cam.render_shard_device(w, depth, B, r, n, bufs[f % F].data_ptr(), sts[f % F].cuda_stream, False)
            else:
                k = f % F
                rtamd.render_frames_device(w, [cam] * NB, depth, B, r, n,
                                           [b.data_ptr() for b in bufs[k * NB:(k + 1) * NB]], sts[k].cuda_stream)
        torch.cuda.synchronize()
        for f in range(3 * F):
            one(f)
        torch.cuda.synchronize()
        calls = max(1, a.frames // NB)
        t0 = time.perf_counter()
        for f in range(calls):
            one(f)
        torch.cuda.synchronize()
        times[r] = (time.perf_counter() - t0) / (calls * NB) * 1e3
        if r == 0:  # per-class times from a separate profiled pass (events would slow the timed frames)
            rtamd._rtamd._wf_profile(w, 1, False)
            for f in range(min(calls, 20)):
                one(f)
            torch.cuda.synchronize()
            p = rtamd._rtamd._wf_profile(w, 0, True)
            cls = " ".join(f"{c}={m:.3f}" for c, m in p["ms"].items())
    mean, worst = sum(times) / n, max(times)
    base = base or worst
    if "--ranks" in sys.argv:
        print("   per rank ms:", " ".join(f"{t:.3f}" for t in times))
    print(f"N={n}: per-GPU frame mean {mean:.3f} ms, worst rank {worst:.3f} ms -> render speedup {base / worst:.2f}x"
          f"  (rank 0 classes, profiled pass: {cls})", flush=True)
