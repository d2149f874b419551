"""Which cross-stream waits slow down frames in flight on CU-masked streams
(dev probe). Renders 100 C3 frames on 4 library streams and times them with
no waits, with the current stream waiting on each frame (main <- render),
and with each render waiting on an event of the current stream (render <- main)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa
import rtamd  # noqa
from rtamd import scenes  # noqa
kind = sys.argv[1] if len(sys.argv) > 1 else "cumask"
rtamd._rtamd._tuning_set("shadow_stream", 0)
w, cam, depth = scenes.c3()
w.upload(0)
F = 4
main = torch.cuda.current_stream()
sts = [rtamd.render_stream(kind == "cumask") for _ in range(F)] if kind != "torch" else [torch.cuda.Stream() for _ in range(F)]
bufs = [torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda") for _ in range(F)]
def run(mode, frames=100):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(frames):
        rs = sts[f % F]
        if mode == "render<-main":
            ev = torch.cuda.Event(); ev.record(main); rs.wait_event(ev)
        cam.render_shard_device(w, depth, 8, 0, 1, bufs[f % F].data_ptr(), rs.cuda_stream, False)
        if mode == "main<-render":
            main.wait_stream(rs)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / frames * 1e3
for m in ("none", "none", "main<-render", "render<-main", "none"):
    print(kind, m, f"{run(m):.3f} ms/frame", flush=True)
