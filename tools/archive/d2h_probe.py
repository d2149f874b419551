"""Device-to-host copy engines (dev tool): a 49.8 MB canvas copied into pinned
host memory with hipMemcpyAsync as hipMemcpyDeviceToHost (ROCclr picks a blit
kernel, which holds CUs) and as hipMemcpyDeviceToDeviceNoCU (the DMA engines);
each alone, and each beside a C3 render on another stream (does the copy slow
the render?). Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
w, cam, depth = scenes.c3()
w.upload(0)
H, W = cam.vsize, cam.hsize
dev = torch.rand((H, W, 3), dtype=torch.float64, device="cuda")
host = torch.empty((H, W, 3), dtype=torch.float64, pin_memory=True)
nbytes = dev.numel() * 8
cs = torch.cuda.Stream()
rs = rtamd.render_stream(False)
rbuf = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
out = {}


def copy(kind):
    rc = hip.hipMemcpyAsync(ctypes.c_void_p(host.data_ptr()), ctypes.c_void_p(dev.data_ptr()), nbytes, kind,
                            ctypes.c_void_p(cs.cuda_stream))
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync kind {kind}: {rc}")


def render():
    cam.render_shard_device(w, depth, 8, 0, 1, rbuf.data_ptr(), rs.cuda_stream, False)


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(sorted(ts)[len(ts) // 2], 4)


for name, kind in (("d2h", 2), ("nocu", 1024)):
    try:
        host.zero_()
        copy(kind)
        torch.cuda.synchronize()
        out[f"{name}_equal"] = bool(torch.equal(host, dev.cpu()))
        out[f"{name}_copy_ms"] = timed(lambda: copy(kind))
        out[f"{name}_copy_and_render_ms"] = timed(lambda: (copy(kind), render()))
    except Exception as e:  # noqa: BLE001
        out[f"{name}_error"] = str(e)
out["render_ms"] = timed(render)
print(json.dumps(out), flush=True)
