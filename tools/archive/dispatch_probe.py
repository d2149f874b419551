"""Device-side dispatch rate of tiny kernels (dev probe). Each stream first
runs torch.cuda._sleep (a spin kernel) long enough for the host to enqueue K
one-block kernels (torch's add_ on a 64-element tensor) behind it; the
backlog then drains at the device's dispatch rate. Drain time = total -
sleep. Done on one stream, then with the launches spread round-robin over
4 and 8 streams, each with its own hardware queue. If the spread backlog
drains no faster than the single-stream one, consecutive dispatches are
serialised device-wide, and a frame's fixed cost is about its launch count
times that per-dispatch time.
Usage: dispatch_probe.py [--launches K]"""
import argparse
import os
import time

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--launches", type=int, default=2000)
ap.add_argument("--sleep-cycles", type=int, default=200_000_000)
a = ap.parse_args()
K = a.launches


def sleep_time(streams):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for st in streams:
        with torch.cuda.stream(st):
            torch.cuda._sleep(a.sleep_cycles)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


for n_streams in (1, 4, 8):
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    xs = [torch.zeros(64, device="cuda") for _ in range(n_streams)]
    for rep in range(2):  # the first pass warms up
        t_sleep = sleep_time(streams)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for st in streams:
            with torch.cuda.stream(st):
                torch.cuda._sleep(a.sleep_cycles)
        for i in range(K):
            k = i % n_streams
            with torch.cuda.stream(streams[k]):
                xs[k].add_(1.0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    ok = "" if t1 - t0 < t_sleep else " (enqueue outlasted the sleep: raise --sleep-cycles)"
    print(f"{n_streams} stream(s): {K} launches, host {(t1 - t0) / K * 1e6:.2f} us/launch, sleep {t_sleep * 1e3:.1f} ms, "
          f"device drain {((t2 - t0) - t_sleep) / K * 1e6:.2f} us/launch{ok}", flush=True)
