#!/usr/bin/env python3
"""Headline benchmark: Mrays/s on the 1920x1080 / 1000-sphere / depth-5 scene.

A "step" renders ONE full frame of the C3 workload (SURVEY.md §8d,
rtamd.scenes.c3): `Camera::render(&World)` with MAX_RECURSION_DEPTH = 5, all
of primary + reflection + refraction + shadow rays (each one a
`World::intersect`, world.rs:71,101). With N GPUs (one process per GPU,
launched by torch.distributed.run) the frame is split into interleaved 8-row
blocks, each rank renders its rows into HBM, and the canvas is assembled on
rank 0 with one RCCL gather (strong scaling: the frame is fixed). F frames
are rendered in batches of NB (--batch, default for C3 8 on 1-2 GPUs and 16 on 4+, for C5 2 on one GPU, 1 on N: one
rt_render_frames_device call renders NB frames, every launch of the pipeline
carrying all of them) on F streams (--inflight, default 4 for C3, 2 for C5 on one GPU and 1 on N),
each with its own library workspace, so one batch's short, latency-bound deep
generations overlap the next batch's work; every frame is complete, gathered
(one gather per batch) and assembled inside the timed region.

The scene is uploaded before timing (inputs resident in HBM). The timed
region holds exactly K steps bracketed by barrier + synchronize; the
reported time is the max over ranks.

Printed JSON line (rank 0): metric/value/unit per BASELINE.json, plus
  roofline      f64 VALU roofline of the dominant trace-kernel class of the
                wavefront pipeline; kernel time from HIP events carried by its
                launches in a serialized pass of the same K frames (one stream,
                kernels alone on the GPU, as in the rocprofv3 kernel trace)
  cpu_baseline  the C oracle (a port of the reference algorithm) on a bounded
                row sample on this host's cores (N=1, rank 0 only)
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]


def _launch_ranks():
    """`python bench.py --gpus N` (N > 1) outside a torch.distributed launcher:
    start the N ranks ourselves, one fresh process per GPU, through
    torch.distributed.run (the driver's own command line for N > 1), and exit
    with its status. Runs before anything touches the GPU (the parent only
    counts devices, which does not initialise HIP) and never re-execs itself.
    Mirrors render_multithreaded owning its workers (camera.rs:150-217)."""
    import socket
    import subprocess
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-launch", action="store_true")
    a, _ = ap.parse_known_args()
    if "WORLD_SIZE" in os.environ:
        ws = int(os.environ["WORLD_SIZE"])
        if a.gpus != ws:
            sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={ws} ranks")
        return
    import torch
    visible = torch.cuda.device_count()  # counts devices without initialising HIP
    if a.gpus > visible and not a.dry_launch:
        sys.exit(f"bench.py: --gpus {a.gpus} but only {visible} GPU(s) are visible")
    if a.gpus <= 1:
        return
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


# Frames in flight render on several streams (--inflight): give the process
# enough hardware queues that they do not share one (HIP's default is 4; the
# current stream, the render streams and RCCL's stream each want their own).
# Read by the HIP runtime at initialisation, so before torch is imported (and
# before _launch_ranks counts the devices).
# With N GPUs each render stream may also have a process group's RCCL stream.
_queues = 8 if int(os.environ.get("WORLD_SIZE", "1") or 1) == 1 else 16
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _queues:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_queues)

if __name__ == "__main__":
    _launch_ranks()

if "--dry-launch" in sys.argv and __name__ == "__main__":  # dev/test: report the rank layout, touch no GPU
    # one write(2) of the whole line: ranks share the stdout pipe, and a write
    # below PIPE_BUF is atomic, so two ranks' lines never interleave
    os.write(1, (json.dumps({"dry_launch": True, "rank": int(os.environ.get("RANK", "0")),
                             "world_size": int(os.environ.get("WORLD_SIZE", "1")),
                             "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}) + "\n").encode())
    sys.exit(0)

import torch  # noqa: E402  (load torch's HIP runtime first: see rtamd/__init__.py)
import torch.distributed as dist  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402
from rtamd.distributed import (FrameAssembler, RcclStreamAssembler, StreamFrameAssembler, block_patterns,  # noqa: E402
                               root_share_default, shard_of)

WF_CLOSEST = 1  # kernel class index (csrc/rt_wavefront.hpp WfClass)
METRIC = "Mrays/s (primary+secondary) on 1920×1080/1000-sphere/depth-5; 1→8 GPU scaling"
METRIC_C5 = "Mrays/s (primary+secondary) on 4096×4096/10000-shape/depth-8 (C5)"
PEAK_F64_VALU_TFLOPS = 39.3  # 256 CU x 64 f64 lanes/clk x 2.4 GHz, non-fused add/mul (MI355X_MICROARCH.md)

# Algorithmic f64 operations per unit of work (DESIGN.md "Roofline"): the
# minimum non-fused add/mul count that reproduces the reference's bits.
#   sphere test, diagonal inverse:   9 (object-space ray) + 5 (a) + 5 (d.o) + 6 (c) + 3 (disc) = 28
#   sphere test, primary ray:        3 (d' = s*d) + 5 (a) + 5 (d'.o') + 3 (disc) = 16  (o', c shared per frame)
#   sphere test, general inverse:   33 (object-space ray) + 5 + 5 + 6 + 3 = 52
#   roots when disc >= 0:            sqrt + 2 add + 2 div, priced 5
#   plane test:                      6 (o'.y) + 5 (d'.y) + 1 (|d'.y| compare) = 12
#   BVH child-box slab test:         binary32: 6 fma + 12 min/max + 1 compare = 19 instructions,
#                                    = 9.5 f64-op issue slots (binary32 VALU issues at twice the rate)
OPS_SPHERE_DIAG, OPS_SPHERE_PRIMARY, OPS_SPHERE_GEN = 28, 16, 52
OPS_ROOTS = 5
OPS_PLANE = 12
OPS_BOX = 9.5
# SURVEY.md §8(d) convention (the reference's general 4x4 path): 57 / 34 / +6
SURVEY_OPS_SPHERE, SURVEY_OPS_PLANE, SURVEY_OPS_ROOTS = 57, 34, 6


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=64)  # whole batches of 8 and 16
    p.add_argument("--warmup", type=int, default=16)
    p.add_argument("--config", default="c3", choices=["c3", "c5"],
                   help="c3: the headline workload (default); c5: 4096x4096, 4 planes + 9996 spheres, 2 lights, "
                        "depth 8 (SURVEY.md §8d C5; sizes below override)")
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--spheres", type=int, default=None)
    p.add_argument("--depth", type=int, default=None)
    p.add_argument("--row-block", type=int, default=8)
    p.add_argument("--batch", type=int, default=None,
                   help="frames per render call (rt_render_frames_device, <= 16; default for C3 8 on 1-2 GPUs, "
                        "16 on 4+; 2 for C5 on one GPU, 1 on N)")
    p.add_argument("--inflight", type=int, default=None,
                   help="frames in flight: consecutive frames render on this many streams (own workspaces)")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget for the CPU baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--stream-kind", default="raw", choices=["cumask", "raw", "torch"],
                   help="render streams: library-made plain (raw), library-made CU-masked (cumask), torch")
    p.add_argument("--fake-shard", default=None,
                   help="dev: r/n renders only rank r's rows of an n-way split on this one process (no gather)")
    p.add_argument("--root-share", type=float, default=None,
                   help="N GPUs: rank 0 (which also assembles every frame) renders this fraction of an equal row "
                        "share, through block patterns (rt_render_block_pattern_device); default: measured per "
                        "config and N (rtamd.distributed.root_share_default); 1 = the plain interleave")
    p.add_argument("--verify", action="store_true",
                   help="dev: check the last assembled frame against a one-GPU render of the whole frame")
    p.add_argument("--dist-backend", default="nccl", help="dev: torch.distributed backend (nccl = RCCL)")
    p.add_argument("--assembler", default="rccl", choices=["rccl", "stream", "main"],
                   help="N GPUs: gathers enqueued by the library on each render stream (rccl), per-stream "
                        "torch process groups (stream), or assembly on the current stream (main, dev)")
    p.add_argument("--emulate-gather", action="store_true",
                   help="dev, 1 GPU: per render stream, a side stream standing in for its RCCL stream copies the "
                        "shard (fenced both ways, as the N-GPU stream assembler), then the un-interleave runs")
    p.add_argument("--event-path", action="store_true",
                   help="dev: on one GPU, run the N-GPU frame pipeline (shard slots, cross-stream events)")
    p.add_argument("--knob", action="append", default=[], help="library tuning knob k=v (dev; see rt_api.cpp)")
    p.add_argument("--exhaustive", action="store_true",
                   help="disable the exact-culling BVH: every ray tests every shape (the reference's loop)")
    p.add_argument("--pmc-summary", default=None,
                   help="HBM traffic per launch measured by rocprofv3 --pmc for this workload "
                        "(default: the newest profiles/r*_pmc_summary*.json that matches it)")
    p.add_argument("--no-verify-frames", action="store_true",
                   help="dev: skip the bitwise check of the last timed frame against the exhaustive frame")
    p.add_argument("--no-end-to-end", action="store_true",
                   help="dev: skip the host-canvas + PPM timing of the drop-in entry point")
    p.add_argument("--no-distinct", action="store_true", help="dev: skip the orbiting-camera (distinct cameras) run")
    p.add_argument("--no-cold", action="store_true", help="dev: skip the cold-start (scene create + first render) run")
    p.add_argument("--dry-launch", action="store_true",
                   help="test: each rank prints its RANK/WORLD_SIZE and exits without touching a GPU")
    return p.parse_args()


def host_cores():
    """CPUs this process may use: its affinity set, capped by a cgroup CPU quota
    (cpu.max) when one is set. `os.cpu_count()` is the whole machine."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(world, cam, depth, budget_s):
    """Oracle (C port of the reference algorithm: full intersection list + sort
    + containers walk, recursive color_at), threads in contiguous row blocks like
    render_multithreaded (camera.rs:157-172): on every core this process may
    use, the whole frame when it takes at most two minutes (C3), else evenly
    spaced rows sized to ~budget_s; and on one core, rows sized to a third of
    budget_s."""
    from oracle import pyoracle
    ow = pyoracle.OracleWorld.from_world(world)
    desc = cam.desc_bytes()
    H = cam.vsize

    def run(rows, nthreads):
        t0 = time.perf_counter()
        _, st = ow.render_rows(desc, depth, rows, nthreads)
        dt = time.perf_counter() - t0
        return dt, st["rays_primary"] + st["rays_reflect"] + st["rays_refract"] + st["rays_shadow"]

    def sample(nthreads, budget, full_limit=0.0):
        # calibrate: one row per thread, spread over the frame
        probe = sorted({int((i + 0.5) * H / nthreads) for i in range(min(nthreads, H))})
        t_probe, r_probe = run(probe, nthreads)
        if t_probe * H / len(probe) <= full_limit:  # the whole frame fits the limit: SURVEY §8(d)'s full frame
            dt, rays = run(list(range(H)), nthreads)
            return list(range(H)), dt, rays, 1
        if t_probe >= 0.5 * budget:  # slow rows (C5): the probe already is the sample
            return probe, t_probe, r_probe, max(1, H // len(probe))
        n_rows = int(max(1, min(H, len(probe) * budget / max(t_probe, 1e-6))))
        stride = max(1, H // n_rows)
        rows = list(range(stride // 2, H, stride))
        dt, rays = run(rows, nthreads)
        return rows, dt, rays, stride

    nthreads = host_cores()
    # the full frame on every core when it takes at most ~2 minutes (C3 on the GPU box's 16 cores: ~52 s;
    # a row sample measured 0.79-1.05x of it, the row blocks' load balance depending on the sample,
    # profiles/r06_cpu_full_frame.json), else evenly spaced rows
    rows, dt, rays, stride = sample(nthreads, budget_s, full_limit=120.0)
    rows1, dt1, rays1, stride1 = sample(1, budget_s / 3)
    return {
        "value": rays / dt / 1e6,
        "unit": "Mrays/s",
        "cores": nthreads,
        "kind": "port",
        "cpu_model": cpu_model(),
        "cpus_on_host": os.cpu_count(),
        "single_core": {"value": rays1 / dt1 / 1e6, "unit": "Mrays/s", "cores": 1,
                        "sample": f"{len(rows1)} of {H} rows (every {stride1}th), {rays1} rays in {dt1:.2f}s"},
        "sample": (f"the full frame ({H} rows), {rays} rays in {dt:.2f}s; " if stride == 1 else
                   f"{len(rows)} of {H} rows (every {stride}th), {rays} rays in {dt:.2f}s; ") +
                  f"C restatement of the reference algorithm (oracle/rt_oracle.c: full intersection list + "
                  f"sort + containers walk, recursion depth {depth}), {nthreads} threads in row blocks "
                  f"(every CPU this process may use: affinity set, cgroup quota)",
    }


def end_to_end(world, cam, depth, frames=3):
    """The drop-in entry point as a caller sees it: `rt_render` (Camera::render,
    camera.rs:133-148: device render + the canvas copied to a host buffer) and
    `rt_canvas_to_ppm` (image/ppm.rs:24-51), per frame, one frame at a time."""
    # warm: the scene's workspaces, and two pooled pinned canvases (a loop holds the
    # previous frame's canvas while the next one renders)
    # (and a few more frames: the band workspaces' arenas settle on their learned sizes)
    warm = [cam.render(world, depth, want_stats=False)[0] for _ in range(2)]
    del warm
    for _ in range(3):
        cam.render(world, depth, want_stats=False)
    t0 = time.perf_counter()
    for _ in range(frames):
        canvas, _ = cam.render(world, depth, want_stats=False)
    t_render = (time.perf_counter() - t0) / frames
    arr = canvas.to_numpy()
    t_ppms = []
    for _ in range(3):  # (each call returns a new bytes object, as a caller's would)
        t0 = time.perf_counter()
        ppm = rtamd.canvas_to_ppm(arr)
        t_ppms.append(time.perf_counter() - t0)
    t_ppm = sorted(t_ppms)[1]
    ref = ppm.encode() if isinstance(ppm, str) else bytes(ppm)
    # rt_render_ppm into the caller's buffer, reused frame after frame (pinned, as rt_host_buffer_alloc gives)
    buf = rtamd._rtamd.host_buffer(len(ref) + 4096)
    n = cam.render_ppm_into(world, buf, depth)  # warm: the scene's PPM buffers
    t0 = time.perf_counter()
    for _ in range(frames):
        n = cam.render_ppm_into(world, buf, depth)
    t_render_ppm = (time.perf_counter() - t0) / frames
    if buf[:n].tobytes() != ref:
        raise SystemExit("bench: rt_render_ppm text differs from rt_canvas_to_ppm of the rendered canvas")
    # the Python binding: a new bytes object per frame
    dev_ppm, _ = cam.render_ppm(world, depth)
    t0 = time.perf_counter()
    for _ in range(frames):
        dev_ppm, _ = cam.render_ppm(world, depth)
    t_bytes = (time.perf_counter() - t0) / frames
    if bytes(dev_ppm) != ref:
        raise SystemExit("bench: the render_ppm binding's text differs from rt_canvas_to_ppm of the rendered canvas")
    return {"ms_render_to_host": round(t_render * 1e3, 3), "ms_canvas_to_ppm": round(t_ppm * 1e3, 3),
            "ms_render_ppm": round(t_render_ppm * 1e3, 3), "ms_render_ppm_bytes": round(t_bytes * 1e3, 3),
            "ppm_bytes": len(ppm), "frames": frames,
            "note": "rt_render (device render + device-to-host copy of the f64 canvas, in row bands, one frame at a "
                    "time), rt_canvas_to_ppm on the host (median of 3 calls), rt_render_ppm (render + PPM encoded on the device + the "
                    "text copied to the host: canvas_to_ppm(&camera.render(&world)) in one call) into the caller's "
                    "reused pinned buffer, and the same through the Python binding, which returns a new bytes object "
                    "per frame (ms_render_ppm_bytes); bytes checked equal; not the headline value"}


def distinct_cameras(world, depth, rstreams, dev, headline, frames=64, nb=8, passes=3):
    """An animation over the C3 scene: `frames` cameras along an arc
    (scenes.c3_orbit), each rendered for the first time, in batches of `nb` on
    the render streams (batch b on stream b % F, as the headline). Nothing is
    calibrated per camera: every generation of every frame sizes itself on the
    device. `passes` timed passes, each over a new arc (0.8, 0.9, 1.0 rad: no
    camera repeats); the value is the median pass. Mrays/s counts each camera's
    own reference rays (one counted fast-path render per camera, after timing);
    the frames left in the buffers (the last batch of every stream) are checked
    bitwise against their exhaustive frames."""
    F = len(rstreams)
    n_batches = frames // nb
    results = []
    for p in range(passes):
        cams = [scenes.c3_orbit(k, frames, arc=0.8 + 0.1 * p) for k in range(frames)]
        H, W = cams[0].vsize, cams[0].hsize
        bufs = [[torch.empty((H, W, 3), dtype=torch.float64, device=dev) for _ in range(nb)] for _ in range(F)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in range(n_batches):
            rs = rstreams[b % F]
            rtamd.render_frames_device(world, cams[b * nb:(b + 1) * nb], depth, 8, 0, 1,
                                       [x.data_ptr() for x in bufs[b % F]], rs.cuda_stream)
        torch.cuda.synchronize()
        results.append((time.perf_counter() - t0, cams, bufs))
    world.check()  # every frame complete (no arena overflow)
    dts = sorted(r[0] for r in results)
    dt, cams, bufs = next(r for r in results if r[0] == dts[len(dts) // 2])
    ok = True
    ref = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
    for b in range(max(0, n_batches - F), n_batches):
        for j in range(nb):
            cams[b * nb + j].render_shard_device(world, depth, 8, 0, 1, ref.data_ptr(),
                                                 torch.cuda.current_stream().cuda_stream, True, exhaustive=True)
            torch.cuda.synchronize()
            ok = ok and bool(torch.equal(ref, bufs[b % F][j]))
    rays = 0
    for c in cams[:n_batches * nb]:
        st = c.render_shard_device(world, depth, 8, 0, 1, ref.data_ptr(), torch.cuda.current_stream().cuda_stream,
                                   True, exhaustive=False)
        rays += st["rays_primary"] + st["rays_reflect"] + st["rays_refract"] + st["rays_shadow"]
    del bufs, ref, results
    value = rays / dt / 1e6
    return {"value": round(value, 3), "unit": "Mrays/s", "frames": n_batches * nb, "batch": nb, "streams": F,
            "ms_per_frame": round(dt / (n_batches * nb) * 1e3, 4), "vs_headline": round(value / headline, 4),
            "passes_ms_per_frame": [round(x / (n_batches * nb) * 1e3, 4) for x in dts],
            "parity": {"vs_exhaustive": "bitwise", "ok": ok, "frames_checked": min(F, n_batches) * nb},
            "note": "C3 scene, a new camera every frame (scenes.c3_orbit: arcs of 0.8, 0.9 and 1.0 rad around the "
                    "look-at point, one timed pass each, the median pass reported), batches of 8 on the render streams, "
                    "no per-camera calibration or cache; value = the cameras' own reference rays / wall time"}


def cold_start(dev_index):
    """The first call of a new caller: rt_scene_create (flatten, hierarchies,
    light buffer, upload) and the first rt_render into a host canvas (render +
    device-to-host copy) of the C3 scene and camera; rt_scene_create of C5.
    The host World's construction (the caller's own code) is not timed."""
    w, cam, depth = scenes.c3()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w.upload(dev_index)
    t1 = time.perf_counter()
    canvas, _ = cam.render(w, depth, want_stats=False)
    t2 = time.perf_counter()
    del canvas, w
    w5, _, _ = scenes.c5()
    t3 = time.perf_counter()
    w5.upload(dev_index)
    t4 = time.perf_counter()
    del w5
    return {"c3_scene_create_ms": round((t1 - t0) * 1e3, 3), "c3_first_render_ms": round((t2 - t1) * 1e3, 3),
            "c3_cold_ms": round((t2 - t0) * 1e3, 3), "c5_scene_create_ms": round((t4 - t3) * 1e3, 3),
            "note": "rt_scene_create + the first rt_render (device render + canvas to host) of a fresh C3 scene "
                    "and camera; rt_scene_create of C5 (10000 shapes: BVH, light buffer, upload)"}


def main():
    a = parse()
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world_size:  # _launch_ranks starts N ranks for --gpus N; never fall back silently
        sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world_size}")
    n = world_size
    srank, sn = shard_of(rank, n), n  # the shard this process renders (rank 0 assembles: the smallest)
    prank, pn = rank, n  # the rank whose rows this process renders (pattern mode)
    if a.fake_shard:
        prank, pn = (int(x) for x in a.fake_shard.split("/"))
        srank, sn = shard_of(prank, pn), pn
    # rank 0 receives and un-interleaves every frame: with a share below 1 it renders fewer
    # row blocks than the others (block patterns, DESIGN.md §6, profiles/r05_assembly_n8.txt)
    share = a.root_share if a.root_share is not None else root_share_default(a.config, pn)
    pattern = block_patterns(pn, share) if pn > 1 and share < 1.0 else None
    my_mask = pattern[1][prank] if pattern else None
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if n > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:  # dev rehearsal of the N-rank pipeline, e.g. 2 ranks sharing one GPU
            dist.init_process_group(a.dist_backend)

    for kv in a.knob:
        k, v = kv.split("=")
        rtamd._rtamd._tuning_set(k, int(v))
    dflt = {"c3": (1920, 1080, 1000), "c5": (4096, 4096, 9996)}[a.config]
    a.width, a.height, a.spheres = a.width or dflt[0], a.height or dflt[1], a.spheres or dflt[2]
    world, cam, depth = getattr(scenes, a.config)(a.width, a.height, a.spheres)
    if a.depth is not None:
        depth = a.depth
    world.upload(local_rank)  # flatten + upload: outside the timed region
    if a.exhaustive:
        world.tune("accel", 0)
    W, H, B = cam.hsize, cam.vsize, a.row_block

    def render(cams, ptrs, stream_handle, want_stats=False, exhaustive=False):
        """This rank's rows of the frames `cams` into the device buffers `ptrs`."""
        if pattern:
            return rtamd.render_block_pattern_device(world, cams, depth, B, pattern[0], my_mask, ptrs, stream_handle,
                                                     want_stats, 1, exhaustive)
        if len(cams) == 1:
            return cams[0].render_shard_device(world, depth, B, srank, sn, ptrs[0], stream_handle, want_stats,
                                               exhaustive=exhaustive)
        return rtamd.render_frames_device(world, cams, depth, B, srank, sn, ptrs, stream_handle)
    # Batches of NB frames (one rt_render_frames_device call: every launch of the
    # pipeline carries the NB frames) on F streams: batch b renders on
    # stream b % F (the library keeps one workspace per stream, so the batches overlap
    # on the device).
    # - 1 GPU: into canvas slots; stream order alone protects a slot.
    # - N GPUs (default "rccl" assembler): each render stream owns a batch of shard
    #   slots, a gather buffer, canvases and an RCCL communicator, and a batch's render,
    #   its ONE gather and rank 0's un-interleave all queue behind its own stream, so
    #   batches on different streams never wait on each other (RcclStreamAssembler;
    #   "stream": the same with torch process groups, StreamFrameAssembler).
    # - "main" assembler (dev): one frame per call, gather and un-interleave on the
    #   current stream, coupled to the render streams by events (FrameAssembler).
    # The render streams are plain streams, each on its own hardware queue
    # (GPU_MAX_HW_QUEUES above); CU-masked streams (--stream-kind cumask) also get
    # their own queue, but any cross-stream wait on them costs ~1 ms.
    # default: 4 streams for C3; two for C5 on one GPU (one on N: the shards' row
    # blocks), whose wavefront workspace (16.8 M primary rays, depth 8) takes tens of
    # GB per frame
    F = max(1, a.inflight if a.inflight is not None else (4 if a.config == "c3" else (2 if n == 1 else 1)))
    # (C3: 8 frames per pass on 1-2 GPUs, 16 on the smaller shards of 4+; C5: 2 per pass on one GPU. A C5
    # frame fills the GPU alone, but two passes of two frames in flight overlap one pass's
    # draining deep generations and combines with the other's work: 43.0 -> 42.2-42.4 ms per
    # frame, profiles/r06_c5_regime.txt)
    NB = max(1, min(16, a.batch if a.batch is not None else ((8 if n < 4 else 16) if a.config == "c3" else
                                                                 (2 if n == 1 else 1))))
    stream = torch.cuda.current_stream()
    kind = a.stream_kind
    if F == 1:
        rstreams = [stream]
    elif kind == "torch":
        rstreams = [torch.cuda.Stream(device=dev) for _ in range(F)]
    else:
        rstreams = [rtamd.render_stream(kind == "cumask") for _ in range(F)]
    if F > 1:  # the frames are the concurrency: no shadow side stream
        world.tune("shadow_stream", 0)
    per_stream = n > 1 and a.assembler in ("stream", "rccl")
    events = not per_stream and (n > 1 or a.event_path)
    if events:
        NB = 1  # the event-coupled dev path assembles frame by frame
    fa = None
    assembler_fallback = None  # why the RCCL stream assembler was not used (reported in the line)
    if n > 1 and a.assembler == "rccl" and F > 1:
        try:
            fa = RcclStreamAssembler(H, W, B, rank, n, dev, streams=rstreams, batch=NB, pattern=pattern)
        except Exception as e:  # fall back to the torch process groups
            assembler_fallback = f"{type(e).__name__}: {e}"
            print(f"warning: RCCL stream assembler unavailable ({e}); using per-stream process groups",
                  file=sys.stderr, flush=True)
            fa = None
    elif n > 1 and a.assembler == "rccl":
        assembler_fallback = "one render stream (--inflight 1): torch process groups on the current stream"
    if fa is not None:
        pass
    elif per_stream:
        groups = [dist.new_group(list(range(n))) for _ in range(F)]
        fa = StreamFrameAssembler(H, W, B, rank, n, dev, streams=rstreams if F > 1 else None, groups=groups,
                                  slots=F, batch=NB, pattern=pattern)
    else:
        fa = FrameAssembler(H, W, B, rank, n, dev, slots=F * NB if not events else (F + 1 if F > 1 else 2),
                            pattern=pattern if n > 1 else None)
    if not a.fake_shard:
        assert len(fa.rows) == (rtamd.pattern_rows(H, B, pattern[0], my_mask) if pattern
                                else rtamd.shard_rows(H, B, srank, n))
    shard = fa.shard
    free_ev = [None] * len(fa.shards)
    frame_no = [0]
    last_frame = [0]

    if a.emulate_gather:
        gstreams = [torch.cuda.Stream(device=dev) for _ in range(F)]
        gbufs = [torch.empty_like(fa.slot(k)) for k in range(F)]
        canv = [torch.empty_like(fa.slot(k)) for k in range(F)]
        perm = torch.randperm(fa.slot(0).shape[0], device=dev)

    def step(nf=None, assemble=True):
        """Render the next batch (nf <= NB frames, default NB) and queue its
        assembly; frame numbers advance by whole batches, so batch b always
        uses stream b % F and its own slots."""
        s = frame_no[0]
        if not events:
            nf = NB if nf is None else nf
            rs = rstreams[(s // NB) % F]
            render([cam] * nf, [fa.slot(s + j).data_ptr() for j in range(nf)], rs.cuda_stream)
            if a.emulate_gather:
                k = s % F
                gs = gstreams[k]
                gs.wait_stream(rs)
                with torch.cuda.stream(gs):
                    gbufs[k].copy_(fa.slot(s))
                rs.wait_stream(gs)
                with torch.cuda.stream(rs):
                    torch.index_select(gbufs[k], 0, perm, out=canv[k])
            if assemble:
                # 1 GPU: the slots are the canvases; N GPUs: one gather + un-interleave per batch, on its stream
                for j in range(nf):
                    submit(fa, s + j, j == nf - 1)
            frame_no[0] = s + NB
            last_frame[0] = s + nf - 1
            return
        rs = rstreams[s % F]
        slot = s % len(fa.shards)
        if rs is not stream and free_ev[slot] is not None:
            rs.wait_event(free_ev[slot])
        render([cam], [fa.slot(s).data_ptr()], rs.cuda_stream)
        if rs is not stream:
            stream.wait_stream(rs)
        fa.submit(s)
        if F > 1 and s > 0:  # frame s-1 is complete once the current stream gets here
            ev = torch.cuda.Event()
            ev.record(stream)
            free_ev[(s - 1) % len(fa.shards)] = ev
        frame_no[0] = s + 1
        last_frame[0] = s

    def settled(fn, tries=4):
        """fn() until no asynchronous pass of it outgrew its arenas (one GPU)."""
        for attempt in range(tries):
            try:
                fn()
                torch.cuda.synchronize()
                world.check()
                return
            except rtamd.RtError as e:
                if "overflow" not in str(e) or attempt == tries - 1:
                    raise
                torch.cuda.synchronize()

    def run_frames(k, assemble=True):
        """k frames: whole batches, then one partial batch."""
        for _ in range(k // NB):
            step(assemble=assemble)
        if k % NB:
            step(k % NB, assemble=assemble)

    # exact work counters of one frame (deterministic), from a counted warm-up launch
    # (this first launch also sizes the wavefront queues of this camera/shard)
    st = render([cam], [shard.data_ptr()], stream.cuda_stream, True, exhaustive=True)
    assert st["exhaustive"]
    # the exhaustive frame (the reference's every-shape loop) that the timed fast-path frames must equal
    ref_shard = shard.clone()
    counts = torch.tensor([st["rays_primary"], st["rays_reflect"], st["rays_refract"], st["rays_shadow"],
                           st["sphere_tests"], st["plane_tests"], st["sphere_disc_ge0"]],
                          dtype=torch.float64, device=dev)
    if n > 1:
        dist.all_reduce(counts)
    rays_per_frame = float(counts[:4].sum())
    # SURVEY §8(d) reference work F of one frame (the reference's exhaustive general-4x4
    # loop): 57 per sphere test, 34 per plane test, +6 per disc >= 0 (exact counters)
    ref_work = (SURVEY_OPS_SPHERE * float(counts[4]) + SURVEY_OPS_PLANE * float(counts[5])
                + SURVEY_OPS_ROOTS * float(counts[6]))
    # setup: one batch on each render stream allocates that stream's workspace
    # (queue arenas, counters), so the timed region never meets a first
    # allocation whatever --warmup is (with batches: a whole batch, and the timed
    # region's partial batch size, on every stream)
    def setup():
        for _ in range(F):
            step()
        if a.steps % NB:
            for _ in range(F):
                step(a.steps % NB)
        fa.flush()
    if n == 1:
        # a new workspace's first asynchronous pass may outgrow its guessed arenas:
        # that pass is poisoned and reported by the next call (rt_scene_check), and
        # the arenas have grown; run the setup again until it completes
        settled(setup)
    else:
        setup()
    torch.cuda.synchronize()
    run_frames(a.warmup)
    fa.flush()
    torch.cuda.synchronize()

    # Timed region: K frames, F in flight, no profiling events.
    rtamd._rtamd._wf_profile(world, 0, False)
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_frames(a.steps)
    last = fa.flush()  # the last frame's gather + un-interleave are inside the timed region
    torch.cuda.synchronize()
    if n > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # every asynchronous frame's device-side check (rt_scene_check): a frame left
    # incomplete raises here instead of passing unnoticed
    world.check()
    # Parity of the timed frames (outside the timed region): the last frame each
    # rank rendered, and rank 0's assembled canvas, must equal the exhaustive frame
    # bit for bit (camera.rs:133-148 renders every pixel with the every-shape loop).
    parity = None if a.no_verify_frames else verify_frames(fa, last, ref_shard, last_frame[0], n, rank, H)
    # Where an N-rank frame's time goes (outside the timed region, same streams and
    # batches): the renders alone, and the assembly (gathers + un-interleave) alone
    split = None
    if n > 1:
        split = phase_split(a, n, rank, dev, run_frames, fa, F, NB)
    # Serialized pass (outside the timed region): the same K frames in the same
    # batches (the benched launches: NB frames per launch), one batch after the
    # other on one stream, every launch carrying its own start/stop HIP events
    # (hipExtLaunchKernel), for the roofline's per-launch kernel time and the
    # per-class table (per frame: a batch's time / NB). With batches in flight the
    # timed region overlaps kernels of different batches, so a launch's duration
    # there includes the CUs it waited for; here each kernel runs alone, as in the
    # rocprofv3 kernel trace.
    sbufs = [torch.empty_like(shard) for _ in range(NB)] if NB > 1 else [shard]
    # (the current stream's workspace has rendered single frames so far: one untimed
    # batch of NB first, so that an outgrown arena is not met inside the pass)
    settled(lambda: render([cam] * NB, [b.data_ptr() for b in sbufs[:NB]], stream.cuda_stream))
    rtamd._rtamd._wf_profile(world, 1, False)
    for s0 in range(0, a.steps, NB):
        nf = min(NB, a.steps - s0)
        render([cam] * nf, [b.data_ptr() for b in sbufs[:nf]], stream.cuda_stream)
    torch.cuda.synchronize()
    del sbufs
    rtamd._rtamd._wf_profile(world, 0, False)
    # the fast path's own counters (what the kernels executed and traced), one counted
    # frame on the same workspace: the timed and profiled kernels do not count
    fst = render([cam], [shard.data_ptr()], stream.cuda_stream, True, exhaustive=False)
    breakdown = rtamd._rtamd._wf_profile(world, -1, True)  # class times of the profiled frames, counters of the counted one
    prof = breakdown
    if a.verify and rank == 0:  # dev: the assembled last frame equals a one-GPU render of the whole frame
        whole = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        cam.render_shard_device(world, depth, B, 0, 1, whole.data_ptr(), stream.cuda_stream, False)
        torch.cuda.synchronize()
        same = last is not None and bool(torch.equal(last, whole))
        print(f"verify: assembled frame {'==' if same else '!='} whole-frame render", file=sys.stderr, flush=True)
        if not same:
            raise SystemExit("verify failed: the assembled frame differs from the whole-frame render")
    traced = torch.tensor([fst["rays_primary"] + fst["rays_reflect"] + fst["rays_refract"] + fst["rays_shadow_traced"],
                           fst["sphere_tests_executed"], fst["box_tests_executed"],
                           fst["rays_primary"] + fst["rays_reflect"] + fst["rays_refract"] + fst["rays_shadow"]],
                          dtype=torch.float64, device=dev)
    if n > 1:
        dist.all_reduce(traced)
    assert float(traced[3]) == rays_per_frame, "fast-path reference ray count differs from the exhaustive count"
    traced_rays = float(traced[0])
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if n > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])

    if rank == 0:
        value = rays_per_frame * a.steps / elapsed / 1e6
        gather_desc = ("library RCCL communicators on the render streams" if isinstance(fa, RcclStreamAssembler)
                       else f"torch.distributed {dist.get_backend() if dist.is_initialized() else ''}".strip())
        out = {
            "metric": METRIC if a.config == "c3" else METRIC_C5,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": (f"c3: {W}x{H}, floor plane + {a.spheres} random spheres (splitmix64 seed 0x5EED0003), "
                             f"1 light, reflect+refract depth {depth}") if a.config == "c3" else
                            (f"c5: {W}x{H}, 4 planes + {a.spheres} random spheres (splitmix64 seed 0x5EED0005), "
                             f"2 lights, reflect+refract depth {depth}"),
                "width": W, "height": H, "spheres": a.spheres, "depth": depth,
                "rays_per_frame": int(rays_per_frame),
                "parallelism": (f"{n} GPUs, one process each: interleaved {B}-row blocks"
                                + (f" (periods of {pattern[0]} blocks, rank 0 {bin(pattern[1][0]).count('1')} and "
                                   f"the others {bin(pattern[1][-1]).count('1')} per period)" if pattern else "")
                                + f", one gather per batch to rank 0 ({gather_desc})" if n > 1
                                else "1 GPU: wavefront pipeline") + f"; batches of {NB} frames on {F} streams",
                "root_share": share if n > 1 else None,
                "frames_in_flight": F * NB,
                "batch": NB,
                "render_streams_n": F,
                "render_streams": kind if F > 1 else "current",
                "assembler": type(fa).__name__ if n > 1 else None,
                "assembler_fallback": assembler_fallback,
                "dist_backend": (dist.get_backend() if n > 1 and dist.is_initialized() else None),
            },
            "roofline": roofline(prof, breakdown, W, H, a, n, ref_work, elapsed / a.steps * 1e3, NB),
            "traced_rays_per_frame": int(traced_rays),
            "traced_mrays_per_s": round(traced_rays * a.steps / elapsed / 1e6, 3),
            "rays_note": "value counts the reference's rays (one per World::intersect call, world.rs:71,101), "
                         "including shadow rays the fast path provably need not trace; traced_* counts what the "
                         "kernels traced",
            "parity": parity,
        }
        if split is not None:
            out["per_rank"] = split
        if n == 1 and not a.no_end_to_end:
            out["end_to_end"] = end_to_end(world, cam, depth, frames=10)
        if n == 1 and a.config == "c3" and not a.no_distinct:
            out["distinct_cameras"] = distinct_cameras(world, depth, rstreams, dev, value)
        if n == 1 and not a.no_cold:
            out["cold_ms"] = cold_start(local_rank)
        if n == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(world, cam, depth, a.cpu_seconds)
        print(json.dumps(out), flush=True)
    if parity is not None and not parity["ok"]:
        raise SystemExit("bench.py: the timed frames differ from the exhaustive frame")
    if n > 1:
        torch.cuda.synchronize()
        if hasattr(fa, "close"):
            fa.close()  # the per-stream RCCL communicators
        dist.destroy_process_group()


def submit(fa, step, end):
    """Frame `step` is rendered (`end`: the last of its batch)."""
    if isinstance(fa, StreamFrameAssembler):
        fa.submit(step, end=end)
    else:
        fa.submit(step)


def phase_split(a, n, rank, dev, run_frames, fa, F, NB):
    """Per-rank frame time of the renders alone and of the assembly alone
    (gathers + rank 0's un-interleave of the same batches), each over K frames
    with a barrier on both sides; collective. Gathered to rank 0."""
    def timed(fn):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3
    render_ms = timed(lambda: run_frames(a.steps, assemble=False))

    def gathers():
        for s in range(0, a.steps, NB):
            nf = min(NB, a.steps - s)
            for j in range(nf):
                submit(fa, s + j, j == nf - 1)
        fa.flush()
    gather_ms = timed(gathers)
    t = torch.tensor([render_ms, gather_ms], dtype=torch.float64, device=dev)
    allt = [torch.empty_like(t) for _ in range(n)] if rank == 0 else None
    dist.gather(t, allt, dst=0)
    if rank != 0:
        return None
    return {"render_ms": [round(float(x[0]), 4) for x in allt], "assemble_ms": [round(float(x[1]), 4) for x in allt],
            "note": "per rank, per frame, outside the timed region: the renders alone and the assembly alone "
                    "(one gather per batch + rank 0's un-interleave), same streams and batches"}


def verify_frames(fa, last, ref_shard, last_step, n, rank, H):
    """Bitwise parity of the benchmarked frames: every rank's last rendered
    shard equals its exhaustive shard, and rank 0's last assembled canvas equals
    the exhaustive shards gathered and un-interleaved the same way. Collective."""
    own = bool(torch.equal(fa.slot(last_step), ref_shard))
    canvas_ok = True
    if n == 1:
        canvas_ok = last is not None and bool(torch.equal(last, ref_shard[:H]))
    else:
        bufs = [torch.empty_like(ref_shard) for _ in range(n)] if rank == 0 else None
        dist.gather(ref_shard, bufs, dst=0)
        if rank == 0:
            ref_canvas = torch.index_select(torch.cat(bufs), 0, fa.inv_idx)
            canvas_ok = last is not None and bool(torch.equal(last, ref_canvas))
    ok = torch.tensor([1.0 if (own and canvas_ok) else 0.0], dtype=torch.float64, device=ref_shard.device)
    if n > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return {"vs_exhaustive": "bitwise", "ok": bool(ok[0] == 1.0),
            "checked": "last timed frame: every rank's shard and rank 0's assembled canvas vs the exhaustive "
                       "(every-shape loop) frame rendered before timing"}


def pmc_summary_path(a, W, H, n, build):
    """The committed PMC summary (tools/profile.sh) of THIS build (its `build`
    field equals rtamd.buildinfo.build_id(), the hash of the library's sources)
    measured on this workload; "" when the kernels benched here were never
    profiled (then the roofline carries no traffic rather than another build's)."""
    if a.pmc_summary:
        return a.pmc_summary
    import glob
    for c in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_summary*.json")), reverse=True):
        try:
            pm = json.load(open(c))
        except (OSError, ValueError):
            continue
        if (pm.get("width"), pm.get("height"), pm.get("spheres"), pm.get("n_gpus"), pm.get("build")) == \
                (W, H, a.spheres, n, build):
            return c
    return ""


def roofline(prof, breakdown, W, H, a, n, ref_work, frame_ms, nb=1):
    """f64 VALU roofline of the dominant kernel (its launches per frame on
    rank 0; with batches, a batch's launches / nb). Its time comes from the
    launch-carried HIP events of the serialized pass (`prof` = `breakdown`),
    like the per-class table."""
    nd, ng, npl = prof["n_diag"], prof["n_gen"], prof["n_planes"]
    fused = bool(prof.get("fused"))
    # the generation pipeline's primary launch uses the shared-origin records (16 ops per test)
    per_sphere = {"primary": OPS_SPHERE_PRIMARY, "closest": OPS_SPHERE_DIAG, "shadow": OPS_SPHERE_DIAG}
    sh_in_r, sh_in_t = prof.get("shadow_rays_in", {}), prof.get("shadow_tests_in", {})

    def class_ops(c):
        # executed work: diag-sphere tests (every sphere per ray when exhaustive, the
        # visited leaves' spheres under the BVH), child-box tests, the rest exhaustively
        ops = (prof["tests"][c] * per_sphere[c] + OPS_BOX * prof["boxes"][c]
               + prof["rays"][c] * (OPS_SPHERE_GEN * ng + OPS_PLANE * npl) + OPS_ROOTS * prof["disc"][c])
        if fused and c in ("primary", "closest"):
            # the fused launches also trace their hits' shadow rays (light buffer: sphere tests only)
            ops += (OPS_SPHERE_DIAG * sh_in_t.get(c, 0.0)
                    + sh_in_r.get(c, 0.0) * (OPS_SPHERE_GEN * ng + OPS_PLANE * npl))
        return ops

    def class_survey_ops(c):
        # SURVEY.md §8(d)'s pricing of the same executed tests: 57 per sphere test, 34 per
        # plane test, +6 per disc >= 0 (the reference's general 4x4 path; boxes unpriced)
        ops = (SURVEY_OPS_SPHERE * (prof["tests"][c] + prof["rays"][c] * ng)
               + SURVEY_OPS_PLANE * prof["rays"][c] * npl + SURVEY_OPS_ROOTS * prof["disc"][c])
        if fused and c in ("primary", "closest"):
            ops += (SURVEY_OPS_SPHERE * (sh_in_t.get(c, 0.0) + sh_in_r.get(c, 0.0) * ng)
                    + SURVEY_OPS_PLANE * sh_in_r.get(c, 0.0) * npl)
        return ops
    kernels = {}
    for c in ("primary", "closest", "shadow"):
        ms_c = breakdown["ms"][c]
        ops_c = class_ops(c)
        kernels[c] = {"ms_per_frame": round(ms_c, 4), "rays": int(prof["rays"][c]),
                      "sphere_tests": int(prof["tests"][c]), "box_tests": int(prof["boxes"][c]),
                      "tflops": round(ops_c / (ms_c * 1e-3) / 1e12, 3) if ms_c > 0 else None}
        if fused and c in ("primary", "closest"):
            kernels[c]["shadow_rays_inside"] = int(sh_in_r.get(c, 0.0))
            kernels[c]["shadow_sphere_tests_inside"] = int(sh_in_t.get(c, 0.0))
    if fused:
        kernels["shadow"]["note"] = "traced inside the fast-path launches (no launch of its own)"
    for c in ("prep", "combine"):
        kernels[c] = {"ms_per_frame": round(breakdown["ms"][c], 4)}
    ms_src = "serialized pass: launch-carried HIP events, one stream, the benched batches"
    dom = max(("primary", "closest", "shadow"), key=lambda c: breakdown["ms"][c])
    kernel_ms = breakdown["ms"][dom]
    ops = class_ops(dom)
    survey_ops = class_survey_ops(dom)
    kname = (f"wf_trace_fused ({dom} launches: closest hit + shading + shadow rays + spawn) in one frame"
             if fused else f"wf_trace_{dom}: its launches in one frame")
    if kernel_ms <= 0:
        return {"bound": "valu_f64", "kernel": None, "achieved": None, "peak": PEAK_F64_VALU_TFLOPS,
                "unit": "TFLOP/s", "frac": None, "traffic": None}
    achieved = ops / (kernel_ms * 1e-3) / 1e12
    achieved_survey = survey_ops / (kernel_ms * 1e-3) / 1e12
    traffic, traffic_src, counters = None, None, None
    from rtamd.buildinfo import build_id
    build = build_id()
    traffic_src = f"no PMC summary of this build ({build}) on this workload in profiles/"
    pmc_path = pmc_summary_path(a, W, H, n, build)
    if pmc_path and os.path.exists(pmc_path):
        a.pmc_summary = pmc_path
        try:
            pm = json.load(open(a.pmc_summary))
            if (pm.get("width"), pm.get("height"), pm.get("spheres"), pm.get("n_gpus"), pm.get("kernel_class"),
                    pm.get("traversal")) == (W, H, a.spheres, n, dom, "bvh" if prof["bvh"] else "exhaustive"):
                traffic, traffic_src = pm.get("hbm_bytes_per_frame"), os.path.relpath(a.pmc_summary, REPO)
                c = pm["per_frame"][dom]
                # SQ_ACTIVE_INST_VALU counts quad-cycles summed over the SIMDs; GRBM_GUI_ACTIVE
                # is summed over the 8 XCDs (MI355X: 256 CUs x 4 SIMDs)
                simd_cycles = c["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0
                counters = {"valu_busy": round(4.0 * c["SQ_ACTIVE_INST_VALU"] / simd_cycles, 3),
                            "f64_valu_insts_per_frame": c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"]
                            + c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_TRANS_F64"],
                            "valu_insts_per_frame": c["SQ_INSTS_VALU"],
                            "build": pm.get("build")}
        except Exception:
            pass
    return {
        "bound": "valu_f64",
        "kernel": kname,
        # achieved / frac: SURVEY.md §8(d)'s pricing of the executed tests (the survey's per-unit figure x
        # the units this kernel's launches process in one frame, / their time)
        "achieved": round(achieved_survey, 3),
        "peak": PEAK_F64_VALU_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved_survey / PEAK_F64_VALU_TFLOPS, 4),
        "pricing": "SURVEY.md §8(d): 57 f64 ops per executed sphere test, 34 per plane test, +6 per "
                   "disc >= 0; box tests unpriced",
        # the same launches priced by the minimum op count of this code (box tests at 9.5, diagonal
        # sphere tests at 28; DESIGN.md 'Roofline')
        "achieved_executed": round(achieved, 3),
        "frac_executed": round(achieved / PEAK_F64_VALU_TFLOPS, 4),
        "traffic": traffic,
        "kernel_ms": round(kernel_ms, 4),
        "kernel_ms_source": ms_src,
        "kernel_regime": (f"serialized: one batch of {nb} frames at a time (the benched launches, each carrying "
                          f"{nb} frames), time per frame = the batch's / {nb}; the timed region keeps several "
                          "batches in flight, so its per-frame time (ms_per_step) can be below kernel_ms"),
        "ops_per_frame": survey_ops,
        "ops_per_frame_executed": ops,
        "per_unit_executed": f"{OPS_SPHERE_DIAG} f64 ops per sphere test ({OPS_SPHERE_PRIMARY} for the generation "
                    f"pipeline's primary rays), {OPS_BOX} per BVH box test, {OPS_PLANE} per plane test, "
                    f"{OPS_ROOTS} per root pair (DESIGN.md 'Roofline'); executed tests counted on the device",
        "traversal": "bvh" if prof["bvh"] else "exhaustive",
        "reference_work_tflops": round(ref_work / (frame_ms * 1e-3) / 1e12, 3),
        "traffic_source": traffic_src,
        "build": build,
        "pmc": counters,
        "kernels": kernels,
    }


if __name__ == "__main__":
    main()
