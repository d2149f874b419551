"""Round-5 measurement probe (dev tool, one GPU).

Sections (--what, comma separated):
  e2e       the drop-in entry point (rt_render -> host Canvas, camera.rs:133-148):
            one frame's render alone, the 49.8 MB device-to-host copy alone, rt_render
            as shipped, and row bands rendered on two streams with each band's copy
            queued behind its render (the overlap the banded rt_render would get)
  assembly  rank 0's budget at N = 8 on C3 (rtamd.distributed): the
            un-interleave of a 16-frame batch, rank 0's shard (7/8) and a full shard
            (6/8) rendered alone in the bench's regime (batches of 16 on 4 streams), and
            rank 0's shard with an emulated receive stream (7 x 6.27 MB per frame
            written into its gather buffer by a copy on a side stream) plus the
            un-interleave behind each batch
  assembly_share  the same with rank 0 rendering a block pattern of --share of an
            equal split (rtamd.distributed.block_patterns), projected N = 8 speedup
  bands     rt_render into a host canvas per (bands, band_pct) knob pair, round-robin
  pow       channels of the fast frame that differ from the oracle (material.rs:76
            powf vs the device pow) on 4096 C3 and 2048 C5 pixels, and how close
            any channel's v*255 comes to a .5 rounding boundary of the PPM quantiser
Prints one JSON object per section.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtamd  # noqa: E402
from rtamd import scenes  # noqa: E402
from rtamd.distributed import StreamFrameAssembler  # noqa: E402


def sync():
    torch.cuda.synchronize()


def timeit(fn, reps):
    fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t0) / reps * 1e3


def e2e(reps):
    w, cam, depth = scenes.c3()
    w.upload(0)
    H, W = cam.vsize, cam.hsize
    dev = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    host = torch.empty((H, W, 3), dtype=torch.float64).pin_memory()
    s0 = torch.cuda.current_stream()
    out = {}
    out["render_only_ms"] = timeit(lambda: cam.render_shard_device(w, depth, 8, 0, 1, dev.data_ptr(), s0.cuda_stream,
                                                                   False), reps)
    out["d2h_only_ms"] = timeit(lambda: host.copy_(dev, non_blocking=True), reps)
    out["d2h_GBps"] = dev.numel() * 8 / out["d2h_only_ms"] / 1e6
    ts = []
    cam.render(w, depth, want_stats=False)
    for _ in range(reps):
        t0 = time.perf_counter()
        cam.render(w, depth, want_stats=False)
        ts.append((time.perf_counter() - t0) * 1e3)
    out["rt_render_ms"] = ts
    for bands, pct in ((1, 55), (2, 50), (2, 55), (2, 60), (3, 40), (3, 50), (4, 34)):  # rt_render's row bands
        w.tune("bands", bands)
        w.tune("band_pct", pct)
        cam.render(w, depth, want_stats=False)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            cam.render(w, depth, want_stats=False)
            ts.append((time.perf_counter() - t0) * 1e3)
        out[f"rt_render_bands{bands}_{pct}_ms"] = sorted(ts)[len(ts) // 2]
    w.tune("bands", 4)
    w.tune("band_pct", 35)
    ref = dev.clone()
    streams = [rtamd.render_stream(False) for _ in range(2)]
    for K in (2, 3, 4, 6, 8):
        rb = (H + K - 1) // K

        def banded():
            for k in range(K):
                y0 = k * rb
                y1 = min(H, y0 + rb)
                st = streams[k % 2]
                cam.render_shard_device(w, depth, rb, k, K, dev[y0:y1].data_ptr(), st.cuda_stream, False)
                with torch.cuda.stream(st):
                    host[y0:y1].copy_(dev[y0:y1], non_blocking=True)
        out[f"banded_{K}_ms"] = timeit(banded, reps)
    dev.fill_(-1)
    banded()
    sync()
    out["banded_bitwise"] = bool(torch.equal(host, ref.cpu()))
    # bands on streams of descending priority: the first band gets the CUs first, so it
    # finishes early and its copy overlaps the later bands' renders
    lo, hi = torch.cuda.Stream.priority_range()
    out["priority_range"] = [lo, hi]
    pstreams = [torch.cuda.Stream(priority=p) for p in sorted({hi, (lo + hi) // 2, lo})]
    out["stream_priorities"] = [s.priority for s in pstreams]
    for K in (2, 3, 4):
        rb = (H + K - 1) // K
        for mode in ("prio", "stagger"):
            evs = [torch.cuda.Event() for _ in range(K)]

            def pbanded():
                for k in range(K):
                    y0 = k * rb
                    y1 = min(H, y0 + rb)
                    st = pstreams[min(k, len(pstreams) - 1)] if mode == "prio" else streams[k % 2]
                    if mode == "stagger" and k > 0:
                        st.wait_event(evs[k - 1])  # band k starts when band k-1's render is done
                    cam.render_shard_device(w, depth, rb, k, K, dev[y0:y1].data_ptr(), st.cuda_stream, False)
                    evs[k].record(st)
                    with torch.cuda.stream(st):
                        host[y0:y1].copy_(dev[y0:y1], non_blocking=True)
            out[f"{mode}_{K}_ms"] = timeit(pbanded, reps)
            dev.fill_(-1)
            pbanded()
            sync()
            out[f"{mode}_{K}_bitwise"] = bool(torch.equal(host, ref.cpu()))
    for K in (2, 3, 4):  # one band alone (render only), for the model
        rb = (H + K - 1) // K
        out[f"band_1of{K}_render_ms"] = timeit(
            lambda: cam.render_shard_device(w, depth, rb, 0, K, dev.data_ptr(), s0.cuda_stream, False), reps)
    return out


def bands(reps):
    """rt_render (host canvas) on C3 per (bands, band_pct), round-robin over the
    configurations so that clock drift hits all of them alike; median and min."""
    w, cam, depth = scenes.c3()
    w.upload(0)
    cfgs = [(1, 50, -1, 100), (4, 35, 1, 100), (4, 30, 1, 100), (5, 30, 1, 100), (5, 25, 1, 100), (6, 25, 1, 100),
            (6, 20, 1, 100), (8, 20, 1, 100), (8, 15, 1, 100), (6, 30, 1, 80), (8, 25, 1, 80), (5, 30, 2, 100),
            (6, 25, 2, 100), (6, 25, 0, 100), (8, 20, 0, 100)]
    ts = {c: [] for c in cfgs}

    def setc(c):
        w.tune("bands", c[0])
        w.tune("band_pct", c[1])
        w.tune("band_gen", c[2])
        w.tune("band_ratio", c[3])
    ref = None
    for c in cfgs:  # warm every configuration's workspaces; every frame bitwise equal
        setc(c)
        img = cam.render(w, depth, want_stats=False)[0].to_numpy().tobytes()
        ref = ref or img
        assert img == ref, c
    for _ in range(reps):
        for c in cfgs:
            setc(c)
            t0 = time.perf_counter()
            cam.render(w, depth, want_stats=False)
            ts[c].append((time.perf_counter() - t0) * 1e3)
    setc((4, 35, 1, 100))
    return {f"bands{b}_{p}_gen{g}_r{r}": {"median_ms": round(sorted(v)[len(v) // 2], 4), "min_ms": round(min(v), 4)}
            for (b, p, g, r), v in ts.items()}


def assembly(reps, share=None):
    """Rank 0's cost at N = 8 on C3, measured on one GPU: rank 0's rows and a full
    rank's rows rendered alone in the bench's regime (batches of 16 on 4 streams),
    then rank 0's rows with its receive emulated (the 7 peers' shards of each batch
    copied into its gather buffer by a side stream, 7 x ~6.3 MB per frame) and the
    un-interleave (index_select through the inverse row map) behind each batch, as
    RcclStreamAssembler queues it. `share`: rank 0's share of an equal split (block
    patterns, rtamd.distributed.block_patterns); None = the plain interleave."""
    from rtamd.distributed import block_patterns
    w, cam, depth = scenes.c3()
    w.upload(0)
    w.tune("shadow_stream", 0)
    H, W, B, N, NB, F = cam.vsize, cam.hsize, 8, 8, 16, 4
    pattern = block_patterns(N, share) if share is not None and share < 1.0 else None
    out = {"config": "C3 1920x1080, N=8, 8-row blocks, batches of 16 on 4 streams",
           "root_share": share if pattern else 1.0,
           "pattern": {"period": pattern[0], "blocks_per_period": [bin(m).count("1") for m in pattern[1]]}
           if pattern else None}
    fa = StreamFrameAssembler(H, W, B, 0, N, torch.device("cuda", 0), slots=F, batch=NB, pattern=pattern)
    gb, cv = fa.gather_buf[0], fa.canvas[0]
    out["gather_buf_MB"] = gb.numel() * 8 / 1e6
    out["unweave_batch_ms"] = timeit(lambda: torch.index_select(gb, 0, fa.inv_batch, out=cv), reps)
    out["unweave_per_frame_ms"] = out["unweave_batch_ms"] / NB
    rstreams = [rtamd.render_stream(False) for _ in range(F)]
    rx_stream = torch.cuda.Stream()

    def rows_of(r):
        if pattern:
            return rtamd.pattern_rows(H, B, pattern[0], pattern[1][r])
        return rtamd.shard_rows(H, B, N - 1 - r, N)

    def render(r, cams, ptrs, st):
        if pattern:
            rtamd.render_block_pattern_device(w, cams, depth, B, pattern[0], pattern[1][r], ptrs, st)
        else:
            rtamd.render_frames_device(w, cams, depth, B, N - 1 - r, N, ptrs, st)
    rmax = max(range(1, N), key=rows_of)  # the peer with the most rows
    out["rows_rank0"], out["rows_peer_max"], out["peer_max_rank"] = rows_of(0), rows_of(rmax), rmax
    out["rx_MB_per_frame"] = sum(rows_of(r) for r in range(1, N)) * W * 24 / 1e6
    bufs = {r: [torch.empty((NB, rows_of(r), W, 3), dtype=torch.float64, device="cuda") for _ in range(F)]
            for r in (0, rmax)}
    peers = torch.empty(((N - 1) * NB * fa.max_rows, W, 3), dtype=torch.float64, device="cuda")
    frames = 64

    def run(r, rx=False, unweave=False):
        for b in range(frames // NB):
            k = b % F
            rs = rstreams[k]
            render(r, [cam] * NB, [bufs[r][k][j].data_ptr() for j in range(NB)], rs.cuda_stream)
            if rx:  # the 7 peers' shards of this batch land in the gather buffer
                with torch.cuda.stream(rx_stream):
                    fa.gather_buf[k][fa.max_rows * NB:].copy_(peers, non_blocking=True)
                rs.wait_stream(rx_stream)
            if unweave:
                with torch.cuda.stream(rs):
                    torch.index_select(fa.gather_buf[k], 0, fa.inv_batch, out=fa.canvas[k])

    for label, r, rx, uw in (("render_rank0", 0, False, False), ("render_peer_max", rmax, False, False),
                             ("rank0_rx", 0, True, False), ("rank0_unweave", 0, False, True),
                             ("rank0_rx_unweave", 0, True, True)):
        out[label + "_ms_per_frame"] = timeit(lambda: run(r, rx, uw), max(1, reps // 2)) / frames
    out["rx_copy_alone_ms_per_frame"] = timeit(lambda: fa.gather_buf[0][fa.max_rows * NB:].copy_(peers), reps) / NB
    whole = [torch.empty((H, W, 3), dtype=torch.float64, device="cuda") for _ in range(8 * F)]

    def run_whole():
        for b in range(frames // 8):
            k = b % F
            rtamd.render_frames_device(w, [cam] * 8, depth, B, 0, 1, [whole[k * 8 + j].data_ptr() for j in range(8)],
                                       rstreams[k].cuda_stream)
    out["whole_frame_ms"] = timeit(run_whole, max(1, reps // 2)) / frames
    t_root = out["rank0_rx_unweave_ms_per_frame"]
    t_peer = out["render_peer_max_ms_per_frame"]
    out["projection"] = {
        "rank0_ms": t_root, "peer_render_ms": t_peer, "frame_ms": max(t_root, t_peer),
        "speedup_vs_1gpu": out["whole_frame_ms"] / max(t_root, t_peer),
        "xgmi_ms_per_frame_at_64GBps_per_link": rows_of(rmax) * W * 24 / 64e9 * 1e3,
        "xgmi_ms_per_frame_at_50GBps_per_link": rows_of(rmax) * W * 24 / 50e9 * 1e3,
        "note": "one GPU: rank 0's receive is a device copy on a side stream; the peers' sends and the xGMI "
                "link time (each peer's shard over its own link, overlapped with later batches) are not "
                "measured: a peer's link carries rows_peer_max x W x 24 B per frame"}
    del fa, bufs, peers, whole
    torch.cuda.empty_cache()
    return out


def pow_ulps():
    from oracle import pyoracle
    out = {}
    nthreads = 16
    for name, n, seed in (("c3", 4096, 3), ("c5", 2048, 5)):
        w, cam, depth = getattr(scenes, name)()
        buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
        cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), torch.cuda.current_stream().cuda_stream, False)
        sync()
        rng = np.random.default_rng(seed)
        xy = np.stack([rng.integers(0, cam.hsize, n), rng.integers(0, cam.vsize, n)], 1)
        ow = pyoracle.OracleWorld.from_world(w)
        ref, _ = ow.render_pixels(cam.desc_bytes(), depth, xy, nthreads)
        got = buf[xy[:, 1], xy[:, 0]].cpu().numpy()
        d = got - ref
        ulps = np.abs(got.view(np.int64) - ref.view(np.int64))
        s = ref * 255.0
        dist = np.abs(s - np.floor(s) - 0.5)  # distance of v*255 from the nearest .5 (quantiser boundary)
        diff = d != 0
        out[name] = {"pixels": n, "channels": int(d.size), "channels_differ": int(diff.sum()),
                     "differing_min_dist_to_half_of_v255": float(dist[diff].min()) if diff.any() else None,
                     "max_abs_delta": float(np.abs(d).max()), "max_ulps": int(ulps.max()),
                     "min_dist_to_half_of_v255": float(dist.min()),
                     "ppm_same": rtamd.canvas_to_ppm(got[None]) == pyoracle.canvas_to_ppm(ref[None])}
        del buf
        torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="e2e,assembly,pow")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--share", type=float, default=0.75, help="assembly_share: rank 0's share of an equal split")
    a = ap.parse_args()
    for what in a.what.split(","):
        t0 = time.perf_counter()
        res = {"e2e": lambda: e2e(a.reps), "assembly": lambda: assembly(a.reps),
               "assembly_share": lambda: assembly(a.reps, a.share), "pow": pow_ulps,
               "bands": lambda: bands(a.reps)}[what]()
        res["section"] = what
        res["seconds"] = round(time.perf_counter() - t0, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
