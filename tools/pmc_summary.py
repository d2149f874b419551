"""Summarise rocprofv3 PMC passes of the bench workload per kernel class (dev tool).

Usage: pmc_summary.py OUT.json [--width W --height H --spheres S --n-gpus N
       --dominant CLASS] DIR [DIR ...]
Each DIR holds one --pmc pass (*_counter_collection.csv). Counters are summed
over all dispatches of a kernel class and divided by the number of frames
(= wf_frame_init dispatches, one per render call, x --batch frames per call),
i.e. per-FRAME values of that class's launches — the same unit as bench.py's
roofline.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) under-reports a
wide coalesced stream by 2x on gfx950, so hbm_read = 2 * FETCH_SIZE * 1024 is
an upper estimate; WRITE_SIZE (KiB) is exact for 16-B stores.
"""
import argparse, collections, csv, glob, json

def _targs(n, name):
    i = n.index(name + "<") + len(name) + 1
    return [t.strip() for t in n[i:n.index(">", i)].split(",")]


def klass(n):
    """Kernel class of a demangled name: primary / closest / shadow / prep /
    combine / frame (wf_frame_init: one per rendered frame)."""
    if "wf_walk<" in n:  # split generation's walk launch (WfTuning::split): closest hits only
        return "walk_primary" if _targs(n, "wf_walk")[1] == "true" else "walk"
    if "wf_trace_fused<" in n:  # fused generation: closest hit + shading + shadow rays + spawn
        # generation 0 of a camera render: PRIMARY (the wave traversal) or CAM (the per-lane
        # walks over the LDS images read camera rays: template argument 5); SPLIT (argument 6):
        # a split generation's shading launch
        t = _targs(n, "wf_trace_fused")
        prim = t[0] == "true" or (len(t) >= 5 and t[4] == "true")
        if len(t) >= 6 and t[5] == "true":
            return "shade_primary" if prim else "shade"
        return "primary" if prim else "closest"
    if "wf_trace_closest_bvh<" in n:
        return "primary" if _targs(n, "wf_trace_closest_bvh")[0] == "true" else "closest"
    if "wf_trace_closest<" in n:
        return "primary" if _targs(n, "wf_trace_closest")[1] == "true" else "closest"
    if "wf_trace_shadow" in n:
        return "shadow"
    if "wf_prep(" in n:
        return "prep"
    if "wf_combine(" in n or "wf_combine_parents(" in n or "wf_average(" in n:
        return "combine"
    if "wf_frame_init(" in n or "wf_prim_prep(" in n:
        return "frame"
    return None


ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("dirs", nargs="+")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--spheres", type=int, default=1000)
ap.add_argument("--n-gpus", type=int, default=1)
ap.add_argument("--dominant", default="closest")
ap.add_argument("--traversal", default="bvh", help="bvh (fast path) or exhaustive")
ap.add_argument("--build", default=None, help="the build the passes profiled (git describe / tag)")
ap.add_argument("--batch", type=int, default=1, help="frames per render call (rt_render_frames_device)")
a = ap.parse_args()

tot = collections.defaultdict(lambda: collections.defaultdict(float))
frames = {}
for d in a.dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            c = klass(r["Kernel_Name"])
            if c is None:
                continue
            if c == "frame":  # one frame_init dispatch per rendered frame (batch)
                seen.add(r["Dispatch_Id"])
            if c == "frame":
                continue
            tot[c][r["Counter_Name"]] += float(r["Counter_Value"])
        frames[f] = len(seen)
nf = (max(frames.values()) if frames else 0) * max(1, a.batch)
res = {"width": a.width, "height": a.height, "spheres": a.spheres, "n_gpus": a.n_gpus, "traversal": a.traversal,
       "frames_per_pass": nf, "batch": max(1, a.batch), "per_frame": {}, "build": a.build}
for c, cs in tot.items():
    pf = {k: v / max(nf, 1) for k, v in cs.items()}
    if "FETCH_SIZE" in pf or "WRITE_SIZE" in pf:
        fetch = pf.get("FETCH_SIZE", 0.0) * 1024
        write = pf.get("WRITE_SIZE", 0.0) * 1024
        pf["hbm_read_bytes_raw"] = fetch
        pf["hbm_read_bytes_corrected"] = 2 * fetch
        pf["hbm_write_bytes"] = write
        pf["hbm_bytes"] = 2 * fetch + write
    res["per_frame"][c] = pf
dom = res["per_frame"].get(a.dominant, {})
res["kernel_class"] = a.dominant
res["hbm_bytes_per_frame"] = dom.get("hbm_bytes")
json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)
print(json.dumps(res, indent=1, sort_keys=True))
