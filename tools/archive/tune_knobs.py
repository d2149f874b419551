"""A/B runtime tuning knobs on the C3 frame in one process, interleaved
rounds; every variant must reproduce the first variant's image (dev tool).
Usage: tune_knobs.py bvh_leaf=2,3 lb_res=128,256 [--c5] [--no-check]  (knobs: rtamd_tuning_set in rt_api.cpp)
(--no-check: timing experiments whose images differ, e.g. exp=0,1)"""
import itertools, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa
import rtamd
from rtamd import scenes
args = [x for x in sys.argv[1:] if "=" in x]
scene = "c5" if "--c5" in sys.argv else "c3"
knobs = [(k, [int(v) for v in vs.split(",")]) for k, vs in (x.split("=") for x in args)]
SCENE_KNOBS = ("bvh_leaf", "bvh_ct", "lb_res")  # applied at scene creation: one world per value


def make_world():
    if scene == "c5":
        return scenes.c5(1024, 1024)
    return scenes.c3()


worlds = {}
w, cam, depth = make_world()
buf = torch.empty((cam.vsize, cam.hsize, 3), dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
combos = list(itertools.product(*[vs for _, vs in knobs]))
res, ref = {}, None
for r in range(4):
    for combo in combos:
        for (k, _), v in zip(knobs, combo):
            if k in SCENE_KNOBS:
                rtamd._rtamd._tuning_set(k, v)
        skey = tuple(v for (k, _), v in zip(knobs, combo) if k in SCENE_KNOBS)
        if skey not in worlds:
            worlds[skey] = make_world()[0]
            worlds[skey].upload(0)
        w = worlds[skey]
        for (k, _), v in zip(knobs, combo):  # render-time knobs are per scene (WfTuning)
            if k not in SCENE_KNOBS:
                w.tune(k, v)
        rtamd._rtamd._wf_profile(w, 1, False)
        for _ in range(3):
            cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s, False)
        torch.cuda.synchronize()
        p = rtamd._rtamd._wf_profile(w, 0, True)
        lds = (max(int(p["bvh_depth"]), 1) * 4096 + 64 * p["n_bvh_nodes"] + 64 * p["n_diag"]) / 1024
        res.setdefault(combo, []).append((sum(p["ms"].values()), p["ms"], p["tests"], p["boxes"],
                                          f"lb {p['lb_res']:.0f}/{p['lb_items']:.0f} nodes {p['n_bvh_nodes']} depth {p['bvh_depth']} lane-LDS {lds:.0f}KB"))
        chk = buf.cpu().numpy().tobytes()
        ref = ref or chk
        assert chk == ref or "--no-check" in sys.argv, combo
for combo, v in res.items():
    tot, ms, tests, boxes, info = min(v, key=lambda x: x[0])
    name = " ".join(f"{k}={c}" for (k, _), c in zip(knobs, combo))
    print(f"{name}: frame {tot:.3f} ms  " + " ".join(f"{c}={m:.3f}" for c, m in ms.items())
          + "  tests " + " ".join(f"{c}={t/1e6:.0f}M" for c, t in tests.items())
          + "  boxes " + " ".join(f"{c}={t/1e6:.0f}M" for c, t in boxes.items()) + "  " + info, flush=True)
