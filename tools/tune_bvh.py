"""A/B the BVH knobs in one process, interleaved rounds (dev tool):
leaf size (scene rebuilt per value) x trace occupancy (4 / 8 waves per SIMD)."""
import os, sys, statistics, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "raytracer-challenge-rs_amd")]
import torch  # noqa
import rtamd
from rtamd import scenes
leaves = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8").split(",")]
waves = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "8,4").split(",")]
worlds = {}
for lf in leaves:
    rtamd._rtamd._tuning_set("bvh_leaf", lf)
    w, cam, depth = scenes.c3()
    w.upload(0)
    worlds[lf] = w
buf = torch.empty((1080, 1920, 3), dtype=torch.float64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
res = {}
ref = None
for r in range(4):
    for lf, w in worlds.items():
        for tw in waves:
            rtamd._rtamd._tuning_set("wf_waves", tw)
            rtamd._rtamd._wf_profile(w, 1, False)
            for _ in range(3):
                cam.render_shard_device(w, depth, 8, 0, 1, buf.data_ptr(), s, False)
            torch.cuda.synchronize()
            p = rtamd._rtamd._wf_profile(w, 0, True)
            tot = sum(p["ms"].values())
            res.setdefault((lf, tw), []).append((tot, p["ms"]))
            chk = buf.cpu().numpy().tobytes()
            if ref is None:
                ref = chk
            assert chk == ref, (lf, tw)
for k, v in sorted(res.items()):
    best = min(v, key=lambda x: x[0])
    print(f"leaf={k[0]} waves={k[1]}: best frame {best[0]:.3f} ms  " +
          " ".join(f"{c}={m:.3f}" for c, m in best[1].items()), flush=True)
