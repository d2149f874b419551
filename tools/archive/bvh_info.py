"""BVH node count and depth of the C3 scene per leaf size, and of C5 (dev
tool; needs a GPU: the hierarchy is built at upload)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'raytracer-challenge-rs_amd')]
import torch, rtamd
from rtamd import scenes
for lf in (1, 2, 4, 8):
    rtamd._rtamd._tuning_set("bvh_leaf", lf)
    w, cam, depth = scenes.c3()
    w.upload(0)
    p = rtamd._rtamd._wf_profile(w, -1, True)
    print("leaf", lf, "nodes", p["n_bvh_nodes"], "depth", p["bvh_depth"], flush=True)
w, cam, depth = scenes.c5(256, 256)
w.upload(0)
p = rtamd._rtamd._wf_profile(w, -1, True)
print("c5 nodes", p["n_bvh_nodes"], "depth", p["bvh_depth"])
