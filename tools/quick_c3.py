"""Quick C3 timing probe (dev tool): renders the headline frame a few times."""
import os, sys, time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracer-challenge-rs_amd")]
import rtamd
from rtamd import scenes
w, cam, depth = scenes.c3()
t = time.time(); w.upload(); print("upload", time.time() - t, flush=True)
for i in range(3):
    t = time.time()
    canvas, st = cam.render(w, depth)
    dt = time.time() - t
    n = st["rays_primary"] + st["rays_reflect"] + st["rays_refract"] + st["rays_shadow"]
    print(f"iter {i}: wall {dt*1e3:.1f} ms kernel {st['ms_kernel']:.2f} ms rays {n} -> {n/st['ms_kernel']/1e3:.1f} Mrays/s", st, flush=True)
