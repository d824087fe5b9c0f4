"""Interleaved A/B of traversal-kernel variants (TMPT_TUNE) in ONE process on
the bench frame (sponza stand-in 1920x1080, pixel seeding).  Prints per-variant
MRays/s (median over rounds) and the extend/shadow kernel times."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

variants = sys.argv[1].split(";") if len(sys.argv) > 1 else ["32,8,16"]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
W, H = 1920, 1080
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=True)
sc = tm.Scene(tris)
res = {v: [] for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        os.environ["TMPT_TUNE"] = v
        t0 = time.perf_counter()
        img, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_PIXEL)
        dt = time.perf_counter() - t0
        st = sc.stats()
        if ref is None:
            ref = img
        assert np.array_equal(img, ref), v
        res[v].append((rays / dt / 1e6, st.extend_ms, st.shadow_ms, dt * 1e3))
for v, xs in res.items():
    a = np.array(xs)
    print(f"{v:>12}: {np.median(a[:,0]):8.1f} MRays/s  extend {np.median(a[:,1]):7.1f} ms  shadow {np.median(a[:,2]):7.1f} ms  frame {np.median(a[:,3]):7.1f} ms", flush=True)
