"""Per-pixel traversal work split into closest-hit and shadow queries (instrumented
persistent engine, TMPT_COST_MAP=1 total / 2 shadow only): how much of the
heaviest pixels' chains are shadow queries (which feed neither the RNG stream
nor the path, main.cpp:57-67, so could run off the chain).
  python tools/cost_split.py [spp]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
W, H = 1920, 1080
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=True)
sc = tm.Scene(tris)
maps = {}
for mode in (1, 2):
    os.environ["TMPT_COST_MAP"] = str(mode)
    img, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_PERSISTENT,
                               count_visits=True)
    maps[mode] = np.ascontiguousarray(img).view(np.uint32).reshape(-1).astype(np.int64)
tot, sh = maps[1], maps[2]
print(f"spp {spp}: work/pixel mean {tot.mean():.0f} max {tot.max()}; shadow share overall "
      f"{sh.sum() / tot.sum() * 100:.1f}%")
order = np.argsort(-tot)
for q in (0.0001, 0.001, 0.01, 0.05, 0.1, 0.25, 0.5, 1.0):
    k = max(1, int(len(tot) * q))
    sel = order[:k]
    print(f"  heaviest {q * 100:7.2f}% ({k:7d} px): work mean {tot[sel].mean():8.0f}, shadow share "
          f"{sh[sel].sum() / tot[sel].sum() * 100:5.1f}%, closest-hit-only max {np.max(tot[sel] - sh[sel])}")
ce = tot - sh
print(f"  max total {tot.max()} -> max closest-hit-only {ce.max()} ({ce.max() / tot.max() * 100:.1f}%)")
