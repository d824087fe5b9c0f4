"""Per-pixel traversal work of the bench frame (instrumented persistent engine,
TMPT_COST_MAP=1) and a list-scheduling model of one rank's shard: how much of
the N-GPU frame time is the per-pixel chain and how much is pixel order.

  python tools/cost_map.py [spp] [out.npy]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import heapq  # noqa: E402

import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402
from toymeshpathtracer_amd import shard  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out", "cost_map.npy")
W, H = 1920, 1080
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=True)
sc = tm.Scene(tris)
os.environ["TMPT_COST_MAP"] = "1"
img, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_PERSISTENT,
                           band_rows=16, count_visits=True)
cost = np.ascontiguousarray(img).view(np.uint32).reshape(H, W).astype(np.int64)
os.makedirs(os.path.dirname(out), exist_ok=True)
np.save(out, cost)
tot = cost.sum()
print(f"rays {rays}, work {tot} (node visits + tri tests), per pixel mean {cost.mean():.0f} "
      f"max {cost.max()} p50 {np.percentile(cost, 50):.0f} p90 {np.percentile(cost, 90):.0f} "
      f"p99 {np.percentile(cost, 99):.0f} p99.9 {np.percentile(cost, 99.9):.0f}")
rowm = cost.mean(1)
print("row means (every 60th row):", " ".join(f"{v:.0f}" for v in rowm[::60]))


def schedule(costs, lanes):
    """Greedy list scheduling: each free lane takes the next pixel in order."""
    if len(costs) <= lanes:
        return int(costs.max())
    h = list(costs[:lanes])
    heapq.heapify(h)
    for c in costs[lanes:]:
        t = heapq.heappop(h)
        heapq.heappush(h, t + int(c))
    return max(h)


lanes = 131072
for n in (1, 8):
    rows = shard.all_rows(H, 16, n)[0]
    c = cost[rows].ravel()
    ideal = c.sum() / lanes
    for name, order in (("index", c), ("reverse", c[::-1]), ("LPT", np.sort(c)[::-1]),
                        ("random", np.random.default_rng(0).permutation(c))):
        mk = schedule(order, lanes)
        print(f"N={n} shard0 {len(c)} px: {name:>7} makespan {mk:>9} work units = "
              f"{mk / ideal:5.2f}x the balanced {ideal:.0f}; max pixel {c.max()}")
