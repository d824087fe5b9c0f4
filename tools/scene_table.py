"""MRays/s and algorithmic-HBM roofline fraction per scene and per-rank load
(BASELINE.json configs + the other data/*.obj scenes), for DESIGN.md.

For each config: node visits / triangle tests per query from an instrumented
render (count_visits, 4 spp, sample seeding) give B_ray = 48 + 64 N_node +
36 N_tri; then shard 0 of N (1-row bands, as bench.py deals them)
is timed for N = 1, 2, 4, 8 in sample seeding, and the whole frame in row
seeding (the reference's own RNG) where it is at most 1080p x 64 spp.
Per-rank rate = shard-0 rays / shard-0 time; the N-GPU aggregate is
projected as all rays / shard-0 time (bench.py measures the real one).

  python tools/scene_table.py [rounds]     -> one JSON line per config + a markdown table
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

PEAK = 8.0e12
CONFIGS = [  # name, obj, W, H, spp, is_sponza
    ("triangle640", "triangle.obj", 640, 360, 4, False),
    ("cube640", "cube.obj", 640, 360, 4, False),           # configs[0]
    ("suzanne640", "suzanne.obj", 640, 360, 4, False),     # configs[1]
    ("teapot720", "teapot.obj", 1280, 720, 16, False),     # configs[2]
    ("sponza1080", "sponza", 1920, 1080, 64, True),        # configs[3]
    ("sponza4k", "sponza", 3840, 2160, 256, True),         # configs[4]
]


def timed(fn, rounds):
    fn()  # warm
    ts = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), r


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    rows_out = []
    for name, obj, W, H, spp, sponza in CONFIGS:
        path = gen_standin_sponza.ensure() if obj == "sponza" else os.path.join(ROOT, "data", obj)
        tris, bmin, bmax = tm.load_scene(path)
        cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=sponza)
        # the reference's octree (main.cpp:312): its tie order and root box,
        # as bench.py renders (TABLE_OCTREE=0: ties by index, round-3 table)
        with tm.Scene(tris, bounds=None if os.environ.get("TABLE_OCTREE") == "0" else (bmin, bmax)) as sc:
            cw, ch = min(W, 1920), min(H, 1080)  # visit counts on at most the 1080p frame
            ccam = tm.Camera.for_scene(bmin, bmax, cw, ch, is_sponza=sponza)
            _, q = sc.trace_image(ccam, cw, ch, 4, seed_mode=tm.SEED_SAMPLE, band_rows=1, count_visits=True)
            st = sc.stats()
            nn = (st.node_visits + st.shadow_node_visits) / q
            nt = (st.tri_tests + st.shadow_tri_tests) / q
            b_ray = 48 + 64 * nn + 36 * nt
            rec = {"config": name, "tris": int(len(tris)), "W": W, "H": H, "spp": spp,
                   "n_node": round(nn, 3), "n_tri": round(nt, 3), "bytes_per_ray": round(b_ray, 1), "sample": {}}
            total = None
            for n in (1, 2, 4, 8):
                dt, (_, rays) = timed(lambda: sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1,
                                                             shard=0, num_shards=n), rounds)
                if n == 1:
                    total = rays
                rate = rays / dt
                rec["sample"][n] = {"ms": round(dt * 1e3, 2), "rank_mrays": round(rate / 1e6, 1),
                                    "agg_mrays": round(total / dt / 1e6, 1), "frac": round(rate * b_ray / PEAK, 4)}
            if W * H * spp <= 1920 * 1080 * 64:
                dt, (_, rays) = timed(lambda: sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_ROW), max(1, rounds - 1))
                rec["row"] = {"ms": round(dt * 1e3, 1), "mrays": round(rays / dt / 1e6, 1)}
        print(json.dumps(rec), flush=True)
        rows_out.append(rec)
    print("\n| config | tris | B_ray | N=1 MRays/s (frac) | N=2 agg | N=4 agg | N=8 agg | row seeding MRays/s |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows_out:
        s = r["sample"]
        print(f"| {r['config']} {r['W']}x{r['H']}x{r['spp']} | {r['tris']} | {r['bytes_per_ray']:.0f} | "
              f"{s[1]['rank_mrays']:.0f} ({s[1]['frac']:.2f}) | {s[2]['agg_mrays']:.0f} | {s[4]['agg_mrays']:.0f} | "
              f"{s[8]['agg_mrays']:.0f} | {r['row']['mrays'] if 'row' in r else '-'} |")


if __name__ == "__main__":
    main()
