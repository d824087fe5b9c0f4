"""Same-process A/B of render options on one data/*.obj config, interleaved:
  python tools/scene_ab.py teapot.obj 1280 720 16 "sample_block=1;" [rounds] [shards]
Prints the median k_path ms per option set (sample seeding, the octree built)."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import toymeshpathtracer_amd as tm  # noqa: E402

name, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
variants = sys.argv[5].split(";")
rounds = int(sys.argv[6]) if len(sys.argv) > 6 else 20
shards = int(sys.argv[7]) if len(sys.argv) > 7 else 1
tris, bmin, bmax = tm.load_scene(os.path.join(ROOT, "data", name))
cam = tm.Camera.for_scene(bmin, bmax, w, h)
res = {v: [] for v in variants}
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
    defaults = {}
    for r in range(rounds + 1):
        for v in variants:
            for k, val in defaults.items():
                sc.set_option(k, val)
            for kv in filter(None, v.split(",")):
                k, _, val = kv.partition("=")
                defaults.setdefault(k, sc.get_option(k))
                sc.set_option(k, float(val))
            sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1, num_shards=shards)
            if r:
                res[v].append(sc.stats().extend_ms)
for v in variants:
    print(f"{name} {w}x{h}x{spp} 1/{shards} [{v or 'default'}]: {statistics.median(res[v]):.3f} ms", flush=True)
